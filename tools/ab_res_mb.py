#!/usr/bin/env python3
"""A/B of the resident kernel's wave-level temporal blocking (GOL_DEV_RES_MB:
1 = life_res_kernel, swaps every generation; 2..4 = life_resident_mb.hip) and of
the resident plan (rows per wavefront, epoch K via resident=2) at the C2 field,
in ONE process, interleaved rounds: wall-clock TCUPS per 1000 generations
(median and best of the rounds), and whether every variant's digest agrees.

    python tools/ab_res_mb.py [--size 4096] [--rule ref] [--rounds 7]
        [--variants auto:1,auto:2,auto:3,4x24:2,...]   (rows x K : MB; auto = the planner's)
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--rule", default="ref")
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--variants", default="auto:1,auto:2,auto:3")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    n = a.size
    engines = []
    for v in a.variants.split(","):
        plan, mb = v.split(":")
        os.environ["GOL_DEV_RES_MB"] = mb
        kw = {}
        if plan != "auto":
            rows, K = (int(x) for x in plan.split("x"))
            kw = dict(resident=2, rows_per_wave=rows, tb_depth=K)
        try:
            e = pkg.Engine(n, n, rule=rule, device=0, **kw)
        except pkg.GolError as ex:
            print(json.dumps({"variant": v, "error": str(ex)}), flush=True)
            continue
        e.init_random(1)
        e.step(a.gens)
        e.sync()
        engines.append((v, e, []))
    os.environ.pop("GOL_DEV_RES_MB", None)
    for _ in range(a.rounds):
        for v, e, ts in engines:
            t0 = time.perf_counter()
            e.step(a.gens)
            e.sync()
            ts.append(time.perf_counter() - t0)
    digests = {e.digest() for _, e, _ in engines}
    cells = float(n) * n * a.gens
    for v, e, ts in engines:
        print(json.dumps({
            "size": n, "rule": a.rule, "variant": v, "resident_rows": e.resident_rows,
            "resident": e.resident, "gens": a.gens,
            "tcups_median": round(cells / statistics.median(ts) / 1e12, 2),
            "tcups_best": round(cells / min(ts) / 1e12, 2),
            "ms_median": round(statistics.median(ts) * 1e3, 4),
            "digests_equal": len(digests) == 1}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
