#!/usr/bin/env python3
"""A/B of an engine planning knob read from the environment at gol_create (e.g.
GOL_DEV_PAIRS, the packed half strip; GOL_DEV_AGE_SKEW) in ONE process,
interleaved rounds: one single-stream engine per value, wall-clock TCUPS (median
of the rounds), kernel time per launch, work ratio, and whether every variant's
field digest agrees after the same generations.

    python tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto \
        [--shapes 65536,8448,32768x262144] [--rule ref] [--gens 512] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

# engines of this tool are stepped one at a time: no waiting-kernel registry
os.environ.setdefault("GOL_DEV_SHARED_WAITS", "1")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--var", default="GOL_DEV_PAIRS")
    p.add_argument("--values", default="0,auto", help="auto = unset")
    p.add_argument("--shapes", default="65536,8448")
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--gens", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--rule", default="ref")
    p.add_argument("--lib", default="", help="library build to load (GOL_LIB), dev A/B")
    p.add_argument("--handoff", type=int, default=0)
    a = p.parse_args()
    if a.lib:
        os.environ["GOL_LIB"] = os.path.abspath(a.lib)
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    for sh in a.shapes.split(","):
        h, w = (int(x) for x in sh.split("x")) if "x" in sh else (int(sh), a.width)
        engines = []
        for v in a.values.split(","):
            if v == "auto":
                os.environ.pop(a.var, None)
            else:
                os.environ[a.var] = v
            e = pkg.Engine(h, w, rule=rule, device=0, handoff=a.handoff, streams=1, resident=1)
            e.init_random(1)
            e.step(a.gens)  # warm-up (graph capture)
            e.sync()
            engines.append((v, e, []))
        os.environ.pop(a.var, None)
        for _ in range(a.rounds):
            for v, e, ts in engines:
                t0 = time.perf_counter()
                e.step(a.gens)
                e.sync()
                ts.append(time.perf_counter() - t0)
        digests = {e.digest() for _, e, _ in engines}
        for v, e, ts in engines:
            e.set_timing(1)
            e.reset_timing()
            e.step(a.gens)
            e.sync()
            tm = e.timing()
            e.set_timing(0)
            cells = float(h) * w * a.gens
            print(json.dumps({
                "lib": os.path.basename(os.environ.get("GOL_LIB", "libgol.so")),
                "shape": f"{h}x{w}", "rule": a.rule, a.var: v,
                "handoff": e.handoff, "tb_depth": e.tb_depth, "rows_per_wave": e.rows_per_wave,
                "age_skew": e.age_skew, "gens": a.gens,
                "tcups_wall_median": round(cells / statistics.median(ts) / 1e12, 2),
                "tcups_wall_best": round(cells / min(ts) / 1e12, 2),
                "kernel_us_avg": round(tm["kernel_ms"] / max(tm["launches"], 1) * 1e3, 2),
                "work_ratio": round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1), 4),
                "digests_equal": len(digests) == 1}), flush=True)
            e.close()


if __name__ == "__main__":
    main()
