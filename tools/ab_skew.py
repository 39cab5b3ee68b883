#!/usr/bin/env python3
"""A/B of age-skewed row blocks (plan.cpp age_skew) in ONE process, interleaved
rounds: single-stream engines of the per-GPU stripe shapes built with
GOL_DEV_AGE_SKEW = each value of --rhos (0 = equal blocks), wall-clock TCUPS
(median of the rounds), the plan, and whether every variant's field digest
agrees after the same generations.

    python tools/ab_skew.py [--shapes 8448,16640,33024] [--rhos 0,auto] [--handoffs 0,1]
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
    p.add_argument("--shapes", default="8448,16640,33024")
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--rhos", default="0,auto", help="GOL_DEV_AGE_SKEW values; auto = unset")
    p.add_argument("--handoffs", default="0")
    p.add_argument("--gens", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--rule", default="ref")
    p.add_argument("--streams", default="1", help="gol_config.streams values (0 = auto)")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    for sh in a.shapes.split(","):
        h, w = (int(x) for x in sh.split("x")) if "x" in sh else (int(sh), a.width)
        for ho in (int(x) for x in a.handoffs.split(",")):
            engines = []
            for st in (int(x) for x in a.streams.split(",")):
                for rho in a.rhos.split(","):
                    if rho == "auto":
                        os.environ.pop("GOL_DEV_AGE_SKEW", None)
                    else:
                        os.environ["GOL_DEV_AGE_SKEW"] = rho
                    e = pkg.Engine(h, w, rule=rule, device=0, handoff=ho, streams=st, resident=1)
                    e.init_random(1)
                    e.step(a.gens)  # warm-up (graph capture)
                    e.sync()
                    engines.append(((rho, st), e, []))
            os.environ.pop("GOL_DEV_AGE_SKEW", None)
            for _ in range(a.rounds):
                for rho, e, ts in engines:
                    t0 = time.perf_counter()
                    e.step(a.gens)
                    e.sync()
                    ts.append(time.perf_counter() - t0)
            digests = {e.digest() for _, e, _ in engines}
            for rho, e, ts in engines:
                e.set_timing(1)
                e.reset_timing()
                e.step(a.gens)
                e.sync()
                tm = e.timing()
                e.set_timing(0)
                cells = float(h) * w * a.gens
                print(json.dumps({
                    "shape": f"{h}x{w}", "rule": a.rule, "handoff_cfg": ho,
                    "streams_cfg": rho[1], "streams": tm.get("streams", 1),
                    "handoff": e.handoff, "tb_depth": e.tb_depth, "rows_per_wave": e.rows_per_wave,
                    "rho": rho[0], "age_skew": e.age_skew, "gens": a.gens,
                    "tcups_wall_median": round(cells / statistics.median(ts) / 1e12, 2),
                    "tcups_wall_best": round(cells / min(ts) / 1e12, 2),
                    "kernel_us_avg": round(tm["kernel_ms"] / max(tm["launches"], 1) * 1e3, 2),
                    "digests_equal": len(digests) == 1}), flush=True)
                e.close()


if __name__ == "__main__":
    main()
