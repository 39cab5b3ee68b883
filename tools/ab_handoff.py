#!/usr/bin/env python3
"""A/B of the row-block hand-off (gol_config.handoff) on the per-GPU shapes of the
C3/C4 configs, in ONE process, interleaved rounds (cdna_hip_programming.md §5.4
rule 24).  Shapes: the default 65536^2 engine (composite, 2 streams) and single
stripes of R + 2 x 128 rows x 65536 (the per-rank field of 2/4/8-way 65536^2).
Prints one JSON line per (shape, handoff) with wall-clock TCUPS (median of the
rounds), the plan (K, R, hand-off), and the work ratio cell_gens_computed /
cell_gens from the engine's HIP-event timing (separate timed pass).

    python tools/ab_handoff.py [--gens 512] [--rounds 5] [--rule ref]
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
    p.add_argument("--gens", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--rule", default="ref")
    p.add_argument("--shapes", default="65536c,33024,16640,8448")
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--handoffs", default="1,2")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    engines = []
    for sh in a.shapes.split(","):
        comp = sh.endswith("c")
        h = int(sh.rstrip("c"))
        for ho in (int(x) for x in a.handoffs.split(",")):
            e = pkg.Engine(h, a.width, rule=rule, device=0, handoff=ho,
                           streams=0 if comp else 1)
            e.init_random(1)
            e.step(a.gens)  # warm-up (graph capture)
            e.sync()
            engines.append((sh, ho, h, e, []))
    for _ in range(a.rounds):
        for sh, ho, h, e, ts in engines:
            e.sync()
            t0 = time.perf_counter()
            e.step(a.gens)
            e.sync()
            ts.append(time.perf_counter() - t0)
    for sh, ho, h, e, ts in engines:
        e.set_timing(1)
        e.reset_timing()
        e.step(a.gens)
        e.sync()
        tm = e.timing()
        e.set_timing(0)
        cells = float(h) * a.width * a.gens
        rec = {"shape": f"{h}x{a.width}" + (" composite" if sh.endswith("c") else " single stream"),
               "handoff_cfg": ho, "handoff": e.handoff, "tb_depth": e.tb_depth,
               "rows_per_wave": e.rows_per_wave, "gens": a.gens, "rule": a.rule,
               "tcups_wall_median": round(cells / statistics.median(ts) / 1e12, 2),
               "tcups_wall_best": round(cells / min(ts) / 1e12, 2),
               "work_ratio": round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1), 4),
               "kernel_ms_avg": round(tm["kernel_ms"] / max(tm["launches"], 1), 4)}
        print(json.dumps(rec), flush=True)
        e.close()


if __name__ == "__main__":
    main()
