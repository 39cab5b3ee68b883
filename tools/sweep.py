#!/usr/bin/env python3
"""Dev tool: sweep stencil launch parameters in ONE process (interleaved rounds,
cdna_hip_programming.md §5.4 rule 24) and print GCUPS per variant.

    python tools/sweep.py --size 4096 --gens 1000 --depths 8,16 --rpw 0,4,6,10 \
        --lanes 0,32 --handoffs 1,2

Timing is wall clock over gol_step(gens) + gol_sync (graph replay included, as
bench.py and the CLI see it); a separate pass with HIP events on every launch
gives the mean launch time and the engine's work ratio.
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

# engines of this tool are stepped one at a time: no waiting-kernel registry
os.environ.setdefault("GOL_DEV_SHARED_WAITS", "1")


def ints(s):
    return [int(x) for x in s.split(",")]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--gens", type=int, default=96)
    p.add_argument("--depths", default="0")
    p.add_argument("--rpw", default="0")
    p.add_argument("--lanes", default="0", help="strip widths (gol_config.strip_lanes)")
    p.add_argument("--handoffs", default="0")
    p.add_argument("--resident", default="1", help="gol_config.resident values (0 auto, 1 off, 2 on)")
    p.add_argument("--streams", type=int, default=0, help="gol_config.streams (0 = auto)")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--rule", default="ref")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    h = a.size
    w = a.width or a.size
    variants = list(itertools.product(ints(a.depths), ints(a.rpw), ints(a.lanes), ints(a.handoffs),
                                      ints(a.resident)))
    engines = {}
    for v in variants:
        d, r, sl, ho, res = v
        try:
            e = pkg.Engine(h, w, rule=rule, device=0, tb_depth=d, rows_per_wave=r,
                           streams=a.streams, strip_lanes=sl, handoff=ho, resident=res)
        except pkg.GolError as ex:
            print(json.dumps({"variant": v, "error": str(ex)}), flush=True)
            continue
        e.init_random(1)
        e.step(a.gens)  # warm-up + graph capture
        e.sync()
        engines[v] = e
    res = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, e in engines.items():
            t0 = time.perf_counter()
            e.step(a.gens)
            e.sync()
            res[v].append(h * w * a.gens / (time.perf_counter() - t0) / 1e9)
    for v, e in engines.items():
        e.set_timing(1)
        e.reset_timing()
        e.step(a.gens)
        e.sync()
        tm = e.timing()
        e.set_timing(0)
        r = sorted(res[v])
        print(json.dumps({"size": f"{h}x{w}", "gens": a.gens, "rule": a.rule,
                          "tb_depth": e.tb_depth, "rows_per_wave": e.rows_per_wave,
                          "strip_lanes": e.strip_lanes, "handoff": e.handoff,
                          "resident": e.resident,
                          "request": {"tb_depth": v[0], "rpw": v[1], "lanes": v[2],
                                      "handoff": v[3], "resident": v[4]},
                          "gcups_wall_median": round(r[len(r) // 2], 1),
                          "gcups_wall_best": round(r[-1], 1),
                          "kernel_us_avg": round(tm["kernel_ms"] / max(tm["launches"], 1) * 1e3, 2),
                          "launches": tm["launches"],
                          "work_ratio": round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1),
                                              3)}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
