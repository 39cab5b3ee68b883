#!/usr/bin/env python3
"""Dev tool: sweep stencil launch parameters in ONE process (interleaved rounds,
cdna_hip_programming.md §5.4 rule 24) and print GCUPS per variant.

    python tools/sweep.py --size 65536 --gens 96 --depths 4,8,16 --rpw 0,64,128,256
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--gens", type=int, default=96)
    p.add_argument("--depths", default="4,8,16")
    p.add_argument("--rpw", default="0")
    p.add_argument("--variants", default="0")
    p.add_argument("--lanes", default="0", help="strip widths (gol_config.strip_lanes)")
    p.add_argument("--planes", default="0", help="planes per lane group (gol_config.word_planes)")
    p.add_argument("--streams", type=int, default=0, help="gol_config.streams (0 = auto)")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--rule", default="ref")
    p.add_argument("--no-events", action="store_true", help="time wall clock only")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    h = a.size
    w = a.width or a.size
    variants = list(itertools.product([int(x) for x in a.depths.split(",")],
                                      [int(x) for x in a.rpw.split(",")],
                                      [int(x) for x in a.variants.split(",")],
                                      [int(x) for x in a.lanes.split(",")],
                                      [int(x) for x in a.planes.split(",")]))
    engines = {}
    for d, r, kv, sl, wp in variants:
        e = pkg.Engine(h, w, rule=rule, device=0, tb_depth=d, rows_per_wave=r,
                       kernel_variant=kv, streams=a.streams, strip_lanes=sl, word_planes=wp)
        e.init_random(1)
        e.step(d or 8)  # warm
        e.sync()
        engines[(d, r, kv, sl, wp)] = e
        if len(engines) > 6:  # bound HBM use: 1 GiB per engine at 65536^2
            pass
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            e = engines[v]
            e.set_timing(0 if a.no_events else 8)
            e.reset_timing()
            t0 = time.perf_counter()
            e.step(a.gens)
            e.sync()
            dt = time.perf_counter() - t0
            tm = e.timing()
            res[v].append((h * w * a.gens / dt / 1e9,
                           tm["kernel_ms"] / max(tm["launches"], 1),
                           tm["cell_gens"] / max(tm["kernel_ms"], 1e-9) / 1e6))
    for v in variants:
        r = sorted(res[v])
        med = r[len(r) // 2]
        print(json.dumps({"tb_depth": v[0] or f"auto({engines[v].tb_depth})",
                          "rows_per_wave": v[1] or f"auto({engines[v].rows_per_wave})",
                          "variant": v[2], "strip_lanes": engines[v].strip_lanes,
                          "word_planes": engines[v].word_planes,
                          "gcups_wall_median": round(med[0], 1),
                          "gcups_wall_best": round(r[-1][0], 1),
                          "kernel_ms_avg": round(med[1], 4),
                          "gcups_kernel": round(med[2], 1)}), flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
