#!/usr/bin/env python3
"""Dev tool: throughput of the stripe group (gol_create_group) on the visible
GPUs -- S row stripes with k-deep halo rounds, round-robin over the devices.
On one GPU this prices the multi-stripe machinery (halo rounds, band/interior
split, exchange copies) against a single engine on the same field.

    python tools/group_bench.py --size 65536 --stripes 1,2,4,8 --gens 192
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

# engines of this tool are stepped one at a time: no waiting-kernel registry
os.environ.setdefault("GOL_DEV_SHARED_WAITS", "1")

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--width", type=int, default=0)
p.add_argument("--stripes", default="1,2,4,8")
p.add_argument("--gens", type=int, default=192)
p.add_argument("--gpus", type=int, default=1)
p.add_argument("--tb-depth", type=int, default=0)
p.add_argument("--halo-depth", type=int, default=0)
a = p.parse_args()
pkg = entry.load_package()
n = a.size
wd = a.width or a.size
for s in [int(x) for x in a.stripes.split(",")]:
    devs = [r % a.gpus for r in range(s)]
    if s == 1:
        obj = pkg.Engine(n, wd, device=0, tb_depth=a.tb_depth)
    else:
        obj = pkg.Group(n, wd, s, devices=devs, tb_depth=a.tb_depth, halo_depth=a.halo_depth)
    obj.init_random(1)
    obj.step(a.gens)
    obj.sync()
    best = 0
    for _ in range(3):
        t0 = time.perf_counter()
        obj.step(a.gens)
        obj.sync()
        best = max(best, n * wd * a.gens / (time.perf_counter() - t0) / 1e9)
    info = obj if s == 1 else obj.members[min(1, s - 1)]
    print(json.dumps({"stripes": s, "gpus": a.gpus, "gcups": round(best, 1),
                      "halo_depth": info.halo_depth, "tb_depth": info.tb_depth,
                      "rows_per_wave": info.rows_per_wave}), flush=True)
    obj.close()
