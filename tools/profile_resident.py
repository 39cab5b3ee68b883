#!/usr/bin/env python3
"""Dev tool run under rocprofv3: the resident kernel at a small field (default
the C2 job, 4096^2 x 1000 generations of B/S2, one launch per step), `steps`
steps after one warm-up step.  Prints the plan as one JSON line.

    rocprofv3 --pmc SQ_... -- python3 tools/profile_resident.py --size 4096
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=4096)
p.add_argument("--rule", default="ref", choices=["ref", "conway"])
p.add_argument("--gens", type=int, default=1000)
p.add_argument("--steps", type=int, default=3)
p.add_argument("--tb-depth", type=int, default=0)
p.add_argument("--rows-per-wave", type=int, default=0)
a = p.parse_args()
pkg = entry.load_package()
rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
kw = {}
if a.tb_depth or a.rows_per_wave:
    kw = dict(resident=2, tb_depth=a.tb_depth, rows_per_wave=a.rows_per_wave)
e = pkg.Engine(a.size, a.size, rule=rule, device=0, **kw)
assert e.resident is not None, "resident plan expected"
e.init_random(1)
e.step(a.gens)
e.sync()
t0 = time.perf_counter()
for _ in range(a.steps):
    e.step(a.gens)
e.sync()
dt = (time.perf_counter() - t0) / a.steps
print(json.dumps({"size": a.size, "rule": a.rule, "gens": a.gens, "tb_depth": e.tb_depth,
                  "rows_per_wave": e.rows_per_wave, "resident": e.resident,
                  "tcups_wall": round(a.size * a.size * a.gens / dt / 1e12, 3),
                  "digest": e.digest()}))
e.close()
