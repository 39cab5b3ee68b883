#!/usr/bin/env python3
"""Dev tool run under rocprofv3: a fixed number of full-depth launches of one
field shape and hand-off setting (for PMC A/B of the stencil kernel).

    rocprofv3 --pmc ... -- python3 tools/profile_shape.py --rows 8448 --handoff 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=int, default=8448)
p.add_argument("--width", type=int, default=65536)
p.add_argument("--handoff", type=int, default=2)
p.add_argument("--streams", type=int, default=1)
p.add_argument("--launches", type=int, default=8)
a = p.parse_args()
pkg = entry.load_package()
with pkg.Engine(a.rows, a.width, device=0, handoff=a.handoff, streams=a.streams) as e:
    e.init_random(1)
    e.step(e.tb_depth * a.launches)
    e.sync()
    print("plan", e.tb_depth, e.rows_per_wave, e.handoff, e.digest())
