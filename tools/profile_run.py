#!/usr/bin/env python3
"""Dev tool run under rocprofv3: a fixed sequence of kernels with known byte
counts, so PMC counters can be calibrated for this access width (8 B per lane)
before pricing the stencil kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE is
uncalibrated for widths other than 16 B/lane).

  init_random_kernel : writes exactly rows*stride*8 bytes (8 B/lane stores)
  digest_kernel      : reads exactly rows*wq*8 bytes (8 B/lane loads)
  life_tb_kernel     : `launches` launches of depth K over the field
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--tb-depth", type=int, default=0, help="0 = the engine's auto layout")
p.add_argument("--word-planes", type=int, default=0)
p.add_argument("--rows-per-wave", type=int, default=0)
p.add_argument("--launches", type=int, default=4)
a = p.parse_args()
pkg = entry.load_package()
e = pkg.Engine(a.size, a.size, device=0, tb_depth=a.tb_depth, rows_per_wave=a.rows_per_wave,
               word_planes=a.word_planes)
print("layout", e.tb_depth, e.word_planes)
e.init_random(1)
print("digest", e.digest())
e.step(e.tb_depth * a.launches)
e.sync()
print("digest", e.digest())
e.close()
