#!/usr/bin/env python3
"""Dev tool run under rocprofv3: the benchmark's default engine (or a variant)
for a fixed number of full-depth launch rounds, plus kernels with known byte
counts so PMC counters can be calibrated for this access width (8 B per lane)
before pricing the stencil kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE is
uncalibrated for widths other than 16 B/lane).

  init_random_kernel : writes exactly rows*stride*8 bytes (8 B/lane stores)
  digest_kernel      : reads exactly rows*wq*8 bytes (8 B/lane loads)
  life_tb_kernel     : `launches` x tb_depth generations of the field (or, for a
                       field the resident kernel takes, `launches` launches of
                       `gens` generations: life_res_kernel)

Prints one JSON line with the engine's configuration (bench.py's record keys),
which tools/pmc_counters.py reads back.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--rule", default="ref", choices=["ref", "conway"])
p.add_argument("--tb-depth", type=int, default=0, help="0 = the engine's auto layout")
p.add_argument("--rows-per-wave", type=int, default=0)
p.add_argument("--handoff", type=int, default=0)
p.add_argument("--streams", type=int, default=0)
p.add_argument("--launches", type=int, default=16)
p.add_argument("--ranks", type=int, default=1,
               help="> 1: the middle rank (N // 2) of the N-way row-stripe split as one rank "
                    "engine over an RCCL self-loop communicator (GOL_DEV_RCCL_SELF=1; its "
                    "launches are the N-GPU run's per-rank launches, tools/rank_proxy.py)")
p.add_argument("--gens", type=int, default=1000,
               help="resident engines: generations per launch (one launch per gol_step)")
a = p.parse_args()
pkg = entry.load_package()
rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
kw = dict(rule=rule, device=0, tb_depth=a.tb_depth, rows_per_wave=a.rows_per_wave,
          handoff=a.handoff)
if a.ranks > 1:
    os.environ["GOL_DEV_RCCL_SELF"] = "1"
    e = pkg.Engine(a.size, a.size, rank=a.ranks // 2, nranks=a.ranks, uid=pkg.unique_id(), **kw)
else:
    e = pkg.Engine(a.size, a.size, streams=a.streams, **kw)
e.init_random(1)
d0 = e.digest()
e.set_timing(1)
if e.resident:  # the bench's launches: one per gol_step of `gens` generations
    for _ in range(a.launches):
        e.step(a.gens)
    gens_per_launch = a.gens
else:
    e.step(e.tb_depth * a.launches)
    gens_per_launch = e.tb_depth
e.sync()
tm = e.timing()
print(json.dumps({"size": a.size, "rule": a.rule, "tb_depth": e.tb_depth,
                  "streams": max(1, tm["streams"]), "n_gpus": a.ranks,
                  "own_rows": e.rows, "halo_depth": e.halo_depth,
                  "rows_per_launch": round(tm["launch_rows"] / max(1, tm["launches"]), 1),
                  "rows_per_wave": e.rows_per_wave, "handoff": e.handoff,
                  "kernel": "life_res_kernel" if e.resident else "life_tb_kernel",
                  "gens_per_launch": gens_per_launch,
                  "launches": tm["launches"], "digest0": d0, "digest": e.digest()}))
e.close()
