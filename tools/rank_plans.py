#!/usr/bin/env python3
"""Dev tool (run under rocprofv3 --kernel-trace): one rank engine of the N-way
65536^2 split over the RCCL self-loop, GOL_DEV_PLANS=1 (the launch plans go to
stderr), `rounds` full rounds after a warm-up.  Pair the trace's life_tb_kernel
durations (in order) with the plans: launch j of a round runs plan j.

    rocprofv3 --kernel-trace -d out -o t --output-format csv -- python3 tools/rank_plans.py --nranks 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--nranks", type=int, default=8)
p.add_argument("--rounds", type=int, default=4)
p.add_argument("--halo-depth", type=int, default=0)
a = p.parse_args()
os.environ["GOL_DEV_PLANS"] = "1"
os.environ["GOL_DEV_RCCL_SELF"] = "1"
pkg = entry.load_package()
n = a.size
e = pkg.Engine(n, n, device=0, rank=a.nranks // 2, nranks=a.nranks, uid=pkg.unique_id(),
               halo_depth=a.halo_depth)
e.init_random(1)
e.step(e.halo_depth)
e.sync()
e.step(e.halo_depth * a.rounds)
e.sync()
print(json.dumps({"nranks": a.nranks, "rows": e.rows, "halo_depth": e.halo_depth,
                  "tb_depth": e.tb_depth, "handoff": e.handoff, "age_skew": e.age_skew,
                  "launches_per_round": e.halo_depth // e.tb_depth, "rounds": a.rounds + 1}))
e.close()
