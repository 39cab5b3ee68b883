#!/usr/bin/env python3
"""Dev tool: run the RCCL rank-engine path with N processes on the visible GPUs
(device = rank % ngpus; on a 1-GPU box all ranks share device 0, which RCCL may
refuse) and compare the summed digest with a single-field engine.

    python tools/rccl_selftest.py --nranks 2
"""
import argparse
import os
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, n, uid, h, w, gens, q):
    import __graft_entry__ as entry
    pkg = entry.load_package()
    import torch
    dev = rank % max(1, torch.cuda.device_count())
    try:
        e = pkg.Engine(h, w, rule=pkg.CONWAY, device=dev, rank=rank, nranks=n, uid=uid)
        e.init_random(3)
        e.step(gens)
        e.sync()
        q.put((rank, e.digest(), None))
        e.close()
    except Exception as ex:  # report, do not hang the parent
        q.put((rank, None, repr(ex)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nranks", type=int, default=2)
    p.add_argument("--h", type=int, default=4096)
    p.add_argument("--w", type=int, default=8192)
    p.add_argument("--gens", type=int, default=200)
    a = p.parse_args()
    import __graft_entry__ as entry
    pkg = entry.load_package()
    uid = pkg.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, a.nranks, uid, a.h, a.w, a.gens, q))
             for r in range(a.nranks)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    errs = [r for r in res if r[2]]
    if errs:
        print("RCCL path failed:", errs)
        sys.exit(3)
    live = sum(r[1][0] for r in res)
    hsh = sum(r[1][1] for r in res) & 0xFFFFFFFFFFFFFFFF
    with pkg.Engine(a.h, a.w, rule=pkg.CONWAY, device=0) as e:
        e.init_random(3)
        e.step(a.gens)
        want = e.digest()
    print("ranks", (live, hsh), "single", want, "OK" if (live, hsh) == want else "MISMATCH")
    sys.exit(0 if (live, hsh) == want else 1)


if __name__ == "__main__":
    main()
