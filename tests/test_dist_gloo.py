"""CPU suite, world_size 2 over gloo: the multi-rank protocol of the RCCL rank
engines (engine.cpp `exchange` + `run_round`), restated with torch.distributed
send/recv and a small numpy stepper, must reproduce the single-field evolution.

What is exercised is the protocol: the partition (libgol's own gol_rank_rows),
the halo layout (a rank's buffer holds field rows [row0-Hx, row0+R+Hx); it sends
buffer rows [Hx, 2Hx) up and [R, R+Hx) down and receives into [0, Hx) and
[R+Hx, R+2Hx)), and the rounds of Hx generations in launches of depth d that
shrink the valid region by d rows per side.  The oracle is only the checker.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def life_step(cells, birth, survive, glob0, field_h):
    """One generation of a bool field; rows whose field index is outside
    [0, field_h) are dead, columns beyond the array are dead."""
    h, w = cells.shape
    p = np.zeros((h + 2, w + 2), dtype=np.uint8)
    p[1:-1, 1:-1] = cells
    n = sum(p[1 + dy:h + 1 + dy, 1 + dx:w + 1 + dx]
            for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dy, dx) != (0, 0))
    nb = ((birth >> n) & 1).astype(bool)
    ns = ((survive >> n) & 1).astype(bool)
    out = np.where(cells, ns, nb)
    rows = glob0 + np.arange(h)
    out[(rows < 0) | (rows >= field_h)] = False
    return out


def pick_depth(K, left):
    for d in (16, 8, 4, 2, 1):
        if d <= K and d <= left:
            return d
    return 1


def worker(rank, world, port, h, w, gens, K, Hx, rule, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as entry
    pkg = entry.load_package()
    orc = entry.load_oracle()
    field = orc.bp_random(h, w, seed)
    cells = np.unpackbits(field.view(np.uint8), axis=1, bitorder="little")[:, :w].astype(bool)
    row0, R = pkg.rank_rows(h, world, rank)
    Hx = min(Hx, h // world)
    buf = np.zeros((R + 2 * Hx, w), dtype=bool)
    glob0 = row0 - Hx
    lo, hi = max(0, glob0), min(h, row0 + R + Hx)
    buf[lo - glob0:hi - glob0] = cells[lo:hi]
    left = gens
    while left > 0:
        rnd = min(left, Hx)
        # exchange (engine.cpp `exchange`): Hx rows each way
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.uint8))
        reqs = []
        recv_up = torch.zeros((Hx, w), dtype=torch.uint8)
        recv_dn = torch.zeros((Hx, w), dtype=torch.uint8)
        if rank > 0:
            reqs.append(dist.isend(t(buf[Hx:2 * Hx]), rank - 1))
            reqs.append(dist.irecv(recv_up, rank - 1))
        if rank < world - 1:
            reqs.append(dist.isend(t(buf[R:R + Hx]), rank + 1))
            reqs.append(dist.irecv(recv_dn, rank + 1))
        for r in reqs:
            r.wait()
        if rank > 0:
            buf[:Hx] = recv_up.numpy().astype(bool)
        if rank < world - 1:
            buf[R + Hx:] = recv_dn.numpy().astype(bool)
        # run_round: launches of depth d, valid region shrinking by d per side
        done = 0
        while done < rnd:
            d = pick_depth(K, rnd - done)
            for _ in range(d):
                buf = life_step(buf, rule[0], rule[1], glob0, h)
            done += d
        left -= rnd
    q.put((rank, row0, buf[Hx:Hx + R].copy()))
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("K,Hx,gens,rule", [(8, 64, 37, "conway"), (4, 12, 30, "highlife"),
                                            (2, 5, 11, "ref"), (1, 3, 7, "conway")])
def test_two_rank_protocol(oracle, K, Hx, gens, rule):
    R = {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[rule]
    h, w, seed = 61, 70, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, h, w, gens, K, Hx, R, seed, q))
             for r in range(2)]
    for p in procs:
        p.start()
    parts = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([b for _, _, b in parts])
    ref = oracle.bp_run(oracle.bp_random(h, w, seed), w, gens, R)
    ref_cells = np.unpackbits(ref.view(np.uint8), axis=1, bitorder="little")[:, :w].astype(bool)
    assert (got == ref_cells).all()
