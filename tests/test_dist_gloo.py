"""CPU suite, world_size 2-3 over gloo: the multi-rank protocol, driven by the
engine's own schedule.

Each rank asks libgol for the schedule its gol_step would run
(gol_round_schedule -- host-only, the same code path gol_step executes: the
partition, the rounds of Hx generations, the launch depths, the shrinking output
rows, the band/interior split and the overlapped exchange) and executes it on a
bool field with numpy: a launch of depth d writes ONLY its scheduled output rows
(every other row of the target buffer is filled with noise), exchanges move the
Hx boundary rows with torch.distributed send/recv as stripes.cpp `exchange` does.
A schedule that reads a row nobody computed, or a round/exchange order change
that breaks the protocol, shows up as a mismatch with the oracle.
"""
import os
import socket
import subprocess

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


def run_launch(cur, nxt, depth, segs, rule, glob0, field_h):
    """A stencil launch: rows [lo, hi) of nxt from rows [lo-d, hi+d) of cur."""
    for lo, hi in segs:
        a, b = max(0, lo - depth), min(cur.shape[0], hi + depth)
        sub = cur[a:b].copy()
        rows = glob0 + a + np.arange(b - a)
        sub[(rows < 0) | (rows >= field_h)] = False  # the kernel reads those rows as dead
        for k in range(depth):
            sub = life_step(sub, rule[0], rule[1], glob0 + a, field_h)
        nxt[lo:hi] = sub[lo - a:hi - a]


def exchange(buf, rank, world, R, Hx):
    """stripes.cpp `exchange`: own rows [Hx, 2Hx) up and [R, R+Hx) down, received
    into [0, Hx) and [R+Hx, R+2Hx)."""
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.uint8))
    w = buf.shape[1]
    reqs = []
    up, dn = torch.zeros((Hx, w), dtype=torch.uint8), torch.zeros((Hx, w), dtype=torch.uint8)
    if rank > 0:
        reqs += [dist.isend(t(buf[Hx:2 * Hx]), rank - 1), dist.irecv(up, rank - 1)]
    if rank < world - 1:
        reqs += [dist.isend(t(buf[R:R + Hx]), rank + 1), dist.irecv(dn, rank + 1)]
    for r in reqs:
        r.wait()
    if rank > 0:
        buf[:Hx] = up.numpy().astype(bool)
    if rank < world - 1:
        buf[R + Hx:] = dn.numpy().astype(bool)


def worker(rank, world, port, h, w, chunks, K, Hx, rule, seed, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import __graft_entry__ as entry
        pkg = entry.load_package()
        orc = entry.load_oracle()
        rng = np.random.default_rng(100 + rank)
        field = orc.bp_random(h, w, seed)
        cells = np.unpackbits(field.view(np.uint8), axis=1, bitorder="little")[:, :w].astype(bool)
        row0, R = pkg.rank_rows(h, world, rank)
        fresh = False
        bufs = None
        kinds = []
        for chunk in chunks:
            ops, k_eng, hx = pkg.round_schedule(h, w, rank, world, chunk, halo_fresh=fresh,
                                                rule=rule, tb_depth=K, halo_depth=Hx)
            assert k_eng == K
            if bufs is None:
                glob0 = row0 - hx
                cur = np.zeros((R + 2 * hx, w), dtype=bool)  # a load clears the buffer
                cur[row0 - glob0:row0 - glob0 + R] = cells[row0:row0 + R]
                bufs = [cur, rng.random(cur.shape) < 0.5]
            for op in ops:
                kind = op["kind"]
                kinds.append(kind)
                if kind in (pkg.OP_EXCHANGE, pkg.OP_EXCHANGE_ASYNC):
                    exchange(bufs[0], rank, world, R, hx)
                elif kind == pkg.OP_WAIT_EXCHANGE:
                    pass
                elif kind == pkg.OP_BAND:
                    bufs[1] = rng.random(bufs[0].shape) < 0.5
                    run_launch(bufs[0], bufs[1], op["depth"], op["segs"], rule, glob0, h)
                elif kind == pkg.OP_INTERIOR:  # same source buffer as the band, then swap
                    run_launch(bufs[0], bufs[1], op["depth"], op["segs"], rule, glob0, h)
                    bufs.reverse()
                else:  # LAUNCH
                    bufs[1] = rng.random(bufs[0].shape) < 0.5
                    run_launch(bufs[0], bufs[1], op["depth"], op["segs"], rule, glob0, h)
                    bufs.reverse()
            fresh = ops[-1]["kind"] == pkg.OP_EXCHANGE_ASYNC
        q.put((rank, row0, bufs[0][hx:hx + R].copy(), sorted(set(kinds)), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:
        import traceback
        q.put((rank, None, None, None, traceback.format_exc() + repr(ex)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("overlap", ["default", "1"])
@pytest.mark.parametrize("world,K,Hx,chunks,rule", [
    (2, 8, 16, (37,), "conway"),           # 2 overlapped rounds + partial
    (2, 4, 12, (12, 5, 30), "highlife"),   # overlap carried across calls
    (3, 2, 5, (11, 10), "ref"),
    (2, 1, 3, (7,), "conway"),
    (2, 16, 0, (70,), "conway"),           # default halo depth (8K, clipped to h/N)
    (3, 7, 21, (50,), "conway"),           # remainder depths (7 = pick_depth list)
    (2, 12, 24, (24, 24, 9), "conway"),
])
def test_rank_protocol_from_engine_schedule(oracle, monkeypatch, world, K, Hx, chunks, rule,
                                            overlap):
    """overlap: rank engines exchange blocking by default; GOL_DEV_OVERLAP=1 gives
    the band/interior split with the overlapped exchange (inherited by the
    spawned ranks)."""
    if overlap != "default":
        monkeypatch.setenv("GOL_DEV_OVERLAP", overlap)
    R = {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[rule]
    h, w, seed = 101, 70, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, h, w, chunks, K, Hx, R, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    parts = sorted((q.get(timeout=180) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [x[4] for x in parts if x[4]]
    assert not errs, errs[0]
    got = np.concatenate([x[2] for x in parts])
    ref = oracle.bp_run(oracle.bp_random(h, w, seed), w, sum(chunks), R)
    ref_cells = np.unpackbits(ref.view(np.uint8), axis=1, bitorder="little")[:, :w].astype(bool)
    assert (got == ref_cells).all()


def test_default_halo_depth(pkg, monkeypatch):
    """Rounds of 8 launches, 12 for K = 16 stripes of 16384+ rows (stripes.cpp
    rank_geometry: the round's full-depth launches share one region, so deeper
    halos cost rows on every launch); with the
    r03 shrinking regions (GOL_DEV_RANK_SHRINK=1) 16 for K = 16 stripes of at most
    12288 rows (the 8-way 65536^2 rank)."""
    for nranks, want in ((2, 192), (4, 192), (8, 128)):
        _, K, Hx = pkg.round_schedule(65536, 65536, 1, nranks, 16)
        assert (K, Hx) == (16, want), nranks
    monkeypatch.setenv("GOL_DEV_RANK_SHRINK", "1")
    for nranks, want in ((2, 128), (4, 128), (8, 256)):
        _, K, Hx = pkg.round_schedule(65536, 65536, 1, nranks, 16)
        assert (K, Hx) == (16, want), nranks
    monkeypatch.delenv("GOL_DEV_RANK_SHRINK")
    _, K, Hx = pkg.round_schedule(1200, 2000, 0, 2, 16, tb_depth=8)
    assert (K, Hx) == (8, 64)


def test_schedule_structure_default(pkg):
    """A rank engine's blocking schedule for the C4 8-rank stripe at Hx = 128:
    rounds of eight 16-deep launches between blocking exchanges."""
    ops, K, Hx = pkg.round_schedule(65536, 65536, 3, 8, 300, halo_depth=128)
    assert (K, Hx) == (16, 128)
    kinds = [pkg.OP_NAMES[o["kind"]] for o in ops]
    assert kinds[:18] == (["EXCHANGE"] + ["LAUNCH"] * 8) * 2
    assert kinds[18] == "EXCHANGE" and set(kinds[19:]) == {"LAUNCH"}
    assert "BAND" not in kinds and "EXCHANGE_ASYNC" not in kinds
    assert sum(o["depth"] for o in ops) == 300


def test_schedule_structure(pkg, monkeypatch):
    """With the overlap on (GOL_DEV_OVERLAP=1; in-process groups' default): a
    round ends in band + interior + overlapped exchange, and the next call starts
    from that exchange."""
    monkeypatch.setenv("GOL_DEV_OVERLAP", "1")
    ops, K, Hx = pkg.round_schedule(65536, 65536, 3, 8, 300, halo_depth=128)
    assert (K, Hx) == (16, 128)
    kinds = [pkg.OP_NAMES[o["kind"]] for o in ops]
    assert kinds[0] == "EXCHANGE"
    assert kinds[1:8] == ["LAUNCH"] * 7
    assert kinds[8:11] == ["BAND", "INTERIOR", "EXCHANGE_ASYNC"]
    assert kinds[11] == "WAIT_EXCHANGE"
    assert ops[8]["segs"] == [(128, 256), (8192, 8320)]  # rows the neighbours need
    assert ops[9]["segs"] == [(256, 8192)]
    assert ops[-1]["kind"] == pkg.OP_LAUNCH and sum(o["depth"] for o in ops[-4:]) == 300 - 256
    fresh_ops, _, _ = pkg.round_schedule(65536, 65536, 3, 8, 128, halo_fresh=True,
                                         halo_depth=128)
    assert fresh_ops[0]["kind"] == pkg.OP_WAIT_EXCHANGE
    # top and bottom ranks have one band segment, and no overlap when R < 2 Hx
    top, _, _ = pkg.round_schedule(65536, 65536, 0, 8, 128, halo_depth=128)
    assert [o["segs"] for o in top if o["kind"] == pkg.OP_BAND] == [[(8192, 8320)]]
    small, _, hx = pkg.round_schedule(100, 64, 0, 2, 50, halo_depth=40)
    assert hx == 40 and pkg.OP_BAND not in [o["kind"] for o in small]


MPIRUN = "/opt/conda/bin/mpirun"


def test_gol_mpi_dry_run_partition(pkg, tmp_path):
    """gol-mpi's argument parsing, config read and partition (mpirun -np 2, no GPU
    touched): each rank reports the rows it would read and the rounds it would
    run, matching gol_rank_rows / gol_round_schedule."""
    path = os.path.join(os.path.dirname(pkg.CLI_PATH), "gol-mpi")
    if not (os.path.exists(path) and os.path.exists(MPIRUN)):
        pytest.skip("gol-mpi not built (no MPI on this host)")
    (tmp_path / "grid_size_data.txt").write_text("1500 500 100")
    r = subprocess.run([MPIRUN, "-np", "2", path, "--dir", str(tmp_path), "--dry-run",
                        "--transport", "mpi", "--tb-depth", "8", "--halo-depth", "16"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = sorted(l for l in r.stdout.splitlines() if l.startswith("rank "))
    assert len(lines) == 2
    for rank, line in enumerate(lines):
        row0, rows = pkg.rank_rows(1500, 2, rank)
        ops, K, Hx = pkg.round_schedule(1500, 500, rank, 2, 100, tb_depth=8, halo_depth=16)
        assert line == (f"rank {rank}/2: rows [{row0}, {row0 + rows}) offset {row0 * 501} "
                        f"K {K} halo {Hx} ops {len(ops)} transport mpi")
    bad = subprocess.run([MPIRUN, "-np", "2", path, "--dir", str(tmp_path), "--dry-run",
                          "--transport", "carrier-pigeon"], capture_output=True, text=True,
                         timeout=120)
    assert bad.returncode != 0


def test_resident_epoch_length_maps_to_streaming_depth(pkg):
    """resident = 2 takes any epoch length (tb_depth 1..63); a rank engine runs
    the streaming kernel, whose depth is then the auto one when that length has no
    stencil kernel (22 -> 16 at the 8-way 65536^2 stripe, 8 for short stripes)."""
    _, K, Hx = pkg.round_schedule(65536, 65536, 1, 8, 100, resident=2, tb_depth=22)
    assert (K, Hx) == (16, 128)
    _, K, _ = pkg.round_schedule(4096, 4096, 0, 2, 40, resident=2, tb_depth=22)
    assert K == 8
    _, K, _ = pkg.round_schedule(4096, 4096, 0, 2, 40, resident=2, tb_depth=12)
    assert K == 12
