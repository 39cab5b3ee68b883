"""The multi-rank path with more than one rank on ONE GPU: gol_create_rank_transport.

RCCL refuses two ranks on one device, so these tests run the rank engines of
gol_create_rank -- partition, halo rounds (blocking exchanges by default, the
band/interior overlap with GOL_DEV_OVERLAP=1), gol_step's
schedule -- with the halo rows moved by a caller's host transport instead: here
torch.distributed over gloo between 2-4 processes that share cuda:0 (the same
transport shape as the reference's MPI_Sendrecv of boundary rows,
Parallel_Life_MPI.cpp:104-145, with the receive landing in the halo).  Only the
byte mover differs from the RCCL path (stripes.cpp `exchange`).  Also the
`gol-mpi --transport mpi` launcher under mpirun -np 2 / 4 on one GPU.
"""
import hashlib
import json
import os
import socket
import subprocess

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gloo_exchange(rank, world):
    """A gol_transport over gloo: isend/irecv of the boundary rows."""
    def xchg(send_up, send_dn):
        n = len(send_up if send_up is not None else send_dn)
        reqs, ru, rd = [], None, None
        if send_up is not None:
            ru = torch.empty(n, dtype=torch.uint8)
            reqs.append(dist.isend(torch.frombuffer(bytearray(send_up), dtype=torch.uint8), rank - 1))
            reqs.append(dist.irecv(ru, rank - 1))
        if send_dn is not None:
            rd = torch.empty(n, dtype=torch.uint8)
            reqs.append(dist.isend(torch.frombuffer(bytearray(send_dn), dtype=torch.uint8), rank + 1))
            reqs.append(dist.irecv(rd, rank + 1))
        for r in reqs:
            r.wait()
        return (ru.numpy().tobytes() if ru is not None else None,
                rd.numpy().tobytes() if rd is not None else None)
    return xchg


def worker(rank, world, port, h, w, chunks, rule, seed, cfg, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import __graft_entry__ as entry
        pkg = entry.load_package()
        orc = entry.load_oracle()
        g = orc.bp_random(h, w, seed)
        out = []
        with pkg.Engine(h, w, rule=rule, device=0, rank=rank, nranks=world,
                        transport=gloo_exchange(rank, world), **cfg) as e:
            e.load_packed(g[e.row0:e.row0 + e.rows])
            for chunk in chunks:
                e.step(chunk)  # no sync: store/digest must order after the band stream
                out.append((e.store_packed(), e.digest()))
            info = (e.row0, e.rows, e.tb_depth, e.halo_depth)
        q.put((rank, info, out, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, traceback.format_exc() + repr(ex)))


def run_ranks(world, h, w, chunks, rule, seed, **cfg):
    # ranks sharing one GPU: classic row blocks (one waiting launch per device at a
    # time, stripes.cpp gol_create_group)
    cfg.setdefault("handoff", 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, h, w, chunks, rule, seed, cfg, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[3] for r in res if r[3]]
    assert not errs, errs[0]
    return res


@pytest.mark.parametrize("overlap", ["default", "1"])
@pytest.mark.parametrize("world,K,Hx,rule", [(2, 8, 32, "conway"), (3, 4, 16, "highlife"),
                                             (4, 16, 64, "conway"), (2, 16, 0, "ref")])
def test_rank_engines_over_host_transport(oracle, monkeypatch, world, K, Hx, rule, overlap):
    """overlap: blocking exchanges (the rank engines' default) or the band /
    interior split with the overlapped exchange (GOL_DEV_OVERLAP=1, inherited by
    the spawned ranks)."""
    if overlap != "default":
        monkeypatch.setenv("GOL_DEV_OVERLAP", overlap)
    R = {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[rule]
    h, w, seed = 1200, 2000, 11 + world
    chunks = [Hx or 128, 5, 2 * (Hx or 128) + 3, 40]  # full rounds, partial ones, carried overlap
    res = run_ranks(world, h, w, chunks, R, seed, tb_depth=K, halo_depth=Hx)
    g = oracle.bp_random(h, w, seed)
    done = 0
    for i, chunk in enumerate(chunks):
        done += chunk
        want = oracle.bp_run(g, w, done, R)
        got = np.concatenate([r[2][i][0] for r in res])
        assert (got == want).all(), f"after {done} generations"
        live = sum(r[2][i][1][0] for r in res)
        hsh = sum(r[2][i][1][1] for r in res) & 0xFFFFFFFFFFFFFFFF
        assert (live, hsh) == oracle.bp_digest(want, w)


@pytest.mark.parametrize("overlap", ["default", "1"])
def test_rank_engines_c4_shape_over_host_transport(pkg, monkeypatch, overlap):
    """The C4 per-rank shape (65536^2 over 4 ranks) with default K / halo depth
    (age-skewed launches), over 2 rounds and a partial one, equals the single
    field."""
    if overlap != "default":
        monkeypatch.setenv("GOL_DEV_OVERLAP", overlap)
    n, world, gens = 65536, 4, 300
    with pkg.Engine(n, n, rule=pkg.CONWAY, device=0) as e:
        e.init_random(3)
        e.step(gens)
        want = e.digest()
    res = run_ranks_digest(world, n, n, gens, 3)
    assert res == want


def digest_worker(rank, world, port, h, w, gens, seed, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import __graft_entry__ as entry
        pkg = entry.load_package()
        with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, rank=rank, nranks=world,
                        transport=gloo_exchange(rank, world), handoff=1) as e:
            e.init_random(seed)
            e.step(gens)
            d = e.digest()
        q.put((rank, d, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:
        q.put((rank, None, repr(ex)))


def run_ranks_digest(world, h, w, gens, seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=digest_worker, args=(r, world, port, h, w, gens, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[2]]
    assert not errs, errs
    return (sum(r[1][0] for r in res), sum(r[1][1] for r in res) & 0xFFFFFFFFFFFFFFFF)


# ---- gol-mpi --transport mpi: mpirun -np P on one GPU ----

MPIRUN = "/opt/conda/bin/mpirun"
GOLD = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))


def gol_mpi(pkg):
    path = os.path.join(os.path.dirname(pkg.CLI_PATH), "gol-mpi")
    if not (os.path.exists(path) and os.path.exists(MPIRUN)):
        pytest.skip("gol-mpi not built (no MPI on this host)")
    return path


@pytest.mark.parametrize("np_", [2, 4])
def test_gol_mpi_host_transport_reference_output(pkg, tmp_path, np_):
    """mpirun -np P gol-mpi --transport mpi: P rank engines on one GPU exchanging
    halos with MPI_Sendrecv, each reading/writing its own rows of the files; the
    result is the reference's intended (= -np 1) output for any P."""
    case = [c for c in GOLD["cases"] if c["np"] == 1 and c["gens"] == 100][0]
    (tmp_path / "data.txt").write_bytes(open(os.path.join(GOLDEN, "data.txt"), "rb").read())
    (tmp_path / "grid_size_data.txt").write_text("1500 500 100")
    r = subprocess.run([MPIRUN, "-np", str(np_), gol_mpi(pkg), "--dir", str(tmp_path),
                        "--transport", "mpi", "--halo-depth", "16"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = (tmp_path / "output.txt").read_bytes()
    assert hashlib.sha256(out).hexdigest() == case["sha256"]
    # mpirun forwards the ranks' stdout through one pipe and may splice their
    # lines together: count the messages, not the line starts
    for i in range(np_):
        assert r.stdout.count(f"Process {i} wrote data to the file.") == 1, r.stdout
    assert r.stdout.count("Total time = ") == 1, r.stdout


def test_gol_mpi_host_transport_conway(pkg, oracle, tmp_path):
    h, w, gens = 700, 900, 77
    g = oracle.bp_random(h, w, 8)
    (tmp_path / "data.txt").write_bytes(oracle.bp_unpack(g, w))
    (tmp_path / "grid_size_data.txt").write_text(f"{h} {w} {gens}")
    r = subprocess.run([MPIRUN, "-np", "3", gol_mpi(pkg), "--dir", str(tmp_path),
                        "--transport", "mpi", "--rule", "conway", "--tb-depth", "8",
                        "--halo-depth", "24"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "output.txt").read_bytes() == oracle.bp_unpack(
        oracle.bp_run(g, w, gens, oracle.CONWAY), w)
