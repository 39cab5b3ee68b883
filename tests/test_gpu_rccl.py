"""The RCCL halo path itself (gol_create_rank + ncclSend/Recv over xGMI), one
process per GPU.  RCCL refuses two ranks on one device, so this needs a box with
at least two GPUs and is skipped elsewhere (test_gpu_transport.py runs the same
rank engines and schedule with a host transport on one GPU; bench.py --gpus N
repeats this check as `rccl_selfcheck` before its timed run).

Each rank advances its stripe of a B3/S23 field over several Hx-generation
rounds; the stripe digests (order-independent sums) must add up to the digest of
the whole field evolved by one engine, which the rest of the suite pins to the
oracle.
"""
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def worker(rank, n, uid, h, w, gens, q):
    try:
        import __graft_entry__ as entry
        pkg = entry.load_package()
        with pkg.Engine(h, w, rule=pkg.CONWAY, device=rank, rank=rank, nranks=n, uid=uid) as e:
            e.init_random(3)
            e.step(gens)
            q.put((rank, e.digest(), e.halo_depth, None))
    except Exception as ex:  # report, never leave the parent waiting
        q.put((rank, None, None, repr(ex)))


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_rccl_ranks_equal_single_field(pkg, nranks):
    if torch.cuda.device_count() < nranks:
        pytest.skip(f"needs {nranks} GPUs (RCCL refuses two ranks on one device)")
    h, w, gens = 4096, 8192, 3 * 64 + 21
    uid = pkg.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, nranks, uid, h, w, gens, q))
             for r in range(nranks)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[3] for r in res if r[3]]
    assert not errs, errs
    live = sum(r[1][0] for r in res)
    hsh = sum(r[1][1] for r in res) & 0xFFFFFFFFFFFFFFFF
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0) as e:
        e.init_random(3)
        e.step(gens)
        assert (live, hsh) == e.digest()
