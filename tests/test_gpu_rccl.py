"""The RCCL halo path itself (gol_create_rank + ncclSend/Recv), stripes.cpp
`exchange`, which replaces the reference's MPI_Sendrecv pair
(Parallel_Life_MPI.cpp:113-116, :129-132, called at :218).

* On ONE GPU (every box): RCCL refuses two ranks on one device, so a rank engine
  of an N-way split runs its byte mover against a 1-rank communicator whose up
  and down peers are itself (GOL_DEV_RCCL_SELF=1: ncclCommInitRank with nranks 1,
  then ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd on the engine's
  stream every round).  Its halos then receive the stripe's own boundary rows.
  That is checked three ways: against the oracle evolving the same "mirrored"
  extended stripe round by round, against the same engine over a host transport
  that returns what it is sent (bytewise, every chunk), and against a transport
  that delivers dead rows (the exchange must change the result).
* On boxes with >= 2 GPUs: one process per GPU, the stripe digests of a B3/S23
  field must add up to the whole field evolved by one engine (bench.py --gpus N
  repeats this as `rccl_selfcheck` before timing).
"""
import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def mirrored_round(oracle, own, w, gens, rule, Hx, has_up, has_dn):
    """One round of a self-looped rank: its halos hold its own first / last Hx
    rows (where it has that neighbour), the extended stripe evolves `gens`
    generations with dead cells beyond it, and its own rows are kept."""
    parts = ([own[:Hx]] if has_up else []) + [own] + ([own[-Hx:]] if has_dn else [])
    ext = np.concatenate(parts)
    out = oracle.bp_run(ext, w, gens, rule)
    top = Hx if has_up else 0
    return out[top:top + own.shape[0]]


def mirrored_steps(oracle, own, w, chunks, rule, Hx, has_up, has_dn):
    """Every gol_step call starts a round; rounds are Hx generations, the last
    one of a call what is left (stripes.cpp step_schedule)."""
    outs = []
    for c in chunks:
        left = c
        while left:
            g = min(left, Hx)
            own = mirrored_round(oracle, own, w, g, rule, Hx, has_up, has_dn)
            left -= g
        outs.append(own)
    return outs


@pytest.mark.parametrize("overlap", [1, 2])
@pytest.mark.parametrize("world,rank,K,Hx,rule", [
    (2, 0, 8, 32, "conway"),     # bottom neighbour only
    (2, 1, 16, 64, "conway"),    # top neighbour only
    (3, 1, 8, 24, "highlife"),   # both
    (4, 2, 16, 0, "ref"),        # both, default halo depth
])
def test_rccl_self_loop(pkg, oracle, monkeypatch, world, rank, K, Hx, rule, overlap):
    """overlap 1: blocking exchanges on the compute stream; 2: the band launch,
    then the exchange on the comm stream beside the interior launch."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    R = {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[rule]
    h, w, seed = 1200, 2000, 21 + rank
    g = oracle.bp_random(h, w, seed)
    cfg = dict(rule=R, device=0, tb_depth=K, halo_depth=Hx, exchange_overlap=overlap)
    with pkg.Engine(h, w, rank=rank, nranks=world, uid=pkg.unique_id(), **cfg) as e:
        Hx_ = e.halo_depth
        own = g[e.row0:e.row0 + e.rows]
        chunks = [Hx_, 5, 2 * Hx_ + 3, 40]  # full rounds, partial ones, carried overlap
        got = []
        e.load_packed(own)
        for c in chunks:
            e.step(c)  # no sync: store/digest must order after the comm stream
            got.append((e.store_packed(), e.digest()))
    has_up, has_dn = rank > 0, rank < world - 1
    want = mirrored_steps(oracle, own, w, chunks, R, Hx_, has_up, has_dn)
    for i, (c, (a, dg), b) in enumerate(zip(chunks, got, want)):
        assert (a == b).all(), f"chunk {i} ({c} generations)"
        # the rank's live count covers its own rows
        assert dg[0] == int(np.unpackbits(b.view(np.uint8)).sum())
    # bytewise against the host transport that loops back what it is sent, and the
    # exchange must matter: dead rows in the halos give a different field
    loop = lambda su, sd: (su, sd)  # noqa: E731
    dead = lambda su, sd: (None if su is None else bytes(len(su)),  # noqa: E731
                           None if sd is None else bytes(len(sd)))
    for tp, same in ((loop, True), (dead, False)):
        with pkg.Engine(h, w, rank=rank, nranks=world, transport=tp, **cfg) as t:
            t.load_packed(own)
            res = []
            for c in chunks:
                t.step(c)
                res.append((t.store_packed(), t.digest()))
        if same:
            for i, ((a, da), (b, db)) in enumerate(zip(got, res)):
                assert (a == b).all() and da == db, f"RCCL vs host loopback, chunk {i}"
        else:
            assert any((a != b).any() for (a, _), (b, _) in zip(got, res)), \
                "dead halos gave the same field: the exchange had no effect"


def test_rccl_self_loop_c4_rank_shape(pkg, monkeypatch):
    """The 8-way C4 per-rank shape (8192 own rows of 65536^2 + 2 x 128 halo rows,
    default K = 16, age-skewed one-round launches, default block kind): 1 MiB
    messages through RCCL every round, bytewise equal to the host loopback."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    n, world, rank, gens = 65536, 8, 3, 2 * 256 + 40
    out = []
    for mode in ("rccl", "host"):
        kw = dict(uid=pkg.unique_id()) if mode == "rccl" else dict(transport=lambda su, sd: (su, sd))
        with pkg.Engine(n, n, rule=pkg.CONWAY, device=0, rank=rank, nranks=world, **kw) as e:
            assert e.halo_depth == 128
            e.init_random(3)
            e.step(gens)
            out.append((e.digest(), e.store_packed()))
    assert out[0][0] == out[1][0]
    assert (out[0][1] == out[1][1]).all()


@pytest.mark.parametrize("overlap", [1, 2])
def test_rccl_self_loop_c5_rank_shape(pkg, oracle, monkeypatch, overlap):
    """The C5 per-rank shape (rank 3 of 8 of 262144^2: 32768 own rows x 262144
    columns + 2 x Hx halo rows, default K = 16 and Hx = 12K = 192, 6 MiB messages)
    through RCCL every round, both exchange modes: one partial round (16
    generations) against the oracle evolving the mirrored extended stripe
    (Parallel_Life_MPI.cpp:37-54 on :70-81's stripe, with the halo rows the
    exchange :104-145 is meant to deliver), then two full rounds and a partial one
    bytewise against the same engine over the host loopback transport."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    n, world, rank = 262144, 8, 3
    chunks = [16, 2 * 192 + 40]
    out = []
    for mode in ("rccl", "host"):
        kw = dict(uid=pkg.unique_id()) if mode == "rccl" else dict(transport=lambda su, sd: (su, sd))
        with pkg.Engine(n, n, rule=pkg.CONWAY, device=0, rank=rank, nranks=world,
                        exchange_overlap=overlap, **kw) as e:
            assert (e.rows, e.tb_depth, e.halo_depth) == (32768, 16, 192)
            e.init_random(5)
            res = []
            for c in chunks:
                e.step(c)
                res.append((e.digest(), e.store_packed()))
            row0 = e.row0
        out.append(res)
    for i, ((da, a), (db, b)) in enumerate(zip(*out)):
        assert da == db and (a == b).all(), f"RCCL vs host loopback, chunk {i}"
    # the first chunk against the oracle's mirrored stripe (the field's rows of
    # this rank, splitmix64 seed 5)
    own = oracle.bp_random_rows(row0, 32768, n, 5)
    want = mirrored_round(oracle, own, n, 16, oracle.CONWAY, 192, True, True)
    assert (out[0][0][1] == want).all()
    assert out[0][0][0][0] == int(np.unpackbits(want.view(np.uint8)).sum())


@pytest.mark.parametrize("overlap", [1, 2])
def test_rank_timing_spans_add_up(pkg, monkeypatch, overlap):
    """gol_timing's round spans (r06, bench.py rank_breakdown): per halo round
    one compute-stream span, the exchange split into its exposed and hidden
    parts; spans + exposed exchange fit in the wall time of the steps, both
    exchange modes."""
    import time
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    with pkg.Engine(16384, 16384, rule=pkg.CONWAY, device=0, rank=1, nranks=4,
                    uid=pkg.unique_id(), exchange_overlap=overlap) as e:
        hx = e.halo_depth
        e.init_random(1)
        e.step(4 * hx)
        e.sync()
        e.set_timing(8)
        e.reset_timing()
        t0 = time.perf_counter()
        e.step(4 * hx)
        e.sync()
        wall = (time.perf_counter() - t0) * 1e3
        t = e.timing()
    assert t["rounds"] == 4 and t["exchanges"] == 4, t
    assert t["round_ms"] > 0 and t["exchange_ms"] > 0
    assert 0 <= t["exchange_exposed_ms"] <= t["exchange_ms"] + 1e-6
    if overlap == 1:  # blocking: every exchange sits between two rounds
        assert t["exchange_exposed_ms"] == pytest.approx(t["exchange_ms"])
    assert t["round_ms"] + t["exchange_exposed_ms"] <= wall * 1.01 + 0.05, (t, wall)


@pytest.mark.parametrize("world,rank,size", [(4, 1, 4096), (8, 3, 65536)])
def test_rccl_exchange_mode_chosen_at_create(pkg, monkeypatch, world, rank, size):
    """exchange_overlap = 0 (late r06): a rank engine over RCCL times rounds of both
    exchange modes at create on its communicator (stripes.cpp tune_exchange; the
    self-loop here, xGMI between two MI355X) and keeps the faster.  Whichever it
    keeps, its field equals the host loopback transport's (which blocks) bytewise
    over full rounds, partial ones and a carried overlapped exchange; the choice
    follows the reported timings; forced modes report themselves untimed."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    chunks = None
    out = []
    for mode in ("rccl", "host"):
        kw = dict(uid=pkg.unique_id()) if mode == "rccl" else dict(transport=lambda su, sd: (su, sd))
        with pkg.Engine(size, size, rule=pkg.CONWAY, device=0, rank=rank, nranks=world, **kw) as e:
            if mode == "rccl":
                chosen, tb, to = e.exchange
                assert chosen in ("blocking", "overlapped") and tb > 0 and to > 0, e.exchange
                if abs(to - 0.98 * tb) > 1e-3 * tb:  # (the rounded report at the margin)
                    assert (chosen == "overlapped") == (to < 0.98 * tb), e.exchange
            else:
                assert e.exchange == ("blocking", 0.0, 0.0)
            hx = e.halo_depth
            chunks = [hx, 7, 2 * hx + 3]
            e.init_random(11)
            res = []
            for c in chunks:
                e.step(c)
                res.append((e.digest(), e.store_packed()))
        out.append(res)
    for i, ((da, a), (db, b)) in enumerate(zip(*out)):
        assert da == db and (a == b).all(), f"auto exchange mode vs host loopback, chunk {i}"
    for ov, name in ((1, "blocking"), (2, "overlapped")):
        with pkg.Engine(4096, 4096, rule=pkg.CONWAY, device=0, rank=1, nranks=4,
                        uid=pkg.unique_id(), exchange_overlap=ov) as e:
            assert e.exchange == (name, 0.0, 0.0)


def test_rccl_self_loop_two_communicators(pkg, monkeypatch):
    """A second engine on another self-loop communicator in the same process, and
    destroy/re-create: communicators are per engine."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    for _ in range(2):
        a = pkg.Engine(512, 640, rule=pkg.CONWAY, device=0, rank=1, nranks=3, uid=pkg.unique_id())
        b = pkg.Engine(512, 640, rule=pkg.CONWAY, device=0, rank=1, nranks=3, uid=pkg.unique_id())
        a.init_random(1)
        b.init_random(1)
        a.step(100)
        a.sync()
        b.step(100)
        assert a.digest() == b.digest()
        a.close()
        b.close()


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
