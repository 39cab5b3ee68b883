"""GPU parity of multi-pass launches (life_stencil.h, r05; dev switch
GOL_DEV_PASSES = 2 or 3 at engine create).

A multi-pass launch runs P passes of K generations over the same row blocks,
odd passes bottom-up, with per-pass head/done flags between row neighbours, the
hand-off side rows and flags per pass parity, and the halo lanes' own values
kept across passes in a shadow half of each buffer.  Checked against the oracle
(Parallel_Life_MPI.cpp:37-54 update, :21-27 dead border) for classic and
hand-off blocks, forced and auto (age-skewed) block lengths, B/S2, B3/S23 and the
generic-mask kernel, generation counts that mix multi-pass and single-pass
launches, narrow fields (32/16-lane strips); and for rank engines (host loopback
transport) against the same engine without passes, bytewise, at the 8-way C4
rank shape.

Since r06 the multi-pass kernels are compiled into the dev build only (make dev;
the shipped libgol.so carries none, tests/test_abi.py): run this module with
GOL_LIB=mpi-game-of-life_amd/libgol_dev.so.  Against the shipped library it skips.
"""
import re

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _needs_multipass_kernels(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    if not re.search(rb"life_tb_kernelILi\d+ELi\dELi\dELb\dELi\dELb1E", blob):
        pytest.skip("multi-pass kernels are in the dev build only (GOL_LIB=.../libgol_dev.so)")

W = 62 * 64 * 2 + 100  # 8036 columns: 3 strips, the last group ragged


def rule_of(oracle, name):
    return {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[name]


@pytest.mark.parametrize("passes", [2, 3])
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife"])
@pytest.mark.parametrize("handoff", [1, 2])
@pytest.mark.parametrize("rpw", [0, 64, 90])
def test_multipass_single_field(pkg, oracle, monkeypatch, passes, rule, handoff, rpw):
    monkeypatch.setenv("GOL_DEV_PASSES", str(passes))
    R = rule_of(oracle, rule)
    K = 12 if rule == "highlife" else 16
    h = 3000 + 7 * passes + rpw
    seed = 5 * passes + rpw + handoff
    g = oracle.bp_random(h, W, seed)
    kw = dict(rows_per_wave=rpw) if rpw else {}
    with pkg.Engine(h, W, rule=R, device=0, tb_depth=K, handoff=handoff, **kw) as e:
        assert e.passes == passes, (e.passes, e.handoff, e.rows_per_wave)
        if handoff == 2:
            assert e.handoff
        for gens in (passes * K, passes * K + 5, 2 * passes * K + K):
            e.init_random(seed)
            e.step(gens)
            want = oracle.bp_run(g, W, gens, R)
            assert (e.store_packed() == want).all(), f"gens {gens}"


@pytest.mark.parametrize("w", [700, 1500, 4000])
@pytest.mark.parametrize("passes", [2, 3])
def test_multipass_narrow_fields(pkg, oracle, monkeypatch, w, passes):
    """Narrow fields: 16/32-lane strips (several strips per wavefront) and the
    edge-aligned single strip."""
    monkeypatch.setenv("GOL_DEV_PASSES", str(passes))
    h, K = 2500, 16
    g = oracle.bp_random(h, w, w)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, tb_depth=K) as e:
        assert e.passes == passes
        for gens in (passes * K, 3 * passes * K + 3):
            e.init_random(w)
            e.step(gens)
            want = oracle.bp_run(g, w, gens, oracle.CONWAY)
            assert (e.store_packed() == want).all(), f"w {w} gens {gens}"


def test_multipass_graph_replay(pkg, oracle, monkeypatch):
    """Repeated gol_step calls replay one captured graph: the flags every launch
    leaves at 0 (each reset by its reader) must hold across replays."""
    monkeypatch.setenv("GOL_DEV_PASSES", "3")
    h, w, K = 4000, W, 16
    g = oracle.bp_random(h, w, 77)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, tb_depth=K) as e:
        assert e.passes == 3
        e.load_packed(g)
        for _ in range(4):
            e.step(6 * K)
        want = oracle.bp_run(g, w, 24 * K, oracle.CONWAY)
        assert (e.store_packed() == want).all()


@pytest.mark.parametrize("passes", [2, 3])
@pytest.mark.parametrize("world,rank,handoff", [(2, 0, 0), (3, 1, 2), (4, 3, 1)])
def test_multipass_rank_equals_single_pass(pkg, oracle, monkeypatch, passes, world, rank, handoff):
    """Rank engines (host loopback transport): consecutive full-depth launches of
    a round merge into multi-pass launches; the field is bytewise the one the same
    engine computes without passes."""
    h, w = 3000, 5000
    own_g = oracle.bp_random(h, w, 9)
    loop = lambda su, sd: (su, sd)  # noqa: E731
    out = []
    for np_ in (1, passes):
        if np_ > 1:
            monkeypatch.setenv("GOL_DEV_PASSES", str(np_))
        else:
            monkeypatch.delenv("GOL_DEV_PASSES", raising=False)
        with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, rank=rank, nranks=world, tb_depth=16,
                        handoff=handoff, transport=loop) as e:
            assert e.passes == np_
            e.load_packed(own_g[e.row0:e.row0 + e.rows])
            res = []
            for c in (e.halo_depth, 37, 2 * e.halo_depth + 16):
                e.step(c)
                res.append((e.store_packed(), e.digest()))
            out.append(res)
    for i, ((a, da), (b, db)) in enumerate(zip(*out)):
        assert da == db and (a == b).all(), f"chunk {i}"


def test_multipass_c4_rank_shape(pkg, monkeypatch):
    """The 8-way C4 per-rank shape (8192 own rows + 2 x 128 halo rows of 65536^2,
    default plan kind), 2 and 3 passes against single-pass launches, bytewise."""
    n, world, rank, gens = 65536, 8, 3, 2 * 128 + 40
    loop = lambda su, sd: (su, sd)  # noqa: E731
    out = []
    for np_ in (1, 2, 3):
        if np_ > 1:
            monkeypatch.setenv("GOL_DEV_PASSES", str(np_))
        else:
            monkeypatch.delenv("GOL_DEV_PASSES", raising=False)
        with pkg.Engine(n, n, rule=pkg.REF_RULE, device=0, rank=rank, nranks=world,
                        transport=loop) as e:
            assert e.passes == np_
            e.init_random(3)
            e.step(gens)
            out.append((e.digest(), e.store_packed()))
    for d, f in out[1:]:
        assert d == out[0][0]
        assert (f == out[0][1]).all()
