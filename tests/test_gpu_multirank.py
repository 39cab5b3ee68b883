"""GPU parity of the multi-stripe path (row stripes + k-deep halo rounds).

gol_create_group runs the same partition (gol_rank_rows), halo layout and
shrinking launch rounds as the RCCL rank engines (gol_create_rank), with the
halo rows moved by device copies, so every stripe count can be checked on one
GPU against the oracle's single-field evolution.
"""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nranks", [2, 3, 4, 8])
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife"])
def test_group_matches_single_field(pkg, oracle, nranks, rule):
    R = {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE}[rule]
    h, w = 203, 4000
    g = oracle.bp_random(h, w, 3 + nranks)
    for tb, hx, gens, ho, lanes, rpw in ((8, 0, 37, 0, 0, 0), (4, 12, 30, 0, 0, 0),
                                         (2, 5, 11, 0, 0, 0), (1, 3, 7, 0, 0, 0),
                                         (16, 16, 33, 0, 0, 0), (8, 0, 37, 1, 0, 0),
                                         (16, 24, 50, 1, 0, 0), (16, 0, 70, 0, 32, 0),
                                         (8, 0, 37, 0, 16, 0), (8, 0, 37, 2, 0, 22),
                                         (16, 0, 40, 2, 0, 46), (4, 16, 45, 2, 0, 14)):
        ref = oracle.bp_run(g, w, gens, R)
        with pkg.Group(h, w, nranks, rule=R, tb_depth=tb, halo_depth=hx, handoff=ho,
                       strip_lanes=lanes, rows_per_wave=rpw) as grp:
            grp.load_packed(g)
            grp.step(gens)
            grp.sync()
            got = grp.store_packed()
            assert (got == ref).all(), f"tb {tb} hx {hx} gens {gens} handoff {ho}"
            assert grp.digest() == oracle.bp_digest(ref, w)


def test_group_reference_data(pkg, ref_data):
    """Intended semantics of the reference (its halo exchange actually working)
    == the reference's own -np 1 output."""
    gold = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))
    h, w = gold["h"], gold["w"]
    for case in gold["cases"]:
        if case["np"] != 1 or case["gens"] not in (1, 2, 3, 4, 100):
            continue
        with pkg.Group(h, w, 4) as grp:
            grp.load_ascii(ref_data)
            grp.step(case["gens"])
            out = grp.store_ascii()
        assert hashlib.sha256(out).hexdigest() == case["sha256"], case


def test_group_large_equals_single(pkg):
    """Size-independent property: 8 stripes of 2048 rows (hand-off row blocks,
    overlapped rounds) equal the single field."""
    h, w = 16384, 65536
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0) as e:
        e.init_random(9)
        e.step(100)
        want = e.digest()
    with pkg.Group(h, w, 8, rule=pkg.CONWAY) as grp:
        grp.init_random(9)
        grp.step(100)
        assert grp.digest() == want


def test_grouped_engine_refuses_solo_step(pkg):
    with pkg.Group(64, 64, 2) as grp:
        with pytest.raises(pkg.GolError) as ei:
            grp.members[0].step(1)
        assert ei.value.status == pkg.GOL_ESTATE


def test_rank_engine_single_rank(pkg, oracle):
    """gol_create_rank with nranks = 1 (no communicator) is a plain field."""
    h, w = 100, 130
    g = oracle.bp_random(h, w, 4)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, rank=0, nranks=1,
                    uid=pkg.unique_id()) as e:
        e.load_packed(g)
        e.step(20)
        assert (e.store_packed() == oracle.bp_run(g, w, 20, oracle.CONWAY)).all()


@pytest.mark.parametrize("nranks", [2, 4])
def test_group_overlap_across_calls(pkg, oracle, nranks):
    """Overlapped exchanges (R >= 2*halo) carried across gol_step calls, partial
    rounds, and reset by a reload."""
    h, w = 400, 1000
    g = oracle.bp_random(h, w, 17)
    with pkg.Group(h, w, nranks, rule=pkg.CONWAY, tb_depth=4, halo_depth=16) as grp:
        grp.load_packed(g)
        done = 0
        for chunk in (16, 16, 5, 32, 11, 16):
            grp.step(chunk)
            done += chunk
            want = oracle.bp_run(g, w, done, oracle.CONWAY)
            assert (grp.store_packed() == want).all(), f"after {done}"
        g2 = oracle.bp_random(h, w, 18)
        grp.load_packed(g2)
        grp.step(40)
        assert (grp.store_packed() == oracle.bp_run(g2, w, 40, oracle.CONWAY)).all()


@pytest.mark.parametrize("streams", [2, 3])
def test_composite_engine(pkg, oracle, ref_data, streams):
    """gol_create with streams = S: the field as S same-device stripes on S streams,
    behind the single-engine API (load/step/store/digest/timing)."""
    h, w = 1100, 777
    g = oracle.bp_random(h, w, 23)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, streams=streams, tb_depth=8) as e:
        assert (e.rows, e.row0) == (h, 0)
        e.load_packed(g)
        e.set_timing(1)
        for chunk in (7, 64, 129):
            e.step(chunk)
        e.sync()
        want = oracle.bp_run(g, w, 200, oracle.CONWAY)
        assert (e.store_packed() == want).all()
        assert e.digest() == oracle.bp_digest(want, w)
        t = e.timing()
        assert t["streams"] == streams and t["launches"] > 0
    gold = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))
    case = [c for c in gold["cases"] if c["np"] == 1 and c["gens"] == 100][0]
    with pkg.Engine(1500, 500, device=0, streams=streams) as e:
        e.load_ascii(ref_data)
        e.step(100)
        assert hashlib.sha256(e.store_ascii()).hexdigest() == case["sha256"]


def test_group_overlap_uneven_stripes(pkg, oracle):
    """Stripes of 2*halo and 2*halo-1 rows in one group: the overlap decision must
    be the same for every member."""
    h, w = 3 * 32 - 1, 300  # stripes 32, 32, 31 rows with halo 16
    g = oracle.bp_random(h, w, 5)
    with pkg.Group(h, w, 3, rule=pkg.CONWAY, tb_depth=4, halo_depth=16) as grp:
        grp.load_packed(g)
        for _ in range(3):
            grp.step(16)
        assert (grp.store_packed() == oracle.bp_run(g, w, 48, oracle.CONWAY)).all()


@pytest.mark.parametrize("h,n", [(12289, 2), (32767, 2)])
def test_group_stripes_straddling_depth_thresholds(pkg, oracle, h, n):
    """Auto depth and halo depth with stripes one row apart across a threshold
    (6145 / 6144 rows: K 16 vs 8 if decided per stripe; 16384 / 16383: Hx 192 vs
    128): every member runs the smallest stripe's K and Hx (stripes.cpp
    rank_geometry, late r06), and the group equals the single field (oracle)."""
    w, gens = 1024, 3 * 192 + 21
    g = oracle.bp_random(h, w, 9)
    with pkg.Group(h, w, n, rule=pkg.CONWAY) as grp:
        assert len({(m.tb_depth, m.halo_depth) for m in grp.members}) == 1
        grp.load_packed(g)
        grp.step(gens)
        assert (grp.store_packed() == oracle.bp_run(g, w, gens, oracle.CONWAY)).all()


@pytest.mark.parametrize("kind", ["group", "composite"])
def test_store_and_digest_without_sync_after_overlap(pkg, oracle, kind):
    """The last launch of an overlapped round writes the band rows on a second
    stream; store/digest right after gol_step (no gol_sync) must still see them.
    A Conway field keeps changing, so stale band rows would show."""
    h, w = 2000, 3000
    g = oracle.bp_random(h, w, 99)
    want = oracle.bp_run(g, w, 96, oracle.CONWAY)
    if kind == "group":
        eng = pkg.Group(h, w, 2, rule=pkg.CONWAY, tb_depth=8, halo_depth=32)
    else:
        eng = pkg.Engine(h, w, rule=pkg.CONWAY, device=0, streams=2, tb_depth=8, halo_depth=32)
    with eng:
        eng.load_packed(g)
        eng.step(96)  # 3 full rounds: ends with a band launch + overlapped exchange
        assert eng.digest() == oracle.bp_digest(want, w)
        eng.step(96)
        assert (eng.store_packed() == oracle.bp_run(want, w, 96, oracle.CONWAY)).all()


def test_group_reload_one_member(pkg, oracle):
    """A member reloaded after an overlapped step (its halos cleared) makes the next
    round exchange afresh for every member."""
    h, w = 600, 700
    g = oracle.bp_random(h, w, 5)
    with pkg.Group(h, w, 3, rule=pkg.CONWAY, tb_depth=4, halo_depth=16) as grp:
        grp.load_packed(g)
        grp.step(32)
        mid = oracle.bp_run(g, w, 32, oracle.CONWAY)
        m = grp.members[1]
        m.load_packed(mid[m.row0:m.row0 + m.rows])  # same rows, halos now stale
        grp.step(48)
        assert (grp.store_packed() == oracle.bp_run(mid, w, 48, oracle.CONWAY)).all()



def test_one_waiting_launch_per_device(pkg, oracle):
    """Hand-off row blocks wait for other wavefronts of their own launch; two such
    launches side by side could hold each other's slots.  Stripes sharing a device
    run concurrently, so only the first member on a device keeps hand-off blocks
    (and a rank's band launch, which runs beside its interior launch, is classic);
    results stay exact."""
    h, w = 6 * 3000, 8000
    g = oracle.bp_random(h, w, 12)
    with pkg.Group(h, w, 3, rule=pkg.CONWAY, tb_depth=16, handoff=2) as grp:
        assert [m.handoff for m in grp.members] == [True, False, False]
        grp.load_packed(g)
        grp.step(300)
        got = grp.store_packed()
    assert (got == oracle.bp_run(g, w, 300, oracle.CONWAY, threads=16)).all()


def test_waiting_kernel_registry_two_default_engines(pkg, oracle, model_plans):
    """Two default engines of one process on one GPU at a hand-off shape (8448 x
    65536: one-round launches with hand-off blocks when alone), stepped without
    syncs in between: only the first keeps hand-off blocks (engine.cpp wait
    registry), both fields exact; a small field created while it lives runs the
    streaming kernel, and gets the resident kernel again once it is gone."""
    h, w, gens = 8448, 65536, 48
    want = oracle.bp_digest(oracle.bp_run(oracle.bp_random(h, w, 5), w, gens, oracle.CONWAY,
                                          threads=16), w)
    a = pkg.Engine(h, w, rule=pkg.CONWAY, device=0)
    b = pkg.Engine(h, w, rule=pkg.CONWAY, device=0)
    small = pkg.Engine(2048, 4096, rule=pkg.CONWAY, device=0)
    try:
        assert a.handoff and not b.handoff, (a.handoff, b.handoff)
        assert small.resident is None
        for e in (a, b):
            e.init_random(5)
        for _ in range(3):
            a.step(gens // 3)
            b.step(gens // 3)
        assert a.digest() == want and b.digest() == want
    finally:
        for e in (a, b, small):
            e.close()
    with pkg.Engine(2048, 4096, device=0) as r, pkg.Engine(h, w, device=0) as c:
        assert r.resident is not None and not c.handoff
