"""GPU parity of age-skewed row blocks (plan.cpp age_skew, life_stencil.h).

A one-round launch at 2 wavefronts per SIMD gives the units dispatched first
(the older wave of each SIMD) longer row blocks than the others.  The blocks of a
strip then have two lengths and the block count differs from ceil(rows / R), so
the row ranges, the hand-off roles and the last (truncated) block all move.  The
per-GPU stripe shapes of the 2/4/8-way 65536^2 split are checked bit-exact
against the CPU oracle (one K = 16 launch), and over several launches against
the same engine with equal blocks.
"""
import pytest

# plan properties: the cost models' plans (conftest.py model_plans)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("model_plans")]

W = 65536
THREADS = 16


def rule_of(oracle, rule):
    return oracle.REF_RULE if rule == "ref" else oracle.CONWAY


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("handoff", [1, 2])
@pytest.mark.parametrize("rows", [8448, 16640])
def test_skewed_stripe_vs_oracle(pkg, oracle, rows, handoff, rule):
    R = rule_of(oracle, rule)
    with pkg.Engine(rows, W, rule=R, device=0, handoff=handoff, streams=1) as e:
        assert e.tb_depth == 16 and e.age_skew is not None, (e.tb_depth, e.age_skew)
        ro, ry, uo = e.age_skew
        assert ro > ry > 0 and uo > 0
        e.init_random(3)
        e.step(16)  # one K = 16 launch
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(rows, W, 3), W, 16, R, threads=THREADS)
    assert got == oracle.bp_digest(g, W)


@pytest.mark.parametrize("rows", [8448, 12288, 33024])
def test_skewed_equals_equal_blocks(pkg, monkeypatch, rows):
    """Several full-depth launches and a remainder (Conway keeps the field
    changing) with the planner's automatic choice, against equal blocks."""
    gens = 5 * 16 + 8
    with pkg.Engine(rows, W, rule=pkg.CONWAY, device=0, streams=1) as e:
        assert e.age_skew is not None
        e.init_random(5)
        e.step(gens)
        got = e.digest()
    monkeypatch.setenv("GOL_DEV_AGE_SKEW", "0")
    with pkg.Engine(rows, W, rule=pkg.CONWAY, device=0, streams=1) as e:
        assert e.age_skew is None
        e.init_random(5)
        e.step(gens)
        assert e.digest() == got


def test_default_c3_engine_is_one_skewed_stream(pkg):
    """gol_create(65536, 65536) runs one stream of skewed one-round launches
    (it beats the 2-stripe composite), and says so in its plan."""
    with pkg.Engine(W, W, device=0) as e:
        assert e.age_skew is not None and e.tb_depth == 16
        e.set_timing(1)
        e.init_random(1)
        e.step(16)
        e.sync()
        assert e.timing()["streams"] == 1


def test_no_skew_when_launches_share_the_device(pkg):
    """Composite stripes and group members on one GPU launch concurrently, so the
    dispatch-order premise does not hold: equal blocks."""
    with pkg.Engine(W, W, device=0, streams=2) as e:
        assert e.age_skew is None
    with pkg.Group(16640 * 2, W, 2) as grp:
        assert all(m.age_skew is None for m in grp.members)


def test_no_skew_for_forced_rows_or_multi_round(pkg):
    with pkg.Engine(8448, W, device=0, streams=1, rows_per_wave=74) as e:
        assert e.age_skew is None  # a caller's rows_per_wave is kept as given
    with pkg.Engine(2048, W, device=0, streams=1, resident=1) as e:
        assert e.age_skew is None  # fewer units than one workgroup per CU x 4


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("h,w,skewed", [
    (9000, 20000, True),     # 6 strips, blocks of 35 / 19 rows
    (12001, 65613, True),    # odd height, a partial last lane group, hand-off blocks
    (7001, 40000, True),     # 11 strips, a partial 11th
    (6500, 65536, True),     # the shortest stripe at K = 16, hand-off
    (20000, 3000, False),    # one strip at the minimum block length: nothing to skew
    (5003, 65613, False),    # K = 8 (more than 2 waves per SIMD): equal blocks
])
def test_skew_shapes_vs_oracle(pkg, oracle, h, w, skewed, rule):
    """Skewed launches on shapes away from the bench's: a few strips, odd widths
    and heights (a partial last lane group and last block), both block kinds, and
    shapes the planner leaves unskewed -- 27 generations (full-depth launches and
    the remainder depths)."""
    R = rule_of(oracle, rule)
    gens = 16 + 8 + 3
    with pkg.Engine(h, w, rule=R, device=0, streams=1, resident=1) as e:
        assert (e.age_skew is not None) == skewed, e.age_skew
        e.init_random(11)
        e.step(gens)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(h, w, 11), w, gens, R, threads=THREADS)
    assert got == oracle.bp_digest(g, w)


@pytest.mark.parametrize("shift", ["11310011:1", "33000000:1", "01230123:2", "30303030:1"])
@pytest.mark.parametrize("handoff", [1, 2])
def test_xcd_row_shift_vs_oracle(pkg, oracle, monkeypatch, shift, handoff):
    """(r06 dev A/B, GOL_DEV_XCD_SHIFT, dev build; green on the shipped-library build
    that carried it, profiles/r06/gpu_tests_xcd_shift.log) paired blocks of a strip trade 8 rows by
    the speed class of their workgroups' XCD: every strip stays tiled exactly, with
    hand-off and classic blocks, the skewed lengths and the launch's remainder
    depths.  B3/S23 so births cross the moved block seams."""
    if b"life_res_mb_kernel" not in open(pkg.LIB_PATH, "rb").read():
        pytest.skip("the row shift is in the dev build only (GOL_LIB=.../libgol_dev.so)")
    monkeypatch.setenv("GOL_DEV_XCD_SHIFT", shift)
    rows, gens = 8448, 16 + 8 + 5
    with pkg.Engine(rows, W, rule=pkg.CONWAY, device=0, handoff=handoff, streams=1) as e:
        assert e.age_skew is not None
        e.init_random(5)
        e.step(gens)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(rows, W, 5), W, gens, oracle.CONWAY, threads=THREADS)
    assert got == oracle.bp_digest(g, W)
