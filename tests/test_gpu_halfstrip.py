"""GPU parity of the edge-aligned strips and the packed half strip
(plan.cpp col_layout / half_units, life_stencil.h).

64-lane strips start at the field's left edge (strip 0 outputs groups 0..62: its
lane 0 sees the DPP shift's zero, the dead border of Parallel_Life_MPI.cpp:26-27)
and, in one-segment launches, the last strip ends at the right edge; the gap of at
most 30 lane groups between it and the strips before it runs as a 32-lane half
strip whose wavefronts carry two row blocks (lanes 32-63 offset by the second
block's rows).  Checked bit-exact against the CPU oracle at widths whose gap is
1, 15 and 30 groups (the last one partial), every rule kind, several launches and
a remainder; and at the full C3 / C5 widths against the same engine without the
half strip (GOL_DEV_PAIRS=0).
"""
import pytest

# plan properties: the cost models' plans (conftest.py model_plans)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("model_plans")]

THREADS = 16


def rule_of(pkg, name):
    return {"ref": pkg.REF_RULE, "conway": pkg.CONWAY,
            "highlife": (1 << 3 | 1 << 6, 1 << 2 | 1 << 3)}[name]


def test_c3_layout_has_half_strip(pkg):
    """65536 columns = 1024 lane groups: 16 strips + a 30-group half strip."""
    with pkg.Engine(65536, 65536, device=0) as e:
        strips, half_units, half_groups = e.columns
        assert (strips, half_groups) == (16, 30), e.columns
        assert half_units > 0


def test_edge_strips_4096_columns_one_strip(pkg):
    """4096 columns = 64 groups fit one edge-aligned strip (no halo lanes)."""
    with pkg.Engine(2048, 4096, device=0, resident=1) as e:
        assert e.columns[0] == 1 and e.columns[1] == 0, e.columns


@pytest.mark.parametrize("rule", ["ref", "conway", "highlife"])
@pytest.mark.parametrize("w", [64 * 127, 9000, 64 * 156, 64 * 189 + 17])
def test_half_strip_vs_oracle(pkg, oracle, w, rule):
    """Short row blocks (many interior pairs plus the border blocks alone), K = 8
    launches and a remainder launch, against the oracle."""
    h, gens, seed = 1500, 2 * 8 + 5, 7
    R = rule_of(pkg, rule)
    with pkg.Engine(h, w, rule=R, device=0, tb_depth=8, rows_per_wave=40, streams=1,
                    resident=1, handoff=1) as e:
        strips, half_units, half_groups = e.columns
        assert half_units > 0 and 1 <= half_groups <= 30, e.columns
        e.init_random(seed)
        e.step(gens)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(h, w, seed), w, gens, R, threads=THREADS)
    assert got == oracle.bp_digest(g, w)


@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_half_strip_depth16_skewed_vs_oracle(pkg, oracle, rule):
    """A per-GPU stripe shape of the 8-way split with classic blocks (age-skewed)
    and the half strip, one K = 16 launch (the hand-off default with it:
    test_gpu_skew.py)."""
    h, w = 8448, 65536
    R = rule_of(pkg, rule)
    with pkg.Engine(h, w, rule=R, device=0, streams=1, handoff=1) as e:
        assert e.columns[1] > 0, e.columns
        e.init_random(3)
        e.step(16)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(h, w, 3), w, 16, R, threads=THREADS)
    assert got == oracle.bp_digest(g, w)


@pytest.mark.parametrize("h,w", [(65536, 65536), (4096, 262144)])
def test_half_strip_equals_full_strips(pkg, monkeypatch, h, w):
    """Full widths of C3 and C5: several launches and a remainder of Conway with
    the half strip against the same engine without it."""
    gens = 3 * 16 + 6
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, streams=1, handoff=1) as e:
        assert e.columns[1] > 0, e.columns
        e.init_random(11)
        e.step(gens)
        got = e.digest()
    monkeypatch.setenv("GOL_DEV_PAIRS", "0")
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, streams=1, handoff=1) as e:
        assert e.columns[1] == 0, e.columns
        e.init_random(11)
        e.step(gens)
        assert e.digest() == got


@pytest.mark.parametrize("h,hand,half", [(8448, True, True), (16640, True, True),
                                         (33024, False, True), (65536, False, True)])
def test_block_kind_policy(pkg, h, hand, half):
    """The planner's choice per stripe height (plan.cpp build_plans,
    kHalfClassicRows): hand-off blocks for short stripes, classic blocks once their
    young blocks reach 160 rows, both with the half strip
    (profiles/r03/ab_half_strip_handoff_scale_sweep.jsonl)."""
    with pkg.Engine(h, 65536, device=0, streams=1) as e:
        assert e.handoff == hand and (e.columns[1] > 0) == half, (e.handoff, e.columns)


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("R,toff", [(62, 0), (64, 2), (66, 4), (68, 6)])
def test_handoff_tail_offsets_vs_oracle(pkg, oracle, R, toff, rule):
    """Hand-off blocks of every tail offset at depth 16 (0, 4 and, r03, 2 and 6:
    (R + 2 - 32) mod 8), with the half strip (8192 columns: a 2-group gap), two
    launches and a remainder, against the oracle."""
    assert (R + 2 - 32) % 8 == toff
    h, w, gens, seed = 900, 8192, 2 * 16 + 5, 13
    Rr = rule_of(pkg, rule)
    with pkg.Engine(h, w, rule=Rr, device=0, tb_depth=16, rows_per_wave=R, handoff=2,
                    streams=1, resident=1) as e:
        assert e.handoff and e.columns[1] > 0, (e.handoff, e.columns)
        e.init_random(seed)
        e.step(gens)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(h, w, seed), w, gens, Rr, threads=THREADS)
    assert got == oracle.bp_digest(g, w)
