"""GPU parity at the births-mask switch of the streaming kernel (life_stencil.h
t_plain_end, r04).

Rules with births run a unit's steady blocks without the mask (kPure) while no
block can emit a row below the field, and masked (kPureMask) from the first one
that can: t_plain_end = f_hi - prefetch + 2, f_hi = h - (rb - K) for the block
starting at row rb.  With rows_per_wave R forced (no skew) the bottom block
starts at rb = (nblk - 1) R and holds x = h - rb rows, so sweeping x over more
than a prefetch block's residues puts the switch exactly at a steady-block start
and one step on either side of it, for classic blocks and under hand-off
consumers (every block but the bottom one).  The width is not a multiple of 64:
the strip holding the ragged last group runs masked throughout, the interior
strips take the switch.  Reference: Parallel_Life_MPI.cpp:21-27 (dead border),
:37-54 (update).  ADVICE r04.
"""
import pytest

pytestmark = pytest.mark.gpu

W = 62 * 64 * 2 + 100  # 8036 columns: 126 groups, the last one ragged


def cases():
    # (K, prefetch, warm-up): the switch lands on a block start when
    # x + K - pf + 2 = warm + m pf
    for K, pf, warm in ((16, 8, 32), (12, 4, 24)):
        R = 64
        for x in range(warm + 2 * pf - K + pf - 2 - 1, warm + 2 * pf - K + 3 * pf):
            if x < 1:
                continue
            yield K, R, x


@pytest.mark.parametrize("K,R,x", list(cases()), ids=lambda v: str(v))
@pytest.mark.parametrize("handoff", [1, 2])
def test_births_mask_switch_conway(pkg, oracle, K, R, x, handoff):
    h = 2 * R + x
    seed = 31 * x + K
    g = oracle.bp_random(h, W, seed)
    with pkg.Engine(h, W, rule=pkg.CONWAY, device=0, tb_depth=K, rows_per_wave=R,
                    handoff=handoff) as e:
        assert e.rows_per_wave == R
        assert e.age_skew is None
        if handoff == 2:
            assert e.handoff
        for gens in (K, 2 * K + 5):
            e.init_random(seed)
            e.step(gens)
            want = oracle.bp_run(g, W, gens, oracle.CONWAY)
            assert (e.store_packed() == want).all(), f"h {h} K {K} gens {gens}"


@pytest.mark.parametrize("x", [38, 39, 40, 41, 42, 43, 44, 45, 46])
def test_births_mask_switch_highlife(pkg, oracle, x):
    """The generic-mask kernel (K = 12, hand-off) at the same switch."""
    K, R = 12, 64
    h = 3 * R + x
    g = oracle.bp_random(h, W, x)
    with pkg.Engine(h, W, rule=oracle.HIGHLIFE, device=0, tb_depth=K, rows_per_wave=R,
                    handoff=2) as e:
        e.init_random(x)
        e.step(K + 7)
        want = oracle.bp_run(g, W, K + 7, oracle.HIGHLIFE)
        assert (e.store_packed() == want).all()
