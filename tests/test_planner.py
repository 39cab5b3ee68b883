"""CPU suite: the launch planner (plan.cpp build_plans, pick_rows_per_wave,
age_skew, col_layout, half_units, rank_geometry) through the host-only model
gol_plan_model -- no GPU.  Also run under the host sanitizers
(tools/asan_cpu_suite.sh).

The model takes the device's CU count and the stencil kernels' occupancy (256-
thread workgroups per CU, 2 for the K = 16 kernels on MI355X) and returns the
first full-depth launch plan before the autotuner times its candidates.  The
checks restate what the kernel relies on (life_stencil.h): every strip's row
blocks tile the launch's rows (the kernel derives each unit's block from
rows_per_wave / rows_old / units_old), hand-off plans have even block lengths
of one tail-offset class (the pair forms take a step's parity from its index,
ADVICE r04) and fit one round of the occupancy (a waiting wavefront must never
hold the slot its producer needs).  Reference: Parallel_Life_MPI.cpp:70-81 (the
stripe arithmetic the planner generalises).
"""
import re

import pytest

CUS, OCC = 256, 2


def handoff_toff(R, K):
    """life_internal.h handoff_toff (2-plane lane groups)."""
    pf = 8 if K >= 16 else 4
    warm = -(-2 * K // pf) * pf
    if K < 4 or R + 2 < warm + 2 * pf:
        return -1
    off = (R + 2 - warm) % pf
    if off not in (0, pf // 2) and not (pf == 8 and off in (2, 6)):
        return -1
    return off if R + 2 - off >= warm + 2 * pf else -1


def strip_blocks(p, s):
    """Row blocks of strip s as the kernel derives them (life_stencil.h, the
    unit's rb / rlen from rows_per_wave, rows_old, units_old; blocks numbered
    bottom-up, the bottom jo of them old)."""
    lo, hi = p["rows_lo"], p["rows_hi"]
    nblk = p["blocks"]
    ry, ro, strips = p["rows_per_wave"], p["rows_old"], p["strips"]
    out = []
    for blk in range(nblk):
        rb, rlen = lo + blk * ry, ry
        if ro:
            jo = min(nblk, max(0, (p["units_old"] - s + strips - 1) // strips))
            ny = nblk - jo
            if blk >= ny:
                rb, rlen = lo + ny * ry + (blk - ny) * ro, ro
        out.append((rb, min(rb + rlen, hi)))
    return out


def check_plan(p, one_round=True):
    lo, hi = p["rows_lo"], p["rows_hi"]
    K = p["tb_depth"]
    assert 0 <= lo < hi
    assert p["blocks"] >= 1 and p["strips"] >= 1
    assert p["total_units"] == p["blocks"] * p["strips"] + p["half_units"]
    if p["lane_shift"] != 0:
        assert p["half_units"] == 0
    for s in range(p["strips"]):
        bl = strip_blocks(p, s)
        # contiguous, covering [lo, hi), every block non-empty
        assert bl[0][0] == lo and bl[-1][1] == hi, (s, bl[0], bl[-1])
        for (a0, a1), (b0, _) in zip(bl, bl[1:]):
            assert a1 == b0
        assert all(b > a for a, b in bl), s
    if p["rows_old"]:
        assert p["rows_old"] > p["rows_per_wave"] > 0
        assert p["units_old"] == 4 * CUS
        # one round of more than one wavefront per SIMD
        assert 4 * CUS < p["total_units"] <= OCC * 4 * CUS
    if p["handoff"]:
        assert p["blocks"] >= 2
        for R in (p["rows_per_wave"], p["rows_old"] or p["rows_per_wave"]):
            assert R % 2 == 0, R
            assert handoff_toff(R, K) == p["tail_off"] >= 0, (R, p["tail_off"])
        if one_round:
            assert p["total_units"] <= OCC * 4 * CUS


# the bench shapes (BASELINE configs 2-4): the plans the GPU runs measured
# (profiles/r05/wave_phases_*.jsonl, rank_proxy_*.jsonl); the autotuner may then
# replace them by a variant
BENCH = [
    # (h, rank, nranks, handoff, young, old, units)
    (65536, 0, 1, 0, 440, 619, 2044),
    (65536, 1, 2, 0, 220, 312, 2044),
    (65536, 2, 4, 1, 118, 158, 2032),
    (65536, 4, 8, 1, 58, 82, 2013),
    (262144, 0, 1, 0, 1775, 2460, 2043),
]


@pytest.mark.parametrize("h,rank,n,hand,young,old,units", BENCH)
def test_bench_shape_plans(pkg, h, rank, n, hand, young, old, units):
    p = pkg.plan_model(h, 65536, rank=rank, nranks=n)
    check_plan(p)
    assert (p["handoff"], p["rows_per_wave"], p["rows_old"], p["total_units"]) == \
        (hand, young, old, units)
    assert p["tb_depth"] == 16 and p["strips"] == 16 and p["half_units"] > 0
    if n > 1:
        # the shared region of a round's full-depth launches: [K, R + 2Hx - K)
        # (rank_geometry), clipped to the field at the first and last rank
        row0, R = pkg.rank_rows(h, n, rank)
        Hx = p["halo_depth"]
        glob0 = row0 - Hx
        lo = max(16, -glob0)
        hi = min(R + 2 * Hx - 16, h - glob0)
        assert (p["rows_lo"], p["rows_hi"]) == (lo, hi)
        assert p["candidates"] >= 1


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 12, 16])
def test_rank_plans_every_split(pkg, rule, n):
    R = pkg.REF_RULE if rule == "ref" else pkg.CONWAY
    for rank in sorted({0, n // 2, n - 1}):
        p = pkg.plan_model(65536, 65536, rank=rank, nranks=n, rule=R)
        check_plan(p)


@pytest.mark.parametrize("seed", range(4))
def test_single_field_plans_sweep(pkg, seed):
    """Many field shapes: every plan kind the planner makes (classic / hand-off,
    skewed or not, 64/32/16-lane strips, with and without the half strip)."""
    import random
    rnd = random.Random(seed)
    for _ in range(40):
        h = rnd.choice([rnd.randint(1, 300), rnd.randint(300, 20000), rnd.randint(20000, 140000)])
        w = rnd.choice([rnd.randint(1, 4200), rnd.randint(4200, 70000), 65536, 65536 + 64 * 62])
        rule = rnd.choice([pkg.REF_RULE, pkg.CONWAY])
        p = pkg.plan_model(h, w, rule=rule)
        check_plan(p)


@pytest.mark.parametrize("seed", range(4))
def test_rank_plans_sweep(pkg, seed):
    """Random splits (2-16 ranks, any rank, uneven stripes, both rules, both
    exchange modes): every rank's first full-depth plan tiles its rows and keeps
    the kernel's invariants."""
    import random
    rnd = random.Random(100 + seed)
    for _ in range(30):
        n = rnd.randint(2, 16)
        h = rnd.choice([rnd.randint(2 * n, 3000), rnd.randint(3000, 70000), rnd.randint(70000, 270000)])
        w = rnd.choice([rnd.randint(1, 4200), rnd.randint(4200, 70000), 65536])
        rank = rnd.randrange(n)
        rule = rnd.choice([pkg.REF_RULE, pkg.CONWAY])
        p = pkg.plan_model(h, w, rank=rank, nranks=n, rule=rule,
                           exchange_overlap=rnd.choice([0, 1, 2]))
        check_plan(p)


@pytest.mark.parametrize("h", [8192 + 2 * 128, 12288, 16384 + 2 * 192, 33024, 40000])
@pytest.mark.parametrize("handoff", [0, 1, 2])
def test_block_kinds_and_forced_lengths(pkg, h, handoff):
    p = pkg.plan_model(h, 65536, handoff=handoff)
    check_plan(p)
    if handoff == 1:
        assert p["handoff"] == 0
    for rpw in (58, 64, 90, 131):
        q = pkg.plan_model(h, 65536, handoff=handoff, rows_per_wave=rpw)
        # a forced length: no skew, several rounds allowed for classic blocks
        assert q["rows_old"] == 0 and q["rows_per_wave"] == rpw
        check_plan(q, one_round=False)


def test_overlap_rank_plans(pkg):
    """exchange_overlap = 2: the band and interior plans exist after the round's
    full-depth plans; the first full-depth plan is unchanged in kind."""
    p = pkg.plan_model(65536, 65536, rank=3, nranks=8, exchange_overlap=2)
    check_plan(p)
    assert p["plans"] == p["halo_depth"] + 2


def test_plan_model_rejects_bad_args(pkg):
    with pytest.raises(pkg.GolError):
        pkg.plan_model(100, 100, cus=0)
    with pytest.raises(pkg.GolError):
        pkg.plan_model(100, 100, rank=1, nranks=1)
    with pytest.raises(pkg.GolError):
        pkg.plan_model(10, 100, rank=0, nranks=20)


@pytest.mark.parametrize("passes", [2, 3])
@pytest.mark.parametrize("h,rank,n", [(65536, 4, 8), (65536, 2, 4), (8416, 0, 1), (3007, 0, 1)])
def test_multipass_plans(pkg, monkeypatch, passes, h, rank, n):
    """Multi-pass launches (GOL_DEV_PASSES, life_stencil.h): every wavefront
    waits for its row neighbours between passes, so the plan must be one round
    of the occupancy, one segment, and without the half strip (its pair units
    have no pass protocol).  Dev build only (GOL_LIB=.../libgol_dev.so)."""
    monkeypatch.setenv("GOL_DEV_PASSES", str(passes))
    p = pkg.plan_model(h, 65536, rank=rank, nranks=n, tb_depth=16)
    check_plan(p)
    if not re.search(rb"life_tb_kernelILi\d+ELi\dELi\dELb\dELi\dELb1E",
                     open(pkg.LIB_PATH, "rb").read()):
        # (r06) the shipped library has no multi-pass kernel: the switch is inert
        assert p["passes"] == 1
        return
    assert p["passes"] == passes
    assert p["half_units"] == 0
    assert p["total_units"] <= OCC * 4 * CUS
    # no multi-pass kernel at depth 8 (multipass_kernel_exists)
    assert pkg.plan_model(h, 65536, rank=rank, nranks=n, tb_depth=8)["passes"] == 1
    monkeypatch.delenv("GOL_DEV_PASSES")
    assert pkg.plan_model(h, 65536, rank=rank, nranks=n, tb_depth=16)["passes"] == 1


@pytest.mark.parametrize("h,n", [(32767, 2), (12289, 2), (65535, 4), (49151, 3), (24577, 4),
                                 (65536, 8), (1200, 3)])
def test_rank_geometry_agrees_across_ranks(pkg, h, n):
    """Every rank of a split must run the same fused depth K and halo depth Hx:
    neighbours exchange Hx rows each way per round, so a rank of 6145 rows beside
    ranks of 6144 (K 16 vs 8) or of 16384 beside 16383 (Hx 192 vs 128) would send
    and expect different row counts (stripes.cpp rank_geometry decides both from the
    smallest stripe, late r06).  The schedules then agree op for op."""
    got = [pkg.round_schedule(h, 4096, r, n, 300) for r in range(n)]
    assert len({(K, Hx) for _, K, Hx in got}) == 1, [(K, Hx) for _, K, Hx in got]
    kinds = [[(o["kind"], o["depth"]) for o in ops] for ops, _, _ in got]
    assert all(k == kinds[0] for k in kinds)


def test_rank_geometry_agrees_sweep(pkg):
    """The same over seeded random heights around every threshold (K at 6144 rows,
    Hx at 16384) and every split of 2..8 ranks, plus the halo's cap (<= the
    smallest stripe) for short stripes."""
    import random
    rnd = random.Random(7)
    hs = [rnd.randrange(n * t - 3 * n, n * t + 3 * n) for t in (6144, 16384) for n in range(2, 9)]
    hs += [rnd.randrange(16, 4000) for _ in range(12)]
    for h in hs:
        for n in range(2, 9):
            if h < n:
                continue
            kh = {pkg.round_schedule(h, 640, r, n, 50)[1:] for r in range(n)}
            assert len(kh) == 1, (h, n, kh)
            assert next(iter(kh))[1] <= h // n, (h, n, kh)
