"""GPU parity at the benchmark sizes (BASELINE.json configs[2..4]).

The timed path itself: gol_create(65536, 65536) with defaults is one stream of
K = 16 launches with age-skewed row blocks (plan.cpp age_skew) -- exactly what
bench.py measures; the 2-stripe composite engine (streams=2: 2 same-device
stripes on 2 streams, 256-row halo rounds) is checked the same way.  Checked
  * against the CPU oracle after one step(16) call (the K = 16 kernel runs);
  * after 600 more generations (two overlapped 256-generation rounds and a
    partial one) against a streams=1, tb_depth=1, classic-block engine, which the
    rest of the suite pins to the oracle at every size;
  * the C4 stripe shapes (row stripes of 65536^2 over 2/4/8 with halo rounds),
  * the C5 per-GPU unit (32768 x 262144) against the oracle.
Bit-exact (integer work): digests (live count + order-independent 64-bit hash)
must be equal.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 65536
THREADS = 16


def digest_of(pkg, h, w, rule, gens, seed=1, **kw):
    with pkg.Engine(h, w, rule=rule, device=0, **kw) as e:
        e.init_random(seed)
        if gens:
            e.step(gens)
        return e.digest()


@pytest.mark.parametrize("streams", [0, 2])
@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_c3_default_engine_vs_oracle_and_depth1(pkg, oracle, rule, streams):
    R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
    with pkg.Engine(N, N, rule=R, device=0, streams=streams) as e:
        assert e.tb_depth == 16 and e.resident is None, (e.tb_depth, e.resident)
        # (the autotuner may keep another variant of the skewed plan)
        assert (e.age_skew is not None) == (streams == 0) or e.tuning[0] != "models", e.age_skew
        e.init_random(1)
        e.step(16)  # one full-depth launch per stripe
        d16 = e.digest()
        e.step(600)  # composite: 2 overlapped 256-generation rounds + a partial one
        d616 = e.digest()
    g = oracle.bp_run(oracle.bp_random(N, N, 1), N, 16, R, threads=THREADS)
    assert d16 == oracle.bp_digest(g, N)
    del g
    assert d616 == digest_of(pkg, N, N, R, 616, streams=1, tb_depth=1)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_c4_stripes_equal_single_field(pkg, nranks):
    """C4 partition: 65536^2 in `nranks` row stripes (gol_rank_rows), default K and
    halo depth (8K = 128 for the 8192-row stripes, 12K = 192 above), 3 rounds + a
    partial one, overlapped exchanges."""
    hx = 128 if nranks == 8 else 192
    gens = 3 * hx + 40
    want = digest_of(pkg, N, N, pkg.CONWAY, gens, seed=4)
    with pkg.Group(N, N, nranks, rule=pkg.CONWAY) as grp:
        m = grp.members[0]
        assert (m.tb_depth, m.halo_depth) == (16, hx)
        grp.init_random(4)
        grp.step(gens)
        assert grp.digest() == want


@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_c5_per_gpu_unit_vs_oracle(pkg, oracle, rule):
    """The C5 weak-scaling unit (262144^2 over 8 GPUs = 32768 x 262144 per GPU)."""
    h, w = 32768, 262144
    R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
    got = digest_of(pkg, h, w, R, 16)
    g = oracle.bp_run(oracle.bp_random(h, w, 1), w, 16, R, threads=THREADS)
    assert got == oracle.bp_digest(g, w)


def test_c3_conway_1000_generations_vs_depth1(pkg):
    """The headline field under B3/S23 (still active after 1000 generations, unlike
    B/S2's fixed point within ~10): the default engine's 1000 generations (62
    full-depth age-skewed launches + a depth-8 one, graph replay) equal 1000
    depth-1 launches of classic blocks."""
    with pkg.Engine(N, N, rule=pkg.CONWAY, device=0) as e:
        assert e.tb_depth == 16 and (e.age_skew is not None or e.tuning[0] != "models")
        e.init_random(7)
        e.step(999)
        d999 = e.digest()
        e.step(1)
        d1000 = e.digest()
    assert d999 != d1000, "field reached a fixed point: the check would be weak"
    assert d1000 == digest_of(pkg, N, N, pkg.CONWAY, 1000, seed=7, streams=1, tb_depth=1,
                              handoff=1)


@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_c5_full_field_one_gpu_vs_oracle(pkg, oracle, rule):
    """The whole C5 field, 262144^2 (8 GiB per buffer), on ONE GPU with the default
    engine (one stream of age-skewed launches; the 144 TCUPS configuration of
    DESIGN.md §5) after one K = 16 launch, against the oracle's digest (24 GiB of
    host memory)."""
    n = 262144
    R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
    with pkg.Engine(n, n, rule=R, device=0) as e:
        assert e.tb_depth == 16 and (e.age_skew is not None or e.tuning[0] != "models"), \
            (e.tb_depth, e.age_skew)
        e.init_random(1)
        e.step(16)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(n, n, 1), n, 16, R, threads=THREADS)
    assert got == oracle.bp_digest(g, n)


def test_c3_headline_1000_generations_vs_oracle_fixed_point(pkg, oracle):
    """The headline job itself (65536^2, seed 1, B/S2, 1000 generations through
    the default engine: 62 age-skewed K = 16 launches + a depth-8 one, graph
    replay) against the oracle.  B/S2 has no births (Parallel_Life_MPI.cpp:44-50),
    so the live set only shrinks and reaches a fixed point: the oracle iterates
    until bp_run(g, 1) == g (about ten generations), which is then its state at
    every later generation, 1000 included."""
    with pkg.Engine(N, N, device=0) as e:
        assert e.tb_depth == 16 and e.resident is None
        e.init_random(1)
        e.step(1000)
        got = e.digest()
    g = oracle.bp_random(N, N, 1)
    for gen in range(1, 201):
        nxt = oracle.bp_run(g, N, 1, oracle.REF_RULE, threads=THREADS)
        if (nxt == g).all():
            break
        g = nxt
    else:
        pytest.fail("the oracle's B/S2 field reached no fixed point in 200 generations")
    assert gen < 1000
    assert got == oracle.bp_digest(g, N), f"fixed point reached at generation {gen}"


def test_conway_16384_1000_generations_vs_oracle(pkg, oracle):
    """B3/S23 for 1000 generations at the largest size the oracle evolves in well
    under a minute on the box (16384^2: 2.7e11 cell-generations), through the
    default engine there (K = 16 streaming launches of the skewed plan), against
    the oracle's own 1000 generations."""
    n = 16384
    with pkg.Engine(n, n, rule=pkg.CONWAY, device=0) as e:
        assert e.tb_depth == 16 and e.resident is None, (e.tb_depth, e.resident)
        e.init_random(3)
        e.step(1000)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(n, n, 3), n, 1000, oracle.CONWAY, threads=THREADS)
    assert got == oracle.bp_digest(g, n)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_c4_group_vs_oracle(pkg, oracle, nranks):
    """(r06) The C4 partition against the oracle itself, not only against the
    single engine: 65536^2 in 2 / 4 / 8 row stripes (gol_rank_rows), default K = 16
    and Hx (192 / 192 / 128), one full halo round and a partial one (Hx + 16
    generations, B3/S23 so births cross every stripe seam).  After G generations a row depends only on
    the rows within G of it, so the oracle evolves a band of +-(G + 32) rows
    around each stripe seam (and around one row in the middle of each stripe) with
    a dead border and its middle 64 rows are the exact global rows there: those
    are compared bytewise with the stripes' stored rows."""
    hx = 128 if nranks == 8 else 192
    G, half = hx + 16, 32
    with pkg.Group(N, N, nranks, rule=pkg.CONWAY) as grp:
        assert (grp.members[0].tb_depth, grp.members[0].halo_depth) == (16, hx)
        seams = [m.row0 for m in grp.members[1:]]
        mids = [m.row0 + m.rows // 2 for m in grp.members]
        grp.init_random(6)
        grp.step(G)
        got = grp.store_packed()
    g0 = oracle.bp_random(N, N, 6)
    for r in seams + mids + [0, N - half]:
        lo, hi = max(0, r - half - G), min(N, r + half + G)
        band = oracle.bp_run(g0[lo:hi], N, G, oracle.CONWAY, threads=THREADS)
        a, b = max(0, r - half), min(N, r + half)
        assert (got[a:b] == band[a - lo:b - lo]).all(), f"rows [{a}, {b})"


def test_c5_group_vs_oracle_at_seams(pkg, oracle):
    """(r06) The C5 partition, 262144^2 in 8 stripes of 32768 rows (Hx = 192,
    device-copy exchanges; 8 GiB per field buffer in all), on one GPU as an
    in-process group: one full halo round and a partial one (208 generations of
    B3/S23), checked against the oracle in light-cone bands around every stripe
    seam (the oracle builds only those rows of the splitmix64 field)."""
    n, half = 262144, 32
    with pkg.Group(n, n, 8, rule=pkg.CONWAY) as grp:
        m0 = grp.members[0]
        assert (m0.rows, m0.tb_depth, m0.halo_depth) == (32768, 16, 192)
        G = m0.halo_depth + 16
        grp.init_random(8)
        grp.step(G)
        for up, dn in zip(grp.members, grp.members[1:]):
            s = dn.row0
            got = np.concatenate([up.store_packed()[-half:], dn.store_packed()[:half]])
            lo, hi = s - half - G, s + half + G
            band = oracle.bp_run(oracle.bp_random_rows(lo, hi - lo, n, 8), n, G, oracle.CONWAY,
                                 threads=THREADS)
            assert (got == band[G:G + 2 * half]).all(), f"seam at row {s}"
