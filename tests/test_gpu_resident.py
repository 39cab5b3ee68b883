"""GPU parity of the resident kernel (life_resident.hip) vs the pinned oracle.

The resident kernel runs a whole gol_step in one launch on fields small enough
to sit in registers across the chip (the C2 regime, 4096^2): one workgroup per
(band, strip) tile, neighbour tiles swapping band rows through the ping-pong
field buffers every K generations under sc1 flags.  Bit-exact bar, every call
through the C ABI.  Covers: one strip with all 64 lanes as field groups and
multi-strip rows (62 groups + halo lanes, corner neighbours), partial last
bands, every rows-per-wavefront instantiation, K from 1 to the largest that
fits (including epoch lengths with no streaming instantiation), rules without and with births (B0 included: the dead border and columns
beyond w must stay masked), flag counts carried across launches, odd/even
epoch counts (buffer parity), and the hand-off under uneven load.
"""
import pytest

pytestmark = pytest.mark.gpu


def mask(ns):
    return sum(1 << n for n in ns)


def rules(oracle):
    return {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE,
            "b0": (mask([0, 1]), mask([8]))}


SHAPES = [(1, 1), (2, 64), (3, 4096), (17, 129), (100, 3969), (64, 4097), (130, 8000),
          (257, 200), (1000, 1000), (2000, 2048)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife", "b0"])
def test_resident_random_fields(pkg, oracle, shape, rule):
    h, w = shape
    R = rules(oracle)[rule]
    seed = 3 * h + w
    g = oracle.bp_random(h, w, seed)
    want = {n: oracle.bp_run(g, w, n, R) for n in (1, 3, 16, 21, 70)}
    for cfg in ({}, {"rows_per_wave": 2, "tb_depth": 1}, {"rows_per_wave": 3, "tb_depth": 7},
                {"rows_per_wave": 8, "tb_depth": 16},
                # epoch lengths the streaming kernel does not instantiate
                {"rows_per_wave": 4, "tb_depth": 22}, {"rows_per_wave": 6, "tb_depth": 5}):
        try:
            e = pkg.Engine(h, w, rule=R, device=0, resident=2, **cfg)
        except pkg.GolError:
            assert cfg, "the auto resident plan must fit every small shape"
            continue  # this (rows, K) does not fit the shape
        with e:
            assert e.resident is not None, cfg
            for n, ref in want.items():
                e.init_random(seed)
                e.step(n)
                assert (e.store_packed() == ref).all(), f"{cfg} gens {n}"
                assert e.digest() == oracle.bp_digest(ref, w)


@pytest.mark.parametrize("rule", ["ref", "conway", "b0"])
def test_resident_chunks_carry_flags_and_parity(pkg, oracle, rule):
    """Consecutive gol_step calls (flag counts continue from the previous launch,
    odd and even epoch counts flip the current buffer) match one long run."""
    h, w = 700, 5000  # 2 strips
    R = rules(oracle)[rule]
    g = oracle.bp_random(h, w, 5)
    with pkg.Engine(h, w, rule=R, device=0, resident=2, rows_per_wave=4, tb_depth=8) as e:
        assert e.resident is not None and e.resident[1] == 2
        e.load_packed(g)
        total = 0
        for n in (1, 1, 8, 9, 16, 3, 40, 1, 1, 1, 24):
            e.step(n)
            total += n
            assert (e.store_packed() == oracle.bp_run(g, w, total, R)).all(), total


def test_resident_auto_only_without_streaming_knobs(pkg):
    with pkg.Engine(4096, 4096, device=0) as e:
        assert e.resident is not None
        bands, strips = e.resident
        assert strips == 1 and bands >= 1
    with pkg.Engine(4096, 4096, device=0, tb_depth=8) as e:
        assert e.resident is None  # a streaming-kernel knob: the streaming kernel
    with pkg.Engine(4096, 4096, device=0, resident=1) as e:
        assert e.resident is None
    with pkg.Engine(65536, 65536, device=0, streams=1) as e:
        assert e.resident is None  # does not fit
    with pytest.raises(pkg.GolError):
        pkg.Engine(4096, 4096, device=0, resident=3)


@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_resident_c2_1000_generations_vs_streaming(pkg, rule):
    """C2 (4096^2 x 1000): the resident engine equals the streaming engine
    (depth 8) and the depth-1 kernel, field for field."""
    R = pkg.REF_RULE if rule == "ref" else pkg.CONWAY
    out = []
    for kw in ({}, {"resident": 1, "tb_depth": 8}, {"resident": 1, "tb_depth": 1}):
        with pkg.Engine(4096, 4096, rule=R, device=0, **kw) as e:
            assert (e.resident is not None) == (not kw)
            e.init_random(1)
            e.step(1000)
            out.append((e.store_packed(), e.digest()))
    for f, d in out[1:]:
        assert d == out[0][1]
        assert (f == out[0][0]).all()


def test_resident_timing(pkg):
    with pkg.Engine(4096, 4096, device=0) as e:
        e.init_random(1)
        e.set_timing(True)
        e.step(100)
        e.step(7)
        e.sync()
        t = e.timing()
    assert t["launches"] == 2
    assert t["kernel_ms"] > 0
    assert t["cell_gens"] == 4096 * 4096 * 107
    assert t["cell_gens_computed"] >= t["cell_gens"]


def test_resident_under_uneven_load(pkg, oracle):
    """The neighbour hand-off with the chip busy: a streaming engine keeps
    launching on its own stream while the resident engine runs (tiles start late
    and unevenly); every word checked."""
    h, w = 2048, 4096
    R = oracle.CONWAY
    g = oracle.bp_random(h, w, 9)
    want = oracle.bp_run(g, w, 300, R)
    # the busy engine uses classic row blocks: one waiting launch per device
    with pkg.Engine(16384, 16384, device=0, resident=1, streams=1, handoff=1) as big, \
            pkg.Engine(h, w, rule=R, device=0) as e:
        assert e.resident is not None
        big.init_random(2)
        for rep in range(3):
            e.load_packed(g)
            big.step(160)  # queued on big's stream: ~10 launches running beside e
            e.step(300)
            got = e.store_packed()
            assert (got == want).all(), f"repetition {rep}"
        big.sync()


def test_two_resident_engines_interleaved(pkg, oracle):
    """Two resident engines of one process stepped without syncs in between: their
    launches share one ordered stream per device (each needs every CU for its
    tiles), so neither waits on tiles the other keeps off the chip."""
    shapes = [(4096, 4096), (3000, 2500)]
    fields = [oracle.bp_random(h, w, h + 1) for h, w in shapes]
    engines = [pkg.Engine(h, w, rule=oracle.CONWAY, device=0) for h, w in shapes]
    try:
        for e, g in zip(engines, fields):
            assert e.resident is not None
            e.load_packed(g)
        for chunk in (40, 7, 33):
            for e in engines:
                e.step(chunk)
        for e, g, (h, w) in zip(engines, fields, shapes):
            assert (e.store_packed() == oracle.bp_run(g, w, 80, oracle.CONWAY, threads=16)).all()
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_resident_cooperative_launch(pkg, oracle, monkeypatch, rule):
    """GOL_DEV_RES_COOP=1: the same kernel through hipLaunchCooperativeKernel (the
    device re-checks that every tile is resident at once), multi-strip rows and
    two launches carrying the epoch flags, against the oracle."""
    monkeypatch.setenv("GOL_DEV_RES_COOP", "1")
    h, w = 1000, 5000
    R = rules(oracle)[rule]
    g = oracle.bp_random(h, w, 21)
    with pkg.Engine(h, w, rule=R, device=0, resident=2) as e:
        assert e.resident is not None
        e.init_random(21)
        e.step(37)
        e.step(40)
        got = e.store_packed()
    assert (got == oracle.bp_run(g, w, 77, R)).all()


# ------------------------------------------------ wave-level temporal blocking
# life_resident_mb.hip (r06): the wavefronts of a tile swap MB rows through LDS
# every MB generations.  GOL_DEV_RES_MB selects it at create (the planner's
# default is reported by Engine.resident_rows[3]).
MB_CASES = [(2, 2), (3, 2), (3, 3), (4, 2), (4, 3), (4, 4)]


@pytest.fixture
def mb_kernels(pkg):
    """The MB kernels are in the dev build only (measured slower):
    these tests run with GOL_LIB=.../libgol_dev.so and skip otherwise."""
    if b"life_res_mb_kernel" not in open(pkg.LIB_PATH, "rb").read():
        pytest.skip("wave-level blocking kernels are in the dev build only (GOL_LIB=libgol_dev.so)")


@pytest.mark.parametrize("rows,mb", MB_CASES, ids=lambda v: str(v))
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife", "b0"])
def test_resident_mb_random_fields(pkg, oracle, monkeypatch, mb_kernels, rows, mb, rule):
    """Every (rows, MB) kernel vs the oracle: one strip and multi-strip rows
    (halo lanes), partial last bands, epoch lengths K that are and are not
    multiples of MB (partial last super-steps), generation counts that end
    inside a super-step and inside an epoch."""
    if rule in ("highlife", "b0") and mb == 4:
        pytest.skip("no generic-mask kernel at MB = 4 (it spills)")
    monkeypatch.setenv("GOL_DEV_RES_MB", str(mb))
    R = rules(oracle)[rule]
    for h, w, K in ((17, 129, 3), (100, 3969, 7), (64, 4097, 8), (257, 200, 5),
                    (1000, 1000, 16), (130, 8000, 11)):
        seed = 3 * h + w + mb
        g = oracle.bp_random(h, w, seed)
        try:
            e = pkg.Engine(h, w, rule=R, device=0, resident=2, rows_per_wave=rows, tb_depth=K)
        except pkg.GolError:
            continue  # (rows, K) does not fit the shape
        with e:
            assert e.resident_rows == (rows, e.resident_rows[1], K, mb), e.resident_rows
            for n in (1, mb, K + 1, 2 * K + mb - 1, 45):
                e.load_packed(g)
                e.step(n)
                ref = oracle.bp_run(g, w, n, R)
                assert (e.store_packed() == ref).all(), f"{h}x{w} K {K} gens {n}"


@pytest.mark.parametrize("mb", [2, 3])
@pytest.mark.parametrize("rule", ["ref", "conway"])
def test_resident_mb_c2_auto_plan(pkg, oracle, monkeypatch, mb_kernels, mb, rule):
    """The C2 field with the auto resident plan (4096^2: 256 tiles of 16 rows,
    K = 16) and wave-level blocking, per generation for the early B/S2
    generations, and 1000 generations against the oracle."""
    monkeypatch.setenv("GOL_DEV_RES_MB", str(mb))
    R = rules(oracle)[rule]
    n = 4096
    g0 = oracle.bp_random(n, n, 1)
    want = {0: g0}
    for gen in range(1, 10):
        want[gen] = oracle.bp_run(want[gen - 1], n, 1, R, threads=16)
    with pkg.Engine(n, n, rule=R, device=0) as e:
        assert e.resident is not None
        rows = e.resident_rows[0]
        assert e.resident_rows[3] == (mb if mb <= rows else 1), e.resident_rows
        for gens in range(1, 10):
            e.init_random(1)
            e.step(gens)
            assert e.digest() == oracle.bp_digest(want[gens], n), gens
        e.init_random(1)
        e.step(1000)
        assert e.digest() == oracle.bp_digest(oracle.bp_run(g0, n, 1000, R, threads=16), n)
