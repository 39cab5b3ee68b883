"""GPU parity: libgol.so (HIP kernels on the MI355X) vs the pinned CPU oracle.

Bar: bit-exact (integer/bit work).  Every call goes through the C ABI; there is
no CPU fallback in the product, so these tests fail if the kernels are wrong or
libgol.so cannot reach a GPU.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))
H, W = GOLD["h"], GOLD["w"]
DEPTHS = [1, 2, 4, 6, 7, 8, 12, 16]  # the shipped library's fused depths
HAND_DEPTHS = [d for d in DEPTHS if d >= 4]  # depths with hand-off row blocks


def mask(ns):
    return sum(1 << n for n in ns)


def rules(oracle):
    return {"ref": oracle.REF_RULE, "conway": oracle.CONWAY, "highlife": oracle.HIGHLIFE,
            "daynight": (mask([3, 6, 7, 8]), mask([3, 4, 6, 7, 8])),
            "seeds": (mask([2]), 0),
            "b0": (mask([0, 1]), mask([8]))}


# ---------------------------------------------------------------- golden (C1)
@pytest.mark.parametrize("case", [c for c in GOLD["cases"] if c["gens"] <= 100],
                         ids=lambda c: f"np{c['np']}-e{c['gens']}")
def test_reference_outputs(pkg, ref_data, case):
    sem = pkg.SEM_GLOBAL if case["np"] == 1 else pkg.SEM_REF_STRIPES
    with pkg.Engine(H, W, device=0, semantics=sem, ref_ranks=case["np"]) as e:
        e.load_ascii(ref_data)
        e.step(case["gens"])
        e.sync()
        out = e.store_ascii(H * (W + 1))
    assert out.count(b"1") == case["live"]
    assert hashlib.sha256(out).hexdigest() == case["sha256"]


def test_reference_1000_generations(pkg, ref_data):
    case = [c for c in GOLD["cases"] if c["gens"] == 1000][0]
    with pkg.Engine(H, W, device=0) as e:
        e.load_ascii(ref_data)
        e.step(1000)
        out = e.store_ascii(H * (W + 1))
    assert hashlib.sha256(out).hexdigest() == case["sha256"]


@pytest.mark.parametrize("depth", DEPTHS)
def test_reference_per_generation(pkg, oracle, ref_data, depth):
    """Gens 1..8 and 12, 16 at every fused depth, each count reached by ONE
    gol_step(g) call on a fresh load, so the fused kernel of that depth (and the
    remainder depths pick_depth chooses) really runs (the B/S2 field reaches a
    fixed point after ~5 gens, so the early gens carry the information)."""
    g0 = oracle.bp_pack(ref_data, H, W)
    want = {0: g0}
    for gen in range(1, 17):
        want[gen] = oracle.bp_run(want[gen - 1], W, 1)
    with pkg.Engine(H, W, device=0, tb_depth=depth) as e:
        for gens in (1, 2, 3, 4, 5, 6, 7, 8, 12, 16):
            e.load_ascii(ref_data)
            e.step(gens)
            assert (e.store_packed() == want[gens]).all(), f"depth {depth} gens {gens}"


# ------------------------------------------------- random fields, all rules
SHAPES = [(1, 1), (1, 70), (2, 64), (3, 63), (5, 65), (17, 129), (64, 500), (100, 3969),
          (33, 3968), (40, 7937), (257, 200)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife"])
def test_random_fields_every_depth(pkg, oracle, shape, rule):
    h, w = shape
    R = rules(oracle)[rule]
    seed = h * 1000 + w
    want = {}
    g = oracle.bp_random(h, w, seed)
    for gens in (1, 3, 16, 21, 70):
        want[gens] = oracle.bp_run(g, w, gens, R)
    for depth in DEPTHS:
        for handoff in ((1, 2) if depth >= 4 else (1,)):
            with pkg.Engine(h, w, rule=R, device=0, tb_depth=depth, handoff=handoff) as e:
                for gens, ref in want.items():
                    e.init_random(seed)
                    e.step(gens)
                    got = e.store_packed()
                    assert (got == ref).all(), f"depth {depth} handoff {handoff} gens {gens}"
                    assert e.digest() == oracle.bp_digest(ref, w)


@pytest.mark.parametrize("lanes", [64, 32, 16])
@pytest.mark.parametrize("rule", ["ref", "conway", "daynight"])
def test_strip_widths(pkg, oracle, lanes, rule):
    """Narrow strips (32/16 lanes, 2/4 per wavefront): strip seams inside a
    wavefront, partial last strip groups, every depth class."""
    R = rules(oracle)[rule]
    for h, w in [(1, 1), (7, 65), (40, 1921), (33, 1983), (129, 4097), (64, 900), (9, 3969)]:
        seed = 7 * h + w
        g = oracle.bp_random(h, w, seed)
        for depth in (1, 4, 8, 16):
            for gens in (3, 33, 70):
                ref = oracle.bp_run(g, w, gens, R)
                with pkg.Engine(h, w, rule=R, device=0, tb_depth=depth, strip_lanes=lanes) as e:
                    assert e.strip_lanes == lanes
                    e.init_random(seed)
                    e.step(gens)
                    assert (e.store_packed() == ref).all(), f"{h}x{w} depth {depth} gens {gens}"


def handoff_toff(R, K):
    """life_internal.h handoff_toff (2-plane lane groups): the tail offset of a
    hand-off launch with R rows per wavefront, or -1 if R does not fit."""
    pf = 8 if K >= 16 else 4
    warm = -(-2 * K // pf) * pf
    if K < 4 or R + 2 < warm + 2 * pf:
        return -1
    off = (R + 2 - warm) % pf
    if off not in (0, pf // 2):
        return -1
    return off if R + 2 - off >= warm + 2 * pf else -1


@pytest.mark.parametrize("rpw", [14, 16, 22, 24, 30, 31, 32, 46, 48, 100])
@pytest.mark.parametrize("handoff", [1, 2])
def test_row_blocking(pkg, oracle, rpw, handoff):
    """Many row blocks per strip (rows_per_wave small): block seams exact, both
    block closures.  Hand-off needs R + 2 - warm-up (16 steps at depth 8) to be 0
    or 2 modulo the 4-step prefetch block and at least 2 blocks: from 22 rows on,
    even R hand over, the others fall back to classic blocks."""
    h, w = 300, 4100
    g = oracle.bp_random(h, w, 5)
    ref = oracle.bp_run(g, w, 16, oracle.CONWAY)
    for lanes in (64, 32, 16):
        with pkg.Engine(h, w, rule=oracle.CONWAY, device=0, tb_depth=8, rows_per_wave=rpw,
                        handoff=handoff, strip_lanes=lanes) as e:
            assert e.handoff == (handoff == 2 and handoff_toff(rpw, 8) >= 0)
            e.init_random(5)
            e.step(16)
            assert (e.store_packed() == ref).all(), (lanes, rpw)


@pytest.mark.parametrize("depth", HAND_DEPTHS)
@pytest.mark.parametrize("rule", ["ref", "conway", "highlife"])
def test_handoff_seams(pkg, oracle, depth, rule):
    """Hand-off row blocks at every depth: the shortest legal rows_per_wave (most
    seams per strip), partial last blocks (h not a multiple of R), births at the
    seams (Conway / HighLife), odd widths, and remainder launches of smaller
    depth in the same call.  Must equal the oracle and the classic blocks."""
    R = rules(oracle)[rule]
    rpw = min(r for r in range(4, 200) if handoff_toff(r, depth) >= 0)
    for h, w in ((5 * rpw + 3, 130), (3 * rpw, 4100), (2 * rpw + 1, 63)):
        g = oracle.bp_random(h, w, h + depth)
        for gens in (depth, 3 * depth + 5):
            ref = oracle.bp_run(g, w, gens, R)
            for handoff in (1, 2):
                with pkg.Engine(h, w, rule=R, device=0, tb_depth=depth, rows_per_wave=rpw,
                                handoff=handoff, streams=1) as e:
                    # no generic-mask hand-off kernel above depth 12 (life_internal.h)
                    assert e.handoff == (handoff == 2 and (rule != "highlife" or depth <= 12))
                    e.load_packed(g)
                    e.step(gens)
                    assert (e.store_packed() == ref).all(), (h, w, gens, handoff)


@pytest.mark.parametrize("depth", [8, 12, 16])
@pytest.mark.parametrize("toff", [0, 1])
def test_handoff_tail_offsets(pkg, oracle, depth, toff):
    """Both hand-off kernels of a depth: R + 2 - warm-up = 0 and = prefetch/2
    (mod the prefetch block), Conway so the tails' stages do real work."""
    pf = 8 if depth >= 16 else 4
    rs = [r for r in range(4, 300) if handoff_toff(r, depth) == toff * pf // 2]
    for rpw in rs[:2]:
        h, w = 4 * rpw + 7, 2000
        g = oracle.bp_random(h, w, rpw + depth)
        ref = oracle.bp_run(g, w, 2 * depth + 3, oracle.CONWAY)
        with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, tb_depth=depth, rows_per_wave=rpw,
                        handoff=2, streams=1) as e:
            assert e.handoff
            e.load_packed(g)
            e.step(2 * depth + 3)
            assert (e.store_packed() == ref).all(), rpw


def test_handoff_repeated_launches_and_graphs(pkg, oracle):
    """Hand-off flags are reset by every consumer, so back-to-back launches, graph
    replays and alternating call sizes (different remainder depths) stay exact."""
    h, w = 1000, 3000
    g = oracle.bp_random(h, w, 77)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, tb_depth=16, rows_per_wave=46,
                    handoff=2, streams=1) as e:
        assert e.handoff
        e.load_packed(g)
        total = 0
        for gens in (64, 64, 37, 64, 37, 5, 100):
            e.step(gens)
            total += gens
        e.sync()
        assert (e.store_packed() == oracle.bp_run(g, w, total, oracle.CONWAY)).all()


def test_load_packed_roundtrip(pkg, oracle):
    h, w = 37, 301
    rng = np.random.default_rng(1)
    g = rng.integers(0, 2**63, size=(h, 5), dtype=np.uint64) * 2 + 1
    with pkg.Engine(h, w, device=0) as e:
        e.load_packed(g)
        out = e.store_packed()
    g[:, 4] &= np.uint64((1 << (301 - 256)) - 1)  # columns >= w are dead
    assert (out == g).all()


def test_ascii_roundtrip_and_errors(pkg, oracle):
    h, w = 9, 70
    g = oracle.bp_random(h, w, 11)
    data = oracle.bp_unpack(g, w)
    with pkg.Engine(h, w, device=0) as e:
        e.load_ascii(data)
        assert e.store_ascii() == data
        with pytest.raises(pkg.GolError):
            e.load_ascii(data[:-1])
        bad = bytearray(data)
        bad[w] = ord("x")  # line 0 has no '\n' at column w
        with pytest.raises(pkg.GolError):
            e.load_ascii(bytes(bad))
    with pytest.raises(pkg.GolError):
        pkg.Engine(0, 5, device=0)
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, tb_depth=3)
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, tb_depth=20)  # dev build only
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, word_planes=4)  # dev build only
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, word_planes=3)
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, handoff=3)
    with pytest.raises(pkg.GolError):
        pkg.Engine(5, 5, device=0, handoff=2, tb_depth=2)


@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_ref_stripes_conway(pkg, oracle, P):
    """REF_STRIPES with a rule that gives births (exercises the stripe borders)."""
    h, w = 203, 190
    g = oracle.bp_random(h, w, P)
    ref = oracle.bp_ref_stripes(g, w, 12, P, oracle.CONWAY)
    with pkg.Engine(h, w, rule=oracle.CONWAY, device=0, semantics=pkg.SEM_REF_STRIPES,
                    ref_ranks=P, tb_depth=4) as e:
        e.load_ascii(oracle.bp_unpack(g, w))
        e.step(12)
        assert (e.store_packed() == ref).all()


@pytest.mark.parametrize("rule", ["daynight", "seeds", "b0"])
def test_generic_rules(pkg, oracle, rule):
    """GENERIC kernel path: births with 0 or 8 neighbours (the 4-bit count), a rule
    with no survivors, and the dead border under B0 (outside cells never count)."""
    R = rules(oracle)[rule]
    for (h, w) in ((1, 1), (7, 65), (129, 4000)):
        g = oracle.bp_random(h, w, h + w)
        for depth in (1, 7, 8):
            with pkg.Engine(h, w, rule=R, device=0, tb_depth=depth) as e:
                e.load_packed(g)
                e.step(11)
                assert (e.store_packed() == oracle.bp_run(g, w, 11, R)).all(), (h, w, depth)


# ------------------------------------------------------------ C2: 4096^2
@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("kernel", ["resident", "streaming"])
def test_c2_4096_per_generation(pkg, oracle, rule, kernel):
    """The default C2 engine (the resident kernel, one launch per call) and the
    streaming engine (K = 8): every checked generation count reached by one
    gol_step call from the initial field, so the depth-8 kernel and the remainder
    depths run (resident: partial and whole epochs), plus gens 1..16 one call
    each for the early B/S2 generations."""
    h = w = 4096
    R = rules(oracle)[rule]
    g0 = oracle.bp_random(h, w, 1)
    want = {0: g0}
    for gen in range(1, 41):
        want[gen] = oracle.bp_run(want[gen - 1], w, 1, R, threads=16)
    kw = {} if kernel == "resident" else {"resident": 1, "tb_depth": 8}
    with pkg.Engine(h, w, rule=R, device=0, **kw) as e:
        assert (e.resident is not None) == (kernel == "resident")
        e.init_random(1)
        assert (e.store_packed() == g0).all()
        for gens in (1, 2, 3, 5, 8, 9, 13, 16, 24, 40):
            e.init_random(1)
            e.step(gens)
            assert e.digest() == oracle.bp_digest(want[gens], w), f"gens {gens}"
        e.init_random(1)
        for gen in range(1, 17):
            e.step(1)
            assert e.digest() == oracle.bp_digest(want[gen], w), f"gen {gen} (one at a time)"
        assert (e.store_packed() == want[16]).all()


_C2_1000 = {}


def c2_oracle_1000(oracle, rule):
    """The oracle's 4096^2 field (seed 1) after 1000 generations (digest), once per
    rule per session (~2-5 s on 16 threads)."""
    if rule not in _C2_1000:
        R = rules(oracle)[rule]
        g = oracle.bp_run(oracle.bp_random(4096, 4096, 1), 4096, 1000, R, threads=16)
        _C2_1000[rule] = oracle.bp_digest(g, 4096)
    return _C2_1000[rule]


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("kernel", ["resident", "streaming"])
def test_c2_4096_1000_generations_vs_oracle(pkg, oracle, rule, kernel):
    """C2 as BASELINE.json states it (4096^2, p = 0.5, 1000 generations, one
    MI355X): the default engine (the resident kernel, ONE launch for the 1000
    generations) and the K = 16 streaming engine (62 full-depth launches + a
    depth-8 one) against the oracle's 1000 generations, both rules (r06; until
    r05 this was "every depth gives the same digest", GPU against GPU).
    Parallel_Life_MPI.cpp:37-54 per generation, :215-221 the loop."""
    R = rules(oracle)[rule]
    want = c2_oracle_1000(oracle, rule)
    kw = {} if kernel == "resident" else {"resident": 1, "tb_depth": 16}
    with pkg.Engine(4096, 4096, rule=R, device=0, **kw) as e:
        assert (e.resident is not None) == (kernel == "resident")
        if kernel == "streaming":
            assert e.tb_depth == 16
        e.init_random(1)
        e.step(1000)
        assert e.digest() == want
        if rule == "conway":  # still active: the check is not a fixed point's
            e.step(1)
            assert e.digest() != want


def test_c2_4096_1000_generations_every_depth_vs_oracle(pkg, oracle):
    """Every fused depth and both block closures after 1000 Conway generations
    (one gol_step call: a depth-d kernel and the remainder depths) against the
    oracle."""
    want = c2_oracle_1000(oracle, "conway")
    for depth in DEPTHS:
        for handoff in ((1, 2) if depth >= 4 else (1,)):
            with pkg.Engine(4096, 4096, rule=pkg.CONWAY, device=0, tb_depth=depth,
                            handoff=handoff) as e:
                e.init_random(1)
                e.step(1000)
                assert e.digest() == want, (depth, handoff)


# ------------------------------------------------------------ timing API
def test_timing_counters(pkg):
    with pkg.Engine(1024, 1024, device=0, tb_depth=8) as e:
        e.init_random(1)
        e.set_timing(True)
        e.step(20)  # 8 + 8 + 4
        e.sync()
        t = e.timing()
    assert t["launches"] == 3
    assert t["kernel_ms"] > 0
    assert t["cell_gens"] == 1024 * 1024 * 20


def test_timing_struct_size(pkg):
    """gol_get_timing never writes past a caller's older gol_timing: without this
    header's struct_size it writes the r04 fields (40 bytes) only."""
    import ctypes
    with pkg.Engine(512, 512, device=0, tb_depth=8) as e:
        e.init_random(1)
        e.set_timing(1)
        e.step(16)
        e.sync()
        full = ctypes.sizeof(pkg.Timing)
        buf = (ctypes.c_uint8 * (full + 16))(*([0xAB] * (full + 16)))
        struct_size = ctypes.c_uint32.from_buffer(buf, 36)
        struct_size.value = 40  # an r04 caller's (garbage) value
        assert pkg.lib().gol_get_timing(e._h, ctypes.cast(buf, ctypes.POINTER(pkg.Timing))) == 0
        assert struct_size.value == 40
        assert bytes(buf[40:]) == bytes([0xAB] * (full + 16 - 40))
        assert ctypes.c_uint64.from_buffer(buf, 0).value == 2  # launches
        struct_size.value = full
        assert pkg.lib().gol_get_timing(e._h, ctypes.cast(buf, ctypes.POINTER(pkg.Timing))) == 0
        assert struct_size.value == full
        assert bytes(buf[full:]) == bytes([0xAB] * 16)


def test_timing_sampled(pkg):
    with pkg.Engine(1024, 1024, device=0, tb_depth=8) as e:
        e.init_random(1)
        e.set_timing(2)
        e.step(40)  # 5 launches of 8; launches 0, 2, 4 are timed
        t = e.timing()
    assert t["launches"] == 3
    assert t["cell_gens"] == 1024 * 1024 * 24


@pytest.mark.parametrize("w", [4100, 4033])
def test_ascii_codec_large_and_malformed(pkg, oracle, w):
    """Device ASCII codec (ballot pack / coalesced unpack) on multi-word rows (odd
    and even word counts), single and composite engines, and a malformed line deep
    inside the field."""
    h = 333
    g = oracle.bp_random(h, w, 31)
    data = oracle.bp_unpack(g, w)
    for streams in (1, 2):
        with pkg.Engine(h, w, device=0, streams=streams, rule=pkg.CONWAY) as e:
            e.load_ascii(data)
            assert (e.store_packed() == g).all()
            assert e.store_ascii() == data
            e.step(9)
            assert e.store_ascii() == oracle.bp_unpack(oracle.bp_run(g, w, 9, oracle.CONWAY), w)
            bad = bytearray(data)
            bad[200 * (w + 1) + w] = ord("1")  # row 200 runs into row 201
            with pytest.raises(pkg.GolError) as ei:
                e.load_ascii(bytes(bad))
            assert ei.value.status == pkg.GOL_EINVAL


def test_graph_replay_matches(pkg, oracle):
    """gol_step(gens) on a single-stream engine replays a captured hipGraph from the
    second call on (keyed by gens and buffer parity); results stay exact."""
    h, w = 513, 2000
    g = oracle.bp_random(h, w, 41)
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, tb_depth=4, streams=1) as e:
        e.load_packed(g)
        total = 0
        for gens in (20, 20, 37, 20, 37, 37, 5):
            e.step(gens)
            total += gens
            assert (e.store_packed() == oracle.bp_run(g, w, total, oracle.CONWAY)).all(), total


@pytest.mark.parametrize("h,w,kw", [
    (1000, 777, {}),                         # resident kernel
    (3000, 5000, dict(resident=1)),          # streaming kernel
    (40000, 1000, dict(streams=2)),          # composite engine: 2 stripes
])
def test_digest_rows_partitions(pkg, oracle, h, w, kw):
    """gol_digest_rows: the digests of a partition of the rows add up to the whole
    field's (the order-independent sums of digest_kernel), the whole range is
    gol_digest, and an empty range is (0, 0)."""
    with pkg.Engine(h, w, rule=pkg.CONWAY, device=0, **kw) as e:
        e.init_random(11)
        e.step(19)
        whole = e.digest()
        assert e.digest_rows(0, h) == whole
        assert e.digest_rows(5, 0) == (0, 0)
        cuts = [0, 1, h // 3, h // 3 + 17, h - 1, h]
        parts = [e.digest_rows(a, b - a) for a, b in zip(cuts, cuts[1:])]
    assert sum(p[0] for p in parts) == whole[0]
    assert sum(p[1] for p in parts) % (1 << 64) == whole[1]
    want = oracle.bp_digest(oracle.bp_run(oracle.bp_random(h, w, 11), w, 19, oracle.CONWAY), w)
    assert whole == want


def test_digest_rows_rank_engine(pkg, monkeypatch):
    """A rank engine's gol_digest_rows covers the part of its own rows inside the
    range; the RCCL communicator as RCCL reports it (self-loop: 1 rank)."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    with pkg.Engine(1200, 640, rule=pkg.CONWAY, device=0, rank=1, nranks=3,
                    uid=pkg.unique_id()) as e:
        e.init_random(2)
        e.step(30)
        d = e.digest()
        assert e.digest_rows(e.row0, e.rows) == d
        assert e.digest_rows(0, 1200) == d
        assert e.digest_rows(0, e.row0) == (0, 0)
        ci = e.comm_info()
    assert ci["count"] == 1 and ci["rank"] == 0 and ci["device"] == 0
    assert ci["peer_up"] == 0 and ci["peer_down"] == 0  # the self-loop's peers
