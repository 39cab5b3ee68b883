"""Seeded differential sweep (late r06): random small fields through random engine
configurations -- single engines (streaming or resident, any depth, block kind,
strip width, rows per wavefront, REF_STRIPES), in-process groups of 2-5 stripes
(halo depth, exchange mode), and several gol_step calls per case -- each against
the oracle (Parallel_Life_MPI.cpp countNeighbours :16-35 + updateGrid :37-54 on
the field, or on :70-81's stripes for REF_STRIPES).  The targeted tests pin each
knob on chosen shapes; this sweep crosses them on shapes nobody chose.  A
configuration the engine rejects (GOL_EINVAL: e.g. a depth too small for hand-off
blocks) must be rejected up front, never produce a wrong field.
"""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
# GOL_FUZZ_SCALE=n runs n times the seeds (a longer sweep by hand; default 1)
SCALE = max(1, int(os.environ.get("GOL_FUZZ_SCALE", "1")))

DEPTHS = [0, 1, 2, 4, 6, 7, 8, 12, 16]
RULES = {
    "ref": (0, 1 << 2),
    "conway": (1 << 3, (1 << 2) | (1 << 3)),
    "highlife": ((1 << 3) | (1 << 6), (1 << 2) | (1 << 3)),
    "seeds": (1 << 2, 0),
    "daynight": ((1 << 3) | (1 << 6) | (1 << 7) | (1 << 8),
                 (1 << 3) | (1 << 4) | (1 << 6) | (1 << 7) | (1 << 8)),
    "b0": ((1 << 0) | (1 << 3), (1 << 2) | (1 << 3)),
}


def draw(rnd):
    """One random case: shape, rule, knobs, and the generation chunks of its steps."""
    h = rnd.choice([rnd.randint(1, 40), rnd.randint(41, 400), rnd.randint(401, 1500),
                    rnd.randint(1501, 5000)])
    w = rnd.choice([rnd.randint(1, 70), rnd.randint(71, 1000), rnd.randint(1001, 5000),
                    rnd.randint(5001, 9000)])
    rule = rnd.choice(sorted(RULES))
    kind = rnd.choice(["single", "single", "single", "ref_stripes", "group"])
    knobs = dict(tb_depth=rnd.choice(DEPTHS))
    if rnd.random() < 0.4:
        knobs["handoff"] = rnd.choice([1, 2])
    if rnd.random() < 0.3:
        knobs["strip_lanes"] = rnd.choice([64, 32, 16])
    if rnd.random() < 0.3:
        knobs["rows_per_wave"] = rnd.randint(1, 120)
    if kind == "single" and rnd.random() < 0.3:
        knobs = dict(resident=2, tb_depth=rnd.choice([0, 1, 3, 8, 16, 21]),
                     rows_per_wave=rnd.choice([0, 2, 3, 4, 6, 8]))
    elif kind == "single" and rnd.random() < 0.15:
        knobs["streams"] = rnd.choice([2, 3])  # the composite engine (stripes on streams)
    n = 1
    if kind == "group":
        n = rnd.randint(2, 5)
        if rnd.random() < 0.5:
            knobs["halo_depth"] = rnd.randint(1, 64)
        knobs["exchange_overlap"] = rnd.choice([0, 1, 2])
    P = rnd.randint(1, 6) if kind == "ref_stripes" else 1
    chunks = [rnd.choice([0, 1, 2, 3, 5, 16, 17, rnd.randint(1, 90)]) for _ in range(rnd.randint(1, 3))]
    return dict(h=h, w=w, rule=rule, kind=kind, n=n, P=P, knobs=knobs, chunks=chunks,
                seed=rnd.randint(1, 1 << 30))


def expected(oracle, g, case, gens):
    R = RULES[case["rule"]]
    if case["kind"] == "ref_stripes" and case["P"] > 1:
        return oracle.bp_ref_stripes(g, case["w"], gens, case["P"], R)
    return oracle.bp_run(g, case["w"], gens, R)


@pytest.mark.parametrize("block", range(8 * SCALE))
def test_random_configurations_vs_oracle(pkg, oracle, block):
    rnd = random.Random(20261018 + block)
    ran = rejected = 0
    for i in range(60):
        case = draw(rnd)
        h, w = case["h"], case["w"]
        if case["kind"] == "group" and h < case["n"]:
            continue
        if case["kind"] == "ref_stripes" and h < case["P"]:
            continue
        g = oracle.bp_random(h, w, case["seed"])
        R = RULES[case["rule"]]
        try:
            if case["kind"] == "group":
                eng = pkg.Group(h, w, case["n"], rule=R, **case["knobs"])
            else:
                sem = pkg.SEM_REF_STRIPES if case["kind"] == "ref_stripes" else pkg.SEM_GLOBAL
                eng = pkg.Engine(h, w, rule=R, device=0, semantics=sem, ref_ranks=case["P"],
                                 **case["knobs"])
        except pkg.GolError as ex:
            assert ex.status == pkg.GOL_EINVAL, (case, ex)
            rejected += 1
            continue
        with eng:
            eng.load_packed(g)
            done = 0
            for c in case["chunks"]:
                eng.step(c)
                done += c
                want = expected(oracle, g, case, done)
                got = eng.store_packed()
                assert got.shape == want.shape, case
                assert (got == want).all(), f"case {block}.{i} after {done} generations: {case}"
                assert eng.digest() == oracle.bp_digest(want, w), case
        ran += 1
    assert ran >= 40, (ran, rejected)
    print(f"block {block}: {ran} configurations run, {rejected} rejected up front")


def mirrored_steps(oracle, own, w, chunks, rule, Hx, has_up, has_dn):
    """A rank whose transport returns what it is sent: each round its halos hold
    its own first / last Hx rows, the extended stripe evolves with dead cells
    beyond it, and its own rows are kept (as tests/test_gpu_rccl.py); every
    gol_step call starts a round, rounds are Hx generations."""
    outs = []
    for c in chunks:
        left = c
        while left:
            g = min(left, Hx)
            parts = ([own[:Hx]] if has_up else []) + [own] + ([own[-Hx:]] if has_dn else [])
            ext = oracle.bp_run(np.concatenate(parts), w, g, rule)
            top = Hx if has_up else 0
            own = ext[top:top + own.shape[0]]
            left -= g
        outs.append(own)
    return outs


@pytest.mark.parametrize("block", range(4 * SCALE))
def test_random_rank_engines_vs_oracle(pkg, oracle, block):
    """Rank engines (gol_create_rank_transport) of random splits with a loopback
    transport: random rank of 2-8, depth, halo depth, exchange mode, block kind and
    step chunks, against the oracle evolving the mirrored extended stripe."""
    rnd = random.Random(7100 + block)
    ran = 0
    for i in range(20):
        n = rnd.randint(2, 8)
        h = rnd.randint(2 * n, 3000)
        w = rnd.randint(1, 6000)
        rule = rnd.choice(sorted(RULES))
        R = RULES[rule]
        rank = rnd.randrange(n)
        knobs = dict(tb_depth=rnd.choice(DEPTHS), exchange_overlap=rnd.choice([0, 1, 2]))
        if rnd.random() < 0.5:
            knobs["halo_depth"] = rnd.randint(1, 80)
        if rnd.random() < 0.3:
            knobs["handoff"] = rnd.choice([1, 2])
        chunks = [rnd.choice([1, 5, 16, rnd.randint(1, 150)]) for _ in range(rnd.randint(1, 3))]
        g = oracle.bp_random(h, w, rnd.randint(1, 1 << 30))
        try:
            e = pkg.Engine(h, w, rule=R, device=0, rank=rank, nranks=n,
                           transport=lambda su, sd: (su, sd), **knobs)
        except pkg.GolError as ex:
            assert ex.status == pkg.GOL_EINVAL, (ex, knobs)
            continue
        with e:
            own = g[e.row0:e.row0 + e.rows]
            e.load_packed(own)
            got = []
            for c in chunks:
                e.step(c)
                got.append(e.store_packed())
            Hx = e.halo_depth
        want = mirrored_steps(oracle, own, w, chunks, R, Hx, rank > 0, rank < n - 1)
        for j, (a, b) in enumerate(zip(got, want)):
            assert (a == b).all(), f"case {block}.{i} chunk {j}: h {h} w {w} rank {rank}/{n} {rule} {knobs} {chunks}"
        ran += 1
    assert ran >= 12


@pytest.mark.parametrize("block", range(2 * SCALE))
def test_random_ascii_round_trips(pkg, oracle, block):
    """The GPU ASCII codec (readGridFromFile's parse :91-99 and writeDataToFile's
    serialisation :157-164) on random shapes: data.txt bytes of a random field load
    to the oracle's packing, step, and store back as the oracle's bytes; a field
    of REF_STRIPES engines likewise (its output keeps each stripe's own rows)."""
    rnd = random.Random(515 + block)
    for _ in range(12):
        h, w = rnd.randint(1, 900), rnd.randint(1, 3000)
        g = oracle.bp_random(h, w, rnd.randint(1, 1 << 30))
        data = oracle.bp_unpack(g, w)
        assert len(data) == h * (w + 1)
        P = rnd.randint(1, 5) if h >= 5 else 1
        sem = pkg.SEM_REF_STRIPES if P > 1 else pkg.SEM_GLOBAL
        gens = rnd.choice([0, 1, 7, 33])
        with pkg.Engine(h, w, device=0, semantics=sem, ref_ranks=P) as e:
            e.load_ascii(data)
            assert (e.store_packed() == g).all()
            e.step(gens)
            out = e.store_ascii(h * (w + 1))
        if h * w <= 200000:  # the scalar restatement of the whole program
            want = oracle.ref_program(data, h, w, gens, P)
        else:
            kind = "ref_stripes" if P > 1 else "single"
            want = oracle.bp_unpack(expected(oracle, g, dict(kind=kind, P=P, w=w, rule="ref"), gens), w)
        assert out == want, (h, w, P, gens)
