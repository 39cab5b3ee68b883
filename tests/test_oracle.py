"""CPU suite: pin the oracle (oracle/gol_oracle.c) before trusting it.

1. The scalar program restatement reproduces every reference output recorded in
   tests/golden/ref_outputs.json (the reference binary run on the
   shipped data.txt at -np 1/2/3/4/8).
2. Known-answer patterns for the reference-effective rule B/S2 and for B3/S23.
3. The bit-packed restatement equals the scalar one on random fields (odd widths,
   h % P != 0, all three rules, REF_STRIPES), so it can serve as the oracle at
   sizes the scalar one cannot reach.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def ascii_of(cells):
    return b"".join(bytes(np.where(r, 49, 48).astype(np.uint8)) + b"\n" for r in cells)


def cells_of(data, h, w):
    a = np.frombuffer(data, dtype=np.uint8).reshape(h, w + 1)
    return a[:, :w] == 49


GOLD = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))


def test_input_fixture_intact(ref_data):
    assert hashlib.sha256(ref_data).hexdigest() == GOLD["input_sha256"]
    with open(os.path.join(GOLDEN, "grid_size_data.txt")) as f:
        assert f.read().split() == ["1500", "500", "100"]


@pytest.mark.parametrize("case", [c for c in GOLD["cases"] if c["gens"] <= 100],
                         ids=lambda c: f"np{c['np']}-e{c['gens']}")
def test_scalar_oracle_matches_reference_outputs(oracle, ref_data, case):
    out = oracle.ref_program(ref_data, GOLD["h"], GOLD["w"], case["gens"], case["np"])
    assert out.count(b"1") == case["live"]
    assert hashlib.sha256(out).hexdigest() == case["sha256"]


def test_stripe_decomposition(oracle):
    # Parallel_Life_MPI.cpp:70-81 on the shipped 1500 rows
    assert oracle.ref_stripe(1500, 1, 0) == (0, 1500)
    assert oracle.ref_stripe(1500, 4, 0) == (0, 376)
    assert oracle.ref_stripe(1500, 4, 1) == (374, 377)
    assert oracle.ref_stripe(1500, 4, 3) == (1124, 376)
    assert oracle.ref_stripe(10, 3, 2) == (5, 5)  # tail 10 % 3 on the last rank
    with pytest.raises(ValueError):
        oracle.ref_stripe(2, 3, 0)  # h < P: the reference crashes


def run(oracle, cells, gens, rule, P=1):
    h, w = cells.shape
    return cells_of(oracle.ref_program(ascii_of(cells), h, w, gens, P, rule), h, w)


def pattern(rows):
    return np.array([[c == "#" for c in r] for r in rows])


def test_kat_reference_rule(oracle):
    R = oracle.REF_RULE
    blinker = pattern([".....", ".....", ".###.", ".....", "....."])
    # B/S2: the ends have 1 neighbour and die, the centre has 2 and lives
    assert (run(oracle, blinker, 1, R) == pattern([".....", ".....", "..#..", ".....", "....."])).all()
    block = pattern(["....", ".##.", ".##.", "...."])
    assert not run(oracle, block, 1, R).any()  # 3 neighbours each: dies under B/S2
    beehive = pattern(["......", "..##..", ".#..#.", "..##..", "......"])
    assert (run(oracle, beehive, 5, R) == beehive).all()  # every cell has exactly 2


def test_kat_conway(oracle):
    C = oracle.CONWAY
    blinker = pattern([".....", ".....", ".###.", ".....", "....."])
    vert = pattern([".....", "..#..", "..#..", "..#..", "....."])
    assert (run(oracle, blinker, 1, C) == vert).all()
    assert (run(oracle, blinker, 2, C) == blinker).all()
    block = pattern(["....", ".##.", ".##.", "...."])
    assert (run(oracle, block, 7, C) == block).all()
    g = np.zeros((12, 12), bool)
    g[1:4, 1:4] = pattern([".#.", "..#", "###"])
    out = run(oracle, g, 4, C)
    assert (out == np.roll(np.roll(g, 1, 0), 1, 1)).all()  # glider moves (1,1) per 4 gens
    # dead border: a glider hitting the edge does not wrap
    g2 = np.zeros((6, 6), bool)
    g2[3:6, 3:6] = pattern([".#.", "..#", "###"])
    assert not run(oracle, g2, 40, C)[:2, :2].any()


@pytest.mark.parametrize("seed", range(24))
def test_bitpacked_equals_scalar(oracle, seed):
    rng = np.random.default_rng(seed)
    h = int(rng.integers(1, 70))
    w = int([1, 63, 64, 65, 127, 128, 129, 200][seed % 8])
    E = int(rng.integers(0, 9))
    rule = [oracle.REF_RULE, oracle.CONWAY, oracle.HIGHLIFE][seed % 3]
    P = int(rng.integers(1, 5))
    if h // P == 0:
        P = 1
    cells = rng.random((h, w)) < rng.uniform(0.2, 0.8)
    data = ascii_of(cells)
    ref = oracle.ref_program(data, h, w, E, P, rule)
    g = oracle.bp_pack(data, h, w)
    out = oracle.bp_ref_stripes(g, w, E, P, rule) if P > 1 else oracle.bp_run(g, w, E, rule)
    assert oracle.bp_unpack(out, w) == ref


def test_bitpacked_reference_data(oracle, ref_data):
    g = oracle.bp_pack(ref_data, 1500, 500)
    for case in GOLD["cases"]:
        if case["gens"] > 6:
            continue
        if case["np"] == 1:
            out = oracle.bp_run(g, 500, case["gens"])
        else:
            out = oracle.bp_ref_stripes(g, 500, case["gens"], case["np"])
        assert hashlib.sha256(oracle.bp_unpack(out, 500)).hexdigest() == case["sha256"]


def test_random_init_and_digest(oracle):
    g = oracle.bp_random(5, 130, seed=3)
    assert g.shape == (5, 3)
    assert int(g[:, 2].max()) < (1 << 2)  # columns >= 130 are dead
    live, h = oracle.bp_digest(g, 130)
    assert live == sum(bin(int(x)).count("1") for x in g.ravel())
    g2 = g.copy()
    g2[4, 0] ^= 1
    assert oracle.bp_digest(g2, 130)[1] != h
    # p = 0.5 on a bigger field
    big = oracle.bp_random(256, 4096, seed=1)
    assert abs(oracle.bp_digest(big, 4096)[0] / (256 * 4096) - 0.5) < 0.01


def test_cpu_baseline_field_is_the_bench_field(oracle):
    """bench.py's cpu_baseline times the reference algorithm on the benchmark's own
    synthetic field: 0 generations leave exactly the live cells of the engine's
    splitmix64 field (gol_init_random == oracle_bp_init_random)."""
    for rows, w, threads in ((3, 200, 2), (5, 64, 3), (2, 65, 1)):
        live = oracle.ref_baseline(rows, w, 0, threads, seed=1)
        assert live == oracle.bp_digest(oracle.bp_random(rows * threads, w, 1), w)[0]
    # and its stepping is the reference's (REF rule on each stripe alone)
    g = oracle.bp_random(40, 90, 1)
    want = sum(oracle.bp_digest(oracle.bp_run(g[t * 20:(t + 1) * 20], 90, 7), 90)[0]
               for t in range(2))
    assert oracle.ref_baseline(20, 90, 7, 2, seed=1) == want
