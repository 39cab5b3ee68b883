"""The stage logic's v_bitop3 networks, checked exhaustively on the CPU.

life_stencil.h computes each generation with 3-input bitwise functions
(v_bitop3_b32, truth table in an 8-bit immediate).  This test reads the immediates
from the header and evaluates the networks bit-sliced over every case they can
meet, against the rule itself (Parallel_Life_MPI.cpp:37-54, restated in
oracle/gol_oracle.c):

  * the 3-row total T = H3(r-2) + H3(r-1) + H3(r) of rule32_total (B/S2, B3/S23);
  * the r04 pair form (GOL_PAIR_SUM): the pair H3(r-1), H3(r) reduced once for two
    rows to three features, then the rule for either third row A.
"""
import itertools
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "mpi-game-of-life_amd", "csrc", "life_stencil.h")


def luts():
    src = open(HDR).read()
    return {m.group(1): int(m.group(2), 16)
            for m in re.finditer(r"constexpr uint32_t (k\w+) = 0x([0-9A-Fa-f]+);", src)}


def bitop3(lut, a, b, c):
    """v_bitop3_b32 on 0/1 inputs: the immediate is the truth table evaluated on
    S0 = 0xF0, S1 = 0xCC, S2 = 0xAA, i.e. bit index 4a + 2b + c."""
    return (lut >> (4 * a + 2 * b + c)) & 1


def h3(left, mid, right):
    """(sum, carry) of a cell and its two horizontal neighbours, as the kernel forms them."""
    L = luts()
    return bitop3(L["kXor3"], left, mid, right), bitop3(L["kMaj"], left, mid, right)


def triples():
    return list(itertools.product((0, 1), repeat=3))


def test_h3_is_the_horizontal_sum():
    for t in triples():
        s, c = h3(*t)
        assert s + 2 * c == sum(t)


def test_pair_rule_matches_b_s2():
    """Every (row r-2, r-1, r, r+1) horizontal triple and cell: the pair step's
    output (row r-1 against H3(r-2)) and the next step's (row r against H3(r+1))
    equal alive && n == 2 with n the 8-neighbour count.  The pair (H3(r-1), H3(r))
    enters as the three features of pair_sum<RULE_REF> and the lower row's carry."""
    L = luts()
    assert GOL_PAIR_SUM_ON()

    def pair(b, e):
        f0 = bitop3(L["kRefF0"], e[0], b[1], b[0])
        f1 = bitop3(L["kRefF1"], e[0], b[0], b[1])
        f2 = bitop3(L["kRefF2"], e[0], b[0], f1)
        return f0, f1, f2, e[1]

    def test(f0, f1, f2, ec, a0, a1, alive):
        u = bitop3(L["kRefT0"], a0, f2, f0)
        v = bitop3(L["kRefT1"], f1, ec, a1)
        return bitop3(L["kRefT2"], u, v, alive)

    n = 0
    for up, mid, low, low2 in itertools.product(triples(), repeat=4):
        a = h3(*up)      # H3(r-2)
        b = h3(*mid)     # H3(r-1): the row emitted at the pair step
        e = h3(*low)     # H3(r): the row emitted at the next step
        f = h3(*low2)    # H3(r+1)
        q = pair(b, e)
        # pair step: row r-1 (cell mid[1]) sees rows r-2, r-1, r
        nb = sum(up) + sum(mid) + sum(low) - mid[1]
        assert test(*q, a[0], a[1], mid[1]) == int(mid[1] == 1 and nb == 2)
        # next step: row r (cell low[1]) sees rows r-1, r, r+1
        nb = sum(mid) + sum(low) + sum(low2) - low[1]
        assert test(*q, f[0], f[1], low[1]) == int(low[1] == 1 and nb == 2)
        n += 1
    assert n == 8 ** 4


def test_pair_rule_matches_b3_s23():
    """The B3/S23 pair form (pair_sum<RULE_CONWAY> features, conway_from_pair) on
    every (row r-2, r-1, r, r+1) case: both rows of a pair equal the rule."""
    L = luts()
    assert GOL_PAIR_SUM_ON()

    def pair(b, e):
        f0 = bitop3(L["kConwayF0"], b[0], e[0], e[0])
        f1 = bitop3(L["kConwayF1"], b[1], f0, e[1])
        f2 = bitop3(L["kConwayF2"], f0, e[1], b[1])
        f3 = bitop3(L["kConwayF3"], e[0], b[0], f2)
        return f1, f2, f3

    def test(f1, f2, f3, a0, a1, alive):
        g4 = bitop3(L["kConwayT0"], a0, f3, alive)
        g5 = bitop3(L["kConwayT1"], f2, g4, a1)
        g6 = bitop3(L["kConwayT2"], g4, f1, g5)
        return bitop3(L["kConwayT3"], g4, g6, alive)

    for up, mid, low, low2 in itertools.product(triples(), repeat=4):
        q = pair(h3(*mid), h3(*low))
        a, f = h3(*up), h3(*low2)
        nb = sum(up) + sum(mid) + sum(low) - mid[1]
        assert test(*q, a[0], a[1], mid[1]) == int(nb == 3 or (mid[1] == 1 and nb == 2))
        nb = sum(mid) + sum(low) + sum(low2) - low[1]
        assert test(*q, f[0], f[1], low[1]) == int(nb == 3 or (low[1] == 1 and nb == 2))


def test_three_row_rules_match():
    """rule32_total's B/S2 and B3/S23 networks against the rule on every 3 x 3 case."""
    L = luts()

    def total(a, b, e, alive, rule):
        s0 = bitop3(L["kXor3"], a[0], b[0], e[0])
        k0 = bitop3(L["kMaj"], a[0], b[0], e[0])
        p = bitop3(L["kXor3"], a[1], b[1], e[1])
        mj = bitop3(L["kMaj"], a[1], b[1], e[1])
        three = bitop3(L["kTwoThree"], p, k0, mj)
        if rule == "ref":
            return bitop3(L["kAnd3"], alive, s0, three)
        four = bitop3(L["kFour"], p, k0, mj)
        stay = bitop3(L["kAndNot"], alive, four, s0)
        return bitop3(L["kOrAnd2"], s0, three, stay)

    for up, mid, low in itertools.product(triples(), repeat=3):
        alive = mid[1]
        nb = sum(up) + sum(mid) + sum(low) - alive
        a, b, e = h3(*up), h3(*mid), h3(*low)
        assert total(a, b, e, alive, "ref") == int(alive == 1 and nb == 2)
        assert total(a, b, e, alive, "conway") == int(nb == 3 or (alive == 1 and nb == 2))


def GOL_PAIR_SUM_ON():
    m = re.search(r"#define GOL_PAIR_SUM (\d)", open(HDR).read())
    return m is not None and m.group(1) == "1"
