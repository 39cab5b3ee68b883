// life_stencil.h -- the gfx950 stencil kernel of the Game of Life engine.
//
// Hot path: the per-generation update of Parallel_Life_MPI.cpp (countNeighbours
// :16-35 + updateGrid :37-54), restated on a bit-packed field (64 cells per
// uint64) and fused over K generations per launch (temporal blocking).  Included
// by one translation unit per depth (life_tb_d<K>.hip), which instantiates
// life_tb_kernel<K, RULE, NP, HAND> for the three rule kinds.
//
// Kernel shape (one wavefront = one work unit, no LDS, no block barriers):
//   * A wavefront owns a strip of 64 consecutive lane groups of a row (lane l
//     holds group strip*62 - 1 + l); lanes 0 and 63 are the horizontal halo, so
//     each strip outputs 62 groups.  A lane group is NP = 2 (or, dev build, 4)
//     planes of 32 cells (bitlayout.h: column NP*j + k of the group at bit j of
//     plane k), so the horizontal neighbours of every plane but the first and
//     last are other planes at the same bit; those two take one v_alignbit each,
//     with the carry bit from the adjacent lane by a DPP wave shift.  After g
//     fused generations the contamination from the unknown groups beyond the
//     halo lanes has moved g columns into lanes 0/63, so K <= 63 keeps lanes
//     1..62 exact.  64-lane strips are edge-aligned (StepArgs::edge): a lane
//     next to the DPP shift's zero (lane 0 / 63) or to a lane outside the field
//     sees the dead border, so strip 0 starts at group 0 and the last strip of a
//     one-segment launch ends at group ng - 1; the gap of <= 30 groups before it
//     is a 32-lane "half strip" whose wavefronts carry two row blocks.
//   * The wavefront streams down the rows of its row block.  Generation g
//     (stage g-1, g = 1..K) keeps a 3-row window in registers: for each incoming
//     row it forms the horizontal 3-cell sum H3 (bit-sliced sum + carry) once and
//     emits the previous row from the 9-cell total H3(r-2) + H3(r-1) + H3(r).
//     Stage s consumes the row stage s-1 emitted in the same step.  Each input row
//     is read once from HBM and each output row written once per K generations.
//   * Field rows outside [0, field_h) are dead (Parallel_Life_MPI.cpp:21-22) and
//     columns >= w are dead (:26-27): masked on load and -- for rules that can
//     give birth -- re-masked after every generation.
//
// Row blocks (R output rows each, rb..re).  Step t ingests input row rb - K + t;
// stage s emits row rb - K + t - (s+1) at step t, so generation g is computed
// for rows [rb - K + g, ...) and the K rows of input above the block are its
// vertical halo.  Two ways to close the block at the bottom:
//   * classic (HAND = false, and the last block of every segment): keep
//     streaming K rows past re; stage s computes R + 2(K - s - 1) rows, i.e. every
//     block recomputes K(K-1) stage-steps of its neighbour's rows.
//   * hand-off (HAND = true): the block's generation-g rows end at re - K + g and
//     the two generation-(g-1) rows stage g-1 needs beyond that come from the
//     block below, which computed them first thing (its first two rows of every
//     generation).  Each block writes those 2(K-1) "side rows" to its slot,
//     signals a flag, and the block above reads them at the end of its stream:
//     stage s computes exactly R + 2 rows.  Blocks are numbered bottom-up: each
//     XCD starts its share of a launch's blocks in order, so the block a waiting
//     consumer depends on has a smaller index and cannot be queued behind waiting
//     blocks of the same launch.  A second launch that waits could hold an XCD's
//     slots, so the engine runs at most one hand-off launch per device at a time
//     (engine.cpp: band launches and group members after the first on a device
//     use classic blocks).  Waits are bounded; a timeout sets *err (reported by
//     gol_sync) instead of hanging.
//     Hand-off memory protocol (MI355X_MICROARCH.md, inter-workgroup
//     visibility, first table row): side rows stored write-through (sc1), the
//     producer's s_waitcnt vmcnt(0), an sc1 flag store by one lane; the consumer
//     polls with sc1 loads and reads the rows with sc1 loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <type_traits>

#include "bitlayout.h"
#include "life_internal.h"
#include "loop_place.h"

namespace gol {

namespace {

// Lane shifts by DPP.  (r04: the LDS crossbar instead, ds_bpermute_b32 + a
// full-rate AND for the zero fill, lost 25% at B/S2; removed in r06.)
__device__ __forceinline__ uint32_t lane_from_left(uint32_t v)
{
    // DPP wave_shr:1 -- lane l receives lane l-1's value; lane 0 receives 0.
    return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t lane_from_right(uint32_t v)
{
    // DPP wave_shl:1 -- lane l receives lane l+1's value; lane 63 receives 0.
    return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xf, 0xf, true);
}

// The NP 32-bit cell planes of one lane group (bitlayout.h): NP/2 words, 32*NP
// columns; plane k bit j = column NP*j + k of the group.
template <int NP>
struct Pl {
    uint32_t v[NP];
};

// The group's words as stored in HBM: one 8- (NP = 2) or 16-byte (NP = 4) access.
template <int NP>
struct alignas(4 * NP) Grp {
    uint64_t w[NP / 2];
};

template <int NP>
__device__ __forceinline__ Pl<NP> planes_of(const Grp<NP>& g)
{
    Pl<NP> p;
#pragma unroll
    for (int i = 0; i < NP / 2; ++i) {
        p.v[2 * i] = (uint32_t)g.w[i];
        p.v[2 * i + 1] = (uint32_t)(g.w[i] >> 32);
    }
    return p;
}
template <int NP>
__device__ __forceinline__ Grp<NP> words_of(const Pl<NP>& p)
{
    Grp<NP> g;
#pragma unroll
    for (int i = 0; i < NP / 2; ++i) g.w[i] = ((uint64_t)p.v[2 * i + 1] << 32) | p.v[2 * i];
    return g;
}

// Loads and stores of the row stream.  Every load of the stream is an agent-scope
// relaxed atomic (global_load ... sc1: served by L2, not the CU's L1), so the same
// code reads the input field and, at the end of a hand-off block, the side rows
// another wavefront stored write-through.
template <int NP>
__device__ __forceinline__ Grp<NP> load_grp(const uint64_t* p)
{
    Grp<NP> g;
#pragma unroll
    for (int i = 0; i < NP / 2; ++i)
        g.w[i] = __hip_atomic_load(const_cast<uint64_t*>(p + i), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    return g;
}
// Field rows (written by an earlier launch, so plain loads would see them too).
// (r05: non-temporal loads and stores -- all of them, or the warm-up rows only --
// shortened the start burst but lost in the kernel, 65536^2 156.7-156.9 vs
// 158.0-158.3 TCUPS, the 8-way rank 107.5-107.9 vs 117.4-118.3: the rows a block
// shares with its neighbours no longer stay in L2; nt stores 111.6-111.7;
// profiles/r05/ab_nt_loads_stores_rejected.jsonl.  The switches were removed in r06.)
template <int NP>
__device__ __forceinline__ Grp<NP> load_field(const uint64_t* p)
{
    return load_grp<NP>(p);
}

template <int NP>
__device__ __forceinline__ void store_side(uint64_t* p, const Pl<NP>& x)
{
    const Grp<NP> g = words_of(x);
#pragma unroll
    for (int i = 0; i < NP / 2; ++i)
        __hip_atomic_store(p + i, g.w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// v_bitop3_b32: any 3-input bitwise function in one VALU op.  The immediate is
// the function's truth table evaluated on S0 = 0xF0, S1 = 0xCC, S2 = 0xAA.
template <uint32_t LUT>
__device__ __forceinline__ uint32_t lop3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, LUT);
}
constexpr uint32_t kXor3 = 0x96;      // a ^ b ^ c
constexpr uint32_t kMaj = 0xE8;       // majority(a, b, c): carry of a + b + c
constexpr uint32_t kTwoThree = 0x14;  // (a ^ b) & ~c
constexpr uint32_t kAnd3 = 0x80;      // a & b & c
constexpr uint32_t kFour = 0x42;      // ~(a ^ b) & (a ^ c)
constexpr uint32_t kAndNot = 0x40;    // a & b & ~c
constexpr uint32_t kOrAnd2 = 0xEA;    // (a & b) | c

// Horizontal neighbours of a lane group x (bitlayout.h).  Plane k's left
// neighbours are plane k-1 and its right neighbours plane k+1, at the same bit,
// except at the two ends: plane 0's left neighbours are plane NP-1 shifted up one
// bit (its bit 0 from the last plane of the group to the left, in lane l-1), and
// plane NP-1's right neighbours are plane 0 shifted down one bit (bit 31 from
// lane l+1).  One DPP wave shift and one v_alignbit each, per group.
struct Ends {
    uint32_t l0, rn;
};
template <int NP>
__device__ __forceinline__ Ends ends(const Pl<NP>& x)
{
    const uint32_t hp = lane_from_left(x.v[NP - 1]);  // bit 31: the column left of the group
    const uint32_t ln = lane_from_right(x.v[0]);      // bit 0: the column right of the group
    Ends e;
    e.l0 = __builtin_amdgcn_alignbit(x.v[NP - 1], hp, 31);  // (last << 1) | (hp >> 31)
    e.rn = __builtin_amdgcn_alignbit(ln, x.v[0], 1);        // (first >> 1) | (ln << 31)
    return e;
}
template <int NP>
__device__ __forceinline__ uint32_t left_of(const Pl<NP>& x, const Ends& e, int k)
{
    return k == 0 ? e.l0 : x.v[k - 1];
}
template <int NP>
__device__ __forceinline__ uint32_t right_of(const Pl<NP>& x, const Ends& e, int k)
{
    return k == NP - 1 ? e.rn : x.v[k + 1];
}

// Stage state (5 planes per fused generation): H3 of rows r-2 and r-1 and the
// cells of row r-1.  The emitted cell sees T = H3(r-2) + H3(r-1) + H3(r), the
// 9-cell sum including itself.  For an alive cell T = n + 1, for a dead one T = n
// (generic masks: survive bit T-1 / birth bit T); the two fixed rules read it off
// directly:
//   REF (B/S2):      next = alive && T == 3   (Parallel_Life_MPI.cpp:47-50)
//   CONWAY (B3/S23): next = T == 3 || (alive && T == 4)
//
// Both fixed rules share work between a stage's consecutive steps (r04,
// GOL_PAIR_SUM): rows r-1 and r emitted at two consecutive steps both see the pair
// H3(r-1), H3(r) (ingest of r: emit r-1 = pair + H3(r-2); ingest of r+1: emit r =
// pair + H3(r+1)).  The pair is reduced once, at the step whose ingested row has
// even index (a "pair step"), to three planes kept in (q0, q1, q2) for the next
// step, and each row tests them against its third row: B/S2 3 features + 3 gates
// per row (ref_from_pair), B3/S23 4 features + 4 gates per row (conway_from_pair).
// Per plane and stage-step 6.5 instead of 8 v_bitop3 (B/S2) and 8 instead of 10
// (B3/S23), H3 included.
template <int NP>
struct StageT {
    Pl<NP> ps, pc;
    Pl<NP> cs, cc;
    Pl<NP> al;
    Pl<NP> q0, q1, q2;  // the pair sum between a pair step and the next step
};

template <int RULE>
__device__ __forceinline__ uint32_t rule32_total(uint32_t as, uint32_t ac, uint32_t bs,
                                                 uint32_t bc, uint32_t es, uint32_t ec,
                                                 uint32_t alive, uint32_t birth,
                                                 uint32_t survive)
{
    // T = A + B + E, each a 2-bit H3 sum: T = s0 + 2*(p + k0) + 4*mj (0..9)
    const uint32_t s0 = lop3<kXor3>(as, bs, es);
    const uint32_t k0 = lop3<kMaj>(as, bs, es);
    const uint32_t p = lop3<kXor3>(ac, bc, ec);
    const uint32_t mj = lop3<kMaj>(ac, bc, ec);
    // T == 3  <=>  s0 && p + k0 == 1 && !mj
    const uint32_t three = lop3<kTwoThree>(p, k0, mj);
    if constexpr (RULE == RULE_REF) {
        // Parallel_Life_MPI.cpp:47-50: alive && n == 2  <=>  alive && T == 3
        return lop3<kAnd3>(alive, s0, three);
    } else if constexpr (RULE == RULE_CONWAY) {
        // T == 4  <=>  !s0 && (p + k0 == 2 && !mj  ||  p + k0 == 0 && mj)
        const uint32_t four = lop3<kFour>(p, k0, mj);
        const uint32_t stay = lop3<kAndNot>(alive, four, s0);  // alive & four & !s0
        return lop3<kOrAnd2>(s0, three, stay);                 // (s0 & three) | stay
    } else {
        // T = s0 + 2*x + 4*t2 + 8*t3; alive cells have n = T - 1, dead ones n = T
        const uint32_t x = p ^ k0, y = p & k0;
        const uint32_t t2 = y ^ mj, t3 = y & mj;
        uint32_t r = 0;
#pragma unroll
        for (int v = 0; v <= 9; ++v) {
            const uint32_t ssel = v >= 1 ? (survive >> (v - 1)) & 1u : 0u;
            const uint32_t bsel = v <= 8 ? (birth >> v) & 1u : 0u;
            if (bsel | ssel) {
                const uint32_t eq = ((v & 1) ? s0 : ~s0) & ((v & 2) ? x : ~x) &
                                    ((v & 4) ? t2 : ~t2) & ((v & 8) ? t3 : ~t3);
                const uint32_t sel = (ssel ? alive : 0u) | (bsel ? ~alive : 0u);
                r |= eq & sel;
            }
        }
        return r;
    }
}

#ifndef GOL_PAIR_SUM
#define GOL_PAIR_SUM 1
#endif

// B/S2 of one plane from a pair (b, e) = (H3 of the upper row, H3 of the lower
// row), the third row's H3 (a0, a1) and the cell: alive && b + e + A == 3.  The
// pair enters as three features formed once for its two rows (kRefF*, from bs, bc,
// es) and each row tests them, the pair's lower carry ec and its own third row in
// 3 v_bitop3 (kRefT*): 4.5 per plane and row against 5 for the binary pair sum
// q0 + 2 q1 + 4 q2 (4 per pair) and its 3-gate test.  Found by
// tools/rule_search_pair_feat.c, checked exhaustively by tests/test_stage_logic.py.
constexpr uint32_t kRefF0 = 0x7B;
constexpr uint32_t kRefF1 = 0x95;
constexpr uint32_t kRefF2 = 0xBC;
constexpr uint32_t kRefT0 = 0xC7;
constexpr uint32_t kRefT1 = 0x9E;
constexpr uint32_t kRefT2 = 0x02;
__device__ __forceinline__ uint32_t ref_from_pair(uint32_t f0, uint32_t f1, uint32_t f2,
                                                  uint32_t ec, uint32_t a0, uint32_t a1,
                                                  uint32_t alive)
{
    const uint32_t u = lop3<kRefT0>(a0, f2, f0);
    const uint32_t v = lop3<kRefT1>(f1, ec, a1);
    return lop3<kRefT2>(u, v, alive);
}

// B3/S23 of one plane from a pair (b, e) the same way: T = b + e + A == 3, or alive
// && T == 4.  Four features per pair (kConwayF*; the first only feeds the others)
// and a 4-gate test per row (kConwayT*): 6 per plane and row against 8 for the
// 3-row total.  No test of <= 4 gates on the binary pair sum exists
// (tools/rule_search_pair.c, exhaustive); this network was found by
// tools/rule_search_pair_feat.c and is checked exhaustively by tests/test_stage_logic.py.
constexpr uint32_t kConwayF0 = 0x1D;
constexpr uint32_t kConwayF1 = 0x4D;
constexpr uint32_t kConwayF2 = 0x18;
constexpr uint32_t kConwayF3 = 0xBC;
constexpr uint32_t kConwayT0 = 0xBC;
constexpr uint32_t kConwayT1 = 0xB5;
constexpr uint32_t kConwayT2 = 0x79;
constexpr uint32_t kConwayT3 = 0x32;
__device__ __forceinline__ uint32_t conway_from_pair(uint32_t f1, uint32_t f2, uint32_t f3,
                                                     uint32_t a0, uint32_t a1, uint32_t alive)
{
    const uint32_t g4 = lop3<kConwayT0>(a0, f3, alive);
    const uint32_t g5 = lop3<kConwayT1>(f2, g4, a1);
    const uint32_t g6 = lop3<kConwayT2>(g4, f1, g5);
    return lop3<kConwayT3>(g4, g6, alive);
}

// A pair of H3 rows (b upper, e lower), one plane, as the rule's test reads it:
// three features in (q0, q1, q2) (kRefF* / kConwayF*) and, for B/S2, the lower
// row's carry ec
struct PairQ {
    uint32_t q0, q1, q2, ec;
};
template <int RULE>
__device__ __forceinline__ PairQ pair_sum(uint32_t bs, uint32_t bc, uint32_t es, uint32_t ec)
{
    PairQ q;
    q.ec = ec;
    if constexpr (RULE == RULE_REF) {
        q.q0 = lop3<kRefF0>(es, bc, bs);
        q.q1 = lop3<kRefF1>(es, bs, bc);
        q.q2 = lop3<kRefF2>(es, bs, q.q1);
    } else {
        const uint32_t f0 = lop3<kConwayF0>(bs, es, es);
        q.q0 = lop3<kConwayF1>(bc, f0, ec);
        q.q1 = lop3<kConwayF2>(f0, ec, bc);
        q.q2 = lop3<kConwayF3>(es, bs, q.q1);
    }
    return q;
}
template <int RULE>
__device__ __forceinline__ uint32_t rule_from_pair(const PairQ& q, uint32_t a0, uint32_t a1,
                                                   uint32_t alive)
{
    if constexpr (RULE == RULE_CONWAY) return conway_from_pair(q.q0, q.q1, q.q2, a0, a1, alive);
    return ref_from_pair(q.q0, q.q1, q.q2, q.ec, a0, a1, alive);
}
// rules with a pair form
constexpr bool pair_rule(int RULE) { return GOL_PAIR_SUM && (RULE == RULE_REF || RULE == RULE_CONWAY); }

// One stage step: ingest row r (x, generation g-1), emit row r-1 at generation g.
// `pair`: the step reduces the pair (even ingested row; a constant once the
// caller's loops are unrolled).
template <int RULE, int NP>
__device__ __forceinline__ Pl<NP> stage_step(StageT<NP>& st, const Pl<NP>& x, uint32_t birth,
                                             uint32_t survive, bool pair)
{
    constexpr bool kPairSum = pair_rule(RULE);
    const Ends e = ends(x);
    Pl<NP> s3, c3, y;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint32_t L = left_of(x, e, k), R = right_of(x, e, k);
        s3.v[k] = lop3<kXor3>(L, x.v[k], R);
        c3.v[k] = lop3<kMaj>(L, x.v[k], R);
        if constexpr (kPairSum) {
            if (pair) {
                // P = H3(r-1) + H3(r); emit r-1 against H3(r-2)
                const PairQ q = pair_sum<RULE>(st.cs.v[k], st.cc.v[k], s3.v[k], c3.v[k]);
                y.v[k] = rule_from_pair<RULE>(q, st.ps.v[k], st.pc.v[k], st.al.v[k]);
                st.q0.v[k] = q.q0;
                st.q1.v[k] = q.q1;
                st.q2.v[k] = q.q2;
            } else {
                // P = H3(r-2) + H3(r-1) from the pair step; emit r-1 against H3(r)
                const PairQ q{st.q0.v[k], st.q1.v[k], st.q2.v[k], st.cc.v[k]};
                y.v[k] = rule_from_pair<RULE>(q, s3.v[k], c3.v[k], st.al.v[k]);
            }
        } else {
            y.v[k] = rule32_total<RULE>(st.ps.v[k], st.pc.v[k], st.cs.v[k], st.cc.v[k], s3.v[k],
                                        c3.v[k], st.al.v[k], birth, survive);
        }
    }
    if (!kPairSum || !pair) {
        st.ps = st.cs;
        st.pc = st.cc;
    }
    st.cs = s3;
    st.cc = c3;
    st.al = x;
    return y;
}

// Steps per block (rows prefetched ahead through the register ring): 8 for the
// 2-plane kernels of depth >= 16, whose 2 waves/SIMD leave VGPRs to spare, 4
// elsewhere (profiles/r01/ab_prefetch_depth.jsonl).  Host copy: prefetch_of().
template <int NP, int K>
constexpr int kPfOf()
{
    return (NP == 2 && K >= 16) ? 8 : 4;
}

// Code placement directive of a steady-state block (see the kernel): every
// plane of the block's inputs passes through it.
#define GOL_PL2(p) "+v"(x[p].v[0]), "+v"(x[p].v[1])
#define GOL_PL4(p) "+v"(x[p].v[0]), "+v"(x[p].v[1]), "+v"(x[p].v[2]), "+v"(x[p].v[3])
template <bool PAD, int NP, int PF>
__device__ __forceinline__ void place_block(Pl<NP> (&x)[PF])
{
    static_assert((NP == 2 && (PF == 4 || PF == 8)) || (NP == 4 && PF == 4),
                  "placement asm names 4 or 8 inputs");
    if constexpr (NP == 2 && PF == 8) {
        if constexpr (PAD)
            asm volatile(".p2align 3\n\ts_nop 0"
                         : GOL_PL2(0), GOL_PL2(1), GOL_PL2(2), GOL_PL2(3), GOL_PL2(4), GOL_PL2(5),
                           GOL_PL2(6), GOL_PL2(7) : : "memory");
        else
            asm volatile(".p2align 3"
                         : GOL_PL2(0), GOL_PL2(1), GOL_PL2(2), GOL_PL2(3), GOL_PL2(4), GOL_PL2(5),
                           GOL_PL2(6), GOL_PL2(7) : : "memory");
    } else if constexpr (NP == 2) {
        if constexpr (PAD)
            asm volatile(".p2align 3\n\ts_nop 0" : GOL_PL2(0), GOL_PL2(1), GOL_PL2(2), GOL_PL2(3)
                         : : "memory");
        else
            asm volatile(".p2align 3" : GOL_PL2(0), GOL_PL2(1), GOL_PL2(2), GOL_PL2(3) : : "memory");
    } else {
        if constexpr (PAD)
            asm volatile(".p2align 3\n\ts_nop 0" : GOL_PL4(0), GOL_PL4(1), GOL_PL4(2), GOL_PL4(3)
                         : : "memory");
        else
            asm volatile(".p2align 3" : GOL_PL4(0), GOL_PL4(1), GOL_PL4(2), GOL_PL4(3) : : "memory");
    }
}
#undef GOL_PL2
#undef GOL_PL4

// Upper bound of a wait for another wavefront (hand-off rows, resident tiles and
// waves): 2 s of the 100 MHz constant clock (s_memrealtime), read only while the
// awaited value is not there yet.  A wait that long means the protocol is broken
// (or the GPU is shared with something that holds it for seconds): flag the
// error and go on, so that the launch always drains and gol_sync reports it.
constexpr uint64_t kWaitTicks = 200000000ull;
__device__ __forceinline__ uint64_t wait_clock() { return __builtin_amdgcn_s_memrealtime(); }

// Block modes of the stencil kernel (see `block`).
constexpr int kWarmBlk = 0, kPure = 1, kSide = 2, kPureMask = 3;

// Dev timing experiments only (tools/exp_build.sh; results are NOT valid): bit 0
// skips the consumer's wait, bit 1 the producer's drain + flag, bit 2 the
// side-row stores, bit 3 the consumer's tail; bit 7 logs every wavefront's start/end
// stamps and hardware id (gol_dev_set_wave_log), bits 8/9 alternate s_setprio
// between the two waves of a SIMD every steady block, bit 10 balances them closed-loop
// (each takes priority while it is not ahead of its partner).
#ifndef GOL_EXP
#define GOL_EXP 0
#endif
// (r05) warm-up rows loaded up front (see the kernel); 0 = the r04 one-block ring
// (r05) The warm-up's first kWarmAheadRows rows are loaded up front and each
// warm-up block issues the rows that many steps ahead of it, with a scheduling
// barrier between the blocks that keeps those loads where they are.  Every
// wavefront of a launch starts at once and its first loads stall at issue on the
// CU's outstanding requests (the start burst): with one block of rows
// up front instead of all 32 the first blocks compute while the rest stream in.
// RCCL per-rank proxy, 5 runs with the build order rotated, one box
// (profiles/r05/ab_warm_ahead.jsonl), mean TCUPS of own rows, all 32 rows up
// front / 16 / 12 / 8 ahead: 8-way 117.8 / 118.4-118.9 / 118.9 / 119.7, 4-way
// 136.0 / 136.1-136.4 / 137.1 / 136.8; 65536^2 157.8-158.0 (16) vs 158.1-158.2
// (8).  (The r04 one-block ring and these dev switches were removed in r06.)
constexpr int kWarmAheadRows = 8;
// the steady ring's first rows are issued this many warm-up blocks before the
// steady loop (r05: 1 or 3 instead of 2 measured no better,
// profiles/r05/ab_steady_lead_rejected.jsonl)
constexpr int kSteadyLeadBlocks = 2;

// MP: the multi-pass form (StepArgs::npass > 1; a separate instantiation, so the
// single-pass kernel's steady loop stays exactly as it was)
template <int K, int RULE, int NP, bool HAND, int TOFF, bool MP = false>
// (capped at 256 registers to keep 2 waves per SIMD: the 8-step-prefetch hand-off
// kernels of tail offset 2, which need 258 VGPRs, with a few scratch spills, and the
// B/S2 and B3/S23 ones with the pair sum, whose hand-off kernels would take 262)
// (depths > 16, dev build only, need 1 wave per SIMD and stay uncapped)
__global__ __launch_bounds__(256, (kPfOf<NP, K>() == 8 && K <= 16 &&
                                   (pair_rule(RULE) ||
                                    (HAND && TOFF == 2 && RULE != RULE_GENERIC))) ? 2 : 1)
void life_tb_kernel(StepArgs a)
{
    constexpr bool kBirths = RULE != RULE_REF;
    constexpr int G = NP / 2;  // words per lane group
    constexpr int kPrefetch = kPfOf<NP, K>();
    constexpr int kSideRows = 2 * (K - 1);  // hand-off rows per block: 2 per generation 1..K-1
    constexpr int kWarmSteps = (2 * K + kPrefetch - 1) / kPrefetch * kPrefetch;  // unrolled warm-up
    constexpr int kWarmAhead = kWarmAheadRows < kWarmSteps ? kWarmAheadRows : kWarmSteps;
    static_assert(K + 2 * kPrefetch <= kGuardRows, "streaming loads must stay in the guard rows");
    static_assert(!HAND || K >= kHandoffMinDepth, "hand-off kernels start at kHandoffMinDepth");
    static_assert(TOFF >= 0 && TOFF < kPrefetch && (HAND || TOFF == 0), "tail offset");
    // stage_rm takes a step's pair parity from its index within the unrolled block:
    // every block start (warm-up, steady, tail offset, tail at t_side = R + 2 with R
    // even, checked on the host in engine.cpp launch) must be an even step
    static_assert(kPrefetch % 2 == 0 && kWarmSteps % 2 == 0 && TOFF % 2 == 0,
                  "pair steps need even block starts");
    const int lane = threadIdx.x & 63;
    const int64_t unit =
        (int64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (unit >= a.total_units) return;
#if GOL_EXP & 128
    const uint64_t wl_t0 = __builtin_amdgcn_s_memrealtime();
#endif
#if GOL_EXP & (256 | 512)
    // priority alternation between the two waves of a SIMD: parity from the wave
    // slot (HW_ID.WAVE_ID, 256) or from dispatch order (first half of the grid, 512)
    const uint32_t prio_par = (GOL_EXP & 256)
                                  ? (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4) & 1u)
                                  : (blockIdx.x < gridDim.x / 2 ? 0u : 1u);
#endif
#if GOL_EXP & 1024
    // closed-loop balance of the two waves of a SIMD: each publishes its count of
    // steady blocks in its SIMD's slot (HW_ID wave slot & 1) and takes priority
    // while it is not ahead of its partner
    uint32_t* prog_me;
    const uint32_t* prog_mate;
    {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 7;
        const uint32_t simd = ((((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 +
                                ((hw >> 8) & 15)) * 4 + ((hw >> 4) & 3));
        prog_me = a.prog + simd * 2 + (hw & 1);
        prog_mate = a.prog + simd * 2 + ((hw & 1) ^ 1);
    }
    uint32_t prog_n = 0, prog_m = 0;
#endif

    // a unit of the packed half strip (uniform): its two row blocks from the table
    const bool pu = a.pair_units > 0 && unit >= a.pair0;
    // (r05) One-segment launches (every launch of a GLOBAL or rank engine) take
    // their segment from the kernel arguments, which arrive with the first scalar
    // loads, instead of a dependent table walk in memory at every wavefront's
    // start; the half strip's units use it with one block from pair0 (the device
    // table's extra segment, plan.cpp build_plans).
    SegDesc sg;
    if (a.seg0_only) {
        sg = a.seg0;
        if (pu) {
            sg.nblk = 1;
            sg.unit0 = a.pair0;
        }
    } else {
        int sidx = 0;
        for (int j = 1; j < a.nseg; ++j)
            if (unit >= a.segs[j].unit0) sidx = j;
        sg = a.segs[sidx];
    }
    const int64_t u = unit - sg.unit0;
    // strip and block-from-the-bottom of the unit: 32-bit (units < 2^31; the 64-bit
    // division is a long VALU/SALU sequence in every wavefront's prologue)
    const uint32_t u_blk = (uint32_t)u / (uint32_t)a.strips;
    const int64_t u_strip = (int64_t)((uint32_t)u - u_blk * (uint32_t)a.strips);
    int64_t pair_a = 0, pair_b = -1, pair_len = 0;
    if (pu) {
        // (row indices < 2^31; readfirstlane keeps them, and every row bound derived
        // from them, in SGPRs)
        const int64_t* pd = a.pairs + 3 * (unit - a.pair0);
        pair_a = __builtin_amdgcn_readfirstlane((int32_t)pd[0]);
        pair_b = __builtin_amdgcn_readfirstlane((int32_t)pd[1]);
        pair_len = __builtin_amdgcn_readfirstlane((int32_t)pd[2]);
    }
    // row blocks bottom-up: the block below (a hand-off producer) has the smaller index
    const int64_t blk = pu ? 0 : sg.nblk - 1 - (int64_t)u_blk;
    // strip `strip` of the row block lives in lanes [sub*L, sub*L + L); the DPP
    // shifts cross from one strip into the next only at halo lanes
    const int lshift = a.lane_shift;
    const int L = 64 >> lshift;
    const int sub = lane >> (6 - lshift);
    const int lin = lane & (L - 1);
    // lane group q of this lane, the group `qfirst` in the strip's first lane, and
    // whether the lane's result is exact (an output lane)
    int64_t q, qfirst;
    bool exact, on = true;
    if (pu) {
        // half strip: lanes 0 and 31 of each half are its halo
        const int hl = lane & 31;
        qfirst = a.half_q0;
        q = qfirst + hl;
        exact = hl >= 1 && q <= a.half_hi;
        on = lane < 32 || pair_b >= 0;
    } else if (a.edge) {
        const int64_t s = u_strip;
        qfirst = s == 0 ? 0 : (s == a.strips - 1 && a.right_q0 >= 0) ? a.right_q0 : 62 * s;
        q = qfirst + lane;
        exact = (lane >= 1 || q == 0) && (lane <= 62 || q == a.ng - 1);
    } else {
        // q = qbase + sub*(L-2) + lin, qbase (uniform) the group one left of the
        // wave's first strip
        const int64_t qbase = u_strip * (int64_t)(1 << lshift) * (L - 2) - 1;
        qfirst = qbase + 1;
        q = qbase + sub * (L - 2) + lin;
        exact = lin >= 1 && lin <= L - 2;
    }
    const bool qin = on && (q >= 0) && (q < a.ng);
    // column mask (columns >= w dead)
    Pl<NP> cm;
#pragma unroll
    for (int k = 0; k < NP; ++k)
        cm.v[k] = qin ? ((q == a.ng - 1) ? (uint32_t)(a.lastmask[k / 2] >> (32 * (k & 1))) : ~0u)
                      : 0u;
    // lanes outside the field read a group of the strip (any word of the row will
    // do; masked to 0)
    const int64_t qc = qin ? q : min(qfirst + 1, a.ng - 1);
    // Every access = a uniform row base (SGPRs) + a per-lane byte offset: the
    // lane's group in field rows (lanes 32-63 of a pair unit: plus their row
    // block's offset), the lane itself in side rows (halo lanes and lanes outside
    // the field share groups with other lanes, so side rows, which every lane
    // stores, are indexed by lane)
    const int64_t row_off = (pu && lane >= 32 && pair_b >= 0) ? (pair_b - pair_a) * a.stride : 0;
    const uint32_t voff = (uint32_t)((qc * G + row_off) * 8);
    const uint32_t voff_side = (uint32_t)(lane * G * 8);

    // row block [rb, re): rows_per_wave rows each, or with age-skewed blocks
    // (one segment) the bottom blocks of a strip whose units start first (u <
    // units_old, the older wave of their SIMD) rows_old rows each; a pair unit's
    // from the table
    int64_t rb = pu ? pair_a : sg.out_lo + blk * a.rows_per_wave;
    int64_t rlen = pu ? pair_len : a.rows_per_wave;
    // (multi-pass) the rows the strip's blocks cover as planned: only the bottom
    // block may end past out_hi, clipped to a length of no hand-off class
    int64_t planned_end = sg.out_lo + sg.nblk * a.rows_per_wave;
    if (a.rows_old && !pu) {
        const int32_t s = (int32_t)u_strip;
        const int64_t jo = min(sg.nblk, (int64_t)(a.units_old > s ? (uint32_t)(a.units_old - s + a.strips - 1) /
                                                                       (uint32_t)a.strips
                                                                 : 0u));
        const int64_t ny = sg.nblk - jo;  // young blocks, on top
        if (blk >= ny) {
            rb = sg.out_lo + ny * a.rows_per_wave + (blk - ny) * a.rows_old;
            rlen = a.rows_old;
        }
        planned_end = sg.out_lo + ny * a.rows_per_wave + jo * a.rows_old;
    }
    // (r06 dev A/B, GOL_DEV_XCD_SHIFT, dev build only; measured 7% slower at the
    // 8-way rank shape whatever the table) Per-XCD row shift: inside a strip,
    // blocks pair up from the top as (1, 2), (3, 4), ... (never the first or the
    // last block), and in the pairs of every m-th strip the block whose wavefront's
    // workgroup lands on the faster XCD class (blockIdx mod 8 under round-robin
    // dispatch; codes in 2-bit fields, higher = faster) takes 8 rows from its
    // partner.  A pair's rows stay its rows, so every strip is still tiled exactly
    // whatever XCD the workgroups really land on; 8 rows keep the hand-off
    // tail-offset class and the even block starts.
#if GOL_DEV_KERNELS
    if (a.xcd_shift && !pu) {
        const uint32_t m = (a.xcd_shift >> 16) & 0xffu;
        const int32_t j = (int32_t)blk, nb = (int32_t)sg.nblk;
        const int32_t jp = (j & 1) ? j : j - 1;  // the pair's upper block
        if (m && jp >= 1 && jp + 1 <= nb - 2 && (uint32_t)u_strip % m == 0) {
            auto code_of = [&](int32_t jj) {
                const uint32_t uu = (uint32_t)sg.unit0 + (uint32_t)(nb - 1 - jj) * (uint32_t)a.strips +
                                    (uint32_t)u_strip;
                return (a.xcd_shift >> (2 * ((uu / kWavesPerBlock) & 7u))) & 3u;
            };
            const uint32_t cu = code_of(jp), cl = code_of(jp + 1);
            const int32_t d = cu > cl ? 8 : (cu < cl ? -8 : 0);  // rows the upper block gains
            if (j == jp) {
                rlen += d;
            } else {
                rb += d;
                rlen -= d;
            }
        }
    }
#endif
    const int64_t re = min(rb + rlen, sg.out_hi);
    // step counts and indices are 32-bit (a block has at most rows_per_wave + 2K
    // steps): uniform 32-bit compares stay on the scalar unit, 64-bit ones do not
    const int32_t T = (int32_t)(re - rb) + 2 * K;  // steps (input rows of a classic block)
    // hand-off roles: every block but the top one produces side rows for the block
    // above; every block but the bottom one consumes those of the block below
    // (pair units close their blocks the classic way: their segment, the last of
    // the launch, is one block deep.  A pu term here instead costs the hand-off
    // kernels ~80 VGPRs: the compiler specializes the stream on it.)
    const int64_t row_bytes = a.stride * 8;
    constexpr int64_t kSideRowBytes = 64 * G * 8;
    const bool st_lane = qin && exact;
    // buffer rows that are inside the buffer and the field (dead border)
    const int64_t vlo = max((int64_t)0, -sg.glob0), vhi = min(sg.in_rows, sg.field_h - sg.glob0);
    const bool has_above = blk > 0, has_below = blk < sg.nblk - 1;
    // a clipped bottom block takes no hand-off in bottom-up passes (its length has
    // no tail offset class, maybe not even an even one): it closes classically,
    // and the block above it produces no side rows
    const bool bottom_clipped = planned_end != sg.out_hi;
    const bool up_consumer = has_above && !(bottom_clipped && blk == sg.nblk - 1);
    const bool up_producer = has_below && !(bottom_clipped && blk == sg.nblk - 2);

    // Multi-pass launches (r05).  A launch runs `npass` passes of K generations
    // over the same row blocks, pass p reading buffer pbuf[p] and writing
    // pbuf[p + 1] (the host gives npass + 1 distinct buffers, so no pass writes
    // rows another wavefront may still read in an earlier pass).  Odd passes
    // stream their block bottom-up: a block's first rows in one pass are then its
    // last ones in the next, so the rows beyond its start (the block in front,
    // "front") were computed at that block's start of the previous pass, long
    // done, and only the rows beyond its end (the block behind, "back") wait for
    // a neighbour to finish the previous pass -- at the end of this one.  Flags:
    // a unit raises head[p] once its first K output rows of pass p are stored and
    // done[p] at the end of pass p, each read (and reset) by the one unit that
    // needs it.  Halo lanes (lanes whose group another strip outputs) keep their
    // own values across passes in a shadow half of each buffer (a.shadow_off
    // bytes on): after P passes of K generations their outer P*K columns are wrong
    // and the exact lanes beside them still see exact columns (P*K <= 48 < 64).
    // The stencil is symmetric under a vertical flip, so a bottom-up pass is the
    // same code on rows addressed with a negative stride.  (Measured slower than
    // single-pass launches: the extra per-pass state spills the hand-off kernels
    // and lengthens the address arithmetic; a dev switch, GOL_DEV_PASSES)
    const int npass = MP ? a.npass : 1;
    const bool halo_lane = qin && !exact && !pu;
    bool up = false, producer = false, consumer = false, head_sent = false;
    int32_t t_side = INT32_MAX, t_lo = 0, t_hi = 0, f_lo = 0, f_hi = 0;
    int32_t s_back = INT32_MAX;  // first stream step beyond the block's far end
    int64_t rs = row_bytes;      // bytes per stream step (negative bottom-up)
    const char* in_rows = nullptr;
    char* out_rows = nullptr;
    char* my_side = nullptr;
    const char* dn_side = nullptr;
    uint32_t* my_flag = nullptr;
    uint32_t* dn_flag = nullptr;
    uint32_t voff_ld = voff, voff_st = voff;
    bool st_ok = st_lane, wt_stores = false, done_need = false, back_need = false;
    int64_t back_unit = 0;
    // one-shot flags of the multi-pass protocol: wait until *f is set, reset it
    auto mp_wait = [&](uint32_t* f) {
        if (a.mp_dev & 2) return;  // dev timing: no inter-pass waits (field not valid)
        uint32_t v = 0;
        uint64_t w0 = 0;
        for (int it = 0;; ++it) {
            v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (v) break;
            if (it == 0) w0 = wait_clock();
            else if (wait_clock() - w0 > kWaitTicks) break;
            __builtin_amdgcn_s_sleep(4);
        }
        if (lane == 0) {
            if (!v) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(f, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("" ::: "memory");
    };
    auto mp_raise = [&](uint32_t* f) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this pass's stores drained
        if (lane == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // flags of unit x for pass p: head at [p][x], done at [2 + p][x]
    auto head_flag = [&](int p, int64_t x) { return a.mpflags + (int64_t)p * a.total_units + x; };
    auto done_flag = [&](int p, int64_t x) { return a.mpflags + (int64_t)(2 + p) * a.total_units + x; };

#if GOL_EXP & 128
    uint64_t wl_tb = 0, wl_tb1 = 0, wl_tw = 0, wl_ts = 0;
#endif
#if GOL_EXP & 16384
    uint64_t wl_pi = 0, wl_pl = 0;
#endif
    for (int pass = 0; pass < npass; ++pass) {
    {
        up = (pass & 1) != 0;
        const int64_t start_row = up ? re - 1 + K : rb - K;  // local row of step 0
        const int64_t out_first = up ? re - 1 : rb;          // row of the first output
        rs = up ? -row_bytes : row_bytes;
        in_rows = reinterpret_cast<const char*>(a.pbuf[pass] + (sg.base_row + start_row) * a.stride);
        out_rows = reinterpret_cast<char*>(a.pbuf[pass + 1] + (sg.base_row + out_first) * a.stride);
        // steps [t_lo, t_hi) read rows inside the buffer and the field
        t_lo = (int32_t)(up ? start_row - vhi + 1 : vlo - start_row);
        t_hi = (int32_t)(up ? start_row - vlo + 1 : vhi - start_row);
        // stage g at step t emits the row t - (g + 1) steps from start_row: a field
        // row (glob0 + that row) alive only in [0, field_h) when x in [f_lo, f_hi)
        f_lo = (int32_t)(up ? sg.glob0 + start_row - sg.field_h + 1 : -(sg.glob0 + start_row));
        f_hi = (int32_t)(up ? sg.glob0 + start_row + 1 : sg.field_h - (sg.glob0 + start_row));
        // hand-off roles: a block takes its last side rows from the block behind it
        // (top-down: the block below, bottom-up: the block above) and produces them
        // for the block in front (pair units close their blocks the classic way:
        // their segment, the last of the launch, is one block deep)
        producer = HAND && (up ? up_producer : has_above);
        consumer = HAND && (up ? up_consumer : has_below);
        // a consumer streams R + 2 input rows (steps < t_side), then side rows
        t_side = consumer ? (int32_t)(re - rb) + 2 : INT32_MAX;
        // the first stream step beyond the block's far end (a consumer reads none)
        s_back = consumer ? INT32_MAX : (int32_t)(re - rb) + K;
        const int64_t par = pass & 1;
        const int64_t prod = up ? unit + a.strips : unit - a.strips;  // a consumer's producer
        if constexpr (HAND) {
            my_side = reinterpret_cast<char*>(a.side + (par * a.total_units + unit) * a.side_slot);
            dn_side = reinterpret_cast<const char*>(a.side + (par * a.total_units + prod) * a.side_slot);
            my_flag = a.flags + par * a.total_units + unit;
            dn_flag = a.flags + par * a.total_units + prod;
        }
        voff_ld = voff + ((pass > 0 && halo_lane && !(a.mp_dev & 8)) ? a.shadow_off : 0u);
        const bool wr_shadow = pass < npass - 1 && halo_lane && !(a.mp_dev & 8);
        voff_st = voff + (wr_shadow ? a.shadow_off : 0u);
        st_ok = st_lane || wr_shadow;
        // rows another wavefront reads in the next pass go out write-through
        wt_stores = pass < npass - 1;
        // the next pass's reader of this pass's head / done flags (see above)
        head_sent = !(pass < npass - 1 && (up ? has_below : has_above));
        done_need = pass < npass - 1 && (up ? has_above : has_below);
        back_need = pass > 0 && !consumer && (up ? has_above : has_below);
        back_unit = up ? unit + a.strips : unit - a.strips;
        // the block in front's first rows of the previous pass
        if (pass > 0 && (up ? has_below : has_above))
            mp_wait(head_flag(pass - 1, up ? unit - a.strips : unit + a.strips));
        // the block behind's last rows of the previous pass, when the rows the pass
        // loads up front reach them (later: mp_sync)
        if (back_need && s_back < kWarmSteps + 2 * kPrefetch) mp_wait(done_flag(pass - 1, back_unit));
    }
    StageT<NP> st[K];
#pragma unroll
    for (int g = 0; g < K; ++g) st[g] = {};

    // the row streamed at step s: input row start_row + s (rows in stream order), or for a consumer from
    // step t_side on the block below's side row s - t_side (uniform select)
    auto load_step = [&](int32_t s) -> Grp<NP> {
        if constexpr (!HAND)
            return load_field<NP>(reinterpret_cast<const uint64_t*>(in_rows + (int64_t)s * rs + voff_ld));
        if (s < t_side)
            return load_field<NP>(reinterpret_cast<const uint64_t*>(in_rows + (int64_t)s * rs + voff_ld));
        // side rows: stored sc1 by another wavefront of this launch, loaded sc1
        return load_grp<NP>(reinterpret_cast<const uint64_t*>(
            dn_side + (int64_t)(s - t_side) * kSideRowBytes + voff_side));
    };
    Grp<NP> ring[kPrefetch];
    // (r05) The warm-up rows have a ring of their own (the first kWarmAhead loaded
    // up front, each warm-up block issuing the rows kWarmAhead steps ahead), and
    // the steady ring is filled kSteadyLeadBlocks warm-up blocks before the steady
    // loop.  With the r04 one-block ring the compiler pulled each warm-up block's
    // ingest up into the block before (no scheduling barriers there), so every
    // refill was consumed right after its issue: a chain of HBM round trips
    // (s_waitcnt vmcnt(0/1) after each load) that made the 2K warm-up steps take
    // 16-20 us per wavefront at every shape (profiles/r05/wave_phases_*.jsonl).
    Grp<NP> wring[kWarmSteps];
#pragma unroll
    for (int p = 0; p < kWarmAhead; ++p)  // (input rows: t_side >= warm-up + 2 blocks)
        wring[p] = load_field<NP>(reinterpret_cast<const uint64_t*>(in_rows + (int64_t)p * rs + voff_ld));
    constexpr int kSteadyIssue =
        kWarmSteps >= kSteadyLeadBlocks * kPrefetch ? kWarmSteps - kSteadyLeadBlocks * kPrefetch : 0;
#if GOL_EXP & 16384
    // dev probe of a wavefront's start (tools/wave_log.py --probe): the initial
    // loads issued, and all of them landed (results stay valid, timing does not)
    wl_pi = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wl_pl = __builtin_amdgcn_s_memrealtime();
#endif

    // row of step t: an input row is dead outside the field / buffer; a side row
    // comes as the block below computed it; columns >= w masked.  SIDE: the step
    // may be a side row (a consumer's last blocks); else it is an input row.
    auto ingest = [&](int32_t t, const Grp<NP>& xv, auto side) -> Pl<NP> {
        const bool ok = (decltype(side)::value && t >= t_side) || ((t >= t_lo) && (t < t_hi));
        Pl<NP> x = planes_of(xv);
#pragma unroll
        for (int k = 0; k < NP; ++k) x.v[k] = ok ? (x.v[k] & cm.v[k]) : 0u;
        return x;
    };
    auto load_in = [&](int32_t s) -> Grp<NP> {
        return load_field<NP>(reinterpret_cast<const uint64_t*>(in_rows + (int64_t)s * rs + voff_ld));
    };
    // stage g (generation g+1) at step t: emits the row t - (g+1) steps from start_row
    // With births (rules other than B/S2) nothing may come alive outside the field:
    // rm is the uniform row test of the emitted row (all ones or 0, a scalar), the
    // column mask is per lane; one v_bitop3 AND3 per plane (8-byte encoding, like the
    // rest of the hot loop).
    auto row_mask = [&](int32_t r) -> uint32_t {  // r: steps from start_row of the emitted row
        return __builtin_amdgcn_readfirstlane((r >= f_lo) && (r < f_hi) ? ~0u : 0u);
    };
    // (the ingested row of stage g at step t is t - g; every caller's t has the parity
    // of its unrolled step index p: blocks start at multiples of kPrefetch, the tail
    // at t_side = R + 2 with R even for hand-off plans)
    auto stage_rm = [&](int g, int p, Pl<NP> x, uint32_t rm, auto masked) -> Pl<NP> {
        x = stage_step<RULE>(st[g], x, a.birth, a.survive, ((p - g) & 1) == 0);
        if constexpr (kBirths && decltype(masked)::value) {
#pragma unroll
            for (int k = 0; k < NP; ++k) x.v[k] = lop3<kAnd3>(x.v[k], cm.v[k], rm);
        }
        return x;
    };
    auto stage = [&](int g, int p, int32_t t, Pl<NP> x) -> Pl<NP> {
        return stage_rm(g, p, x, kBirths ? row_mask(t - (g + 1)) : 0u, std::true_type{});
    };
    // Steady blocks without the births mask (r04).  The mask only changes cells the
    // unit holds outside the field: lanes outside it or bits >= w of the last
    // group (a per-lane column mask that is not all ones), and rows outside
    // [0, field_h).  Rows above the field are emitted only in the warm-up (stage g
    // emits row t - g - 1 at step t, and the first row of the field is at most K
    // rows below the stream's first, f_lo <= K, so t < f_lo + K <= 2K <= warm-up),
    // rows below it only by the last blocks of a stream that reaches past the
    // field.  So a unit whose lanes are all inside the field runs its steady blocks
    // up to the first that can emit row f_hi unmasked (kPure) and the rest masked
    // (kPureMask); in a B3/S23 launch that is every unit but those of the field's
    // last row blocks and of narrow or ragged columns (two v_bitop3 fewer per
    // stage-step of 30.6 issue slots).
    int32_t t_plain_end = INT32_MAX;  // steady blocks from t0 >= t_plain_end mask
    if constexpr (kBirths) {
        bool full = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) full = full && cm.v[k] == ~0u;
        const bool lanes_in = __builtin_amdgcn_ballot_w64(!full) == 0;
        t_plain_end = (lanes_in && f_lo + K <= kWarmSteps) ? f_hi - kPrefetch + 2 : INT32_MIN;
#if defined(GOL_DEV_MASK_MODE) && GOL_DEV_MASK_MODE == 1
        t_plain_end = INT32_MIN;  // dev A/B: every steady block masked (r03 behaviour)
#endif
    }
    // (wt: wt_stores as the caller's opaque copy, see `opaque`)
    auto store = [&](int32_t t, const Pl<NP>& x, uint32_t wt) {
        if (t >= 2 * K && t < T && st_ok) {
            char* o = out_rows + (int64_t)(t - 2 * K) * rs + voff_st;
            if (wt) {
                store_side<NP>(reinterpret_cast<uint64_t*>(o), x);
            } else {
                *reinterpret_cast<Grp<NP>*>(o) = words_of(x);
            }
        }
    };
    // A uniform value the compiler must treat as new in every block: tests of the
    // per-pass state (write-through stores, the multi-pass flags) would otherwise
    // be hoisted out of the steady loop, which then exists twice (unswitched) and
    // loses its code placement (tools/loop_align.py).
    auto opaque = [](uint32_t v) {
        v = __builtin_amdgcn_readfirstlane(v);
        asm volatile("" : "+s"(v));
        return v;
    };
    // (multi-pass) write-through stores for the steps [t_first, t_last] of a
    // non-final pass where they hold rows another wavefront reads next pass: the
    // block's first and last K output rows (its other rows, and its halo lanes'
    // shadow rows, only this wavefront reads back, through its own XCD's L2)
    auto wt_for = [&](int32_t t_first, int32_t t_last) -> uint32_t {
        if constexpr (!MP) return 0u;
        const bool w = wt_stores && (t_first < 3 * K || t_last >= T - K);
        return opaque(w ? 1u : 0u);
    };
    // (multi-pass) after the stores of the steps up to t_last: the head flag once
    // the block's first K output rows (steps 2K .. 3K-1) are out
    auto head_check = [&](int32_t t_last) {
        if (!head_sent && t_last >= 3 * K - 1) {
            mp_raise(head_flag(pass, unit));
            head_sent = true;
        }
    };
    // (multi-pass) in the steady block from t0, before the refill of the block after
    // it: the block behind's done flag when that refill reaches step s_back
    auto mp_sync = [&](int32_t t0) {
        if (back_need && s_back >= t0 + 2 * kPrefetch && s_back < t0 + 3 * kPrefetch)
            mp_wait(done_flag(pass - 1, back_unit));
    };

    // Hand-off signalling (HAND kernels), done in steady blocks after the compute:
    //  * a producer (every block but the top one) raises its flag after its first
    //    steady block -- its side rows were all stored in the warm-up blocks, and
    //    s_waitcnt vmcnt(0) there finds them long complete;
    //  * a consumer waits for the flag of the block below at the end of the block
    //    before the one whose refill first fetches side rows (the planner keeps
    //    R + 2 >= warm-up + 2 blocks + tail offset, handoff_toff).
    auto signal = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(my_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto wait_below = [&]() {
        const uint32_t* f = dn_flag;
        uint32_t v = 0;
        uint64_t t0 = 0;
        for (int it = 0; !(GOL_EXP & 1); ++it) {
            v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(const_cast<uint32_t*>(f), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT));
            if (v) break;
            if (it == 0) t0 = wait_clock();
            else if (wait_clock() - t0 > kWaitTicks) break;
            __builtin_amdgcn_s_sleep(8);
        }
        if (lane == 0) {
            if (!v && !(GOL_EXP & 1))
                __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // flags are all 0 between launches (and passes of one parity): reset
            // the producer's
            __hip_atomic_store(const_cast<uint32_t*>(f), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("" ::: "memory");
    };
    auto sync_point = [&](int32_t t0) {
        const uint32_t r0 = (producer ? 1u : 0u) | (consumer ? 2u : 0u);
        const uint32_t role = MP ? opaque(r0) : r0;
        if ((role & 1u) && t0 == kWarmSteps && !(GOL_EXP & 2)) signal();
        if ((role & 2u) && t0 + 3 * kPrefetch + TOFF > t_side && t0 + 2 * kPrefetch + TOFF <= t_side)
            wait_below();
    };

    // One block of kPrefetch steps from step t0, in one of four modes:
    //  * kWarmBlk (warm-up blocks): stage g first emits a row that can reach a valid
    //    output at step 2g+2 and needs the two ingests before it, so it only runs
    //    from step 2g on; skipping it earlier saves K*(K-1) of the 2K*K warm-up
    //    stage-steps.  In the warm-up blocks of a hand-off kernel, stage g's outputs
    //    at steps 2g+2 and 2g+3 (its first two rows, generation g+1) are also stored
    //    as side rows 2g and 2g+1 for the block above;
    //  * kPure: the steady-state loop -- input rows only (a hand-off kernel's
    //    signal and wait are scalar-guarded calls in it);
    //  * kSide (hand-off consumers): the last 1-2 steady blocks, whose refill may
    //    reach the side rows (a per-load select).  Peeling them keeps the selects
    //    out of the hot loop; a third copy for the first steady block cost more in
    //    instruction cache than it saved (profiles/r02/ab_handoff_peeled.jsonl).
    auto block = [&](int32_t t0, auto mode) {
        constexpr int kMode = decltype(mode)::value;
        constexpr bool kGuard = kMode == kWarmBlk;
        constexpr bool kSideMode = HAND && kMode == kSide;
        // births masked everywhere but in kPure blocks (t_plain_end)
        constexpr bool kMask = kBirths && kMode != kPure;
        Pl<NP> x[kPrefetch];
        if constexpr (kGuard) __builtin_amdgcn_sched_barrier(0);
        if constexpr (kGuard) {
#pragma unroll
            for (int p = 0; p < kPrefetch; ++p) {
                x[p] = ingest(t0 + p, wring[t0 + p], std::false_type{});
                if (t0 + kWarmAhead + p < kWarmSteps)
                    wring[t0 + kWarmAhead + p] = load_in(t0 + kWarmAhead + p);
                if (t0 == kSteadyIssue) ring[p] = load_in(kWarmSteps + p);
            }
        } else
#pragma unroll
        for (int p = 0; p < kPrefetch; ++p) {
            x[p] = ingest(t0 + p, ring[p], std::integral_constant<bool, kSideMode>{});
            if constexpr (kSideMode)
                ring[p] = load_step(t0 + kPrefetch + p);
            else
                ring[p] = load_in(t0 + kPrefetch + p);
        }
        // Code placement (steady-state blocks).  gfx950 issues this kernel's
        // instruction mix (DPP move, v_alignbit, v_bitop3 chains; all 8-byte
        // encodings) 10-25% faster when those instructions sit at addresses =
        // 4 mod 8 with 2+ waves per SIMD, and faster at 0 mod 8 with one
        // (profiles/r01/loop_alignment_ab.jsonl).  The scheduling barriers keep
        // the 4-byte encodings (loads, ingest masks, SALU, stores) out of the
        // compute, so one alignment directive places all of it; the compiler may
        // add a hazard s_nop after it, so the 4-byte pad that gives the wanted
        // parity is per kernel: loop_place.h, generated by tools/loop_align.py.
        // the block's row masks, computed ahead of the compute (scalar code stays out
        // of the placed region): stage g at step t0 + p emits row t0 + p - g - 1
        uint32_t rmv[kPrefetch + K - 1];
        if constexpr (kMask) {
#pragma unroll
            for (int j = 0; j < kPrefetch + K - 1; ++j) rmv[j] = row_mask(t0 - K + j);
        }
        if constexpr (!kGuard) {
            __builtin_amdgcn_sched_barrier(0);
            place_block<life_loop_pad(K, RULE, NP, HAND, TOFF, (kMask ? 1 : 0) | (MP ? 2 : 0)) != 0, NP,
                        kPrefetch>(x);
            __builtin_amdgcn_sched_barrier(0);
        }
        // stage g of step p only needs stage g-1 of step p and stage g of step
        // p-1: issue the block's (p, g) pairs by anti-diagonal d = p + g so
        // independent stage steps sit next to each other for the scheduler
#pragma unroll
        for (int d = 0; d < K + kPrefetch - 1; ++d) {
#pragma unroll
            for (int p = 0; p < kPrefetch; ++p) {
                const int g = d - p;
                if (g >= 0 && g < K && (!kGuard || t0 + p >= 2 * g)) {
                    x[p] = stage_rm(g, p, x[p], kMask ? rmv[p - g - 1 + K] : 0u,
                                    std::integral_constant<bool, kMask>{});
                    if constexpr (HAND && kGuard && !(GOL_EXP & 4)) {
                        if (g <= K - 2 && (t0 + p == 2 * g + 2 || t0 + p == 2 * g + 3))
                            store_side<NP>(reinterpret_cast<uint64_t*>(
                                               my_side + (int64_t)(t0 + p - 2) * kSideRowBytes +
                                               voff_side),
                                           x[p]);
                    }
                }
            }
        }
#if GOL_EXP & (256 | 512)
        if constexpr (!kGuard) {
            if (__builtin_amdgcn_readfirstlane(((uint32_t)t0 / kPrefetch ^ prio_par) & 1u))
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
#endif
#if GOL_EXP & 1024
        if constexpr (!kGuard) {
            // the partner's count loaded one block ago (its latency hidden by this
            // block's compute); then publish ours and load theirs for the next block
            if (__builtin_amdgcn_readfirstlane(prog_m) < prog_n)
                __builtin_amdgcn_s_setprio(0);
            else
                __builtin_amdgcn_s_setprio(1);
            ++prog_n;
            if (lane == 0)
                __hip_atomic_store(prog_me, prog_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            prog_m = __hip_atomic_load(const_cast<uint32_t*>(prog_mate), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
#endif
        if constexpr (!kGuard) {
            __builtin_amdgcn_sched_barrier(0);
            // hand-off signalling between this block's compute and its stores: the
            // memory operations still outstanding here (this block's refill, the
            // previous block's stores) were issued a whole block of compute ago
            if constexpr (HAND) sync_point(t0);
        }
        const uint32_t wt = wt_for(t0, t0 + kPrefetch - 1);
        if constexpr (MP && !kGuard) mp_sync(t0);
#pragma unroll
        for (int p = 0; p < kPrefetch; ++p) store(t0 + p, x[p], wt);
        if constexpr (MP) head_check(t0 + kPrefetch - 1);
    };

    // Warm-up blocks, unrolled (compile-time guards).
    constexpr int kWarm = kWarmSteps;
    static_assert(!HAND || kWarm >= 2 * K, "side rows are all stored in the warm-up blocks");
#if GOL_EXP & 128
    // (wl_tb / wl_tb1: after the first / second warm-up block)
#pragma unroll
    for (int t0 = 0; t0 < kWarm; t0 += kPrefetch) {
        block(t0, std::integral_constant<int, kWarmBlk>{});
        if (t0 == 0) wl_tb = __builtin_amdgcn_s_memrealtime();
        if (t0 == kPrefetch) wl_tb1 = __builtin_amdgcn_s_memrealtime();
    }
#else
#pragma unroll
    for (int t0 = 0; t0 < kWarm; t0 += kPrefetch) block(t0, std::integral_constant<int, kWarmBlk>{});
#endif
#if GOL_EXP & 128
    // phase stamps (r05): issue time of the warm-up's end and the steady blocks' end
    wl_tw = __builtin_amdgcn_s_memrealtime();
#endif

    // Steady state: whole blocks of input steps.  A consumer stops TOFF steps
    // before t_side; its last whole block's refill is the first to reach t_side.
    // The hand-off kernel's first block and a consumer's last blocks (whose
    // refills reach the side rows) are peeled off the hot loop.
    int32_t t0 = kWarm;
    if constexpr (!HAND) {
        for (; t0 < T && t0 < t_plain_end; t0 += kPrefetch)
            block(t0, std::integral_constant<int, kPure>{});
#if !(defined(GOL_DEV_MASK_MODE) && GOL_DEV_MASK_MODE == 2)  // 2: timing only, no masked loop
        if constexpr (kBirths)
            for (; t0 < T; t0 += kPrefetch) block(t0, std::integral_constant<int, kPureMask>{});
#endif
    } else {
        // the consumer's wait is in the last pure block
        const int32_t t_pure_end = consumer ? t_side - 2 * kPrefetch - TOFF + 1 : T;
        auto pure_more = [&](int32_t t) { return t < t_pure_end; };
        for (; pure_more(t0) && t0 < t_plain_end; t0 += kPrefetch)
            block(t0, std::integral_constant<int, kPure>{});
        if constexpr (kBirths)
            for (; pure_more(t0); t0 += kPrefetch)
                block(t0, std::integral_constant<int, kPureMask>{});
        if (consumer)
            for (; t0 + kPrefetch + TOFF <= t_side; t0 += kPrefetch)
                block(t0, std::integral_constant<int, kSide>{});
    }
    // a producer whose stream had no steady block (a short last block) signals here
    if constexpr (HAND)
        if (producer && T <= kWarm && !(GOL_EXP & 2)) signal();
#if GOL_EXP & 128
    wl_ts = __builtin_amdgcn_s_memrealtime();
#endif

    if constexpr (HAND && !(GOL_EXP & 8)) {
        if (consumer) {
            // The planner keeps t_side - warm-up = TOFF (mod kPrefetch): TOFF more
            // input steps, then the ring holds the tail's first rows after a
            // compile-time shift by TOFF slots.
            if constexpr (TOFF > 0) {
                Pl<NP> x[TOFF];
#pragma unroll
                for (int p = 0; p < TOFF; ++p) x[p] = ingest(t0 + p, ring[p], std::true_type{});
#pragma unroll
                for (int p = 0; p + TOFF < kPrefetch; ++p) ring[p] = ring[p + TOFF];
#pragma unroll
                for (int p = 0; p < TOFF; ++p)
                    ring[kPrefetch - TOFF + p] = load_step(t0 + kPrefetch + p);
#pragma unroll
                for (int d = 0; d < K + TOFF - 1; ++d) {
#pragma unroll
                    for (int p = 0; p < TOFF; ++p) {
                        const int g = d - p;
                        if (g >= 0 && g < K) x[p] = stage(g, p, t0 + p, x[p]);
                    }
                }
                const uint32_t wt = wt_for(t0, t0 + TOFF - 1);
#pragma unroll
                for (int p = 0; p < TOFF; ++p) store(t0 + p, x[p], wt);
                if constexpr (MP) head_check(t0 + TOFF - 1);
            }
            // Tail: steps t_side + tau, tau = 0 .. 2K-3.  Side row tau (generation
            // tau/2 + 1) enters at stage s0 = tau/2 + 1 in place of stage s0-1's
            // output; stages below s0 are done (their rows are the block below's).
            const int32_t tb = t_side;
            auto tail = [&](int tau0) {  // tau0: a constant once the loop below is unrolled
                Pl<NP> x[kPrefetch];
#pragma unroll
                for (int p = 0; p < kPrefetch; ++p) {
                    x[p] = ingest(tb + tau0 + p, ring[p], std::true_type{});
                    if (tau0 + kPrefetch + p < kSideRows)
                        ring[p] = load_step(tb + tau0 + kPrefetch + p);
                }
#pragma unroll
                for (int d = 0; d < K + kPrefetch - 1; ++d) {
#pragma unroll
                    for (int p = 0; p < kPrefetch; ++p) {
                        const int g = d - p, tau = tau0 + p;
                        if (tau < kSideRows && g >= tau / 2 + 1 && g < K)
                            x[p] = stage(g, p, tb + tau, x[p]);
                    }
                }
                const uint32_t wt = wt_for(tb + tau0, tb + tau0 + kPrefetch - 1);
#pragma unroll
                for (int p = 0; p < kPrefetch; ++p)
                    if (tau0 + p < kSideRows) store(tb + tau0 + p, x[p], wt);
                if constexpr (MP) head_check(tb + tau0 + kPrefetch - 1);
            };
#pragma unroll
            for (int tau0 = 0; tau0 < kSideRows; tau0 += kPrefetch) tail(tau0);
        }
    }
    if (pass < npass - 1) {
        // this pass's rows are out (this wavefront reads them next pass) and, for
        // the wavefronts beside it, flagged
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!head_sent) mp_raise(head_flag(pass, unit));
        if (done_need) mp_raise(done_flag(pass, unit));
    }
    }  // pass
#if GOL_EXP & 128
    if (a.wlog && lane == 0) {
        // 8 words per wavefront: start, end, HW_ID | XCC_ID, block | workgroup,
        // warm-up end, steady end (tools/wave_log.py)
        uint64_t* wl = a.wlog + unit * 8;
#if GOL_EXP & 16384
        wl[4] = wl_pi;
        wl[5] = wl_pl;
#else
        wl[4] = wl_tw;
        wl[5] = wl_ts;
#endif
        wl[6] = (uint64_t)(re - rb) | ((wl_tb1 - wl_t0) << 32);
        wl[7] = wl_tb;
        wl[0] = wl_t0;
        wl[1] = __builtin_amdgcn_s_memrealtime();
        wl[2] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) |
                ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) << 32);
        wl[3] = (uint64_t)blk | ((uint64_t)blockIdx.x << 32);
    }
#endif
}

}  // namespace

template <int K, int NP, bool HAND, int TOFF>
hipError_t launch_kernel(const StepArgs& a, RuleKind rule, hipStream_t s)
{
    const dim3 grid((unsigned)((a.total_units + kWavesPerBlock - 1) / kWavesPerBlock));
    const dim3 block(64 * kWavesPerBlock);
    if (a.npass > 1) {
        if constexpr (multipass_kernel_exists(K, RULE_REF, NP)) {
            switch (rule) {
            case RULE_REF:
                hipLaunchKernelGGL((life_tb_kernel<K, RULE_REF, NP, HAND, TOFF, true>), grid, block, 0, s, a);
                break;
            case RULE_CONWAY:
                hipLaunchKernelGGL((life_tb_kernel<K, RULE_CONWAY, NP, HAND, TOFF, true>), grid, block, 0, s, a);
                break;
            default:
                if constexpr (multipass_kernel_exists(K, RULE_GENERIC, NP))
                    hipLaunchKernelGGL((life_tb_kernel<K, RULE_GENERIC, NP, HAND, TOFF, true>), grid, block, 0, s, a);
                else
                    return hipErrorInvalidValue;
                break;
            }
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
    switch (rule) {
    case RULE_REF:
        hipLaunchKernelGGL((life_tb_kernel<K, RULE_REF, NP, HAND, TOFF>), grid, block, 0, s, a);
        break;
    case RULE_CONWAY:
        hipLaunchKernelGGL((life_tb_kernel<K, RULE_CONWAY, NP, HAND, TOFF>), grid, block, 0, s, a);
        break;
    default:
        if constexpr (!HAND || handoff_kernel_exists(K, RULE_GENERIC))
            hipLaunchKernelGGL((life_tb_kernel<K, RULE_GENERIC, NP, HAND, TOFF>), grid, block, 0, s, a);
        else
            return hipErrorInvalidValue;
        break;
    }
    return hipGetLastError();
}

template <int K, int NP, bool HAND, int TOFF>
int occupancy_kernel(RuleKind rule, bool mp)
{
    int blocks = 0;
    hipError_t e = hipErrorInvalidValue;
    const int threads = 64 * kWavesPerBlock;
    if (mp) {
        if constexpr (multipass_kernel_exists(K, RULE_REF, NP)) {
            if (rule == RULE_REF)
                e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &blocks, life_tb_kernel<K, RULE_REF, NP, HAND, TOFF, true>, threads, 0);
            else if (rule == RULE_CONWAY)
                e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &blocks, life_tb_kernel<K, RULE_CONWAY, NP, HAND, TOFF, true>, threads, 0);
            else if constexpr (multipass_kernel_exists(K, RULE_GENERIC, NP))
                e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &blocks, life_tb_kernel<K, RULE_GENERIC, NP, HAND, TOFF, true>, threads, 0);
        }
        return e == hipSuccess ? blocks : 0;
    }
    if (rule == RULE_REF)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_REF, NP, HAND, TOFF>, threads, 0);
    else if (rule == RULE_CONWAY)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_CONWAY, NP, HAND, TOFF>, threads, 0);
    else if constexpr (!HAND || handoff_kernel_exists(K, RULE_GENERIC))
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_GENERIC, NP, HAND, TOFF>, threads, 0);
    return e == hipSuccess ? blocks : 0;
}

// 2-plane lane groups at every depth; 4-plane ones (dev build) up to depth 16,
// where 5 planes x 4 x K state words still fit the register file.  Hand-off
// kernels from kHandoffMinDepth on, with tail offsets 0, kPrefetch/2 and (8-step
// prefetch) 6 (handoff_toff in life_internal.h).
constexpr bool depth_has_planes(int K, int NP) { return NP == 2 || (kDevKernels && NP == 4 && K <= 16); }

template <int K, int NP>
hipError_t launch_planes(const StepArgs& a, RuleKind rule, bool hand, hipStream_t s)
{
    if constexpr (K >= kHandoffMinDepth) {
        if (hand) {
            // tail offsets 0, pf/2 and (pf = 8) 2, 6: handoff_toff_exists
            constexpr int pf = kPfOf<NP, K>();
            if (a.tail_off == 0) return launch_kernel<K, NP, true, 0>(a, rule, s);
            if (a.tail_off == pf / 2) return launch_kernel<K, NP, true, pf / 2>(a, rule, s);
            if constexpr (pf == 8) {
                if (a.tail_off == 6) return launch_kernel<K, NP, true, (pf == 8 ? 6 : 0)>(a, rule, s);
                if (a.tail_off == 2) return launch_kernel<K, NP, true, (pf == 8 ? 2 : 0)>(a, rule, s);
            }
            return hipErrorInvalidValue;
        }
    }
    return launch_kernel<K, NP, false, 0>(a, rule, s);
}

template <int K>
hipError_t launch_depth(const StepArgs& a, RuleKind rule, int planes, bool hand, hipStream_t s)
{
    if (hand && K < kHandoffMinDepth) return hipErrorInvalidValue;
    if (planes == 4) {
        if constexpr (depth_has_planes(K, 4)) return launch_planes<K, 4>(a, rule, hand, s);
        return hipErrorInvalidValue;
    }
    return launch_planes<K, 2>(a, rule, hand, s);
}

// Blocks per CU of the hand-off kernels of one depth: the LEAST over every tail
// offset that launch_planes can pick (their register use differs: offset 2 needs
// 258 VGPRs and is capped), since a hand-off launch must fit in one round of
// whichever offset its row lengths select (pick_rows_per_wave).
template <int K, int NP>
int occupancy_hand(RuleKind rule, bool mp)
{
    constexpr int pf = kPfOf<NP, K>();
    int occ = occupancy_kernel<K, NP, true, 0>(rule, mp);
    occ = std::min(occ, occupancy_kernel<K, NP, true, pf / 2>(rule, mp));
    if constexpr (pf == 8) {
        occ = std::min(occ, occupancy_kernel<K, NP, true, (pf == 8 ? 2 : 0)>(rule, mp));
        occ = std::min(occ, occupancy_kernel<K, NP, true, (pf == 8 ? 6 : 0)>(rule, mp));
    }
    return occ;
}

template <int K>
int occupancy_depth(RuleKind rule, int planes, bool hand, bool mp)
{
    if (hand && K < kHandoffMinDepth) return 0;
    if (planes == 4) {
        if constexpr (depth_has_planes(K, 4)) {
            if constexpr (K >= kHandoffMinDepth)
                if (hand) return occupancy_hand<K, 4>(rule, mp);
            return occupancy_kernel<K, 4, false, 0>(rule, mp);
        }
        return 0;
    }
    if constexpr (K >= kHandoffMinDepth)
        if (hand) return occupancy_hand<K, 2>(rule, mp);
    return occupancy_kernel<K, 2, false, 0>(rule, mp);
}

// Instantiation per depth.  A depth's hand-off kernels can be split into their
// own translation units (GOL_EXTERN_HAND in the depth's unit, GOL_INSTANTIATE_HAND
// in the others) to keep the build parallel.
#define GOL_INSTANTIATE_DEPTH(K)                                                              \
    template hipError_t launch_depth<K>(const StepArgs&, RuleKind, int, bool, hipStream_t);   \
    template int occupancy_depth<K>(RuleKind, int, bool, bool);
#define GOL_INSTANTIATE_HAND(K, T)                                                            \
    template hipError_t launch_kernel<K, 2, true, T>(const StepArgs&, RuleKind, hipStream_t); \
    template int occupancy_kernel<K, 2, true, T>(RuleKind, bool);
#define GOL_EXTERN_HAND(K, T)                                                                 \
    extern template hipError_t launch_kernel<K, 2, true, T>(const StepArgs&, RuleKind,        \
                                                            hipStream_t);                     \
    extern template int occupancy_kernel<K, 2, true, T>(RuleKind, bool);

}  // namespace gol
