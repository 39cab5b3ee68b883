// life_kernels.hip -- gfx950 kernels of the Game of Life engine.
//
// Hot path: the per-generation update of Parallel_Life_MPI.cpp (countNeighbours
// :16-35 + updateGrid :37-54), restated on a bit-packed field (64 cells per
// uint64, bit j of word q = column 64q+j) and fused over K generations per
// launch (temporal blocking).
//
// Kernel shape (one wavefront = one work unit, no LDS, no barriers):
//   * A wavefront owns a strip of 64 consecutive lane groups of a row (lane l
//     holds group strip*62 - 1 + l); lanes 0 and 63 are the horizontal halo, so
//     each strip outputs 62 groups.  A lane group is NP = 2 or 4 planes of 32
//     cells (bitlayout.h: column NP*j + k of the group at bit j of plane k), so
//     the horizontal neighbours of every plane but the first and last are other
//     planes at the same bit; those two take one v_alignbit each, with the carry
//     bit from the adjacent lane by a DPP wave shift (wave_shr:1 / wave_shl:1).
//     NP = 4 (two words per lane) pays that once per 128 columns.  After g fused
//     generations the contamination from the unknown groups beyond the halo
//     lanes has moved g columns into lanes 0/63, so K <= 63 keeps lanes 1..62
//     exact.
//   * The wavefront streams down `rows_per_wave` output rows of its strip, K rows
//     of vertical halo on each side.  Generation g (1..K) is a pipeline stage that
//     keeps a 3-row window in registers: for each incoming row it forms the
//     horizontal 3-cell (H3) and 2-cell (H2, centre excluded) bit-sliced sums
//     once, and emits the previous row as H3(r-1) + H2(r) + H3(r+1) -> rule.
//     Stage g consumes the row stage g-1 emitted in the same step.  Each input
//     row is read once from HBM and each output row written once per K
//     generations: HBM bytes per cell-generation = 0.25 / K (x halo overhead).
//   * Field rows outside [0, field_h) are dead (Parallel_Life_MPI.cpp:21-22) and
//     columns >= w are dead (:26-27): masked on load and -- for rules that can
//     give birth -- re-masked after every generation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "bitlayout.h"
#include "life_internal.h"
#include "loop_place.h"

#ifndef GOL_WARM_ROLLED
#define GOL_WARM_ROLLED 0
#endif

namespace gol {

namespace {

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
constexpr uint32_t kRefEmit = 0x20;   // a & ~b & c
constexpr uint32_t kConwayEmit = 0xE0;// a & (b | c)

template <int RULE>
__device__ __forceinline__ uint32_t rule32(uint32_t as, uint32_t ac, uint32_t bs, uint32_t bc,
                                           uint32_t es, uint32_t ec, uint32_t alive,
                                           uint32_t birth, uint32_t survive)
{
    // n = A + B + E with A = H3(r-2), B = H2(r-1), E = H3(r): each a 2-bit number.
    const uint32_t s0 = lop3<kXor3>(as, bs, es);  // bit 0 of n
    const uint32_t k0 = lop3<kMaj>(as, bs, es);   // carry into weight 2
    const uint32_t p = lop3<kXor3>(ac, bc, ec);   // weight-2 column sum, bit 0
    const uint32_t mj = lop3<kMaj>(ac, bc, ec);   // weight-2 column sum, carry
    // n = s0 + 2*(p + k0) + 4*mj;  n in {2,3}  <=>  mj == 0 && p + k0 == 1
    if constexpr (RULE == RULE_REF) {
        // Parallel_Life_MPI.cpp:47-50: next = alive && n == 2
        return lop3<kRefEmit>(alive, s0, lop3<kTwoThree>(p, k0, mj));
    } else if constexpr (RULE == RULE_CONWAY) {
        return lop3<kConwayEmit>(lop3<kTwoThree>(p, k0, mj), s0, alive);
    } else {
        const uint32_t n1 = p ^ k0;
        const uint32_t k1 = p & k0;
        const uint32_t n2 = mj ^ k1;
        const uint32_t n3 = mj & k1;
        uint32_t r = 0;
#pragma unroll
        for (int n = 0; n <= 8; ++n) {
            const uint32_t bsel = (birth >> n) & 1u, ssel = (survive >> n) & 1u;
            if (bsel | ssel) {
                const uint32_t eq = ((n & 1) ? s0 : ~s0) & ((n & 2) ? n1 : ~n1) &
                                    ((n & 4) ? n2 : ~n2) & ((n & 8) ? n3 : ~n3);
                const uint32_t sel = (ssel ? alive : 0u) | (bsel ? ~alive : 0u);
                r |= eq & sel;
            }
        }
        return r;
    }
}

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

// Per-generation pipeline stage state, neighbour-sum form (kernel variant 1):
// H3 (3-cell horizontal sum, bit-sliced sum + carry) of rows r-2 and r-1, H2
// (centre excluded) and the cells of row r-1, where r is the incoming row.
template <int NP>
struct Stage {
    Pl<NP> ps, pc;
    Pl<NP> cs, cc;
    Pl<NP> hs, hc;
    Pl<NP> al;
};

// One stage step: ingest row r (x, generation g-1), emit row r-1 at generation g.
template <int RULE, int NP>
__device__ __forceinline__ Pl<NP> stage_step(Stage<NP>& st, const Pl<NP>& x, uint32_t birth,
                                             uint32_t survive)
{
    const Ends e = ends(x);
    Pl<NP> s2, c2, s3, c3, y;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint32_t L = left_of(x, e, k), R = right_of(x, e, k);
        s2.v[k] = L ^ R;
        c2.v[k] = L & R;
        s3.v[k] = lop3<kXor3>(L, x.v[k], R);
        c3.v[k] = lop3<kMaj>(L, x.v[k], R);
        y.v[k] = rule32<RULE>(st.ps.v[k], st.pc.v[k], st.hs.v[k], st.hc.v[k], s3.v[k], c3.v[k],
                              st.al.v[k], birth, survive);
    }
    st.ps = st.cs;
    st.pc = st.cc;
    st.cs = s3;
    st.cc = c3;
    st.hs = s2;
    st.hc = c2;
    st.al = x;
    return y;
}

// Total-sum stage state (5 planes per fused generation): H3 of rows r-2 and r-1
// and the cells of row r-1.  The emitted cell sees T = H3(r-2) + H3(r-1) + H3(r),
// the 9-cell sum including itself, so no centre-excluded H2 is formed: 4 VALU
// ops and 2 planes per stage fewer than Stage.  For an alive cell T = n + 1, for
// a dead one T = n (generic masks: survive bit T-1 / birth bit T); the two fixed
// rules read it off directly:
//   REF (B/S2):      next = alive && T == 3
//   CONWAY (B3/S23): next = T == 3 || (alive && T == 4)
template <int NP>
struct StageT {
    Pl<NP> ps, pc;
    Pl<NP> cs, cc;
    Pl<NP> al;
};
constexpr uint32_t kAnd3 = 0x80;     // a & b & c
constexpr uint32_t kFour = 0x42;     // ~(a ^ b) & (a ^ c)
constexpr uint32_t kAndNot = 0x40;   // a & b & ~c
constexpr uint32_t kOrAnd2 = 0xEA;   // (a & b) | c

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
        // T == 4  <=>  !s0 && (p + k0 == 2 && !mj  ||  p + k0 == 0 && mj); all
        // three steps are v_bitop3 (8-byte encodings, see loop_place.h)
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

template <int RULE, int NP>
__device__ __forceinline__ Pl<NP> stage_step(StageT<NP>& st, const Pl<NP>& x, uint32_t birth,
                                             uint32_t survive)
{
    const Ends e = ends(x);
    Pl<NP> s3, c3, y;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint32_t L = left_of(x, e, k), R = right_of(x, e, k);
        s3.v[k] = lop3<kXor3>(L, x.v[k], R);
        c3.v[k] = lop3<kMaj>(L, x.v[k], R);
        y.v[k] = rule32_total<RULE>(st.ps.v[k], st.pc.v[k], st.cs.v[k], st.cc.v[k], s3.v[k],
                                    c3.v[k], st.al.v[k], birth, survive);
    }
    st.ps = st.cs;
    st.pc = st.cc;
    st.cs = s3;
    st.cc = c3;
    st.al = x;
    return y;
}

// VAR: 0 = total-sum state, anti-diagonal schedule; 1 = neighbour-sum state,
// anti-diagonal; 2 = as 0 with the plain step-major schedule.
template <int VAR, int NP>
struct StageOf {
    using type = typename std::conditional<VAR != 1, StageT<NP>, Stage<NP>>::type;
};

// Steps per block (rows prefetched ahead through the register ring): 8 for the
// 2-plane kernels of depth >= 16, whose 2 waves/SIMD have VGPRs to spare (203 ->
// 230), 4 elsewhere.  In-process A/B at K = 16, 2 planes: +2.5% at 65536^2
// (129.0 vs 125.8 TCUPS), +0.3% at 8448 rows (profiles/r01/ab_prefetch_depth.jsonl).
// GOL_PF_NP2 overrides it for dev A/B builds.
template <int NP, int K>
constexpr int kPfOf()
{
#ifdef GOL_PF_NP2
    return NP == 2 ? GOL_PF_NP2 : 4;
#else
    return (NP == 2 && K >= 16) ? 8 : 4;
#endif
}
#ifndef GOL_DEV_FLIP_PAD  // dev A/B builds: invert loop_place.h's pads
#define GOL_DEV_FLIP_PAD 0
#endif

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

template <int K, int RULE, int VAR, int NP>
__global__ __launch_bounds__(256) void life_tb_kernel(StepArgs a)
{
    constexpr bool kDiagonal = VAR != 2;
    constexpr bool kBirths = RULE != RULE_REF;
    constexpr int G = NP / 2;  // words per lane group
    constexpr int kPrefetch = kPfOf<NP, K>();
    static_assert(K + 2 * kPrefetch <= kGuardRows, "streaming loads must stay in the guard rows");
    const int lane = threadIdx.x & 63;
    const int64_t unit =
        (int64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (unit >= a.total_units) return;

    int sidx = 0;
    for (int j = 1; j < a.nseg; ++j)
        if (unit >= a.segs[j].unit0) sidx = j;
    const SegDesc sg = a.segs[sidx];
    const int64_t u = unit - sg.unit0;
    const int64_t blk = u / a.strips;
    // strip `strip` of the row block lives in lanes [sub*L, sub*L + L); the DPP
    // shifts cross from one strip into the next only at halo lanes
#ifdef GOL_DEV_FULL_STRIPS
    constexpr int L = 64, lshift = 0;
#else
    const int lshift = a.lane_shift;
    const int L = 64 >> lshift;
#endif
    const int sub = lane >> (6 - lshift);
    const int lin = lane & (L - 1);
    const int strip = (int)(u % a.strips) * (1 << lshift) + sub;

    // lane group of this lane; its column mask (columns >= w are dead)
    const int64_t q = (int64_t)strip * (L - 2) - 1 + lin;
    const bool qin = (q >= 0) && (q < a.ng);
    Pl<NP> cm;
#pragma unroll
    for (int k = 0; k < NP; ++k)
        cm.v[k] = qin ? ((q == a.ng - 1) ? (uint32_t)(a.lastmask[k / 2] >> (32 * (k & 1))) : ~0u)
                      : 0u;
    const int64_t qc = qin ? q : 0;

    const int64_t rb = sg.out_lo + blk * a.rows_per_wave;
    const int64_t re = min(rb + a.rows_per_wave, sg.out_hi);
    const int64_t T = (re - rb) + 2 * K;  // input rows streamed
    const int64_t row_first = rb - K;     // local row of step 0

    const uint64_t* inp = a.in + (sg.base_row + row_first) * a.stride + qc * G;
    uint64_t* outp = a.out + (sg.base_row + rb) * a.stride + qc * G;
    const bool st_lane = qin && lin >= 1 && lin <= L - 2;

    // field-row validity of local row i (dead border) and buffer-row validity
    const int64_t lo_ok = max((int64_t)0, -sg.glob0);             // first local row in field
    const int64_t hi_ok = min(sg.in_rows, sg.field_h - sg.glob0);  // one past last

    typename StageOf<VAR, NP>::type st[K];
#pragma unroll
    for (int g = 0; g < K; ++g) st[g] = {};

    Grp<NP> ring[kPrefetch];
#pragma unroll
    for (int p = 0; p < kPrefetch; ++p)
        ring[p] = *reinterpret_cast<const Grp<NP>*>(inp + (int64_t)p * a.stride);
    const uint64_t* pf = inp + (int64_t)kPrefetch * a.stride;

    // input row of step t: dead outside the field / buffer, columns >= w masked
    auto ingest = [&](int64_t t, const Grp<NP>& xv) -> Pl<NP> {
        const int64_t i = row_first + t;
        const bool ok = (i >= lo_ok) && (i < hi_ok);
        Pl<NP> x = planes_of(xv);
#pragma unroll
        for (int k = 0; k < NP; ++k) x.v[k] = ok ? (x.v[k] & cm.v[k]) : 0u;
        return x;
    };
    // stage g (generation g+1) at step t: emits local row row_first + t - (g+1)
    auto stage = [&](int g, int64_t t, Pl<NP> x) -> Pl<NP> {
        x = stage_step<RULE>(st[g], x, a.birth, a.survive);
        if constexpr (kBirths) {
            const int64_t r = sg.glob0 + row_first + t - (g + 1);  // field row
            const bool rok = (r >= 0) && (r < sg.field_h);
#pragma unroll
            for (int k = 0; k < NP; ++k) x.v[k] = rok ? (x.v[k] & cm.v[k]) : 0u;
        }
        return x;
    };
    auto store = [&](int64_t t, const Pl<NP>& x) {
        if (t >= 2 * K && t < T && st_lane)
            *reinterpret_cast<Grp<NP>*>(outp + (t - 2 * K) * a.stride) = words_of(x);
    };

    // One block of kPrefetch steps.  GUARD (warm-up blocks): stage g first emits a
    // row that can reach a valid output at step 2g+2 and needs the two ingests
    // before it, so it only runs from step 2g on; skipping it earlier saves
    // K*(K-1) of the 2K*K warm-up stage-steps.  The guard is wave-uniform (a
    // scalar branch per stage-step).
    auto block = [&](int64_t t0, auto guard) {
        constexpr bool kGuard = decltype(guard)::value;
        Pl<NP> x[kPrefetch];
#pragma unroll
        for (int p = 0; p < kPrefetch; ++p) {
            x[p] = ingest(t0 + p, ring[p]);
            ring[p] = *reinterpret_cast<const Grp<NP>*>(pf);
            pf += a.stride;
        }
        // Code placement (steady-state blocks).  gfx950 issues this kernel's
        // instruction mix (DPP move, v_alignbit, v_bitop3 chains; all 8-byte
        // encodings) 10-25% faster when those instructions sit at addresses =
        // 4 mod 8 with 2+ waves per SIMD, and faster at 0 mod 8 with one
        // (tools/valu_rate.hip "mix_at_*"; in the kernel: identical code and
        // registers, 89.6 vs 79.9 TCUPS, profiles/r01/loop_alignment_ab.jsonl).
        // The scheduling barriers keep the 4-byte encodings (loads, ingest masks,
        // SALU, stores) out of the compute, so one alignment directive places
        // all of it: the block's inputs pass through the directive, so the
        // compute that depends on them cannot be scheduled above it; "memory"
        // keeps the loads above and the stores below.  The compiler may add a
        // hazard s_nop after it, so the 4-byte pad that gives the wanted parity
        // is per kernel: loop_place.h, generated by tools/loop_align.py.
        if constexpr (!kGuard) {
            __builtin_amdgcn_sched_barrier(0);
            place_block<(life_loop_pad(K, RULE, VAR, NP) != 0) != (GOL_DEV_FLIP_PAD != 0), NP, kPrefetch>(x);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (kDiagonal) {
            // stage g of step p only needs stage g-1 of step p and stage g of step
            // p-1: issue the block's (p, g) pairs by anti-diagonal d = p + g so
            // independent stage steps sit next to each other for the scheduler
#pragma unroll
            for (int d = 0; d < K + kPrefetch - 1; ++d) {
#pragma unroll
                for (int p = 0; p < kPrefetch; ++p) {
                    const int g = d - p;
                    if (g >= 0 && g < K && (!kGuard || t0 + p >= 2 * g))
                        x[p] = stage(g, t0 + p, x[p]);
                }
            }
        } else {
#pragma unroll
            for (int p = 0; p < kPrefetch; ++p) {
#pragma unroll
                for (int g = 0; g < K; ++g)
                    if (!kGuard || t0 + p >= 2 * g) x[p] = stage(g, t0 + p, x[p]);
            }
        }
        if constexpr (!kGuard) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < kPrefetch; ++p) store(t0 + p, x[p]);
    };

    // Warm-up blocks as a rolled loop: unrolled, they would be ~4x the code of
    // the steady-state body and push the kernel past the instruction cache.
    constexpr int kWarm = (2 * K + kPrefetch - 1) / kPrefetch * kPrefetch;
#if GOL_WARM_ROLLED
#pragma clang loop unroll(disable)
    for (int64_t t0 = 0; t0 < kWarm; t0 += kPrefetch) block(t0, std::true_type{});
#else
#pragma unroll
    for (int t0 = 0; t0 < kWarm; t0 += kPrefetch) block(t0, std::true_type{});
#endif
    for (int64_t t0 = kWarm; t0 < T; t0 += kPrefetch) block(t0, std::false_type{});
}

// Instantiated stencil kernels: 2 planes per lane group at every depth (the
// neighbour-sum state up to 16); 4 planes up to depth 16 (neighbour-sum up to 8),
// where 5 planes x 4 x K state words still fit the register file.
constexpr bool has_kernel(int K, int VAR, int NP)
{
    return NP == 2 ? (VAR != 1 || K <= 16) : (K <= 16 && (VAR != 1 || K <= 8));
}

template <int K, int VAR, int NP>
hipError_t launch_depth(const StepArgs& a, RuleKind rule, hipStream_t s)
{
    if constexpr (!has_kernel(K, VAR, NP)) {
        return hipErrorInvalidValue;
    } else {
        const dim3 grid((unsigned)((a.total_units + kWavesPerBlock - 1) / kWavesPerBlock));
        const dim3 block(64 * kWavesPerBlock);
        switch (rule) {
        case RULE_REF:
            hipLaunchKernelGGL((life_tb_kernel<K, RULE_REF, VAR, NP>), grid, block, 0, s, a);
            break;
        case RULE_CONWAY:
            hipLaunchKernelGGL((life_tb_kernel<K, RULE_CONWAY, VAR, NP>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((life_tb_kernel<K, RULE_GENERIC, VAR, NP>), grid, block, 0, s, a);
            break;
        }
        return hipGetLastError();
    }
}

template <int K, int NP>
hipError_t launch_variant(const StepArgs& a, RuleKind rule, int var, hipStream_t s)
{
    switch (var) {
    case 1: return launch_depth<K, 1, NP>(a, rule, s);
    case 2: return launch_depth<K, 2, NP>(a, rule, s);
    default: return launch_depth<K, 0, NP>(a, rule, s);
    }
}

template <int K>
hipError_t launch_planes(const StepArgs& a, RuleKind rule, int var, int planes, hipStream_t s)
{
    return planes == 4 ? launch_variant<K, 4>(a, rule, var, s) : launch_variant<K, 2>(a, rule, var, s);
}

template <int K, int VAR, int NP>
int occupancy_of(RuleKind rule)
{
    if constexpr (!has_kernel(K, VAR, NP)) {
        return 0;
    } else {
        int blocks = 0;
        hipError_t e = hipErrorInvalidValue;
        const int threads = 64 * kWavesPerBlock;
        if (rule == RULE_REF)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &blocks, life_tb_kernel<K, RULE_REF, VAR, NP>, threads, 0);
        else if (rule == RULE_CONWAY)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &blocks, life_tb_kernel<K, RULE_CONWAY, VAR, NP>, threads, 0);
        else
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &blocks, life_tb_kernel<K, RULE_GENERIC, VAR, NP>, threads, 0);
        return e == hipSuccess ? blocks : 0;
    }
}

template <int K>
int occupancy_planes(RuleKind rule, int var, int planes)
{
    if (planes == 4) {
        switch (var) {
        case 1: return occupancy_of<K, 1, 4>(rule);
        case 2: return occupancy_of<K, 2, 4>(rule);
        default: return occupancy_of<K, 0, 4>(rule);
        }
    }
    switch (var) {
    case 1: return occupancy_of<K, 1, 2>(rule);
    case 2: return occupancy_of<K, 2, 2>(rule);
    default: return occupancy_of<K, 0, 2>(rule);
    }
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Memory-bound helpers below work per lane group of NP planes (NP/2 words,
// bitlayout.h); the canonical word index r*wq + c is what the synthetic field
// and the digest are defined on (gol.h), so they match the oracle's.

template <int NP>
__global__ __launch_bounds__(256) void init_random_kernel(uint64_t* buf, int64_t stride,
                                                          int64_t wq, uint64_t lastmask,
                                                          int64_t row_base, int64_t glob_row0,
                                                          int64_t nrows, uint64_t seed)
{
    constexpr int G = NP / 2;
    const int64_t gpr = stride / G;  // lane groups per buffer row
    const int64_t total = nrows * gpr;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / gpr, gq = k - i * gpr;
        uint64_t c[2] = {0, 0}, s[2];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t idx = gq * G + j;
            if (idx < wq) {
                c[j] = splitmix64_at(seed, (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)idx);
                if (idx == wq - 1) c[j] &= lastmask;  // canonical mask
            }
        }
        gol_split_group(c, s, NP);
#pragma unroll
        for (int j = 0; j < G; ++j) buf[(row_base + i) * stride + gq * G + j] = s[j];
    }
}

template <int NP>
__global__ __launch_bounds__(256) void digest_kernel(const uint64_t* buf, int64_t stride,
                                                     int64_t wq, int64_t ng, int64_t row_base,
                                                     int64_t glob_row0, int64_t nrows,
                                                     unsigned long long* acc)
{
    constexpr int G = NP / 2;
    const int64_t total = nrows * ng;
    uint64_t live = 0, hash = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / ng, gq = k - i * ng;
        uint64_t s[2] = {0, 0}, c[2];
#pragma unroll
        for (int j = 0; j < G; ++j) s[j] = buf[(row_base + i) * stride + gq * G + j];
        gol_join_group(s, c, NP);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t idx = gq * G + j;
            if (idx < wq) {
                live += (uint64_t)__popcll(c[j]);
                const uint64_t h = (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)idx;
                hash += splitmix64_at(c[j] ^ splitmix64_at(0, h), 0);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        live += __shfl_xor(live, off);
        hash += __shfl_xor(hash, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], (unsigned long long)live);
        atomicAdd(&acc[1], (unsigned long long)hash);
    }
}

// ASCII codec (data.txt / output.txt bytes <-> stored lane groups), the
// device-side replacement of readGridFromFile's parse (:91-99) and
// writeDataToFile's serialisation (:157-164).  One wavefront per (row, lane
// group): lane j reads the byte of column 64c+j of each of the group's words
// (coalesced), __ballot forms the canonical words, lane 0 stores the group.
// Byte w of every row must be '\n'.
template <int NP>
__global__ __launch_bounds__(256) void ascii_pack_kernel(const char* src, int64_t rows, int64_t w,
                                                         int64_t ng, uint64_t* dst,
                                                         int64_t stride, int* bad)
{
    constexpr int G = NP / 2;
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * ng;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / ng, gq = k - r * ng;
        const char* line = src + r * (w + 1);
        uint64_t c[2] = {0, 0}, s[2];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t col = (gq * G + j) * 64 + lane;
            c[j] = __ballot(col < w && line[col] == '1');
        }
        if (lane == 0) {
            gol_split_group(c, s, NP);
#pragma unroll
            for (int j = 0; j < G; ++j) dst[r * stride + gq * G + j] = s[j];
            if (gq == ng - 1 && line[w] != '\n') atomicOr(bad, 1);
        }
    }
}

template <int NP>
__global__ __launch_bounds__(256) void ascii_unpack_kernel(const uint64_t* src, int64_t stride,
                                                           int64_t rows, int64_t w, int64_t ng,
                                                           char* dst)
{
    constexpr int G = NP / 2;
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * ng;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / ng, gq = k - r * ng;
        uint64_t s[2] = {0, 0}, c[2];
#pragma unroll
        for (int j = 0; j < G; ++j) s[j] = src[r * stride + gq * G + j];
        gol_join_group(s, c, NP);
        char* line = dst + r * (w + 1);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t col = (gq * G + j) * 64 + lane;
            if (col < w) line[col] = ((c[j] >> lane) & 1) ? '1' : '0';
        }
        if (gq == ng - 1 && lane == 0) line[w] = '\n';
    }
}

}  // namespace

hipError_t launch_life(const StepArgs& a, int depth, RuleKind rule, int var, int planes,
                       hipStream_t s)
{
    if (a.total_units <= 0) return hipSuccess;
#ifdef GOL_DEV_ONLY_DEPTH  // dev A/B builds: one depth only (fast compile)
    if (depth != GOL_DEV_ONLY_DEPTH) return hipErrorInvalidValue;
    return launch_planes<GOL_DEV_ONLY_DEPTH>(a, rule, var, planes, s);
#else
    switch (depth) {
    case 1: return launch_planes<1>(a, rule, var, planes, s);
    case 2: return launch_planes<2>(a, rule, var, planes, s);
    case 4: return launch_planes<4>(a, rule, var, planes, s);
    case 6: return launch_planes<6>(a, rule, var, planes, s);
    case 7: return launch_planes<7>(a, rule, var, planes, s);
    case 8: return launch_planes<8>(a, rule, var, planes, s);
    case 12: return launch_planes<12>(a, rule, var, planes, s);
    case 16: return launch_planes<16>(a, rule, var, planes, s);
    case 20: return launch_planes<20>(a, rule, var, planes, s);
    case 24: return launch_planes<24>(a, rule, var, planes, s);
    case 32: return launch_planes<32>(a, rule, var, planes, s);
    default: return hipErrorInvalidValue;
    }
#endif
}

int life_blocks_per_cu(int depth, RuleKind rule, int var, int planes)
{
#ifdef GOL_DEV_ONLY_DEPTH
    return depth == GOL_DEV_ONLY_DEPTH ? occupancy_planes<GOL_DEV_ONLY_DEPTH>(rule, var, planes)
                                       : 0;
#else
    switch (depth) {
    case 1: return occupancy_planes<1>(rule, var, planes);
    case 2: return occupancy_planes<2>(rule, var, planes);
    case 4: return occupancy_planes<4>(rule, var, planes);
    case 6: return occupancy_planes<6>(rule, var, planes);
    case 7: return occupancy_planes<7>(rule, var, planes);
    case 8: return occupancy_planes<8>(rule, var, planes);
    case 12: return occupancy_planes<12>(rule, var, planes);
    case 16: return occupancy_planes<16>(rule, var, planes);
    case 20: return occupancy_planes<20>(rule, var, planes);
    case 24: return occupancy_planes<24>(rule, var, planes);
    case 32: return occupancy_planes<32>(rule, var, planes);
    default: return 0;
    }
#endif
}

bool life_has_kernel(int depth, int var, int planes) { return has_kernel(depth, var, planes); }

static dim3 grid_for(int64_t items, int64_t per_block, int64_t cap)
{
    int64_t blocks = (items + per_block - 1) / per_block;
    if (blocks > cap) blocks = cap;
    return dim3((unsigned)blocks);
}

hipError_t launch_init_random(uint64_t* buf, int64_t stride, int64_t wq, uint64_t lastmask,
                              int64_t row_base, int64_t glob_row0, int64_t nrows, uint64_t seed,
                              int planes, hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const dim3 grid = grid_for(nrows * stride / (planes / 2), 256, 8192);
    if (planes == 4)
        hipLaunchKernelGGL(init_random_kernel<4>, grid, dim3(256), 0, s, buf, stride, wq, lastmask,
                           row_base, glob_row0, nrows, seed);
    else
        hipLaunchKernelGGL(init_random_kernel<2>, grid, dim3(256), 0, s, buf, stride, wq, lastmask,
                           row_base, glob_row0, nrows, seed);
    return hipGetLastError();
}

hipError_t launch_ascii_pack(const char* src, int64_t rows, int64_t w, int64_t ng, uint64_t* dst,
                             int64_t stride, int* bad, int planes, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    const dim3 grid = grid_for(rows * ng, 4, 16384);
    if (planes == 4)
        hipLaunchKernelGGL(ascii_pack_kernel<4>, grid, dim3(256), 0, s, src, rows, w, ng, dst,
                           stride, bad);
    else
        hipLaunchKernelGGL(ascii_pack_kernel<2>, grid, dim3(256), 0, s, src, rows, w, ng, dst,
                           stride, bad);
    return hipGetLastError();
}

hipError_t launch_ascii_unpack(const uint64_t* src, int64_t stride, int64_t rows, int64_t w,
                               int64_t ng, char* dst, int planes, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    const dim3 grid = grid_for(rows * ng, 4, 16384);
    if (planes == 4)
        hipLaunchKernelGGL(ascii_unpack_kernel<4>, grid, dim3(256), 0, s, src, stride, rows, w, ng,
                           dst);
    else
        hipLaunchKernelGGL(ascii_unpack_kernel<2>, grid, dim3(256), 0, s, src, stride, rows, w, ng,
                           dst);
    return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* buf, int64_t stride, int64_t wq, int64_t ng,
                         int64_t row_base, int64_t glob_row0, int64_t nrows,
                         unsigned long long* acc, int planes, hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const dim3 grid = grid_for(nrows * ng, 256, 8192);
    if (planes == 4)
        hipLaunchKernelGGL(digest_kernel<4>, grid, dim3(256), 0, s, buf, stride, wq, ng, row_base,
                           glob_row0, nrows, acc);
    else
        hipLaunchKernelGGL(digest_kernel<2>, grid, dim3(256), 0, s, buf, stride, wq, ng, row_base,
                           glob_row0, nrows, acc);
    return hipGetLastError();
}

}  // namespace gol
