// life_kernels.hip -- gfx950 kernels of the Game of Life engine.
//
// Hot path: the per-generation update of Parallel_Life_MPI.cpp (countNeighbours
// :16-35 + updateGrid :37-54), restated on a bit-packed field (64 cells per
// uint64, bit j of word q = column 64q+j) and fused over K generations per
// launch (temporal blocking).
//
// Kernel shape (one wavefront = one work unit, no LDS, no barriers):
//   * A wavefront owns a strip of 64 consecutive words of a row (lane l holds
//     word strip*62 - 1 + l); lanes 0 and 63 are the horizontal halo, so each
//     strip outputs 62 words.  Words are column-split (bitlayout.h: even columns
//     in the low dword, odd in the high), so two of the four horizontal
//     neighbour planes are free; the other two are one v_alignbit each, with the
//     carry bit from the adjacent lane by a DPP wave shift (wave_shr:1 /
//     wave_shl:1).  After g fused generations the contamination from the unknown
//     words beyond the halo lanes has moved g bits into lanes 0/63, so K <= 63
//     keeps lanes 1..62 exact.
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
#ifndef GOL_HORIZ_BPERM
#define GOL_HORIZ_BPERM 0
#endif
#ifndef GOL_HORIZ_ADDC
#define GOL_HORIZ_ADDC 0
#endif
#ifndef GOL_HORIZ_OR_DPP
#define GOL_HORIZ_OR_DPP 0
#endif

namespace gol {

namespace {

struct u2 {
    uint32_t lo, hi;
};

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

// Per-generation pipeline stage state (all bit-sliced, two 32-bit halves):
//   H3 of row r-2 (sum, carry), H3 of row r-1, H2 of row r-1, cells of row r-1,
// where r is the incoming row.
struct Stage {
    u2 ps, pc;
    u2 cs, cc;
    u2 hs, hc;
    u2 al;
};

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

// Horizontal neighbour planes of a column-split word x (bitlayout.h): lo = even
// columns, hi = odd columns.  An even column's right neighbour and an odd
// column's left neighbour are the other half at the same bit; the remaining two
// planes take one funnel shift each, with the carry bit from the adjacent lane.
struct Horiz {
    uint32_t Le, Ro;  // left of the even columns, right of the odd columns
};
__device__ __forceinline__ Horiz horiz(u2 x)
{
#if GOL_HORIZ_BPERM
    // neighbour lanes through the LDS crossbar (ds_bpermute) instead of DPP moves,
    // which issue on the VALU at half rate; byte address of lane l-1 / l+1
    const int lane4 = (int)__lane_id() * 4;
    const uint32_t hp = (uint32_t)__builtin_amdgcn_ds_bpermute(lane4 - 4, (int)x.hi);
#if GOL_HORIZ_BPERM == 2  // one direction each way: LDS crossbar and DPP
    const uint32_t ln = lane_from_right(x.lo);
#else
    const uint32_t ln = (uint32_t)__builtin_amdgcn_ds_bpermute(lane4 + 4, (int)x.lo);
#endif
    Horiz h;
    h.Le = __builtin_amdgcn_alignbit(x.hi, hp, 31);
    h.Ro = __builtin_amdgcn_alignbit(ln, x.lo, 1);
    return h;
#elif GOL_HORIZ_ADDC
    // left shift with the carry from lane l-1 as an add-with-carry: the carries of
    // all lanes are one wave mask (v_cmp), moved up one lane on the scalar unit
    const uint64_t m = __builtin_amdgcn_ballot_w64((int32_t)x.hi < 0) << 1;
    uint32_t le;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(le), "=s"(co) : "v"(x.hi), "s"(m));
    const uint32_t ln = lane_from_right(x.lo);
    Horiz h;
    h.Le = le;
    h.Ro = __builtin_amdgcn_alignbit(ln, x.lo, 1);
    return h;
#elif GOL_HORIZ_OR_DPP
    // the carry bit is shifted into place in the neighbour lane and merged by a
    // v_or_b32 whose src0 reads it through DPP (the mov folds into the or)
    // (the shifts are opaque asm so the compiler cannot commute them with the lane
    // move and form a half-rate v_lshl_or_b32 instead)
    uint32_t th, tl, sh, sl;
    asm("v_lshrrev_b32 %0, 31, %1" : "=v"(th) : "v"(x.hi));
    asm("v_lshlrev_b32 %0, 31, %1" : "=v"(tl) : "v"(x.lo));
    asm("v_lshlrev_b32 %0, 1, %1" : "=v"(sh) : "v"(x.hi));
    asm("v_lshrrev_b32 %0, 1, %1" : "=v"(sl) : "v"(x.lo));
    Horiz h;
    h.Le = sh | lane_from_left(th);
    h.Ro = sl | lane_from_right(tl);
    return h;
#else
    const uint32_t hp = lane_from_left(x.hi);   // odd columns of word q-1 (bit 31: col 64q-1)
    const uint32_t ln = lane_from_right(x.lo);  // even columns of word q+1 (bit 0: col 64q+64)
    Horiz h;
    h.Le = __builtin_amdgcn_alignbit(x.hi, hp, 31);  // (hi << 1) | (hp >> 31)
    h.Ro = __builtin_amdgcn_alignbit(ln, x.lo, 1);   // (lo >> 1) | (ln << 31)
    return h;
#endif
}

// One stage step: ingest row r (x, generation g-1), emit row r-1 at generation g.
template <int RULE>
__device__ __forceinline__ u2 stage_step(Stage& st, u2 x, uint32_t birth, uint32_t survive)
{
    const Horiz hz = horiz(x);
    // even half: (L, C, R) = (Le, lo, hi); odd half: (lo, hi, Ro)
    u2 s2, c2, s3, c3;
    s2.lo = hz.Le ^ x.hi;
    c2.lo = hz.Le & x.hi;
    s3.lo = lop3<kXor3>(hz.Le, x.lo, x.hi);
    c3.lo = lop3<kMaj>(hz.Le, x.lo, x.hi);
    s2.hi = x.lo ^ hz.Ro;
    c2.hi = x.lo & hz.Ro;
    s3.hi = lop3<kXor3>(x.lo, x.hi, hz.Ro);
    c3.hi = lop3<kMaj>(x.lo, x.hi, hz.Ro);
    u2 y;
    y.lo = rule32<RULE>(st.ps.lo, st.pc.lo, st.hs.lo, st.hc.lo, s3.lo, c3.lo, st.al.lo, birth,
                        survive);
    y.hi = rule32<RULE>(st.ps.hi, st.pc.hi, st.hs.hi, st.hc.hi, s3.hi, c3.hi, st.al.hi, birth,
                        survive);
    st.ps = st.cs;
    st.pc = st.cc;
    st.cs = s3;
    st.cc = c3;
    st.hs = s2;
    st.hc = c2;
    st.al = x;
    return y;
}

// Total-sum stage state (10 dwords): H3 of rows r-2 and r-1 and the cells of row
// r-1.  The emitted cell sees T = H3(r-2) + H3(r-1) + H3(r), the 9-cell sum
// including itself, so no centre-excluded H2 is formed: 4 VALU ops per word and
// 4 VGPRs per stage fewer than Stage.  For an alive cell T = n + 1, for a dead
// one T = n (generic masks: survive bit T-1 / birth bit T); the two fixed rules
// read it off directly:
//   REF (B/S2):      next = alive && T == 3
//   CONWAY (B3/S23): next = T == 3 || (alive && T == 4)
struct StageT {
    u2 ps, pc;
    u2 cs, cc;
    u2 al;
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
        // three steps are v_bitop3 (8-byte encodings, see loop_pad.h)
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

template <int RULE>
__device__ __forceinline__ u2 stage_step(StageT& st, u2 x, uint32_t birth, uint32_t survive)
{
    const Horiz hz = horiz(x);
    u2 s3, c3;
    s3.lo = lop3<kXor3>(hz.Le, x.lo, x.hi);
    c3.lo = lop3<kMaj>(hz.Le, x.lo, x.hi);
    s3.hi = lop3<kXor3>(x.lo, x.hi, hz.Ro);
    c3.hi = lop3<kMaj>(x.lo, x.hi, hz.Ro);
    u2 y;
    y.lo = rule32_total<RULE>(st.ps.lo, st.pc.lo, st.cs.lo, st.cc.lo, s3.lo, c3.lo, st.al.lo,
                                  birth, survive);
    y.hi = rule32_total<RULE>(st.ps.hi, st.pc.hi, st.cs.hi, st.cc.hi, s3.hi, c3.hi, st.al.hi,
                                  birth, survive);
    st.ps = st.cs;
    st.pc = st.cc;
    st.cs = s3;
    st.cc = c3;
    st.al = x;
    return y;
}

// VAR: 0 = total-sum state, anti-diagonal schedule; 1 = neighbour-sum state,
// anti-diagonal; 2 = as 0 with the plain step-major schedule.
template <int RULE, int VAR>
struct StageOf {
    using type = typename std::conditional<VAR != 1, StageT, Stage>::type;
};

constexpr int kPrefetch = 4;


template <int K, int RULE, int VAR>
__global__ __launch_bounds__(256) void life_tb_kernel(StepArgs a)
{
    constexpr bool kDiagonal = VAR != 2;
    constexpr bool kBirths = RULE != RULE_REF;
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

    const int64_t q = (int64_t)strip * (L - 2) - 1 + lin;
    const bool qin = (q >= 0) && (q < a.wq);
    const uint64_t cm = qin ? ((q == a.wq - 1) ? a.lastmask : ~0ull) : 0ull;
    const uint32_t cmlo = (uint32_t)cm, cmhi = (uint32_t)(cm >> 32);
    const int64_t qc = qin ? q : 0;

    const int64_t rb = sg.out_lo + blk * a.rows_per_wave;
    const int64_t re = min(rb + a.rows_per_wave, sg.out_hi);
    const int64_t T = (re - rb) + 2 * K;  // input rows streamed
    const int64_t row_first = rb - K;     // local row of step 0

    const uint64_t* inp = a.in + (sg.base_row + row_first) * a.stride + qc;
    uint64_t* outp = a.out + (sg.base_row + rb) * a.stride + qc;
    const bool st_lane = qin && lin >= 1 && lin <= L - 2;

    // field-row validity of local row i (dead border) and buffer-row validity
    const int64_t lo_ok = max((int64_t)0, -sg.glob0);             // first local row in field
    const int64_t hi_ok = min(sg.in_rows, sg.field_h - sg.glob0);  // one past last

    typename StageOf<RULE, VAR>::type st[K];
#pragma unroll
    for (int g = 0; g < K; ++g) st[g] = {};

    uint64_t ring[kPrefetch];
#pragma unroll
    for (int p = 0; p < kPrefetch; ++p) ring[p] = inp[(int64_t)p * a.stride];
    const uint64_t* pf = inp + (int64_t)kPrefetch * a.stride;

    // input row of step t: dead outside the field / buffer, columns >= w masked
    auto ingest = [&](int64_t t, uint64_t xv) -> u2 {
        const int64_t i = row_first + t;
        const bool ok = (i >= lo_ok) && (i < hi_ok);
        u2 x;
        x.lo = ok ? ((uint32_t)xv & cmlo) : 0u;
        x.hi = ok ? ((uint32_t)(xv >> 32) & cmhi) : 0u;
        return x;
    };
    // stage g (generation g+1) at step t: emits local row row_first + t - (g+1)
    auto stage = [&](int g, int64_t t, u2 x) -> u2 {
        x = stage_step<RULE>(st[g], x, a.birth, a.survive);
        if constexpr (kBirths) {
            const int64_t r = sg.glob0 + row_first + t - (g + 1);  // field row
            const bool rok = (r >= 0) && (r < sg.field_h);
            x.lo = rok ? (x.lo & cmlo) : 0u;
            x.hi = rok ? (x.hi & cmhi) : 0u;
        }
        return x;
    };
    auto store = [&](int64_t t, u2 x) {
        if (t >= 2 * K && t < T && st_lane)
            outp[(t - 2 * K) * a.stride] = ((uint64_t)x.hi << 32) | x.lo;
    };

    // One block of kPrefetch steps.  GUARD (warm-up blocks): stage g first emits a
    // row that can reach a valid output at step 2g+2 and needs the two ingests
    // before it, so it only runs from step 2g on; skipping it earlier saves
    // K*(K-1) of the 2K*K warm-up stage-steps.  The guard is wave-uniform (a
    // scalar branch per stage-step).
    auto block = [&](int64_t t0, auto guard) {
        constexpr bool kGuard = decltype(guard)::value;
        u2 x[kPrefetch];
#pragma unroll
        for (int p = 0; p < kPrefetch; ++p) {
            x[p] = ingest(t0 + p, ring[p]);
            ring[p] = *pf;
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
        // all of it.
        if constexpr (!kGuard) {
            // the block's inputs pass through the directive, so the compute that
            // depends on them cannot be scheduled above it; "memory" keeps the
            // loads above and the stores below.  The compiler may add a hazard
            // s_nop after it, so the 4-byte pad that gives the wanted parity is
            // per kernel: loop_place.h, generated by tools/loop_align.py.
            static_assert(kPrefetch == 4, "placement asm names 4 inputs");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (life_loop_pad(K, RULE, VAR))
                asm volatile(".p2align 3\n\ts_nop 0"
                             : "+v"(x[0].lo), "+v"(x[0].hi), "+v"(x[1].lo), "+v"(x[1].hi),
                               "+v"(x[2].lo), "+v"(x[2].hi), "+v"(x[3].lo), "+v"(x[3].hi)
                             :
                             : "memory");
            else
                asm volatile(".p2align 3"
                             : "+v"(x[0].lo), "+v"(x[0].hi), "+v"(x[1].lo), "+v"(x[1].hi),
                               "+v"(x[2].lo), "+v"(x[2].hi), "+v"(x[3].lo), "+v"(x[3].hi)
                             :
                             : "memory");
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

template <int K, int VAR>
hipError_t launch_depth(const StepArgs& a, RuleKind rule, hipStream_t s)
{
    const dim3 grid((unsigned)((a.total_units + kWavesPerBlock - 1) / kWavesPerBlock));
    const dim3 block(64 * kWavesPerBlock);
    switch (rule) {
    case RULE_REF:
        hipLaunchKernelGGL((life_tb_kernel<K, RULE_REF, VAR>), grid, block, 0, s, a);
        break;
    case RULE_CONWAY:
        hipLaunchKernelGGL((life_tb_kernel<K, RULE_CONWAY, VAR>), grid, block, 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((life_tb_kernel<K, RULE_GENERIC, VAR>), grid, block, 0, s, a);
        break;
    }
    return hipGetLastError();
}

template <int K>
hipError_t launch_variant(const StepArgs& a, RuleKind rule, int var, hipStream_t s)
{
    switch (var) {
    case 1:  // the neighbour-sum state exists up to depth 16 (14 VGPRs per stage)
        if constexpr (K <= 16) return launch_depth<K, 1>(a, rule, s);
        return hipErrorInvalidValue;
    case 2: return launch_depth<K, 2>(a, rule, s);
    default: return launch_depth<K, 0>(a, rule, s);
    }
}

template <int K, int VAR>
int occupancy_of(RuleKind rule)
{
    int blocks = 0;
    hipError_t e = hipErrorInvalidValue;
    const int threads = 64 * kWavesPerBlock;
    if (rule == RULE_REF)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_REF, VAR>, threads, 0);
    else if (rule == RULE_CONWAY)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_CONWAY, VAR>, threads, 0);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks, life_tb_kernel<K, RULE_GENERIC, VAR>, threads, 0);
    return e == hipSuccess ? blocks : 0;
}

template <int K>
int occupancy_variant(RuleKind rule, int var)
{
    switch (var) {
    case 1:
        if constexpr (K <= 16) return occupancy_of<K, 1>(rule);
        return 0;
    case 2: return occupancy_of<K, 2>(rule);
    default: return occupancy_of<K, 0>(rule);
    }
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void init_random_kernel(uint64_t* buf, int64_t stride,
                                                          int64_t wq, uint64_t lastmask,
                                                          int64_t row_base, int64_t glob_row0,
                                                          int64_t nrows, uint64_t seed)
{
    const int64_t total = nrows * stride;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / stride, q = k - i * stride;
        uint64_t v = 0;
        if (q < wq) {
            v = splitmix64_at(seed, (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)q);
            if (q == wq - 1) v &= lastmask;  // canonical mask
        }
        buf[(row_base + i) * stride + q] = gol_split64(v);
    }
}

__global__ __launch_bounds__(256) void digest_kernel(const uint64_t* buf, int64_t stride,
                                                     int64_t wq, int64_t row_base,
                                                     int64_t glob_row0, int64_t nrows,
                                                     unsigned long long* acc)
{
    const int64_t total = nrows * wq;
    uint64_t live = 0, hash = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / wq, q = k - i * wq;
        const uint64_t v = gol_join64(buf[(row_base + i) * stride + q]);
        live += (uint64_t)__popcll(v);
        const uint64_t idx = (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)q;
        hash += splitmix64_at(v ^ splitmix64_at(0, idx), 0);
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

// ASCII codec (data.txt / output.txt bytes <-> column-split words), the
// device-side replacement of readGridFromFile's parse (:91-99) and
// writeDataToFile's serialisation (:157-164).  One wavefront per (row, word):
// lane j reads the byte of column 64q+j (coalesced), __ballot forms the
// canonical word, lane 0 stores it split.  Byte w of every row must be '\n'.
__global__ __launch_bounds__(256) void ascii_pack_kernel(const char* src, int64_t rows, int64_t w,
                                                         int64_t wq, uint64_t* dst,
                                                         int64_t stride, int* bad)
{
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * wq;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / wq, q = k - r * wq;
        const int64_t c = q * 64 + lane;
        const char* line = src + r * (w + 1);
        const bool live = c < w && line[c] == '1';
        const uint64_t word = __ballot(live);
        if (lane == 0) {
            dst[r * stride + q] = gol_split64(word);
            if (q == wq - 1 && line[w] != '\n') atomicOr(bad, 1);
        }
    }
}

__global__ __launch_bounds__(256) void ascii_unpack_kernel(const uint64_t* src, int64_t stride,
                                                           int64_t rows, int64_t w, int64_t wq,
                                                           char* dst)
{
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * wq;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / wq, q = k - r * wq;
        const uint64_t word = gol_join64(src[r * stride + q]);
        const int64_t c = q * 64 + lane;
        char* line = dst + r * (w + 1);
        if (c < w) line[c] = ((word >> lane) & 1) ? '1' : '0';
        if (q == wq - 1 && lane == 0) line[w] = '\n';
    }
}

}  // namespace

hipError_t launch_life(const StepArgs& a, int depth, RuleKind rule, int compact, hipStream_t s)
{
    if (a.total_units <= 0) return hipSuccess;
#ifdef GOL_DEV_ONLY_DEPTH  // dev A/B builds: one depth only (fast compile)
    if (depth != GOL_DEV_ONLY_DEPTH) return hipErrorInvalidValue;
    return launch_variant<GOL_DEV_ONLY_DEPTH>(a, rule, compact, s);
#else
    switch (depth) {
    case 1: return launch_variant<1>(a, rule, compact, s);
    case 2: return launch_variant<2>(a, rule, compact, s);
    case 4: return launch_variant<4>(a, rule, compact, s);
    case 6: return launch_variant<6>(a, rule, compact, s);
    case 7: return launch_variant<7>(a, rule, compact, s);
    case 8: return launch_variant<8>(a, rule, compact, s);
    case 12: return launch_variant<12>(a, rule, compact, s);
    case 16: return launch_variant<16>(a, rule, compact, s);
    case 20: return launch_variant<20>(a, rule, compact, s);
    case 24: return launch_variant<24>(a, rule, compact, s);
    case 32: return launch_variant<32>(a, rule, compact, s);
    default: return hipErrorInvalidValue;
    }
#endif
}

int life_blocks_per_cu(int depth, RuleKind rule, int compact)
{
#ifdef GOL_DEV_ONLY_DEPTH
    return depth == GOL_DEV_ONLY_DEPTH ? occupancy_variant<GOL_DEV_ONLY_DEPTH>(rule, compact) : 0;
#else
    switch (depth) {
    case 1: return occupancy_variant<1>(rule, compact);
    case 2: return occupancy_variant<2>(rule, compact);
    case 4: return occupancy_variant<4>(rule, compact);
    case 6: return occupancy_variant<6>(rule, compact);
    case 7: return occupancy_variant<7>(rule, compact);
    case 8: return occupancy_variant<8>(rule, compact);
    case 12: return occupancy_variant<12>(rule, compact);
    case 16: return occupancy_variant<16>(rule, compact);
    case 20: return occupancy_variant<20>(rule, compact);
    case 24: return occupancy_variant<24>(rule, compact);
    case 32: return occupancy_variant<32>(rule, compact);
    default: return 0;
    }
#endif
}

hipError_t launch_init_random(uint64_t* buf, int64_t stride, int64_t wq, uint64_t lastmask,
                              int64_t row_base, int64_t glob_row0, int64_t nrows, uint64_t seed,
                              hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const int64_t total = nrows * stride;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(init_random_kernel, dim3((unsigned)blocks), dim3(256), 0, s, buf, stride,
                       wq, lastmask, row_base, glob_row0, nrows, seed);
    return hipGetLastError();
}

hipError_t launch_ascii_pack(const char* src, int64_t rows, int64_t w, int64_t wq, uint64_t* dst,
                             int64_t stride, int* bad, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    int64_t blocks = (rows * wq + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(ascii_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, w,
                       wq, dst, stride, bad);
    return hipGetLastError();
}

hipError_t launch_ascii_unpack(const uint64_t* src, int64_t stride, int64_t rows, int64_t w,
                               int64_t wq, char* dst, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    int64_t blocks = (rows * wq + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(ascii_unpack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, stride,
                       rows, w, wq, dst);
    return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* buf, int64_t stride, int64_t wq, int64_t row_base,
                         int64_t glob_row0, int64_t nrows, unsigned long long* acc,
                         hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const int64_t total = nrows * wq;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(digest_kernel, dim3((unsigned)blocks), dim3(256), 0, s, buf, stride, wq,
                       row_base, glob_row0, nrows, acc);
    return hipGetLastError();
}

}  // namespace gol
