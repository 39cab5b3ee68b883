// Internal interface between the host engine (engine.cpp) and the HIP kernels
// (life_stencil.h, life_tb_d*.hip, life_aux.hip).  Not part of the public C ABI
// (include/gol.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef GOL_DEV_KERNELS
#define GOL_DEV_KERNELS 0
#endif

namespace gol {

// Rule specialisations of the stencil kernel.
enum RuleKind : int {
    RULE_REF = 0,     // birth = {}, survive = {2}: the reference's effective rule
    RULE_CONWAY = 1,  // birth = {3}, survive = {2,3}
    RULE_GENERIC = 2  // any 9-bit mask pair, full 0..8 neighbour count
};

// One independent field region streamed by the stencil kernel.
//   Buffer row (base_row + i) holds segment-local row i.  Local row i is field row
//   (glob0 + i); field rows outside [0, field_h) are dead (never loaded, forced 0).
//   The kernel reads local rows [out_lo - K, out_hi + K) (only those inside
//   [0, in_rows) and inside the field; others read as dead) and writes local rows
//   [out_lo, out_hi) of the output buffer.
struct SegDesc {
    int64_t base_row;
    int64_t in_rows;
    int64_t glob0;
    int64_t field_h;
    int64_t out_lo, out_hi;
    int64_t nblk;   // row blocks of rows_per_wave rows
    int64_t unit0;  // index of this segment's first wavefront in the launch
};

// Strips: a strip is L consecutive lanes (L = 64 >> lane_shift: 64, 32 or 16),
// each holding one lane group of a row (NP 32-bit planes = NP/2 words,
// bitlayout.h); its first and last lane are the horizontal halo (exact for up to
// 63 fused generations), so a strip outputs L - 2 groups.  A wavefront runs 64 / L
// strips side by side over the same rows: narrow strips trade 2 halo lanes per
// strip for more wavefronts per row block, which lets short stripes use longer row
// blocks (less vertical halo recompute).
constexpr int kStripOut = 62;  // output lane groups of a full 64-lane strip
constexpr int kWavesPerBlock = 4;
// Zeroed guard rows allocated before/after every state buffer so that the
// streaming loads (K rows of halo + prefetch distance) never leave the allocation.
constexpr int kGuardRows = 64;
constexpr int kMaxDepth = 32;

struct StepArgs {
    // state buffers, row 0 (guard rows precede it): pass p of the launch reads
    // pbuf[p] and writes pbuf[p + 1]
    uint64_t* pbuf[4];
    // multi-pass launches (life_stencil.h): passes (1 = single), the byte offset of
    // the halo lanes' shadow half of each buffer, and the head/done flags (4 x
    // total_units words, all 0 between launches)
    int32_t npass;
    uint32_t shadow_off;
    uint32_t* mpflags;
    // dev timing switches (GOL_DEV_MP_FLAGS, GOL_EXP builds; the field is not valid): 2 = no
    // inter-pass waits, 8 = no shadow for the halo lanes
    uint32_t mp_dev;
    const SegDesc* segs;  // device table
    int32_t nseg;
    int32_t strips;       // strip groups per row: ceil(ceil(wq / (L-2)) / (64/L))
    int32_t lane_shift;   // L = 64 >> lane_shift lanes per strip (0, 1 or 2)
    int32_t tail_off;     // hand-off kernels: (R + 2 - warm-up) mod prefetch block
    int64_t stride;       // words per buffer row
    int64_t ng;           // lane groups per field row = ceil(ceil(w / 64) / (NP/2))
    uint64_t lastmask[2]; // stored-form valid bits of the last group's words
    int64_t rows_per_wave;
    int64_t total_units;  // wavefronts in the launch
    // Age-skewed row blocks (one-segment launches of one round, engine.cpp
    // age_skew): units below units_old start first on their SIMD, win its VALU
    // arbitration and get rows_old rows; the others rows_per_wave.  0 = off.
    int32_t rows_old;
    int32_t units_old;
    uint32_t birth, survive;
    // Row-block hand-off (kernels instantiated with HAND = true; see
    // life_stencil.h): each wavefront's slot of side rows, its ready flag, and a
    // flag the kernel sets when a wait for a neighbour's rows timed out.
    uint64_t* side;       // total_units slots of side_slot words (per pass parity)
    uint32_t* flags;      // total_units words (per pass parity), all 0 between launches
    int* err;
    int64_t side_slot;    // words per slot: 2 (K-1) rows x 64 lanes x NP/2 words
    uint64_t* wlog;       // dev timing builds only (GOL_EXP & 128): 8 words per wavefront
    uint32_t* prog;       // dev (GOL_EXP & 1024): per-SIMD wave progress, 2 words per SIMD
    // Edge-aligned strips and the packed half strip (plan.cpp col_layout;
    // one-segment launches of 64-lane strips).  A lane whose neighbour lane is the
    // DPP shift's zero (lane 0 / 63) or outside the field is exact, so strip 0 starts
    // at group 0 (63 output groups), strip s at group 62 s (lane 0 its halo), and
    // the last strip ends at group ng - 1 in lane 63 (right_q0 = ng - 64; -1: 62 s).
    // The gap of <= 30 groups left between the last two strips is the half strip
    // [half_q0 + 1, half_hi]: 32 lanes.  Units [pair0, pair0 + pair_units) run it,
    // two row blocks per wavefront (lanes 32-63 offset by the second block's rows),
    // with classic block closure (the device segment table carries one more
    // segment for them: a copy of segment 0 with nblk = 1 and unit0 = pair0, so
    // that no unit of theirs is a hand-off producer or consumer); pairs holds
    // (first row A, first row B or -1 for lanes 32-63 idle, rows) per unit.
    int32_t edge;
    // (r05) the launch's one segment (nseg is 1, or 2 with the half strip's
    // copy): the kernel takes it from here instead of the device table
    int32_t seg0_only;
    SegDesc seg0;
    int64_t right_q0;
    int64_t half_q0, half_hi;
    int64_t pair0, pair_units;
    const int64_t* pairs;
    // (r06 dev A/B) per-XCD row shift between paired blocks (life_stencil.h):
    // bits 2x..2x+1 = speed class of blockIdx mod 8 == x, bits 16-23 = strip
    // modulus m; 0 = off
    uint32_t xcd_shift;
};

// Fused depths with an instantiated kernel, largest first.  The shipped library
// builds the depths auto_layout and the remainder launches use; the dev build
// (make dev, GOL_DEV_KERNELS) adds 20/24/32 and the 4-plane lane groups.
#if GOL_DEV_KERNELS
constexpr int kDepthList[] = {32, 24, 20, 16, 12, 8, 7, 6, 4, 2, 1};
#else
constexpr int kDepthList[] = {16, 12, 8, 7, 6, 4, 2, 1};
#endif
constexpr bool kDevKernels = GOL_DEV_KERNELS != 0;

// Row blocks hand their first rows of every fused generation to the block above
// (life_stencil.h) from this depth on.
constexpr int kHandoffMinDepth = 4;
// ... except for the generic-mask rule above depth 12, whose 10-term mask sum
// already spills without the hand-off's extra state (auto_layout gives it K = 12)
constexpr bool handoff_kernel_exists(int K, RuleKind rule)
{
    return K >= kHandoffMinDepth && (rule != RULE_GENERIC || K <= 12);
}

// Multi-pass stencil kernels (StepArgs::npass > 1, life_stencil.h): 2-plane lane
// groups at depths 12 and 16 (the generic-mask rule at 12 only, as its hand-off
// kernels).  Measured slower than single-pass launches (r05): the dev
// build only (make dev), so the shipped library carries no multi-pass kernel.
constexpr bool multipass_kernel_exists(int K, RuleKind rule, int planes)
{
    return kDevKernels && planes == 2 && (K == 12 || (K == 16 && rule != RULE_GENERIC));
}

// Steps per block of the stencil kernel's register prefetch ring (host copy of
// life_stencil.h kPfOf): 8 for 2-plane kernels of depth >= 16, 4 elsewhere.
constexpr int prefetch_of(int K, int planes) { return (planes == 2 && K >= 16) ? 8 : 4; }
// Unrolled warm-up steps (a multiple of the prefetch block covering 2K steps).
constexpr int warm_steps_of(int K, int planes)
{
    return (2 * K + prefetch_of(K, planes) - 1) / prefetch_of(K, planes) * prefetch_of(K, planes);
}
// Tail offsets with a hand-off kernel: 0 and prefetch/2, and 2 and 6 with the
// 8-step prefetch block (offset 2 there would take 258 VGPRs, one wave per SIMD:
// it is built capped at 256, GOL_TOFF2_CAP).
constexpr bool handoff_toff_exists(int off, int pf)
{
    return off == 0 || off == pf / 2 || (pf == 8 && (off == 6 || off == 2));
}
// A consumer block of R rows streams R + 2 input steps after the warm-up, i.e.
// (R + 2 - warm) mod prefetch must be an offset with a kernel, and at least two
// whole steady blocks must precede the tail (the flag wait sits at the end of the
// first of them).  Returns the offset, or -1 if R does not fit.  Every offset with
// a kernel, the warm-up and the prefetch are even, so R is even: the B/S2 pair sum
// (life_stencil.h) relies on the tail starting at an even step t_side = R + 2.
constexpr int handoff_toff(int64_t R, int K, int planes)
{
    const int pf = prefetch_of(K, planes), warm = warm_steps_of(K, planes);
    if (K < kHandoffMinDepth || R + 2 < warm + 2 * pf) return -1;
    const int off = (int)((R + 2 - warm) % pf);
    if (!handoff_toff_exists(off, pf)) return -1;
    return R + 2 - off >= warm + 2 * pf ? off : -1;
}

// Launch `depth` fused generations (depth in kDepthList) on lane groups of
// `planes` (2, or 4 in the dev build).  hand: the row-block hand-off kernel
// (a.side/flags/err set); else every row block recomputes its vertical halo.
hipError_t launch_life(const StepArgs& a, int depth, RuleKind rule, int planes, bool hand,
                       hipStream_t s);
bool life_has_kernel(int depth, int planes);

// Resident 256-thread blocks per CU of the stencil kernel (occupancy query).
// mp: of the multi-pass kernels (0 where none exists)
int life_blocks_per_cu(int depth, RuleKind rule, int planes, bool hand, bool mp = false);

// Per-depth entry points (explicitly instantiated in life_tb_d<K>.hip).
template <int K>
hipError_t launch_depth(const StepArgs& a, RuleKind rule, int planes, bool hand, hipStream_t s);
template <int K>
int occupancy_depth(RuleKind rule, int planes, bool hand, bool mp);

// The resident kernel (life_resident.hip): one launch runs a whole gol_step on a
// small field held in registers by one 1024-thread workgroup per (band, strip)
// tile; neighbouring tiles swap their band rows every K generations through
// the two field buffers (epoch e's result in buf0 if e is even, else buf1;
// buf0 holds the input).
constexpr int kResWaves = 16;                     // wavefronts per workgroup
constexpr int kResRowsList[] = {2, 3, 4, 6, 8};   // rows per wavefront (instantiated)
struct ResArgs {
    uint64_t* buf0;       // row 0 of the input buffer (also the even epochs' output)
    uint64_t* buf1;
    uint32_t* flags;      // one per tile: epochs published, counting from flag_base
    int* err;             // set when a neighbour wait timed out
    int64_t stride;       // words per buffer row
    int64_t h;            // field rows
    int64_t ng;           // lane groups (= words) per row
    uint64_t lastmask;    // stored-form valid bits of group ng - 1
    int32_t strips;       // 1: lane l = group l (ng <= 64); else 62 groups + 2 halo lanes
    int32_t bands;
    int32_t band_rows;    // B; tiles hold B + 2K <= kResWaves * M rows
    int32_t K;            // generations per epoch (<= 63 when strips > 1)
    int32_t span;         // ceil(K / band_rows): bands a halo reaches; (2 span + 1) x
                          // (strips > 1 ? 3 : 1) - 1 <= 64 neighbour tiles
    int32_t gens;         // generations of this launch
    uint32_t flag_base;
    uint32_t birth, survive;
    uint64_t* wlog;       // dev timing builds only (GOL_EXP & 2048): 4 words per wavefront
};
// coop: hipLaunchCooperativeKernel, else a plain launch (engine.cpp Resident::coop)
hipError_t launch_resident(const ResArgs& a, int rows, RuleKind rule, int grid, hipStream_t s,
                           bool coop = false);
int resident_blocks_per_cu(int rows, RuleKind rule);
// The resident kernel with wave-level temporal blocking (life_resident_mb.hip, r06,
// dev build only: slower than life_res_kernel at every MB): wavefronts
// swap MB rows through LDS every MB generations.  (rows, mb) pairs:
// (the generic-mask rule at rows = mb = 4 spills: not offered)
constexpr bool resident_mb_exists(int rows, int mb, RuleKind rule)
{
    return mb >= 2 && mb <= rows && rows <= 4 && !(rule == RULE_GENERIC && mb == 4);
}
hipError_t launch_resident_mb(const ResArgs& a, int rows, int mb, RuleKind rule, int grid,
                              hipStream_t s);
int resident_mb_blocks_per_cu(int rows, int mb, RuleKind rule);

// Device-side synthetic init: buffer rows [row_base, row_base+nrows) get field
// rows [glob_row0, glob_row0+nrows).
hipError_t launch_init_random(uint64_t* buf, int64_t stride, int64_t wq, uint64_t lastmask,
                              int64_t row_base, int64_t glob_row0, int64_t nrows,
                              uint64_t seed, int planes, hipStream_t s);

// ASCII codec: `rows` lines of w cell bytes + '\n' (device memory) <-> stored
// lane groups (ng per row) at dst/src with `stride` words per row.  *bad is set
// if a line does not end in '\n' at byte w.
hipError_t launch_ascii_pack(const char* src, int64_t rows, int64_t w, int64_t ng, uint64_t* dst,
                             int64_t stride, int* bad, int planes, hipStream_t s);
hipError_t launch_ascii_unpack(const uint64_t* src, int64_t stride, int64_t rows, int64_t w,
                               int64_t ng, char* dst, int planes, hipStream_t s);

// Adds popcount and hash of buffer rows [row_base, row_base+nrows) (field rows
// glob_row0..) into acc[0], acc[1].
hipError_t launch_digest(const uint64_t* buf, int64_t stride, int64_t wq, int64_t ng,
                         int64_t row_base, int64_t glob_row0, int64_t nrows,
                         unsigned long long* acc, int planes, hipStream_t s);

}  // namespace gol
