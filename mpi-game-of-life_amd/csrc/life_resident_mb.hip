// life_resident_mb.hip -- the resident kernel with wave-level temporal blocking
// (r06): the same tiles, epochs and epoch hand-off as life_res_kernel
// (life_resident.hip), but the wavefronts of a tile swap rows through LDS every
// MB generations instead of every generation.
//
// The per-generation update is Parallel_Life_MPI.cpp countNeighbours :16-35 +
// updateGrid :37-54 on the bit-packed lane groups (bitlayout.h), with the H3 sums
// and the rule logic of life_stencil.h (pair forms for B/S2 and B3/S23,
// rule32_total for the generic masks).
//
// Why.  In life_res_kernel a wavefront's first and last row need the H3 of its
// neighbour wavefronts' edge rows of the same generation, so every generation is
// an LDS round trip across every wave seam: ~970 cycles per generation of which
// the VALU is busy about a quarter (profiles/r03 res_trace, r05 counters: VALU
// issue 0.265, SQ_WAIT_ANY 63%).  Here a wavefront holds its M own rows plus MB
// halo rows above and below (E = M + 2 MB rows in VGPRs).  At the start of a
// super-step it reads the MB rows above it (the upper wavefront's last MB own
// rows) and the MB rows below (the lower one's first MB), then advances MB
// generations alone, the computed range shrinking by one row per side per
// generation (generation i of the super-step: ext rows [i, E-1-i]), so that
// after MB generations exactly its own rows are new.  It then publishes its first
// and last MB own rows and raises its progress word.  One seam round trip per MB
// generations, for (MB - 1) extra rows of work per generation per wavefront.
//
// Protocol (LDS; all waves of a tile see the same super-step grid: steps start at
// multiples of MB from each epoch's start).  Slot parity p = super-step index & 1;
// a wavefront publishes the rows for super-step j + 1 into slot (j + 1) & 1 after
// computing super-step j and then stores its word = the generation they hold; a
// neighbour starts super-step j + 1 once that word is >= its start.  A slot is
// rewritten two super-steps later, after the wavefront waited for its
// neighbours' words of the super-step in between, which they raise after reading
// the slot (a wavefront's LDS accesses execute in order).  A wavefront whose rows
// are outside the epoch's exact range from some generation on stops computing
// (gmax, as in life_res_kernel) and raises its word to the epoch's end: the rows
// its neighbours then read from it are stale, and so are the rows they would
// compute from it -- outside the exact range too.  Epoch hand-off, flags, bounded
// waits, ping-pong buffers: life_res_kernel's (life_resident.hip header).
#include "life_stencil.h"

namespace gol {

namespace {

// LDS: edge rows [slot 2][wave][top / bottom][MB rows][64 lanes] x 8 bytes, a zero
// row, the per-wave progress words (one copy per lane); at least 96 KB so that a
// CU holds one tile.
template <int MB>
constexpr int res_mb_edge_words()
{
    return 2 * kResWaves * 2 * MB * 64;
}
template <int MB>
constexpr int res_mb_lds_words()
{
    return std::max(96 * 1024 / 8, res_mb_edge_words<MB>() + 64 + kResWaves * 64 / 2);
}

template <int M, int MB, int RULE>
__global__ __launch_bounds__(1024) void life_res_mb_kernel(ResArgs a)
{
    static_assert(MB >= 2 && MB <= M, "a super-step publishes MB of the wavefront's own rows");
    constexpr bool kBirths = RULE != RULE_REF;
    constexpr bool kPair = pair_rule(RULE);
    constexpr int W = kResWaves;
    constexpr int E = M + 2 * MB;  // held rows: MB above, M own, MB below
    __shared__ uint64_t lds[res_mb_lds_words<MB>()];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

    // workgroup -> tile (consecutive tiles on one XCD under round-robin dispatch;
    // speed only)
    const int G = (int)gridDim.x;
    int tile = (int)blockIdx.x;
    if ((G & 7) == 0) tile = (tile & 7) * (G >> 3) + (tile >> 3);
    const int band = tile / a.strips, strip = tile % a.strips;
    const int64_t b0 = (int64_t)band * a.band_rows;
    const int64_t b1 = min(b0 + a.band_rows, a.h);
    const int64_t r0 = b0 - a.K + (int64_t)wv * M;  // field row of own row 0
    const int64_t e0 = r0 - MB;                     // field row of held row 0

    const bool multi = a.strips > 1;
    const int64_t gi = multi ? (int64_t)strip * 62 - 1 + lane : lane;
    const bool lane_ok = gi >= 0 && gi < a.ng;
    const bool halo_lane = multi && (lane == 0 || lane == 63);
    const bool st_lane = lane_ok && !halo_lane;
    Pl<2> cm;
#pragma unroll
    for (int k = 0; k < 2; ++k)
        cm.v[k] = lane_ok ? (gi == a.ng - 1 ? (uint32_t)(a.lastmask >> (32 * k)) : ~0u) : 0u;
    const uint32_t voff = (uint32_t)((lane_ok ? gi : 0) * 8);
    auto row_ptr = [&](const uint64_t* buf, int64_t r) -> const uint64_t* {
        return reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(buf + r * a.stride) +
                                                 voff);
    };
    auto fetch = [&](const uint64_t* buf, int64_t r) -> Pl<2> {
        if (r < 0 || r >= a.h || !lane_ok) {
            Pl<2> z;
            z.v[0] = z.v[1] = 0u;
            return z;
        }
        Pl<2> x = planes_of<2>(load_grp<2>(row_ptr(buf, r)));
        x.v[0] &= cm.v[0];
        x.v[1] &= cm.v[1];
        return x;
    };

    Pl<2> x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) x[e].v[0] = x[e].v[1] = 0u;
#pragma unroll
    for (int i = 0; i < M; ++i) x[MB + i] = fetch(a.buf0, r0 + i);
    // held rows outside the field stay dead (rules with births)
    uint32_t rowm[E];
#pragma unroll
    for (int e = 0; e < E; ++e) rowm[e] = (e0 + e >= 0 && e0 + e < a.h) ? ~0u : 0u;

    // neighbour tiles whose flags this workgroup waits for (life_res_kernel)
    int nb_tile = -1;
    if (wv == 0) {
        const int sw = multi ? 3 : 1;
        const int center = a.span * sw + sw / 2;
        const int j = lane + (lane >= center ? 1 : 0);
        if (j < (2 * a.span + 1) * sw) {
            const int nbd = band + j / sw - a.span, nst = strip + j % sw - sw / 2;
            if (nbd >= 0 && nbd < a.bands && nst >= 0 && nst < a.strips)
                nb_tile = nbd * a.strips + nst;
        }
    }

    uint2* const ed = reinterpret_cast<uint2*>(lds);
    uint2* const zero2 = ed + res_mb_edge_words<MB>();
    uint32_t* const prog = reinterpret_cast<uint32_t*>(zero2 + 64);
    if (wv == 0) zero2[lane] = uint2{0u, 0u};
    // slot (p, wave w, side: 0 = its first MB own rows, 1 = its last MB), row j
    auto slot = [&](int p, int w, int side, int j) -> uint2* {
        return ed + (((p * W + w) * 2 + side) * MB + j) * 64 + lane;
    };
    auto put_edges = [&](int p) {
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            *slot(p, wv, 0, j) = uint2{x[MB + j].v[0], x[MB + j].v[1]};
            *slot(p, wv, 1, j) = uint2{x[M + j].v[0], x[M + j].v[1]};
        }
    };
    const bool has_up = wv > 0, has_dn = wv < W - 1;
    // the first / last wave reads the zero row and waits on its own word
    uint32_t* const wait_up = prog + (has_up ? wv - 1 : wv) * 64;
    uint32_t* const wait_dn = prog + (has_dn ? wv + 1 : wv) * 64;
    uint32_t* const my_word = prog + wv * 64 + lane;
    auto word = [](uint32_t* p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto set_word = [&](uint32_t v) {
        __hip_atomic_store(my_word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // the halo rows of super-step slot p into x[0, MB) and x[MB + M, E)
    auto read_halos = [&](int p) {
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            const uint2 u = has_up ? *slot(p, wv - 1, 1, j) : zero2[lane];
            const uint2 d = has_dn ? *slot(p, wv + 1, 0, j) : zero2[lane];
            x[j].v[0] = u.x;
            x[j].v[1] = u.y;
            x[MB + M + j].v[0] = d.x;
            x[MB + M + j].v[1] = d.y;
        }
    };
    auto spin = [&](uint32_t* p, uint32_t need) {
        const uint64_t t0 = wait_clock();
        for (;;) {
            if (wait_clock() - t0 > kWaitTicks) {  // lost: flag it, go on so the launch drains
                __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(0);
            asm volatile("" ::: "memory");
            if (__builtin_amdgcn_readfirstlane((int32_t)(word(p) - need)) >= 0) break;
        }
        asm volatile("" ::: "memory");
    };

    Pl<2> s[E], c[E];  // H3 of the held rows (bit-sliced horizontal 3-sums)
    auto h3 = [&](int e) {
        const Ends en = ends(x[e]);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t L = left_of(x[e], en, k), R = right_of(x[e], en, k);
            s[e].v[k] = lop3<kXor3>(L, x[e].v[k], R);
            c[e].v[k] = lop3<kMaj>(L, x[e].v[k], R);
        }
    };
    auto finish = [&](int e, int k, uint32_t y) {
        if constexpr (kBirths) y = lop3<kAnd3>(y, cm.v[k], rowm[e]);
        x[e].v[k] = y;
    };
    // one generation of the super-step: held rows [lo, hi] from the H3 of
    // [lo - 1, hi + 1] (all computed before any row is replaced)
    auto generation = [&](int lo, int hi) {
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (e >= lo - 1 && e <= hi + 1) h3(e);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if (e < lo || e > hi) continue;
            if constexpr (kPair) {
                if (((e - lo) & 1) == 0 && e + 1 <= hi) {  // the pair (e, e + 1)
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const PairQ q = pair_sum<RULE>(s[e].v[k], c[e].v[k], s[e + 1].v[k],
                                                       c[e + 1].v[k]);
                        const uint32_t y0 = rule_from_pair<RULE>(q, s[e - 1].v[k], c[e - 1].v[k],
                                                                 x[e].v[k]);
                        const uint32_t y1 = rule_from_pair<RULE>(q, s[e + 2].v[k], c[e + 2].v[k],
                                                                 x[e + 1].v[k]);
                        finish(e, k, y0);
                        finish(e + 1, k, y1);
                    }
                    continue;
                }
                if (((e - lo) & 1) == 1) continue;  // done with its pair
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
                finish(e, k, rule32_total<RULE>(s[e - 1].v[k], c[e - 1].v[k], s[e].v[k], c[e].v[k],
                                                s[e + 1].v[k], c[e + 1].v[k], x[e].v[k], a.birth,
                                                a.survive));
        }
    };

    const int32_t gmax = (int32_t)min<int64_t>(r0 + M - (b0 - a.K) - 1, b1 + a.K - 1 - r0);
    uint32_t epoch = 0;
    bool gave_up = false;
    for (int32_t done = 0; done < a.gens;) {
        const int32_t k = min(a.K, a.gens - done);
        put_edges(0);
        // (a wave whose rows are never exact this epoch releases its neighbours now)
        set_word((uint32_t)(gmax > 0 ? done : done + k));
        __syncthreads();
        const int32_t gend = min(k, gmax);
        int32_t g = 0;
        for (int p = 0; g < gend; p ^= 1) {
            const int32_t mb = min(MB, k - g);
            const uint32_t need = (uint32_t)(done + g);
            // progress words, then the halo rows (LDS in order): speculative, re-read
            // below if a word came back short
            const uint32_t wu = word(wait_up), wd = word(wait_dn);
            asm volatile("" ::: "memory");
            read_halos(p);
            // H3 of the own rows need no halo: the first generation's start covers
            // the LDS round trip
            const bool short_up = __builtin_amdgcn_readfirstlane((int32_t)(wu - need)) < 0;
            const bool short_dn = __builtin_amdgcn_readfirstlane((int32_t)(wd - need)) < 0;
            if (short_up || short_dn) {
                if (short_up) spin(wait_up, need);
                if (short_dn) spin(wait_dn, need);
                read_halos(p);
            }
#pragma unroll
            for (int i = 1; i <= MB; ++i)
                if (i <= mb) generation(i, E - 1 - i);
            g += mb;
            // rows for the next super-step (none after the epoch's last).  Also at
            // g == gend, where this wave stops: its last own row is still exact at
            // generation gmax, and a neighbour's one-generation super-step (an
            // epoch's partial last one) reads it
            if (g < k && g <= gend) {
                put_edges(p ^ 1);
                asm volatile("" ::: "memory");  // the word after the rows
                set_word((uint32_t)(done + g));
            }
        }
        if (gend < k) set_word((uint32_t)(done + k));  // off: release the neighbours
        done += k;
        ++epoch;
        // publish the band rows into the buffer of this epoch's result
        uint64_t* nb = (epoch & 1) ? a.buf1 : a.buf0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int64_t r = r0 + i;
            if (r >= b0 && r < b1 && st_lane)
                __hip_atomic_store(const_cast<uint64_t*>(row_ptr(nb, r)), words_of<2>(x[MB + i]).w[0],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t want = a.flag_base + epoch;
        if (threadIdx.x == 0)
            __hip_atomic_store(a.flags + tile, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done >= a.gens) break;
        if (nb_tile >= 0 && !gave_up) {
            uint64_t t0 = 0;
            for (int n = 0; (int32_t)(__hip_atomic_load(a.flags + nb_tile, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) -
                                      want) < 0;
                 ++n) {
                if (n == 0) t0 = wait_clock();
                else if (wait_clock() - t0 > kWaitTicks) {  // the field is lost: flag it
                    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    gave_up = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        // reload the halo rows (all lanes) and the halo lanes of the band rows
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int64_t r = r0 + i;
            const bool own = r >= b0 && r < b1;
            if (!own || halo_lane) x[MB + i] = fetch(nb, r);
        }
    }
}

template <int M, int MB>
hipError_t launch_mb(const ResArgs& a, RuleKind rule, int grid, hipStream_t s)
{
    switch (rule) {
    case RULE_REF:
        hipLaunchKernelGGL((life_res_mb_kernel<M, MB, RULE_REF>), dim3(grid), dim3(64 * kResWaves), 0, s, a);
        break;
    case RULE_CONWAY:
        hipLaunchKernelGGL((life_res_mb_kernel<M, MB, RULE_CONWAY>), dim3(grid), dim3(64 * kResWaves), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((life_res_mb_kernel<M, MB, RULE_GENERIC>), dim3(grid), dim3(64 * kResWaves), 0, s, a);
        break;
    }
    return hipGetLastError();
}

template <int M, int MB>
int occupancy_mb(RuleKind rule)
{
    int n = 0;
    hipError_t e;
    const int t = 64 * kResWaves;
    switch (rule) {
    case RULE_REF: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_mb_kernel<M, MB, RULE_REF>, t, 0); break;
    case RULE_CONWAY: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_mb_kernel<M, MB, RULE_CONWAY>, t, 0); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_mb_kernel<M, MB, RULE_GENERIC>, t, 0); break;
    }
    return e == hipSuccess ? n : 0;
}

}  // namespace

// (rows, mb) pairs with a kernel: resident_mb_exists (life_internal.h)
hipError_t launch_resident_mb(const ResArgs& a, int rows, int mb, RuleKind rule, int grid,
                              hipStream_t s)
{
#define GOL_RES_MB(M_, MB_) \
    if (rows == M_ && mb == MB_) return launch_mb<M_, MB_>(a, rule, grid, s);
    GOL_RES_MB(2, 2)
    GOL_RES_MB(3, 2)
    GOL_RES_MB(3, 3)
    GOL_RES_MB(4, 2)
    GOL_RES_MB(4, 3)
    GOL_RES_MB(4, 4)
#undef GOL_RES_MB
    return hipErrorInvalidValue;
}

int resident_mb_blocks_per_cu(int rows, int mb, RuleKind rule)
{
#define GOL_RES_MB(M_, MB_) \
    if (rows == M_ && mb == MB_) return occupancy_mb<M_, MB_>(rule);
    GOL_RES_MB(2, 2)
    GOL_RES_MB(3, 2)
    GOL_RES_MB(3, 3)
    GOL_RES_MB(4, 2)
    GOL_RES_MB(4, 3)
    GOL_RES_MB(4, 4)
#undef GOL_RES_MB
    return 0;
}

}  // namespace gol
