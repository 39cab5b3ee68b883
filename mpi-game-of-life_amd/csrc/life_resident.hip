// life_resident.hip -- the resident kernel: small fields advanced for a whole
// gol_step in ONE launch, the field held in registers across the chip.
//
// Same per-generation update as life_tb_kernel (Parallel_Life_MPI.cpp
// countNeighbours :16-35 + updateGrid :37-54 on the bit-packed lane groups of
// bitlayout.h, bit-sliced H3 sums and the rule32_total LUT logic of
// life_stencil.h), but laid out for fields of a few thousand rows (SURVEY C2,
// 4096^2 x 1000), where the streaming kernel is latency-bound: a launch of K
// fused generations there is a ~20-step load/compute chain per wavefront plus
// a kernel boundary, ~1.3 us per generation in all.
//
// Layout.  The field is cut into bands (row ranges of B rows) x strips (64-lane
// column strips; one strip of up to 64 lane groups covers the whole row with no
// halo lanes, wider rows use strips of 62 groups + 2 halo lanes as the
// streaming kernel does).  One 1024-thread workgroup per (band, strip), at most
// one per CU: its 16 wavefronts hold M consecutive rows each in VGPRs, rows
// [b0 - K, b0 - K + 16 M) ⊇ [b0 - K, b1 + K), the band plus K halo rows on each
// side.  A generation is: every wavefront forms the H3 sums (bit-sliced
// horizontal 3-cell sums) of its M rows, puts those of its first and last row in
// LDS, one workgroup barrier, it reads the H3 of the row above its first and
// below its last, and computes its M rows in registers.  Rows at the edge of the
// held range are wrong by one more row per generation, so after K generations
// exactly the band is valid: an epoch.  Waves whose rows are all already
// outside the shrinking exact range skip the work.
//
// Between epochs (every K generations) a workgroup publishes its band rows to
// the ping-pong field buffer of the next epoch (write-through sc1 stores), then
// one lane an sc1 flag = epoch count; it waits for the flags of its neighbours
// (the bands within K rows above and below, in its own strip and the strips
// left and right) and reloads
// its halo rows and halo lanes from that buffer with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility, first table row: sc1
// payload, every storing wave's vmcnt(0) behind a workgroup barrier, one sc1
// flag store per workgroup; the polling wave loads after its poll matched, the
// others after the barrier it joins; hipMalloc buffers, one workgroup per CU --
// enforced by the 96 KB of LDS each workgroup allocates).  Flags only grow:
// the host passes the count reached by earlier launches as flag_base.  Ping-pong
// safety: a workgroup overwrites the buffer of epoch e only in epoch e + 2,
// after its neighbours' epoch e+1 flags, which they publish after reading it.
// Waits are bounded: a timeout sets *err and the launch still drains.
#include "life_stencil.h"

namespace gol {

namespace {

// LDS of a workgroup: the edge H3 rows (2 slots x top/bottom x waves x 16 B per
// lane), a zero row and the per-wave progress words, in a 96 KB block (> 80 KB:
// one workgroup per CU).  Two tiles per CU (8 rows each at 4096^2, 66 KB each, SGPRs
// capped at 80 so that the hardware admits 8 waves per SIMD) ran 17.9 against 22.7
// TCUPS: the halo work grows by half and the extra waves do not hide it
// (profiles/r03/c2_tiles_per_cu.txt).
constexpr int kResEdgeWords = 2 * 2 * kResWaves * 64 * 2;
constexpr int kResLdsWords = 96 * 1024 / 8;
static_assert(kResEdgeWords + 128 + kResWaves * 64 <= kResLdsWords,
              "edge H3 rows, the zero row and the progress words fit the LDS block");

// H3 of a row: bit-sliced sum (s) and carry (c) of each cell and its 2
// horizontal neighbours (life_stencil.h stage_step's first half).
__device__ __forceinline__ void h3_row(const Pl<2>& x, Pl<2>& s, Pl<2>& c)
{
    const Ends e = ends(x);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t L = left_of(x, e, k), R = right_of(x, e, k);
        s.v[k] = lop3<kXor3>(L, x.v[k], R);
        c.v[k] = lop3<kMaj>(L, x.v[k], R);
    }
}

__device__ __forceinline__ Pl<2> zero_pl()
{
    Pl<2> z;
    z.v[0] = z.v[1] = 0u;
    return z;
}

__device__ __forceinline__ Pl<2> load_pl(const uint64_t* p)
{
    return planes_of<2>(load_grp<2>(p));
}

template <int M, int RULE>
__global__ __launch_bounds__(1024) void life_res_kernel(ResArgs a)
{
    constexpr bool kBirths = RULE != RULE_REF;
    constexpr int W = kResWaves;
    __shared__ uint64_t lds[kResLdsWords];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

    // workgroup -> tile; consecutive tiles on blocks b, b + 8, ... which share an
    // XCD under round-robin dispatch (speed only, never correctness)
    const int G = (int)gridDim.x;
    int tile = (int)blockIdx.x;
    if ((G & 7) == 0) tile = (tile & 7) * (G >> 3) + (tile >> 3);
    const int band = tile / a.strips, strip = tile % a.strips;
    const int64_t b0 = (int64_t)band * a.band_rows;
    const int64_t b1 = min(b0 + a.band_rows, a.h);
    const int64_t r0 = b0 - a.K + (int64_t)wv * M;  // field row of this wave's x[0]

    // lane group of this lane
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
        if (r < 0 || r >= a.h || !lane_ok) return zero_pl();
        Pl<2> x = load_pl(row_ptr(buf, r));
        x.v[0] &= cm.v[0];
        x.v[1] &= cm.v[1];
        return x;
    };

    Pl<2> x[M];
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = fetch(a.buf0, r0 + i);
    // rows of the held range outside the field stay dead (rules with births)
    uint32_t rowm[M];
#pragma unroll
    for (int i = 0; i < M; ++i) rowm[i] = (r0 + i >= 0 && r0 + i < a.h) ? ~0u : 0u;

    // the neighbour tiles whose flags this workgroup waits for: bands within
    // a.span = ceil(K / B) (a K-row halo can reach that far), strips within 1;
    // lanes of wave 0 poll one each (the host keeps the count <= 64)
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

    // H3 (bit-sliced horizontal 3-sums) of this wave's rows, kept across steps so
    // that a wave that skips a generation still publishes defined values
    Pl<2> s[M], c[M];
#pragma unroll
    for (int i = 0; i < M; ++i) s[i] = c[i] = zero_pl();
    uint4* const ed4 = reinterpret_cast<uint4*>(lds);

    uint32_t epoch = 0;
    bool gave_up = false;
    // edge H3 rows through LDS: slot p = [top/bottom][wave][lane], 2 slots
    auto put_top = [&](int p) {
        ed4[p * (2 * W * 64) + wv * 64 + lane] = uint4{s[0].v[0], s[0].v[1], c[0].v[0], c[0].v[1]};
    };
    auto put_bot = [&](int p) {
        ed4[p * (2 * W * 64) + (W + wv) * 64 + lane] =
            uint4{s[M - 1].v[0], s[M - 1].v[1], c[M - 1].v[0], c[M - 1].v[1]};
    };
    // after the edge slots: a zero row (the edges of the missing neighbours of the
    // first and last wave), then two progress words per wave: the top / bottom
    // edge of generation n of the launch is in its slot once top[wave] / bot[wave]
    // >= n.  Every lane stores the word into a slot of its own (one conflict-free
    // store, no lane-0 branch); readers read slot 0.
    uint4* const zero4 = ed4 + 4 * W * 64;
    uint32_t* const prog_top = reinterpret_cast<uint32_t*>(zero4 + 64);
    uint32_t* const prog_bot = prog_top + W * 64;
    if (wv == 0) zero4[lane] = uint4{0u, 0u, 0u, 0u};
    // B/S2 and B3/S23 (r04, GOL_PAIR_SUM): the pair sums of the two rows at each edge
    // are formed before the edges arrive, so an edge row is 3 (B/S2) or 4 (B3/S23)
    // v_bitop3 per plane once its neighbour's H3 is in (life_stencil.h
    // rule_from_pair), and the interior rows next to them reuse the same pairs
    constexpr bool kPair = pair_rule(RULE) && M >= 2;
    PairQ pt[2], pb[2];  // rows (0, 1) and (M-2, M-1)
    auto pair_rows = [&](int i, PairQ (&q)[2]) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
            q[k] = pair_sum<RULE>(s[i].v[k], c[i].v[k], s[i + 1].v[k], c[i + 1].v[k]);
    };
    auto pair_row = [&](int i, const PairQ (&q)[2], const Pl<2>& ts, const Pl<2>& tc) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            uint32_t y = rule_from_pair<RULE>(q[k], ts.v[k], tc.v[k], x[i].v[k]);
            if constexpr (kBirths) y = lop3<kAnd3>(y, cm.v[k], rowm[i]);
            x[i].v[k] = y;
        }
    };
    auto rule_row = [&](int i, const Pl<2>& as, const Pl<2>& ac, const Pl<2>& es,
                        const Pl<2>& ec) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            uint32_t y = rule32_total<RULE>(as.v[q], ac.v[q], s[i].v[q], c[i].v[q], es.v[q],
                                            ec.v[q], x[i].v[q], a.birth, a.survive);
            if constexpr (kBirths) y = lop3<kAnd3>(y, cm.v[q], rowm[i]);
            x[i].v[q] = y;
        }
    };
    // After generation g+1 of an epoch only rows [b0 - K + g + 1, b1 + K - g - 1)
    // of the held range are exact: this wave computes generation g+1 iff g < gmax
    // (the rows its neighbours would compute from it otherwise are discarded), and
    // once off it stays off for the rest of the epoch.
    const int32_t gmax = (int32_t)min<int64_t>(r0 + M - (b0 - a.K) - 1, b1 + a.K - 1 - r0);
    const bool has_up = wv > 0, has_dn = wv < W - 1;
    // the first / last wave waits on its own word (always current) instead
    uint32_t* const wait_up = has_up ? prog_bot + (wv - 1) * 64 : prog_top + wv * 64;
    uint32_t* const wait_dn = has_dn ? prog_top + (wv + 1) * 64 : prog_bot + wv * 64;
    uint32_t* const my_top = prog_top + wv * 64 + lane;
    uint32_t* const my_bot = prog_bot + wv * 64 + lane;
    auto word = [](uint32_t* p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto set_word = [&](uint32_t* p, uint32_t v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // spin until *p >= need (after a first read that came back short), then re-read
    // the edge: progress read before edge read, LDS in order per wave
    auto await = [&](uint32_t* p, uint32_t need, const uint4* pe, uint4& t) {
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
        t = *pe;
    };
#if GOL_EXP & 2048
    // dev timing build: per-wave cycles waiting for neighbour waves, in epoch
    // hand-offs, and in all (s_memtime), logged at the end
    uint64_t t_wait = 0, t_epoch = 0, t_beg = __builtin_amdgcn_s_memtime(), t_ep0 = 0;
    uint64_t t_pub = 0, t_flag = 0, t_x = 0;  // epoch pieces: publish + barrier, flag wait + barrier
#endif
    for (int32_t done = 0; done < a.gens;) {
        const int32_t k = min(a.K, a.gens - done);
#pragma unroll
        for (int i = 0; i < M; ++i) h3_row(x[i], s[i], c[i]);
        put_top(0);
        put_bot(0);
        // (a wave whose rows are never exact this epoch releases its neighbours now)
        set_word(my_top, (uint32_t)(gmax > 0 ? done : done + k));
        set_word(my_bot, (uint32_t)(gmax > 0 ? done : done + k));
        __syncthreads();
        // Generations: no workgroup barrier.  A wave's first row needs the upper
        // neighbour wave's bottom edge, its last row the lower neighbour's top edge;
        // each edge has its own progress word in LDS, and each of the wave's edge
        // rows is computed, its H3 published and its word raised as soon as the one
        // edge it needs is in, at raised priority (the neighbour waits for it); the
        // interior rows fill the LDS round trips.  So the chain across a wave seam
        // is one edge row per generation, and the waves of a SIMD drift apart.  LDS
        // executes a wave's accesses in order: edges are stored before their word
        // and read after it.  An edge slot is rewritten two generations later, after
        // the wave that reads it has raised the word it publishes after that read
        // (which this wave waits for before computing the row).
        // generation g of the epoch (g < gmax); `publish`: not the epoch's last
        auto generation = [&](int32_t g, bool publish) {
            const uint32_t need = (uint32_t)(done + g);
            const int p = g & 1, q = (g + 1) & 1;
            const uint4* pu = has_up ? ed4 + p * (2 * W * 64) + (W + wv - 1) * 64 + lane : zero4 + lane;
            const uint4* pd = has_dn ? ed4 + p * (2 * W * 64) + (wv + 1) * 64 + lane : zero4 + lane;
#if GOL_EXP & 2048
            const uint64_t tw0 = __builtin_amdgcn_s_memtime();
#endif
#if GOL_EXP & 4096
            // dev trace (tools/res_trace.py): shader-clock stamps per generation
            uint64_t ts[5];
            auto stamp = [&](int j) { ts[j] = __builtin_amdgcn_s_memtime(); };
            auto stamp_on = [&](int j, uint32_t& v) {
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
                ts[j] = __builtin_amdgcn_s_memtime();
            };
            stamp(0);
#endif
            const uint32_t wu = word(wait_up), wd = word(wait_dn);
            asm volatile("" ::: "memory");  // edge reads issue after the progress reads
            uint4 tu = *pu, td = *pd;
            // interior rows first: no LDS operand, they cover the round trip
            if constexpr (kPair) {
                pair_rows(0, pt);
                if constexpr (M > 2) pair_rows(M - 2, pb);
            }
#pragma unroll
            for (int i = 1; i < M - 1; ++i) {
                if (kPair && i == 1)
                    pair_row(1, pt, s[M > 2 ? 2 : 0], c[M > 2 ? 2 : 0]);
                else if (kPair && i == M - 2)
                    pair_row(M - 2, pb, s[M > 2 ? M - 3 : 0], c[M > 2 ? M - 3 : 0]);
                else
                    rule_row(i, s[i - 1], c[i - 1], s[i + 1], c[i + 1]);
                asm volatile("" : "+v"(x[i].v[0]), "+v"(x[i].v[1]));
            }
            __builtin_amdgcn_sched_barrier(0);
            if (__builtin_amdgcn_readfirstlane((int32_t)(wu - need)) < 0) await(wait_up, need, pu, tu);
#if GOL_EXP & 2048
            {
                uint32_t v = tu.x;
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
                t_wait += __builtin_amdgcn_s_memtime() - tw0;
                if (v == 0x5a5a5a5au) tu.y ^= 1u;  // keeps v live (never taken on real data)
            }
#endif
#if GOL_EXP & 4096
            stamp_on(1, tu.x);
#endif
            __builtin_amdgcn_s_setprio(2);
            Pl<2> us, uc;
            us.v[0] = tu.x; us.v[1] = tu.y; uc.v[0] = tu.z; uc.v[1] = tu.w;
            if constexpr (M == 1) {
                if (__builtin_amdgcn_readfirstlane((int32_t)(wd - need)) < 0) await(wait_dn, need, pd, td);
                Pl<2> ds, dc;
                ds.v[0] = td.x; ds.v[1] = td.y; dc.v[0] = td.z; dc.v[1] = td.w;
                rule_row(0, us, uc, ds, dc);  // (M = 1: no pair)
                if (publish) {
                    h3_row(x[0], s[0], c[0]);
                    put_top(q);
                    put_bot(q);
                    asm volatile("" ::: "memory");  // progress words after the edges
                    set_word(my_top, need + 1u);
                    set_word(my_bot, need + 1u);
                }
            } else {
                if constexpr (kPair)
                    pair_row(0, pt, us, uc);
                else
                    rule_row(0, us, uc, s[1], c[1]);
                // the last row's rule reads row M-2's H3 of this generation: with
                // M = 2 that is row 0's, about to be replaced
                const Pl<2> s_up = s[M - 2], c_up = c[M - 2];
                if (publish) {
                    h3_row(x[0], s[0], c[0]);
                    put_top(q);
                    asm volatile("" ::: "memory");  // progress word after the edge
                    set_word(my_top, need + 1u);
                }
#if GOL_EXP & 4096
                stamp(2);
#endif
                if (__builtin_amdgcn_readfirstlane((int32_t)(wd - need)) < 0) await(wait_dn, need, pd, td);
#if GOL_EXP & 4096
                stamp_on(3, td.x);
#endif
                Pl<2> ds, dc;
                ds.v[0] = td.x; ds.v[1] = td.y; dc.v[0] = td.z; dc.v[1] = td.w;
                if constexpr (kPair && M > 2)
                    pair_row(M - 1, pb, ds, dc);
                else if constexpr (kPair)
                    pair_row(M - 1, pt, ds, dc);
                else
                    rule_row(M - 1, s_up, c_up, ds, dc);
                if (publish) {
                    h3_row(x[M - 1], s[M - 1], c[M - 1]);
                    put_bot(q);
                    asm volatile("" ::: "memory");
                    set_word(my_bot, need + 1u);
                }
#if GOL_EXP & 4096
                stamp(4);
                // per-generation trace of the middle tile, generations 32..95
                const int32_t gg = done + g - 32;
                if (a.wlog && lane == 0 && tile == G / 2 && gg >= 0 && gg < 64) {
                    uint64_t* tl = a.wlog + 262144 + ((int64_t)wv * 64 + gg) * 8;
#pragma unroll
                    for (int j = 0; j < 5; ++j) tl[j] = ts[j];
                    tl[5] = (uint64_t)(uint32_t)gmax;
                }
#endif
            }
            __builtin_amdgcn_s_setprio(0);
            if (publish) {
#pragma unroll
                for (int i = 1; i < M - 1; ++i) h3_row(x[i], s[i], c[i]);
            }
        };
        // this wave computes generations [0, gend) of the epoch; the last one it
        // computes publishes its edges unless it is the epoch's last
        const int32_t gend = min(k, gmax);
        for (int32_t g = 0; g < gend - 1; ++g) generation(g, true);
        if (gend > 0) generation(gend - 1, gend < k);
        if (gend < k) {
            // off from here on: release the neighbours for the rest of the epoch
            set_word(my_top, (uint32_t)(done + k));
            set_word(my_bot, (uint32_t)(done + k));
        }
#if GOL_EXP & 2048
        t_ep0 = __builtin_amdgcn_s_memtime();
#endif
        done += k;
        ++epoch;
        // publish the band rows into the buffer of this epoch's result
        uint64_t* nb = (epoch & 1) ? a.buf1 : a.buf0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int64_t r = r0 + i;
            if (r >= b0 && r < b1 && st_lane)
                __hip_atomic_store(const_cast<uint64_t*>(row_ptr(nb, r)), words_of<2>(x[i]).w[0],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if GOL_EXP & 2048
        t_x = __builtin_amdgcn_s_memtime();
        t_pub += t_x - t_ep0;
#endif
        const uint32_t want = a.flag_base + epoch;
        if (threadIdx.x == 0)
            __hip_atomic_store(a.flags + tile, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done >= a.gens) break;
        // wait for the neighbours' rows of this epoch
        if (nb_tile >= 0 && !gave_up && !(GOL_EXP & 64)) {
            uint64_t t0 = 0;
            for (int n = 0; (int32_t)(__hip_atomic_load(a.flags + nb_tile, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) -
                                      want) < 0;
                 ++n) {
                if (n == 0) t0 = wait_clock();
                else if (wait_clock() - t0 > kWaitTicks) {  // the field is lost: flag it, stop waiting
                    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    gave_up = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
#if GOL_EXP & 2048
        t_flag += __builtin_amdgcn_s_memtime() - t_x;
#endif
        // reload the halo rows (all lanes) and the halo lanes of the band rows
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int64_t r = r0 + i;
            const bool own = r >= b0 && r < b1;
            if (!own || halo_lane) x[i] = fetch(nb, r);
        }
#if GOL_EXP & 2048
        {
            uint32_t v = x[0].v[0];
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(v));
            x[0].v[0] = v;
            t_epoch += __builtin_amdgcn_s_memtime() - t_ep0;
        }
#endif
    }
#if GOL_EXP & 2048
    if (a.wlog && lane == 0) {
        uint64_t* wl = a.wlog + ((int64_t)blockIdx.x * W + wv) * 8;
        wl[0] = __builtin_amdgcn_s_memtime() - t_beg;
        wl[1] = t_wait;
        wl[2] = t_epoch;
        wl[3] = (uint64_t)tile << 32 | (uint32_t)gmax;
        wl[4] = t_pub;
        wl[5] = t_flag;
    }
#endif
}

// Every tile waits for its neighbours, so all of them must be resident at once.
// The planner keeps the grid within the occupancy query x CUs (one tile per CU);
// with `coop`, hipLaunchCooperativeKernel checks it again at launch time against
// what the device can actually hold (CU masking, another process's kernels) and
// refuses (hipErrorCooperativeLaunchTooLarge, reported by gol_step) instead of
// letting queued tiles run the neighbours' bounded waits out -- at ~30 us per
// launch, so it is opt-in (engine.cpp Resident::coop).
template <int M, int RULE>
hipError_t launch_res_coop(const ResArgs& a, int grid, hipStream_t s, bool coop)
{
    if (!coop) {
        hipLaunchKernelGGL((life_res_kernel<M, RULE>), dim3(grid), dim3(64 * kResWaves), 0, s, a);
        return hipGetLastError();
    }
    ResArgs args = a;
    void* params[] = {&args};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&life_res_kernel<M, RULE>),
                                      dim3(grid), dim3(64 * kResWaves), params, 0, s);
}

template <int M>
hipError_t launch_res_m(const ResArgs& a, RuleKind rule, int grid, hipStream_t s, bool coop)
{
    switch (rule) {
    case RULE_REF: return launch_res_coop<M, RULE_REF>(a, grid, s, coop);
    case RULE_CONWAY: return launch_res_coop<M, RULE_CONWAY>(a, grid, s, coop);
    default: return launch_res_coop<M, RULE_GENERIC>(a, grid, s, coop);
    }
}

template <int M>
int occupancy_res_m(RuleKind rule)
{
    int n = 0;
    hipError_t e;
    switch (rule) {
    case RULE_REF: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_kernel<M, RULE_REF>, 64 * kResWaves, 0); break;
    case RULE_CONWAY: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_kernel<M, RULE_CONWAY>, 64 * kResWaves, 0); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, life_res_kernel<M, RULE_GENERIC>, 64 * kResWaves, 0); break;
    }
    return e == hipSuccess ? n : 0;
}

}  // namespace

hipError_t launch_resident(const ResArgs& a, int rows, RuleKind rule, int grid, hipStream_t s,
                           bool coop)
{
    switch (rows) {
    case 2: return launch_res_m<2>(a, rule, grid, s, coop);
    case 3: return launch_res_m<3>(a, rule, grid, s, coop);
    case 4: return launch_res_m<4>(a, rule, grid, s, coop);
    case 6: return launch_res_m<6>(a, rule, grid, s, coop);
    case 8: return launch_res_m<8>(a, rule, grid, s, coop);
    default: return hipErrorInvalidValue;
    }
}

int resident_blocks_per_cu(int rows, RuleKind rule)
{
    switch (rows) {
    case 2: return occupancy_res_m<2>(rule);
    case 3: return occupancy_res_m<3>(rule);
    case 4: return occupancy_res_m<4>(rule);
    case 6: return occupancy_res_m<6>(rule);
    case 8: return occupancy_res_m<8>(rule);
    default: return 0;
    }
}

}  // namespace gol
