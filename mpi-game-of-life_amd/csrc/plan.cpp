// plan.cpp -- launch planning of libgol.so's stencil launches
// (engine_internal.h): the segment tables of a launch, edge-aligned column strips
// and the packed half strip, rows per wavefront, age-skewed row blocks, the
// hand-off vs classic decision, the multi-pass switch (dev build) and the plan
// autotuner that times equally exact variants at create.
#include "engine_internal.h"

namespace golh __attribute__((visibility("hidden"))) {

int64_t plan_units(const std::vector<SegDesc>& segs, int32_t strips)
{
    int64_t u = 0;
    for (const auto& s : segs) u += s.nblk * strips;
    return u;
}

void finish_segs(std::vector<SegDesc>& segs, int64_t rpw, int32_t strips)
{
    int64_t unit = 0;
    for (auto& s : segs) {
        const int64_t n = std::max<int64_t>(0, s.out_hi - s.out_lo);
        s.nblk = (n + rpw - 1) / rpw;
        s.unit0 = unit;
        unit += s.nblk * strips;
    }
}

// 64-lane strips are edge-aligned (StepArgs::edge).  A lane whose neighbour lane
// is the DPP shift's zero (lane 0 / 63) or lies outside the field sees the dead
// border, so it is exact without a halo lane: strip 0 outputs groups 0..62, strip
// s >= 1 groups 62 s + 1 .. 62 s + 62 (lane 0 its halo), and a strip whose lane 63
// holds group ng - 1 outputs that too.  A row of ng groups takes 1 + ceil((ng -
// 64) / 62) strips (4096 columns: 1; with a halo lane at both ends: 2).  With the
// packed half strip (one-segment plans) the last strip is right-aligned (lane 63 =
// group ng - 1) and the gap of <= 30 groups between it and the strips before it is
// a 32-lane half strip whose units run two row blocks each: a 65536-column row
// costs 16.5 wavefronts per row block instead of 17 (262144 columns: 66.5, not 67).
struct ColLayout {
    int32_t strips = 0;
    int64_t right_q0 = -1, half_q0 = 0, half_hi = -1;
    bool half() const { return half_hi > half_q0; }
};

ColLayout col_layout(int64_t ng, bool allow_half)
{
    ColLayout c;
    c.strips = 1;
    if (ng <= 64) return c;
    const int64_t s0 = 1 + (ng - 64 + 61) / 62;
    const int64_t S = s0 - 1, gap = ng - 126 - 62 * (S - 2);
    c.strips = (int32_t)s0;
    if (allow_half && S >= 2 && gap >= 1 && gap <= 30) {
        c.strips = (int32_t)S;
        c.right_q0 = ng - 64;
        c.half_q0 = 62 * (S - 1);
        c.half_hi = c.half_q0 + gap;
    }
    return c;
}

// Strip groups per row block for strips of 64 >> shift lanes (shift 0: edge-aligned,
// with the packed half strip if `half`).
int32_t strip_groups(uint64_t wq, int shift, bool half = false)
{
    if (shift == 0) return col_layout((int64_t)wq, half).strips;
    const uint64_t out = (uint64_t)((64 >> shift) - 2);
    const uint64_t strips = (wq + out - 1) / out;
    const uint64_t per = 1ull << shift;
    return (int32_t)((strips + per - 1) / per);
}

// Rows per block of the half strip's units (classic closure) for a plan whose
// blocks have R rows: as long as the plan's blocks by the cost models below
// (classic R + K + 4; hand-off 1.02 R + 10).
// Under hand-off blocks the half strip's classic blocks get 0.8 of that: the
// classic cost model undercounts short classic blocks (A/B of the scale, one
// process: 8448 rows 111.2 without the half strip, 115.5-116.7 with it at 0.7-0.9
// (109.9 at 1.0); 12288: 117.2 vs 123.5-124.6 (119.5 at 1.0);
// profiles/r03/ab_half_strip_handoff_scale*.jsonl).  GOL_DEV_HALF_SCALE overrides
// it (dev A/B).
constexpr double kHalfHandScale = 0.8;

int64_t half_rows_for(int64_t R, bool hand, int K)
{
    if (!hand) return R;
    double f = kHalfHandScale;
    if (const char* v = std::getenv("GOL_DEV_HALF_SCALE")) f = std::atof(v);
    return std::max<int64_t>(1, (int64_t)(f * (double)((int64_t)(1.02 * (double)R + 10.0) - K - 4)));
}

// The packed half strip's units of a one-segment plan.  Its column is cut into row
// blocks of Rp rows from out_lo; two consecutive blocks share a wavefront (lanes
// 0-31 / 32-63) when they have the same length, every row they stream (with the
// prefetch overrun) and every row mask they compute lies inside the buffer and the
// field (the kernel takes the first block's row validity for both), and the second
// block's row offset fits the 32-bit lane offset.  Other blocks run alone in lanes
// 0-31.  Returns the unit count; `out` gets (first row A, first row B or -1, rows)
// per unit.
int64_t half_units(const SegDesc& sg, int64_t Rp, int K, int planes, int64_t stride,
                   std::vector<int64_t>* out)
{
    if (out) out->clear();
    const int64_t lo = sg.out_lo, hi = sg.out_hi;
    if (hi <= lo) return 0;
    Rp = std::max<int64_t>(1, Rp);
    const int64_t pf = gol::prefetch_of(K, planes);
    auto interior = [&](int64_t rb, int64_t re) {
        return rb - K >= 0 && sg.glob0 + rb >= 2 * (int64_t)K && re + K + pf <= sg.in_rows &&
               sg.glob0 + re + K + 2 * pf <= sg.field_h;
    };
    int64_t units = 0;
    for (int64_t rb = lo; rb < hi; ++units) {
        const int64_t la = std::min(Rp, hi - rb), rb2 = rb + la;
        const int64_t lb = std::min(Rp, hi - rb2);
        const bool pair = rb2 < hi && la == lb && interior(rb, rb2) && interior(rb2, rb2 + lb) &&
                          (la + 1) * stride * 8 < (int64_t(1) << 31);
        if (out) {
            out->push_back(rb);
            out->push_back(pair ? rb2 : -1);
            out->push_back(la);
        }
        rb = pair ? rb2 + lb : rb2;
    }
    return units;
}

// Hand-off constraint on the rows per wavefront R of a launch of depth d
// (gol::handoff_toff): a consumer block streams R + 2 input rows, kernels exist
// for two or three alignments of that count to the prefetch blocks, and the refill that
// first fetches side rows (the flag wait sits in front of it) must come after the
// unrolled warm-up blocks.
bool handoff_fits(int64_t R, int d, int planes) { return gol::handoff_toff(R, d, planes) >= 0; }

// Rows per wavefront and strip width for one launch plan.  Every wavefront of
// a launch does about the same work, so the launch time is set by the most
// loaded SIMD: n = ceil(units / SIMDs) wavefronts run in rounds of `occ`
// resident ones, and a partial round of m wavefronts still costs max(2, m) issue
// slots per instruction (one wavefront alone issues at half the SIMD's VALU rate).
// A wavefront's time in rows of K stage-steps: classic blocks R + K + 1 (+ c0
// fixed); hand-off blocks skip the K - 1 rows of vertical halo, pay their signal,
// wait and side-row blocks: 1.02 R + 10, fitted at K = 16 to the in-process A/B
// of profiles/r02/ab_handoff_hybrid.jsonl (hand-off 9% faster at 8448 rows, 5% at
// 16640, 1% at 33024 and 65536 -- the hot loop is the classic one since the
// side-row refills were peeled off it).  Measured
// (profiles/r01/sweep_rows_per_wave*.jsonl): keeping fewer than `occ`
// wavefronts per SIMD all launch long is 5-10% slower than the model says, so R
// is restricted to n >= occ whenever the field is large enough.  Narrower strips
// (32 or 16 lanes, 2 or 4 per wavefront) multiply the units per row block, so
// short stripes reach `occ` with longer row blocks.
struct RowPlan {
    int64_t rpw;
    int32_t groups, lane_shift;
    bool hand;
};

RowPlan pick_rows_per_wave(const std::vector<SegDesc>& segs, uint64_t wq, int K, int planes,
                           int occ_classic, int occ_hand, int simds, int force_rpw,
                           int force_shift, uint32_t handoff, int64_t half_stride = 0)
{
    const int64_t c0 = 3;  // per-wavefront fixed cost, in rows
    int64_t maxrows = 1;
    for (const auto& s : segs) maxrows = std::max<int64_t>(maxrows, s.out_hi - s.out_lo);
    // the packed half strip (half_stride = the buffer's row stride; 0 = off)
    const bool half = half_stride > 0 && segs.size() == 1 && col_layout((int64_t)wq, true).half();
    // best [hand][filled]: filled = at least `occ` wavefronts per SIMD
    RowPlan best_p[2][2];
    double best[2][2] = {{1e300, 1e300}, {1e300, 1e300}};
    for (int hand = 0; hand <= 1; ++hand) {
        best_p[hand][0] = best_p[hand][1] = {16, strip_groups(wq, 0), 0, hand != 0};
        if (hand && (handoff == 1 || K < gol::kHandoffMinDepth)) continue;
        const int occ = std::max(1, hand ? occ_hand : occ_classic);
        for (int shift = 0; shift <= 2; ++shift) {
            if (force_shift >= 0 && shift != force_shift) continue;
            const bool hs = half && shift == 0;
            const int32_t groups = strip_groups(wq, shift, hs);
            const int64_t r_lo = force_rpw ? force_rpw : std::max<int64_t>(8, K + 2);
            const int64_t r_hi =
                force_rpw ? force_rpw : std::max<int64_t>(r_lo, std::min<int64_t>(1024, maxrows + K));
            for (int64_t R = r_lo; R <= r_hi; ++R) {
                if (hand && !handoff_fits(R, K, planes)) continue;
                int64_t units = 0, blocks_max = 0;
                for (const auto& sg : segs) {
                    const int64_t nb = (std::max<int64_t>(0, sg.out_hi - sg.out_lo) + R - 1) / R;
                    units += groups * nb;
                    if (hs)
                        units += half_units(sg, half_rows_for(R, hand != 0, K), K, planes, half_stride,
                                            nullptr);
                    blocks_max = std::max(blocks_max, nb);
                }
                if (hand && blocks_max < 2) continue;  // nothing to hand over
                const int64_t n = (units + simds - 1) / simds;
                // hand-off blocks wait for other wavefronts of their launch: only
                // launches of one round (every wavefront resident at once, so a
                // producer never queues behind the consumers waiting for it)
                if (hand && n > occ) continue;
                const int64_t full = n / occ, rem = n % occ;
                const double slots =
                    (double)full * std::max(2, occ) + (rem ? (double)std::max<int64_t>(2, rem) : 0.0);
                const double rows = hand ? 1.02 * (double)R + 10.0 : (double)(R + K + 1 + c0);
                const double cost = slots * rows;
                const int filled = n >= occ ? 1 : 0;
                if (cost < best[hand][filled] * 0.999) {
                    best[hand][filled] = cost;
                    best_p[hand][filled] = {R, groups, shift, hand != 0};
                }
            }
        }
    }
    // per kind: a plan that fills the SIMDs if there is one
    const int fc = best[0][1] < 1e300 ? 1 : 0, fh = best[1][1] < 1e300 ? 1 : 0;
    const bool have_hand = best[1][fh] < 1e300;
    if (handoff == 2 && have_hand) return best_p[1][fh];
    if (handoff == 1 || !have_hand) return best_p[0][fc];
    // auto: the cheaper, preferring plans that fill the SIMDs
    if (fh != fc) return fh > fc ? best_p[1][fh] : best_p[0][fc];
    return best[1][fh] <= best[0][fc] ? best_p[1][fh] : best_p[0][fc];
}

// Age-skewed row blocks.  A launch of one round at 2 wavefronts per SIMD first
// gives every CU one workgroup, then a second: on each SIMD the wave of the first
// workgroup (unit < 4 x CUs) is the older one and wins the VALU arbitration by age
// (MI355X_MICROARCH.md, two waves per SIMD, item 2), so with equal blocks it ends
// at ~0.82 of the launch and its partner finishes alone at half the SIMD's issue
// rate (tools/wave_log.py: 69.8 vs 84.3 us at 8448 x 65536, 241 vs 295 us at
// 33024; profiles/r02/wave_log_*.jsonl).  Balancing the pair by priority instead
// (s_setprio flips, closed loop) was measured 9-10% slower.  So the older units
// get longer blocks: the bottom blocks of each strip whose units are < units_old
// have rows_old rows, the others rows_young, with the young/old rate ratio rho of
// the block kind (kAgeRate*; the in-process A/B optimum, profiles/r02/ab_skew*.jsonl).
// GOL_DEV_AGE_SKEW overrides rho (dev A/B; 0 turns the skew off),
// GOL_DEV_AGE_SKEW_HAND the hand-off blocks' rho only.
constexpr double kAgeRateHand = 0.78, kAgeRateClassic = 0.72;

constexpr double kHandSkewCost = 1.05;
// Young block length from which skewed classic blocks are preferred to hand-off
// blocks when both run the packed half strip (build_plans).
constexpr int64_t kHalfClassicRows = 160;

struct Skew {
    int64_t rows_old = 0, rows_young = 0, nblk = 0;  // rows_old 0 = no skew
    double t = 0;  // modelled launch time, in rows of the kernel kind's cost
};

Skew age_skew(const SegDesc& sg, int64_t R, int32_t strips, int64_t units_old, int occ, int K,
              int planes, bool hand, int64_t max_units = INT64_MAX, int64_t half_stride = 0,
              double rho_mult = 1.0)
{
    Skew best_s;
    double rho = hand ? kAgeRateHand : kAgeRateClassic;
    if (const char* v = std::getenv("GOL_DEV_AGE_SKEW")) rho = std::atof(v);
    if (hand)
        if (const char* v = std::getenv("GOL_DEV_AGE_SKEW_HAND")) rho = std::atof(v);
    rho *= rho_mult;
    const int64_t rows = sg.out_hi - sg.out_lo;
    if (rho <= 0 || rho >= 1 || occ != 2 || rows <= 0) return best_s;
    const int pf = gol::prefetch_of(K, planes);
    auto cost = [&](int64_t r) { return hand ? 1.02 * (double)r + 10.0 : (double)(r + K + 4); };
    auto fits = [&](int64_t r) { return r >= std::max(8, K + 2) && (!hand || handoff_fits(r, K, planes)); };
    // the packed half strip's units (half_stride > 0) come after the full strips':
    // young waves, with blocks as long as the young blocks
    auto half_n = [&](int64_t ry) {
        return half_stride > 0 ? half_units(sg, half_rows_for(ry, hand, K), K, planes, half_stride, nullptr)
                               : (int64_t)0;
    };
    // the planned equal blocks: nw wavefronts per SIMD run as pairs (old rate 1,
    // young rho) with refills, and the last pair's young wave ends alone
    const int64_t nb0 = (rows + R - 1) / R;
    const double nw = std::ceil((double)(nb0 * strips + half_n(R)) / (double)units_old);
    double best = std::max(0.0, nw - 2) * cost(R) / (1 + rho) + cost(R) / rho;
    // Lengths step: hand-off blocks keep both lengths in one class mod the
    // prefetch block (one tail offset per launch: R + 2c, the classes whose
    // offset has a kernel pass `fits`), classic ones take any length.
    const int step = hand ? pf : 1;
    // every block count of one round of more than units_old (= one per SIMD)
    // wavefronts: the old blocks from the mean length to twice it
    for (int64_t nblk = std::max<int64_t>(2, units_old / strips + 1);
         nblk * strips <= std::min(2 * units_old, max_units); ++nblk) {
        const int64_t units = nblk * strips;
        if (units <= units_old) continue;
        const int64_t mean = (rows + nblk - 1) / nblk;
        auto jold = [&](int64_t s) {
            return std::min<int64_t>(nblk, std::max<int64_t>(0, (units_old - s + strips - 1) / strips));
        };
        // at most ~256 old lengths per block count (long blocks step coarser), so
        // that plan building stays fast for tall fields and many rank plans
        const int64_t stride = step * std::max<int64_t>(1, mean / (256 * step));
        for (int cls = 0; cls < (hand ? pf / 2 : 1); ++cls)
        for (int64_t ro = mean + ((R + 2 * cls - mean) % step + step) % step;
             ro <= 2 * mean + pf; ro += stride) {
            // the young length: the least in ro's class mod step that covers every
            // strip
            int64_t ry = 1;
            bool ok = true;
            for (int64_t s = 0; s < strips && ok; ++s) {
                const int64_t jo = jold(s), ny = nblk - jo;
                if (ny == 0)
                    ok = jo * ro >= rows;
                else
                    ry = std::max<int64_t>(ry, (rows - jo * ro + ny - 1) / ny);
            }
            if (!ok) continue;
            ry += ((ro - ry) % step + step) % step;
            if (ry >= ro || !fits(ry) || !fits(ro)) continue;
            // every strip's blocks cover the rows and its last block is not empty
            for (int64_t s = 0; s < strips && ok; ++s) {
                const int64_t jo = jold(s), ny = nblk - jo;
                const int64_t total = ny * ry + jo * ro, last = jo ? ro : ry;
                ok = total >= rows && total - last < rows;
            }
            if (!ok) continue;
            const double t = std::max(cost(ro), cost(ry) / rho);
            if (t < best * 0.995 &&
                (half_stride <= 0 || units + half_n(ry) <= std::min(2 * units_old, max_units))) {
                best = t;
                best_s = {ro, ry, nblk, t};
            }
        }
    }
    return best_s;
}

// Whether a single-stream GLOBAL engine of this field would run age-skewed
// one-round launches (build_plans' choice, without allocating it).  gol_create
// then prefers it to the composite engine: 65536^2 ran 133.6 TCUPS on one stream
// with skewed blocks against 130.6 as 2 same-device stripes (profiles/r02/
// ab_skew_single_vs_composite.jsonl) -- the skew hides the pair tails that the
// second stream's launches otherwise fill.
bool single_stream_skews(uint64_t h, uint64_t w, const gol_config* cfg)
{
    if (cfg->rows_per_wave || h > (uint64_t)INT32_MAX) return false;
    const Layout lay = auto_layout(h, cfg);
    const int K = (int)lay.K, planes = lay.planes;
    if (!gol::life_has_kernel(K, planes)) return false;
    gol::RuleKind rule = gol::RULE_GENERIC;
    if (cfg->birth_mask == GOL_REF_BIRTH && cfg->survive_mask == GOL_REF_SURVIVE)
        rule = gol::RULE_REF;
    else if (cfg->birth_mask == GOL_CONWAY_BIRTH && cfg->survive_mask == GOL_CONWAY_SURVIVE)
        rule = gol::RULE_CONWAY;
    int dev = cfg->device, cus = 0;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    const uint64_t wq = (w + 63) / 64, G = (uint64_t)planes / 2, ng = (wq + G - 1) / G;
    const int shift = cfg->strip_lanes == 64 ? 0 : cfg->strip_lanes == 32 ? 1
                    : cfg->strip_lanes == 16 ? 2 : -1;
    const bool hand_ok = gol::handoff_kernel_exists(K, rule);
    const int occ_c = gol::life_blocks_per_cu(K, rule, planes, false);
    const int occ_h = hand_ok ? gol::life_blocks_per_cu(K, rule, planes, true) : 0;
    SegDesc s{};
    s.in_rows = s.field_h = s.out_hi = (int64_t)h;
    const char* dev_pairs = std::getenv("GOL_DEV_PAIRS");
    const int64_t hs =
        (dev_pairs && std::atoi(dev_pairs) == 0) || h >= (1ull << 30) ? 0 : (int64_t)(ng * G);
    for (int hand = 0; hand <= 1; ++hand) {
        if ((hand && (cfg->handoff == 1 || !hand_ok)) || (!hand && cfg->handoff == 2)) continue;
        const RowPlan rp = pick_rows_per_wave({s}, ng, K, planes, occ_c, occ_h, 4 * cus, 0, shift,
                                              hand ? 2u : 1u, hs);
        if (rp.hand != (hand != 0)) continue;
        std::vector<SegDesc> segs{s};
        finish_segs(segs, rp.rpw, rp.groups);
        if (age_skew(segs[0], rp.rpw, rp.groups, (int64_t)gol::kWavesPerBlock * cus,
                     hand ? occ_h : occ_c, K, planes, hand != 0, INT64_MAX,
                     rp.lane_shift == 0 ? hs : 0)
                .rows_old)
            return true;
    }
    return false;
}

// Autotuner variants of a full-depth plan (build_plans, autotune_plans), in the
// order build_plans makes them; gol_plan_tuning reports 1 + the index.
constexpr int kTuneVariants = 4;
constexpr const char* kTuneVariantNames[kTuneVariants] = {"no_half_strip", "skew_0.95",
                                                          "skew_1.05", "other_block_kind"};

void free_plan(gol_engine::Plan& q)
{
    if (q.alias) return;  // the owner's tables
    if (q.dev) (void)hipFree(q.dev);
    if (q.dpairs) (void)hipFree(q.dpairs);
    q.dev = nullptr;
    q.dpairs = nullptr;
}

gol_status build_plans(gol_engine* e, const std::vector<std::vector<SegDesc>>& raw)
{
    int cus = 0, occ_c = 0, occ_h = 0;
    if (e->model.on) {
        cus = e->model.cus;
        occ_c = e->model.occ_c;
        occ_h = e->K >= (uint32_t)gol::kHandoffMinDepth ? e->model.occ_h : 0;
    } else {
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device));
        occ_c = gol::life_blocks_per_cu((int)e->K, e->rule, e->planes, false);
        occ_h = e->K >= (uint32_t)gol::kHandoffMinDepth
                    ? gol::life_blocks_per_cu((int)e->K, e->rule, e->planes, true)
                    : 0;
    }
    // occupancy of the multi-pass kernels (their register use may differ)
    int occ_mp_c = occ_c, occ_mp_h = occ_h;
    if (e->npass > 1 && !e->model.on) {
        occ_mp_c = gol::life_blocks_per_cu((int)e->K, e->rule, e->planes, false, true);
        occ_mp_h = occ_h ? gol::life_blocks_per_cu((int)e->K, e->rule, e->planes, true, true) : 0;
    }
    int64_t max_units = 0;
    bool any_hand = false, any_mp = false;
    // the packed half strip of one-segment plans (col_layout; GOL_DEV_PAIRS=0 turns
    // it off for A/B): the planners count its units
    // (the kernel reads the half strip's row numbers as 32-bit: buffers up to 2^30 rows)
    const char* dev_pairs = std::getenv("GOL_DEV_PAIRS");
    // (multi-pass launches run no half strip: its pair units close their blocks
    // the classic way and have no pass protocol)
    const int64_t hs = (dev_pairs && std::atoi(dev_pairs) == 0) || e->buf_rows >= (1ull << 30) ||
                               e->npass > 1
                           ? 0
                           : (int64_t)e->stride;
    auto units_of = [&](const std::vector<SegDesc>& segs, int32_t groups, int shift, int64_t R,
                        bool hand, int64_t hs_v) {
        int64_t u = plan_units(segs, groups);
        if (hs_v && shift == 0 && segs.size() == 1 && col_layout((int64_t)e->ng, true).half())
            u += half_units(segs[0], half_rows_for(R, hand, (int)e->K), (int)e->K, e->planes, hs_v,
                            nullptr);
        return u;
    };
    // hand-off or classic blocks for the whole engine, decided on its widest plan
    // (all launches of a step then share one kernel kind; a plan where hand-off
    // does not fit still falls back to classic blocks)
    uint32_t handoff = e->handoff;
    if (!gol::handoff_kernel_exists((int)e->K, e->rule)) handoff = 1;
    if (handoff == 0 && !raw.empty())
        handoff = pick_rows_per_wave(raw[0], e->ng, (int)e->K, e->planes, occ_c, occ_h, 4 * cus,
                                     (int)e->rows_per_wave, e->lane_shift, 0, hs)
                          .hand
                      ? 2
                      : 1;
    // With age-skewed blocks both kinds gain, classic blocks more (their halo
    // recompute is per block, and the old units' longer blocks amortize it): per
    // modelled row a skewed hand-off launch ran ~5% slower than a skewed classic one
    // at the per-GPU shapes 8448..33024 x 65536 (profiles/r02/ab_skew.jsonl), which
    // puts the crossover between 16640 rows (hand-off) and 33024 (classic).  When
    // both kinds skew, the modelled times decide -- except where the packed half
    // strip applies: then classic blocks win once their young blocks reach
    // kHalfClassicRows (profiles/r03/ab_half_strip_handoff_scale_sweep.jsonl, TCUPS,
    // hand-off vs classic, both with the half strip: 8448 rows 116.7 vs 104.8, 12288
    // 124.1 vs 119.0, 16640 124.5-126.7 vs 124.3 (classic young blocks 109 rows),
    // 33024 128.1 vs 130.4 (220)), which the row-cost models do not resolve.
    if (e->handoff == 0 && handoff == 2 && raw.size() >= 1 && raw[0].size() == 1 &&
        !e->rows_per_wave && !e->shared_device) {
        const int64_t first = (int64_t)gol::kWavesPerBlock * cus;
        Skew sk[2];
        for (int hand = 0; hand <= 1; ++hand) {
            const RowPlan rp = pick_rows_per_wave(raw[0], e->ng, (int)e->K, e->planes, occ_c, occ_h,
                                                  4 * cus, 0, e->lane_shift, hand ? 2u : 1u, hs);
            if (rp.hand != (hand != 0)) break;
            std::vector<SegDesc> segs = raw[0];
            finish_segs(segs, rp.rpw, rp.groups);
            sk[hand] = age_skew(segs[0], rp.rpw, rp.groups, first, hand ? occ_h : occ_c, (int)e->K,
                                e->planes, hand != 0, INT64_MAX, rp.lane_shift == 0 ? hs : 0);
        }
        if (hs && col_layout((int64_t)e->ng, true).half()) {
            if (sk[0].rows_old && (!sk[1].rows_old || sk[0].rows_young >= kHalfClassicRows))
                handoff = 1;
        } else if (sk[0].rows_old && (!sk[1].rows_old || sk[0].t < sk[1].t * kHandSkewCost)) {
            handoff = 1;
        }
    }
    // One launch plan for raw plan pi into p: hs_v the half strip's row stride (0 =
    // none), rho_mult scales the skew's young/old rate, kind the engine's block
    // kind (1 classic, 2 hand-off).  The autotuner's variants come from here too.
    auto build_one = [&](size_t pi, int64_t hs_v, double rho_mult, uint32_t kind,
                         gol_engine::Plan& p) -> gol_status {
        const auto& r = raw[pi];
        p.segs = r;
        // the band launch runs beside the interior launch: classic blocks, so that
        // at most one launch that waits for its own wavefronts runs at a time
        const bool band = e->band_plans && pi == (size_t)e->Hx;
        const bool inner = e->band_plans && pi == (size_t)e->Hx + 1;
        const RowPlan rp = pick_rows_per_wave(r, e->ng, (int)e->K, e->planes, occ_c, occ_h, 4 * cus,
                                              (int)e->rows_per_wave, e->lane_shift,
                                              band ? 1u : kind, hs_v);
        p.rpw = rp.rpw;
        p.groups = rp.groups;
        p.lane_shift = rp.lane_shift;
        p.hand = rp.hand;
        // Overlapped rounds (rank engines / groups alone on their device): the band
        // launch must find free wavefront slots beside the interior launch, or it
        // runs after it and the exchange waits.  The band's blocks are
        // sized so that its single waves end well inside the interior launch (about
        // 60% of the full launch's per-wave cost, at the young rate), and the
        // interior launch leaves the band's slots free.
        const int64_t slots_first = (int64_t)gol::kWavesPerBlock * cus;  // one workgroup per CU
        if (band && !e->rows_per_wave && !e->shared_device && e->Hx >= 1) {
            const auto& full = e->plans[e->Hx - 1];
            const double cf = full.hand ? 1.02 * (double)full.rpw + 10.0
                                        : (double)(full.rpw + e->K + 4);
            const int64_t rb = (int64_t)(0.6 * cf * kAgeRateClassic) - (int64_t)e->K - 4;
            p.rpw = std::max<int64_t>(std::max<int64_t>(8, e->K + 2), std::min<int64_t>(rb, (int64_t)e->Hx));
            p.hand = false;
        }
        finish_segs(p.segs, p.rpw, p.groups);
        p.total_units = units_of(p.segs, p.groups, p.lane_shift, p.rpw, p.hand, hs_v);
        int64_t cap = INT64_MAX;
        if (inner && !e->rows_per_wave && !e->shared_device) {
            const int occ = p.hand ? occ_h : occ_c;
            cap = (int64_t)occ * slots_first - e->plans[e->Hx].total_units;
            if (cap > slots_first && p.total_units > cap) {
                int64_t R = p.rpw;
                std::vector<SegDesc> segs = p.segs;
                do {
                    ++R;
                    if (p.hand && !handoff_fits(R, (int)e->K, e->planes)) continue;
                    finish_segs(segs, R, p.groups);
                } while (units_of(segs, p.groups, p.lane_shift, R, p.hand, hs_v) > cap && R < 4096);
                p.rpw = R;
                p.segs = segs;
                p.total_units = units_of(p.segs, p.groups, p.lane_shift, p.rpw, p.hand, hs_v);
            }
        }
        if (!band && p.segs.size() == 1 && !e->rows_per_wave && !e->shared_device) {
            const int occ = p.hand ? occ_h : occ_c;
            const int64_t first = slots_first;
            Skew sk = age_skew(p.segs[0], p.rpw, p.groups, first, occ, (int)e->K, e->planes,
                               p.hand, cap, p.lane_shift == 0 ? hs_v : 0, rho_mult);
            // Auto block kind, per plan: hand-off lengths are confined to two classes
            // mod the prefetch block, which can leave a launch without a close
            // one-round fit (8416 rows in 113 blocks of 86/62 rows: 90 vs 77 us); a
            // skewed classic plan is taken when the model says it is faster.
            if (p.hand && e->handoff == 0 && kind == handoff) {
                const RowPlan rc = pick_rows_per_wave(r, e->ng, (int)e->K, e->planes, occ_c, occ_h,
                                                      4 * cus, 0, e->lane_shift, 1u, hs_v);
                std::vector<SegDesc> cs = r;
                finish_segs(cs, rc.rpw, rc.groups);
                const Skew skc = age_skew(cs[0], rc.rpw, rc.groups, first, occ_c, (int)e->K,
                                          e->planes, false, cap, rc.lane_shift == 0 ? hs_v : 0,
                                          rho_mult);
                if (!rc.hand && skc.rows_old &&
                    (!sk.rows_old || skc.t < sk.t * kHandSkewCost)) {
                    p.hand = false;
                    p.rpw = rc.rpw;
                    p.groups = rc.groups;
                    p.lane_shift = rc.lane_shift;
                    p.segs = cs;
                    sk = skc;
                }
            }
            if (sk.rows_old) {
                p.rows_young = (int32_t)sk.rows_young;
                p.rows_old = (int32_t)sk.rows_old;
                p.units_old = (int32_t)first;
                p.segs[0].nblk = sk.nblk;
                p.total_units = plan_units(p.segs, p.groups);
                // the launch's hand-off tail offset follows the lengths' class
                p.rpw = sk.rows_young;
            }
        }
        // 64-lane strips: edge-aligned columns; one-segment plans also pack the
        // half strip into units after the full strips' (young waves, blocks as long
        // as the young ones)
        if (p.lane_shift == 0) {
            const ColLayout cl = col_layout((int64_t)e->ng, hs_v && p.segs.size() == 1);
            p.edge = 1;
            if (p.groups != cl.strips) {  // a planner's fallback plan: equal blocks
                p.groups = cl.strips;
                p.rows_old = p.rows_young = p.units_old = 0;
                finish_segs(p.segs, p.rpw, p.groups);
            }
            p.total_units = plan_units(p.segs, p.groups);
            if (cl.half()) {
                p.right_q0 = cl.right_q0;
                p.half_q0 = cl.half_q0;
                p.half_hi = cl.half_hi;
                p.half_rows = half_rows_for(p.rpw, p.hand, (int)e->K);
                p.pair_units = half_units(p.segs[0], p.half_rows, (int)e->K, e->planes, hs_v,
                                          &p.pairs);
                p.total_units += p.pair_units;
                if (!e->model.on) {
                    HIP_TRY(hipMalloc(&p.dpairs, sizeof(int64_t) * p.pairs.size()));
                    HIP_TRY(hipMemcpy(p.dpairs, p.pairs.data(), sizeof(int64_t) * p.pairs.size(),
                                      hipMemcpyHostToDevice));
                }
            }
        }
        for (const auto& sg : p.segs) {
            p.multi_blk |= sg.nblk > 1;
            // own rows of a segment: rank engines [Hx, Hx+R); REF_STRIPES the
            // rank's output rows; GLOBAL all rows
            int64_t olo = sg.out_lo, ohi = sg.out_hi;
            if (e->nranks > 1) {
                olo = std::max<int64_t>(olo, (int64_t)e->Hx);
                ohi = std::min<int64_t>(ohi, (int64_t)(e->Hx + e->R));
            } else if (e->sem == GOL_SEM_REF_STRIPES) {
                for (const auto& ur : e->user_regions)
                    if ((int64_t)ur.buf_row >= sg.base_row &&
                        (int64_t)ur.buf_row < sg.base_row + sg.in_rows) {
                        olo = std::max<int64_t>(olo, (int64_t)ur.buf_row - sg.base_row);
                        ohi = std::min<int64_t>(ohi, (int64_t)(ur.buf_row + ur.rows) - sg.base_row);
                    }
            }
            p.own_rows += (double)std::max<int64_t>(0, ohi - olo);
        }
        // Multi-pass launches: every wavefront waits for its row neighbours between
        // passes, so the plan must be one round of the occupancy (all units resident)
        {
            const int occ = std::min(p.hand ? occ_h : occ_c, p.hand ? occ_mp_h : occ_mp_c);
            p.npass = e->npass > 1 && !band && !inner && p.segs.size() == 1 && !p.pair_units &&
                              p.total_units <= (int64_t)occ * slots_first
                          ? (int32_t)e->npass
                          : 1;
        }
        max_units = std::max(max_units, p.total_units);
        any_hand |= p.hand && p.multi_blk;
        any_mp |= p.npass > 1;
        if (std::getenv("GOL_DEV_PLANS"))  // dev: the launch plans as built
            std::fprintf(stderr, "plan %zu: rows [%lld, %lld) x %zu segs, R %lld, strips %d, units %lld, "
                         "hand %d, skew %d/%d, half-strip units %lld (rows %lld)\n", pi,
                         (long long)p.segs[0].out_lo, (long long)p.segs[0].out_hi, p.segs.size(),
                         (long long)p.rpw, p.groups, (long long)p.total_units, (int)p.hand,
                         p.rows_old, p.rows_young, (long long)p.pair_units, (long long)p.half_rows);
        // device segment table: + the half strip's one-block segment (StepArgs::pairs)
        std::vector<SegDesc> dsegs = p.segs;
        if (p.pair_units) {
            SegDesc hs_seg = p.segs[0];
            hs_seg.nblk = 1;
            hs_seg.unit0 = p.total_units - p.pair_units;
            dsegs.push_back(hs_seg);
        }
        if (e->model.on) return GOL_OK;
        HIP_TRY(hipMalloc(&p.dev, sizeof(SegDesc) * dsegs.size()));
        HIP_TRY(hipMemcpy(p.dev, dsegs.data(), sizeof(SegDesc) * dsegs.size(),
                          hipMemcpyHostToDevice));
        return GOL_OK;
    };
    // Autotuner candidates (autotune_plans): for the plans of full-depth launches of
    // an engine alone on its device, variants the row-cost models rank within their
    // error -- without the half strip, the skew rate x 0.95 / 1.05, the other block
    // kind -- are timed on the GPU after planning, and the fastest stays.
    // GOL_DEV_AUTOTUNE=0 keeps the models' plans.
    const char* dev_tune = std::getenv("GOL_DEV_AUTOTUNE");
    const bool tune = !(dev_tune && std::atoi(dev_tune) == 0) && !e->rows_per_wave &&
                      !e->shared_device;
    auto same_plan = [](const gol_engine::Plan& a, const gol_engine::Plan& b) {
        return a.hand == b.hand && a.rpw == b.rpw && a.rows_old == b.rows_old &&
               a.rows_young == b.rows_young && a.groups == b.groups &&
               a.pair_units == b.pair_units && a.segs[0].nblk == b.segs[0].nblk;
    };
    // GOL_DEV_PLAN_VARIANT=<name> (tests/test_gpu_autotune.py): every full-depth plan
    // that has the named autotuner variant runs it instead of the models' plan,
    // without timing -- so each plan kind the autotuner can pick is pinned against
    // the oracle at the shapes where it appears.
    int forced = 0;
    if (const char* fv = std::getenv("GOL_DEV_PLAN_VARIANT")) {
        for (int i = 0; i < kTuneVariants; ++i)
            if (std::strcmp(fv, kTuneVariantNames[i]) == 0) forced = i + 1;
        if (!forced) return fail(GOL_EINVAL, std::string("GOL_DEV_PLAN_VARIANT: unknown variant ") + fv);
    }
    e->plan_alts.assign(raw.size(), {});
    e->plan_alias.assign(raw.size(), -1);
    for (size_t pi = 0; pi < raw.size(); ++pi) {
        // rows already planned (rank engines: the full-depth launches of a round
        // share one region, rank_geometry): the same plan, resolved after the
        // autotuner (resolve_aliases)
        const bool role = e->band_plans && pi >= (size_t)e->Hx;  // band / interior
        for (size_t pj = 0; pj < pi && !role; ++pj) {
            if (e->plan_alias[pj] >= 0 || raw[pj].size() != raw[pi].size()) continue;
            bool same = true;
            for (size_t k = 0; k < raw[pi].size() && same; ++k)
                same = std::memcmp(&raw[pi][k], &raw[pj][k], sizeof(SegDesc)) == 0;
            if (same) {
                e->plan_alias[pi] = (int)pj;
                break;
            }
        }
        if (e->plan_alias[pi] >= 0) {
            gol_engine::Plan a = e->plans[(size_t)e->plan_alias[pi]];
            a.alias = true;
            e->plans.push_back(a);
            continue;
        }
        gol_engine::Plan p;
        GOL_TRY(build_one(pi, hs, 1.0, handoff, p));
        e->plans.push_back(p);
        const bool full = e->nranks > 1 ? (pi < (size_t)e->Hx && (pi + 1) % e->K == 0) : pi == 0;
        if ((!tune && !forced) || !full || p.segs.size() != 1 || p.lane_shift != 0 || !p.rows_old)
            continue;
        struct Variant {
            int64_t hs;
            double rho;
            uint32_t kind;
        };
        // kTuneVariantNames order
        std::vector<Variant> vs = {{0, 1.0, handoff}, {hs, 0.95, handoff}, {hs, 1.05, handoff}};
        if (e->handoff == 0 && gol::handoff_kernel_exists((int)e->K, e->rule))
            vs.push_back({hs, 1.0, p.hand ? 1u : 2u});
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            if (forced && (int)vi + 1 != forced) continue;
            const Variant& v = vs[vi];
            gol_engine::Plan q;
            GOL_TRY(build_one(pi, v.hs, v.rho, v.kind, q));
            bool dup = q.segs.size() != 1 || same_plan(q, p);
            for (const auto& o : e->plan_alts[pi]) dup = dup || same_plan(q, o);
            if (dup) {
                free_plan(q);
                continue;
            }
            q.tuned = (int32_t)vi + 1;
            if (forced) {  // the named variant replaces the models' plan
                free_plan(e->plans[pi]);
                e->plans[pi] = q;
                continue;
            }
            e->plan_alts[pi].push_back(q);
        }
    }
    if (e->model.on) return GOL_OK;
    HIP_TRY(hipMalloc(&e->d_err, sizeof(int)));
#if GOL_EXP
    if (!g_dev_prog) {
        HIP_TRY(hipMalloc(&g_dev_prog, 8192 * 2 * sizeof(uint32_t)));
        HIP_TRY(hipMemset(g_dev_prog, 0, 8192 * 2 * sizeof(uint32_t)));
    }
#endif
    HIP_TRY(hipMemset(e->d_err, 0, sizeof(int)));
    if ((any_hand || any_mp) && max_units > 0) {
        // (multi-pass: hand-off slots and flags per pass parity)
        const size_t slot = (size_t)2 * (e->K - 1) * 64 * (size_t)(e->planes / 2);
        const size_t par = any_mp ? 2 : 1;
        const int regions = e->band_plans ? 2 : 1;
        for (int r = 0; r < regions; ++r) {
            HIP_TRY(hipMalloc(&e->side[r], par * (size_t)max_units * slot * sizeof(uint64_t)));
            HIP_TRY(hipMalloc(&e->flags[r], par * (size_t)max_units * sizeof(uint32_t)));
            HIP_TRY(hipMemset(e->flags[r], 0, par * (size_t)max_units * sizeof(uint32_t)));
        }
    }
    if (any_mp && max_units > 0) {
        HIP_TRY(hipMalloc(&e->mpflags, 4 * (size_t)max_units * sizeof(uint32_t)));
        HIP_TRY(hipMemset(e->mpflags, 0, 4 * (size_t)max_units * sizeof(uint32_t)));
    }
    return GOL_OK;
}

// Multi-pass launches (GOL_DEV_PASSES = 2 or 3; life_stencil.h, measured slower
// than single-pass launches in r05): single-GPU engines alone on their
// device and rank engines, fields whose shadow offset fits the kernel's 32-bit
// lane offsets (`words` per buffer), depths whose P K outer halo columns stay
// inside the halo lane (P K < 64)
void decide_passes(gol_engine* e, size_t words)
{
    if (!gol::kDevKernels) return;  // multi-pass kernels: dev build only
    if (const char* v = std::getenv("GOL_DEV_PASSES")) {
        const int np = std::atoi(v);
        // (group members launch single-pass: gol_group_step runs each launch op)
        if (np >= 2 && np <= 3 && !e->shared_device && !e->grouped && np * (int)e->K < 64 &&
            gol::multipass_kernel_exists((int)e->K, e->rule, e->planes) &&
            (words + e->stride) * sizeof(uint64_t) < (1ull << 32))
            e->npass = (uint32_t)np;
    }
}

// Autotuner (candidates from build_plans): each full-depth plan and its variants
// run interleaved on the engine's buffers, 1 + 4 pairs of launches each timed with
// HIP events (on a random field, see below); the fastest by its median pair
// replaces the models' plan if it is at least 3% faster (timings at
// create scatter by ~2%: at 65536^2 a variant "2% faster" there ran the same in
// steady state).  The variants are all plan kinds the parity tests pin, so this
// changes speed only.  8-way rank launch shapes (one process, TCUPS, models' plan
// vs autotuned, profiles/r03/ab_autotune.jsonl): 8224 rows 103.7 vs 112.6, 8608
// 105.8 vs 116.1, 8672 105.8 vs 114.7; 8448 and 16640 keep the models' plan.  A
// resident engine drops its candidates.
constexpr float kTuneMargin = 0.97f;

gol_status check_err(gol_engine* e);

gol_status autotune_plans(gol_engine* e)
{
    bool any = false;
    for (const auto& a : e->plan_alts) any = any || !a.empty();
    if (!any) return GOL_OK;
    if (e->res.on) {
        for (auto& a : e->plan_alts) {
            for (auto& q : a) free_plan(q);
            a.clear();
        }
        return GOL_OK;
    }
    hipEvent_t t0 = nullptr, t1 = nullptr;
    HIP_TRY(hipEventCreate(&t0));
    HIP_TRY(hipEventCreate(&t1));
    // (r04) Time the candidates as they run in a step: on a p = 0.5 field (a
    // zero field draws less power and runs at a higher clock) and as pairs of
    // back-to-back launches (each launch's tail overlaps the next one's start),
    // the median of 4 pairs after one untimed pair.  At 16640 x 65536 single
    // launches on the zero field kept the models' plan, 3.9% slower in steady state
    // than its skew x 1.05 variant (profiles/r04/ab_plan_variants_forced.jsonl).
    // The field is zeroed again afterwards: a new engine holds a dead field.
    const size_t words_all = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    HIP_TRY(gol::launch_init_random(e->buf[e->cur], (int64_t)e->stride, (int64_t)e->wq,
                                    e->lastmask, 0, 0, (int64_t)e->buf_rows, 0x5eedull,
                                    e->planes, e->stream));
    constexpr int kPairs = 4;
    gol_status st = GOL_OK;
    for (size_t pi = 0; pi < e->plan_alts.size() && st == GOL_OK; ++pi) {
        auto& alts = e->plan_alts[pi];
        if (alts.empty()) continue;
        std::vector<gol_engine::Plan> cand{e->plans[pi]};
        cand.insert(cand.end(), alts.begin(), alts.end());
        alts.clear();
        std::vector<std::vector<float>> times(cand.size());
        for (int rep = 0; rep <= kPairs && st == GOL_OK; ++rep)
            for (size_t c = 0; c < cand.size() && st == GOL_OK; ++c) {
                e->plans[pi] = cand[c];
                float ms = 0;
                if (hipEventRecord(t0, e->stream) != hipSuccess) st = fail(GOL_EHIP, "autotune event");
                for (int l = 0; l < 2 && st == GOL_OK; ++l) st = launch(e, (int)pi, e->K, false);
                if (st == GOL_OK && (hipEventRecord(t1, e->stream) != hipSuccess ||
                                     hipEventSynchronize(t1) != hipSuccess ||
                                     hipEventElapsedTime(&ms, t0, t1) != hipSuccess))
                    st = fail(GOL_EHIP, "autotune timing");
                if (rep > 0) times[c].push_back(0.5f * ms);
            }
        std::vector<float> best(cand.size(), 1e30f);
        for (size_t c = 0; c < cand.size(); ++c)
            if (!times[c].empty()) {
                std::sort(times[c].begin(), times[c].end());
                best[c] = 0.5f * (times[c][(times[c].size() - 1) / 2] + times[c][times[c].size() / 2]);
            }
        size_t pick = 0;
        for (size_t c = 1; c < cand.size(); ++c)
            if (best[c] < best[pick] && best[c] < kTuneMargin * best[0]) pick = c;
        e->plans[pi] = cand[pick];
        e->plans[pi].tune_ms = best[pick];
        e->plans[pi].tune_ms_model = best[0];
        for (size_t c = 0; c < cand.size(); ++c)
            if (c != pick) free_plan(cand[c]);
        if (std::getenv("GOL_DEV_PLANS"))
            std::fprintf(stderr, "autotune plan %zu: candidate %zu of %zu (%.1f us vs %.1f us), R %lld, "
                         "hand %d, skew %d/%d, half-strip units %lld\n", pi, pick, cand.size(),
                         1e3 * best[pick], 1e3 * best[0], (long long)e->plans[pi].rpw,
                         (int)e->plans[pi].hand, e->plans[pi].rows_old, e->plans[pi].rows_young,
                         (long long)e->plans[pi].pair_units);
    }
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (st == GOL_OK) st = check_err(e);  // a hand-off wait that timed out is a failure here too
    for (int b = 0; b < e->nbuf && st == GOL_OK; ++b)
        if (hipMemsetAsync(e->alloc[b], 0, words_all * sizeof(uint64_t), e->stream) != hipSuccess)
            st = fail(GOL_EHIP, "autotune: clearing the field");
    return st;
}

// Plans that share rows with an earlier plan (build_plans) become copies of it as
// the autotuner left it: one block plan for every full-depth launch of a round.
void resolve_aliases(gol_engine* e)
{
    for (size_t pi = 0; pi < e->plans.size() && pi < e->plan_alias.size(); ++pi)
        if (e->plan_alias[pi] >= 0) {
            e->plans[pi] = e->plans[(size_t)e->plan_alias[pi]];
            e->plans[pi].alias = true;
        }
}

}  // namespace golh
