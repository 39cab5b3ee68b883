// engine.cpp -- host side of libgol.so: the C ABI of include/gol.h.
//
// Owns device memory, the HIP streams, the halo transport (RCCL communicator,
// a caller's host transport, or device copies inside a group) and the launch
// plans.  Mirrors main()'s flow in Parallel_Life_MPI.cpp:190-240: create
// (readGridFromFile's allocation :88-89) -> load (:91-99) -> step (the epoch loop
// :215-221 with the halo exchange :104-145) -> store (:157-164).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gol.h"
#include "bitlayout.h"
#include "life_internal.h"

using gol::SegDesc;
using gol::StepArgs;

namespace {

thread_local std::string g_last_error;

#if GOL_EXP
// Dev timing builds (tools/exp_build.sh): device buffer the stencil kernel logs
// per-wavefront (start, end, hardware id, unit) into; set by gol_dev_set_wave_log.
uint64_t* g_dev_wave_log = nullptr;
uint32_t* g_dev_prog = nullptr;  // GOL_EXP & 1024: per-SIMD progress words
#endif

// gol_create splits GLOBAL fields of at least this many rows into 2 same-device
// stripes on 2 streams (measured +11% at 65536^2; no gain at <= 16384 rows,
// profiles/r01/group_bench_*.jsonl)
constexpr uint64_t kCompositeMinRows = 32768;
// captured step graphs kept per engine (least recently used evicted)
constexpr size_t kGraphCache = 8;

// Auto launch layout: fused depth K and planes per lane group (bitlayout.h).
//  * K = 16 with 2 planes (one word per lane; ~230 VGPRs, 2 waves/SIMD, enough
//    for full VALU issue) for stripes of more than 6144 rows: 124.5 TCUPS at
//    65536^2 vs 122.4 (K = 8) and 106.0 (K = 12); K >= 20 drops to 1 wave/SIMD
//    and loses 30-35% (profiles/r01/sweep_total_sum_depth.jsonl).
//  * Short fields are launch-latency bound and keep K = 8 (4096^2: 11.0-11.6
//    TCUPS vs 8.7 at K = 16).
//  * Rules other than B/S2 and B3/S23 evaluate a 10-term mask sum whose K = 16
//    state spills: K = 12.
//  * 4 planes (two words per lane) only on request (dev build), with K = 8.
struct Layout {
    uint32_t K;
    int planes;
};

Layout auto_layout(uint64_t rows, const gol_config* cfg)
{
    const bool fixed = (cfg->birth_mask == GOL_REF_BIRTH && cfg->survive_mask == GOL_REF_SURVIVE) ||
                       (cfg->birth_mask == GOL_CONWAY_BIRTH &&
                        cfg->survive_mask == GOL_CONWAY_SURVIVE);
    Layout l;
    l.planes = cfg->word_planes ? (int)cfg->word_planes : 2;
    // resident = 2 takes any epoch length; the streaming launches of an engine
    // that cannot run the resident kernel (rank engines, composite parts, fields
    // it does not fit) then use the auto depth when that length has no stencil
    // kernel, instead of failing
    const bool res_only = cfg->resident == 2 && cfg->tb_depth &&
                          !gol::life_has_kernel((int)cfg->tb_depth, l.planes);
    if (cfg->tb_depth && !res_only)
        l.K = cfg->tb_depth;
    else if (cfg->word_planes == 4 || rows <= 6144)
        l.K = 8;
    else
        l.K = fixed ? 16 : 12;
    return l;
}

gol_status fail(gol_status st, const std::string& msg)
{
    g_last_error = msg;
    return st;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return fail(_e == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP,                  \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                 \
    } while (0)

#define NCCL_TRY(expr)                                                                      \
    do {                                                                                    \
        ncclResult_t _r = (expr);                                                           \
        if (_r != ncclSuccess)                                                              \
            return fail(GOL_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(_r));     \
    } while (0)

#define GOL_TRY(expr)                                                                       \
    do {                                                                                    \
        gol_status _s = (expr);                                                             \
        if (_s != GOL_OK) return _s;                                                        \
    } while (0)

uint64_t last_mask(uint64_t w)
{
    const unsigned rem = (unsigned)(w & 63);
    return rem ? ((1ull << rem) - 1ull) : ~0ull;
}

// Parallel_Life_MPI.cpp:70-81 -- rank r's extended stripe [start, start+rows).
bool ref_stripe(uint64_t h, uint64_t P, uint64_t r, uint64_t* start, uint64_t* rows)
{
    if (P == 0 || r >= P || h / P == 0) return false;
    uint64_t chunk = h / P, s = r * chunk;
    if (r != 0) {
        s--;
        chunk++;
    }
    chunk += (r == P - 1) ? h % P : 1;
    *start = s;
    *rows = chunk;
    return true;
}

// Scoped device allocation (staging for the ASCII codec).
struct DeviceBytes {
    char* p = nullptr;
    ~DeviceBytes()
    {
        if (p) (void)hipFree(p);
    }
};

// A host-visible region of the field: buffer rows [buf_row, buf_row+rows) are field
// rows [glob_row, glob_row+rows); it corresponds to the caller's ASCII/packed rows
// [user_row, user_row+rows).
struct Region {
    uint64_t buf_row, glob_row, user_row, rows;
};

// Geometry of stripe `rank` of `nranks` (GLOBAL field), host-only: its rows, the
// halo depth, the fused depth, and the segment tables of its launch plans --
// plans[c-1] computes the local rows still valid after a cumulative shrink c of a
// round (c = 1..Hx); with overlap, plans[Hx] (band: the rows the neighbours need)
// and plans[Hx+1] (interior) split the round's last launch.  Shared by the rank
// engines and gol_round_schedule, so the exported schedule is the one run.
// `overlap`: the mode the schedule starts in; `band`: the band and interior plans
// exist (overlap, or an exchange mode to be chosen by timing: `tune`).
struct RankGeom {
    uint64_t row0 = 0, R = 0, Hx = 0, buf_rows = 0;
    uint32_t K = 8;
    bool overlap = false, band = false, tune = false;
    std::vector<std::vector<SegDesc>> raw;
};

gol_status rank_geometry(uint64_t h, const gol_config* cfg, int rank, int nranks, RankGeom* g,
                         bool group = false, bool tune_ok = false);

}  // namespace

// The kinds of exchange a stripe engine does (gol_create_rank /
// gol_create_rank_transport / gol_create_group).
enum XferKind { XFER_NONE = 0, XFER_RCCL = 1, XFER_HOST = 2, XFER_GROUP = 3 };

struct gol_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t H = 0, W = 0, wq = 0, stride = 0, lastmask = 0;
    int planes = 2;                      // planes per lane group (bitlayout.h)
    uint64_t ng = 0;                     // lane groups per row
    uint64_t lastmask_split[2] = {0, 0};  // stored form of the last group's valid bits
    uint32_t birth = 0, survive = 0;
    gol::RuleKind rule = gol::RULE_REF;
    uint32_t K = 8;
    uint32_t rows_per_wave = 0;
    int lane_shift = -1;  // strip width 64 >> lane_shift; -1 = chosen per plan
    uint32_t handoff = 0; // gol_config.handoff
    uint32_t sem = GOL_SEM_GLOBAL;
    uint32_t P = 1;

    // rank geometry (single-GPU: rank 0 of 1, Hx = 0)
    int rank = 0, nranks = 1;
    uint64_t row0 = 0, R = 0, Hx = 0;
    XferKind xfer = XFER_NONE;
    ncclComm_t comm = nullptr;
    // RCCL peers of the up/down halo (rank -+ 1; both 0 for the self-loop test
    // communicator of GOL_DEV_RCCL_SELF, gol_create_rank)
    int peer_up = -1, peer_dn = -1;
    gol_transport tp{nullptr, nullptr};
    uint64_t* host_xfer = nullptr;  // pinned: send_up | recv_up | send_dn | recv_dn

    // in-process group (gol_create_group): halo exchange by device copies
    gol_engine* up = nullptr;
    gol_engine* down = nullptr;
    bool grouped = false;
    // other engines launch on this device concurrently (composite parts, group
    // members sharing a GPU): the age skew's dispatch-order premise does not hold
    bool shared_device = false;
    // registered in the device's waiting-kernel registry (wait_registry) as the
    // hand-off engine / as a resident engine
    bool reg_hand = false, reg_res = false;
    hipEvent_t ev_ready = nullptr, ev_copied = nullptr;

    // exchange/compute overlap (multi-rank): the last launch of a full round is
    // split into a band launch (the rows the neighbours need) and an interior
    // launch; the exchange runs on `comm_stream` between them.  halo_fresh: the
    // current buffer's halo rows were already exchanged (completion signalled by
    // ev_xdone on comm_stream).  The band launch runs on its own stream,
    // concurrently with the interior launch: it is a few hundred rows, far too
    // few wavefronts to fill the GPU.
    hipStream_t comm_stream = nullptr, band_stream = nullptr;
    hipEvent_t ev_band = nullptr, ev_xdone = nullptr, ev_in = nullptr, ev_join = nullptr;
    bool overlap = false;     // the mode gol_step runs (RankGeom::overlap at create)
    bool band_plans = false;  // the band and interior plans exist (RankGeom::band)
    bool halo_fresh = false;
    // (r07) exchange_overlap = 0 on a rank engine over RCCL: both modes timed at
    // create (tune_exchange), the max over ranks of each mode's best sample (ms);
    // 0 = not timed
    bool xchg_tune = false;
    float xchg_ms[2] = {0.f, 0.f};  // blocking, overlapped

    // composite engine (gol_create, large GLOBAL fields): the field is S row
    // stripes on S streams of this device (a gol_create_group), so one stripe's
    // launch tail overlaps the others' work; every call is routed to the parts
    std::vector<gol_engine*> parts;

    uint64_t buf_rows = 0;
    // state buffers: 2, or 4 with multi-pass launches (a launch of P <= 3 passes
    // reads buf[cur] and writes buf[cur + 1 .. cur + P], mod nbuf); those also hold
    // a shadow half (shadow_off bytes after each row) for the strips' halo lanes
    uint64_t* alloc[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t* buf[4] = {nullptr, nullptr, nullptr, nullptr};
    int cur = 0;
    int nbuf = 2;
    uint32_t npass = 1;       // passes per full-depth launch the engine may run
    uint32_t xcd_shift = 0;   // (r06 dev A/B) StepArgs::xcd_shift, GOL_DEV_XCD_SHIFT
    uint32_t shadow_off = 0;  // bytes from a buffer word to its shadow
    uint32_t* mpflags = nullptr;  // multi-pass head/done flags: 4 x max units

    // plans: plan p = a device table of nseg SegDesc (+ host copy)
    struct Plan {
        std::vector<SegDesc> segs;
        int32_t groups = 0;      // strip groups per row block (StepArgs::strips)
        int32_t lane_shift = 0;  // strips of 64 >> lane_shift lanes
        double own_rows = 0;  // output rows of this plan that are the caller's rows
        int64_t rpw = 0;      // rows per wavefront
        int64_t total_units = 0;
        bool multi_blk = false;  // some segment has more than one row block
        bool hand = false;       // the planner chose hand-off row blocks
        // age-skewed row blocks (age_skew; 0 = off): the same blocks per strip, the
        // first-dispatched units rows_old rows, the others rows_young (both = rpw
        // mod the prefetch block, so the hand-off tail offset is rpw's)
        int32_t rows_old = 0, rows_young = 0, units_old = 0;
        // 64-lane strips: edge-aligned columns (col_layout) and the packed half
        // strip's units after the full strips' (pairs: 3 words per unit)
        int32_t edge = 0;
        int64_t right_q0 = -1, half_q0 = 0, half_hi = -1;
        int64_t pair_units = 0, half_rows = 0;
        std::vector<int64_t> pairs;
        int64_t* dpairs = nullptr;
        SegDesc* dev = nullptr;
        // a copy of an earlier plan of the same rows (rank engines: the full-depth
        // launches of a round share one plan); its device tables are the owner's
        bool alias = false;
        // passes per full-depth launch of this plan (multi-pass launches, life_stencil.h:
        // one-segment plans of one round without the half strip; 1 = single pass)
        int32_t npass = 1;
        // autotuner: the candidate that runs (0 = the models' plan, else 1 + the
        // index in kTuneVariantNames) and its best create-time launch vs the
        // models' plan (ms; 0 = not tuned)
        int32_t tuned = 0;
        float tune_ms = 0.f, tune_ms_model = 0.f;
    };
    std::vector<Plan> plans;  // GLOBAL/REF: plans[0]; rank: see RankGeom
    std::vector<int> plan_alias;  // plans[i] copies plans[plan_alias[i]] (-1: own plan)
    std::vector<std::vector<Plan>> plan_alts;  // autotuner candidates per plan (build_plans)
    // host-only planning (gol_plan_model): build_plans takes the device's CU count
    // and occupancies from here and makes no device call or allocation
    struct DevModel {
        bool on = false;
        int cus = 0, occ_c = 0, occ_h = 0;
    } model;

    // row-block hand-off buffers (life_stencil.h): region 0 serves launches on
    // `stream`, region 1 those on `band_stream` (the two may run concurrently)
    uint64_t* side[2] = {nullptr, nullptr};
    uint32_t* flags[2] = {nullptr, nullptr};
    int* d_err = nullptr;

    // resident kernel (life_resident.hip): small GLOBAL fields, one launch per
    // gol_step; flags count the epochs published, from flag_base on
    struct Resident {
        bool on = false;
        int rows = 0;  // rows per wavefront
        int32_t strips = 0, bands = 0, band_rows = 0, K = 0;
        uint32_t* flags = nullptr;
        uint32_t flag_base = 0;
        // hipLaunchCooperativeKernel (GOL_DEV_RES_COOP=1): the device re-checks that
        // every tile fits at once, but the launch costs ~30 us more (C2: 640 vs
        // 609-614 us per 1000 generations, profiles/r03/ab_resident_coop.jsonl);
        // the planner's occupancy check and the bounded waits cover it by default
        bool coop = false;
        // wave-level temporal blocking (life_resident_mb.hip): wavefronts swap rows
        // through LDS every `mb` generations; 1 = every generation (life_res_kernel)
        int mb = 1;
        hipEvent_t ev_in = nullptr, ev_out = nullptr;  // ordering with the shared stream
    } res;

    std::vector<Region> user_regions;  // load/store mapping (own output rows)
    std::vector<Region> load_regions;  // rows loaded (REF_STRIPES loads overlaps too)

    unsigned long long* d_acc = nullptr;
    int* d_flag = nullptr;  // ASCII codec error flag

    // single-stream engines replay a captured hipGraph of the launch sequence of a
    // gol_step(gens) call (keyed by gens and the starting buffer), so a step of
    // many short launches costs one graph launch of host work
    struct GraphEntry {
        hipGraphExec_t exec;
        int cur_after;
        uint64_t used;
    };
    std::map<std::pair<uint64_t, int>, GraphEntry> graphs;
    uint64_t graph_clock = 0;

    // timing: HIP events around every `timing_every`-th stencil launch (0 = off)
    uint32_t timing_every = 0;
    uint64_t launch_count = 0;
    std::vector<hipEvent_t> ev_free;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<double> pending_cells, pending_cells_comp, pending_rows;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_xpending;  // exchanges
    std::vector<char> xpending_blocking;  // ... on the compute stream (1) or comm (0)
    // rank engines, per round: the compute stream's span from before the round's
    // first launch to after its last (band launch joined), and the end of the
    // overlapped exchange issued in that round (null when it blocks)
    struct RoundEv {
        hipEvent_t start, end, xend;
    };
    std::vector<RoundEv> ev_rpending;
    gol_timing tm{};
};

namespace {

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

gol_status check_cfg(const gol_config* cfg)
{
    if (!cfg) return fail(GOL_EINVAL, "null config");
    if (cfg->birth_mask >= 512 || cfg->survive_mask >= 512)
        return fail(GOL_EINVAL, "rule masks must be 9-bit");
    // (the resident kernel takes any epoch length K <= 63: resident = 2 with tb_depth)
    if (cfg->tb_depth != 0 && !(cfg->resident == 2 && cfg->tb_depth <= 63) &&
        std::find(std::begin(gol::kDepthList), std::end(gol::kDepthList),
                  (int)cfg->tb_depth) == std::end(gol::kDepthList))
        return fail(GOL_EINVAL, gol::kDevKernels
                                    ? "tb_depth must be 0 (auto) or one of 1,2,4,6,7,8,12,16,20,24,32"
                                    : "tb_depth must be 0 (auto) or one of 1,2,4,6,7,8,12,16 "
                                      "(20/24/32: dev build)");
    if (cfg->handoff > 2) return fail(GOL_EINVAL, "handoff must be 0 (auto), 1 (off) or 2 (on)");
    if (cfg->handoff == 2 && cfg->tb_depth != 0 && cfg->tb_depth < (uint32_t)gol::kHandoffMinDepth)
        return fail(GOL_EINVAL, "handoff on needs tb_depth >= 4");
    if (cfg->strip_lanes != 0 && cfg->strip_lanes != 64 && cfg->strip_lanes != 32 &&
        cfg->strip_lanes != 16)
        return fail(GOL_EINVAL, "strip_lanes must be 0 (auto), 64, 32 or 16");
    if (cfg->semantics > GOL_SEM_REF_STRIPES) return fail(GOL_EINVAL, "bad semantics");
    if (cfg->resident > 2) return fail(GOL_EINVAL, "resident must be 0 (auto), 1 (off) or 2 (on)");
    if (cfg->exchange_overlap > 2)
        return fail(GOL_EINVAL, "exchange_overlap must be 0 (auto), 1 (blocking) or 2 (overlapped)");
    if (cfg->word_planes != 0 && cfg->word_planes != 2 && cfg->word_planes != 4)
        return fail(GOL_EINVAL, "word_planes must be 0 (auto), 2 or 4");
    if (cfg->word_planes == 4 && !gol::kDevKernels)
        return fail(GOL_EINVAL, "word_planes 4 is built only in the dev library (make dev)");
    if (cfg->word_planes == 4 && cfg->tb_depth > 16)
        return fail(GOL_EINVAL, "word_planes 4 needs tb_depth <= 16");
    return GOL_OK;
}

gol_status rank_geometry(uint64_t h, const gol_config* cfg, int rank, int nranks, RankGeom* g,
                         bool group, bool tune_ok)
{
    gol_status st = gol_rank_rows(h, nranks, rank, &g->row0, &g->R);
    if (st != GOL_OK) return st;
    const uint64_t minR = h / (uint64_t)nranks;
    if (minR == 0) return fail(GOL_EINVAL, "fewer rows than ranks");
    // Depth and halo depth from the smallest stripe, which every rank computes
    // alike: balanced stripes differ by one row, and a rank of 6145 rows beside
    // ranks of 6144 (or 16384 beside 16383) would otherwise pick another K or Hx
    // than its neighbours, whose exchanges then move different row counts (r07 fix;
    // tests/test_planner.py::test_rank_geometry_agrees_across_ranks).
    g->K = auto_layout(minR, cfg).K;
    // Rounds of halo_depth generations between exchanges: 8 launches (r03, with
    // shrinking regions: 16 for K = 16 stripes of at most 12288 rows).  Per-rank
    // proxy over the RCCL byte mover
    // (self-loop communicator, tools/rank_proxy.py, profiles/r03/rank_proxy_rccl.jsonl):
    // the 8-way 65536^2 rank (8192 rows) ran 107.8 TCUPS at Hx = 128 and 109.3 at
    // 256 -- half the rounds, each with an exchange and a launch sequence whose
    // first, longest launch fits the one-round plans worst -- against 1.6% more halo
    // rows; the 4-way rank was 117.2 at 128 and 116.5-116.7 at 192-256.
    //
    // r04: with one region for the round's full-depth launches (below), each launch
    // computes R + 2 Hx - 2K rows, so deeper halos cost rows on every launch (RCCL
    // per-rank proxy, TCUPS of own rows, Hx = 128 vs 256: 8-way 110.0 vs 107.9,
    // 4-way 120.9 vs 120.4; profiles/r04/rank_proxy_rccl_halo_depth.jsonl).  The
    // shrinking regions (GOL_DEV_RANK_SHRINK=1) keep the r03 depths.
    const char* shrink_env = std::getenv("GOL_DEV_RANK_SHRINK");
    const bool shrinking = shrink_env && shrink_env[0] == '1';
    // Stripes of 16384+ rows take 12 launches per round (Hx = 192 at K = 16): 4-way
    // 121.2-122.6 vs 118.3-121.2 TCUPS at 128, 2-way equal, both in one process
    // (profiles/r04/rank_proxy_rccl_halo_depth_sweep.jsonl); the 8-way rank keeps 8
    // (64 / 96 / 128 / 160: 106.2 / 108.3 / 109.6 / 107.9).
    const uint64_t launches_per_round =
        shrinking ? ((g->K >= 16 && minR <= 12288) ? 16 : 8)
                  : ((g->K >= 16 && minR >= 16384) ? 12 : 8);
    uint64_t Hx = cfg->halo_depth ? cfg->halo_depth : launches_per_round * (uint64_t)g->K;
    if (Hx > minR) Hx = minR;  // a rank sends its first/last Hx own rows
    g->Hx = nranks > 1 ? Hx : 0;
    g->raw.clear();
    g->overlap = g->band = g->tune = false;
    if (nranks <= 1) {
        g->buf_rows = h;
        return GOL_OK;
    }
    // local row i <-> field row row0 - Hx + i; buffer holds R + 2Hx rows
    g->buf_rows = g->R + 2 * g->Hx;
    const int64_t glob0 = (int64_t)g->row0 - (int64_t)g->Hx;
    const int64_t in_field_lo = std::max<int64_t>(0, -glob0);
    const int64_t in_field_hi = std::min<int64_t>((int64_t)g->buf_rows, (int64_t)h - glob0);
    // One region for the full-depth launches of a round (r04).  Launch j of a
    // round (cumulative shrink c = jK; round_ops issues every full-depth launch
    // before any shorter one) only needs the rows still valid, [c, buf - c), but
    // it computes the first launch's rows [K, buf - K): the extra rows are
    // computed from rows that are no longer valid, and no valid row ever reads
    // them (row r after c generations needs rows [r - c, r + c] of the round's
    // start).  Every full-depth launch then runs one block plan: the RCCL
    // per-rank proxy's 4-way launches ran 148.7-155.0 us with the 8 shrinking
    // plans of a round and 141.5 us with one plan repeated
    // (profiles/r03/rocprof_kernel_stats_rank4_*.csv).  GOL_DEV_RANK_SHRINK=1
    // restores the shrinking regions (dev A/B).
    const bool shared = !shrinking;
    for (uint64_t c = 1; c <= g->Hx; ++c) {
        const uint64_t cr = (shared && c % g->K == 0) ? g->K : c;
        SegDesc s{};
        s.base_row = 0;
        s.in_rows = (int64_t)g->buf_rows;
        s.glob0 = glob0;
        s.field_h = (int64_t)h;
        s.out_lo = std::max<int64_t>((int64_t)cr, in_field_lo);
        s.out_hi = std::min<int64_t>((int64_t)(g->buf_rows - cr), in_field_hi);
        g->raw.push_back({s});
    }
    // overlap plans: rows neighbours need = own rows [Hx, 2Hx) (to rank-1) and
    // [R, R+Hx) (to rank+1); interior = the rest of the own rows.  Decided from
    // the smallest stripe so every rank / group member agrees (balanced stripes
    // differ by one row).
    //
    // Only in-process groups overlap by default.  A rank engine (one per GPU) runs
    // one-round launches that take every wavefront slot: a band launch beside the
    // interior launch gets slots only as interior waves retire, ends after the
    // interior and the exchange waits for it (rocprofv3 trace of one 8-way rank:
    // +28 us per 640 us round, profiles/r02/trace_rank8_overlap_kernels.csv);
    // blocking exchanges were 1.3-5.7% faster per rank.  With the planner's cap
    // (band blocks sized to end early, the interior launch leaving their slots free,
    // build_plans) the band does run concurrently (trace_rank8_overlap_capped.csv),
    // but per-rank rates through the host-transport proxy stayed within -3..+3% of
    // blocking and bimodal at 2 ranks, and an RCCL exchange is itself a kernel that
    // needs free slots: blocking was the rank default through r06, measured on the
    // RCCL self-loop, where the exchange is a device-local copy.  Over xGMI the
    // exchange costs more and may be worth hiding, so (r07) with
    // gol_config.exchange_overlap = 0 a rank engine over RCCL (tune_ok) builds both
    // schedules' plans, starts blocking, and gol_create_rank times both modes on
    // the real communicator and keeps the faster (tune_exchange).
    // gol_config.exchange_overlap = 1 / 2 forces a mode (bench.py --gpus N times
    // both); with it at 0, GOL_DEV_OVERLAP = 1 / 0 forces the overlap on / off (dev
    // A/B).
    const int64_t Hx_ = (int64_t)g->Hx, R = (int64_t)g->R;
    bool want = group, tune = false;
    if (cfg->exchange_overlap)
        want = cfg->exchange_overlap == 2;
    else if (const char* ov = std::getenv("GOL_DEV_OVERLAP"))
        want = ov[0] == '1';
    else
        tune = tune_ok;
    if ((int64_t)(h / (uint64_t)nranks) >= 2 * Hx_ && (want || tune)) {
        SegDesc b = g->raw.back()[0];  // shrink Hx: out = own rows
        std::vector<SegDesc> band, inner;
        int64_t ilo = Hx_, ihi = Hx_ + R;
        if (rank > 0) {
            SegDesc t = b;
            t.out_lo = Hx_;
            t.out_hi = 2 * Hx_;
            band.push_back(t);
            ilo = 2 * Hx_;
        }
        if (rank < nranks - 1) {
            SegDesc t = b;
            t.out_lo = R;
            t.out_hi = R + Hx_;
            band.push_back(t);
            ihi = R;
        }
        SegDesc t = b;
        t.out_lo = ilo;
        t.out_hi = ihi;
        inner.push_back(t);
        g->raw.push_back(band);
        g->raw.push_back(inner);
        g->overlap = want;
        g->band = true;
        g->tune = tune;
    }
    return GOL_OK;
}

uint32_t pick_depth(uint32_t K, uint64_t remaining)
{
    for (int d : gol::kDepthList)
        if ((uint32_t)d <= K && (uint64_t)d <= remaining) return (uint32_t)d;
    return 1;
}

// One operation of a stripe engine's step (gol_sched_op without the rows).
struct SchedOp {
    uint32_t kind, depth;
    int plan;  // launch ops: index into the plans (RankGeom)
};

// The launches of one round of `round` generations after a halo exchange: each
// launch of depth d shrinks the valid region by d rows per side (plan c-1 for a
// cumulative shrink of c).  With overlap, the last launch of a full round runs
// as band + interior, with the next round's exchange started between them.
void round_ops(uint32_t K, uint64_t Hx, bool overlap, uint64_t round, std::vector<SchedOp>& ops)
{
    uint64_t done = 0;
    while (done < round) {
        const uint32_t d = pick_depth(K, round - done);
        done += d;
        if (overlap && done == Hx) {
            ops.push_back({GOL_OP_BAND, d, (int)Hx});
            ops.push_back({GOL_OP_INTERIOR, d, (int)Hx + 1});
            ops.push_back({GOL_OP_EXCHANGE_ASYNC, 0, -1});
        } else {
            ops.push_back({GOL_OP_LAUNCH, d, (int)(done - 1)});
        }
    }
}

// A stripe engine's gol_step(generations): rounds of Hx generations, each after
// an exchange -- blocking, or the overlapped one the previous round started.
void step_schedule(uint32_t K, uint64_t Hx, bool overlap, bool halo_fresh, uint64_t gens,
                   std::vector<SchedOp>& ops)
{
    uint64_t left = gens;
    while (left > 0) {
        const uint64_t round = std::min<uint64_t>(left, Hx);
        ops.push_back({halo_fresh ? (uint32_t)GOL_OP_WAIT_EXCHANGE : (uint32_t)GOL_OP_EXCHANGE, 0, -1});
        const size_t n0 = ops.size();
        round_ops(K, Hx, overlap, round, ops);
        halo_fresh = ops.back().kind == GOL_OP_EXCHANGE_ASYNC && ops.size() > n0;
        left -= round;
    }
}

gol_status plan_resident(gol_engine* e, const gol_config* cfg);
void decide_passes(gol_engine* e, size_t words);
gol_status autotune_plans(gol_engine* e);
void resolve_aliases(gol_engine* e);

// Kernels that wait for other wavefronts of their own launch -- hand-off row blocks
// (life_stencil.h) and the resident kernel -- need every wavefront they wait for
// to get a slot.  Their plans guarantee it for the launch alone on the device:
// hand-off launches are one round of the occupancy query (pick_rows_per_wave), the
// resident grid is at most one workgroup per CU (plan_resident).  Launches of
// other engines of this process would share the slots, so the process keeps, per
// device: at most one engine with hand-off blocks, and none while a resident engine
// lives (resident launches of several engines are ordered on one stream,
// resident_stream; classic blocks and composite parts never wait, so they may run
// beside either).  An engine that cannot get the kind it would plan runs classic
// blocks / the streaming kernel instead (gol_plan_handoff, gol_plan_resident
// report it).  GOL_DEV_SHARED_WAITS=1 turns the registry off (dev sweeps that
// step their engines one at a time).
struct WaitReg {
    gol_engine* hand = nullptr;
    int resident = 0;
};
std::mutex g_wait_mu;
std::map<int, WaitReg> g_wait_reg;

bool wait_registry_off()
{
    const char* v = std::getenv("GOL_DEV_SHARED_WAITS");
    return v && v[0] == '1';
}

void wait_release(gol_engine* e)
{
    if (!e->reg_hand && !e->reg_res) return;
    std::lock_guard<std::mutex> lock(g_wait_mu);
    WaitReg& r = g_wait_reg[e->device];
    if (e->reg_hand && r.hand == e) r.hand = nullptr;
    if (e->reg_res) r.resident--;
    e->reg_hand = e->reg_res = false;
}

// Host-side layout of an engine (no GPU): rule kind, depth and lane-group
// layout, row stride and the last group's mask.  Geometry (row0, R, Hx, rank)
// already set.
gol_status host_layout(gol_engine* e, uint64_t h, uint64_t w, const gol_config* cfg)
{
    e->H = h;
    e->W = w;
    e->wq = (w + 63) / 64;
    e->stride = (e->wq + 7) / 8 * 8;
    e->lastmask = last_mask(w);
    e->birth = cfg->birth_mask;
    e->survive = cfg->survive_mask;
    if (e->birth == GOL_REF_BIRTH && e->survive == GOL_REF_SURVIVE)
        e->rule = gol::RULE_REF;
    else if (e->birth == GOL_CONWAY_BIRTH && e->survive == GOL_CONWAY_SURVIVE)
        e->rule = gol::RULE_CONWAY;
    else
        e->rule = gol::RULE_GENERIC;
    const Layout lay = auto_layout(e->R, cfg);
    e->K = lay.K;
    e->rows_per_wave = cfg->rows_per_wave;
    e->lane_shift = cfg->strip_lanes == 64 ? 0 : cfg->strip_lanes == 32 ? 1
                  : cfg->strip_lanes == 16 ? 2 : -1;
    e->handoff = cfg->handoff;
    e->planes = lay.planes;
    if (!gol::life_has_kernel((int)e->K, e->planes))
        return fail(GOL_EINVAL, "no stencil kernel for this tb_depth / word_planes");
    {
        const uint64_t G = (uint64_t)e->planes / 2;
        e->ng = (e->wq + G - 1) / G;
        uint64_t c[2] = {0, 0};
        for (uint64_t j = 0; j < G; ++j) {
            const uint64_t idx = (e->ng - 1) * G + j;
            c[j] = idx + 1 < e->wq ? ~0ull : idx + 1 == e->wq ? e->lastmask : 0ull;
        }
        gol_split_group(c, e->lastmask_split, e->planes);
    }
    e->sem = cfg->semantics;
    return GOL_OK;
}

// The raw launch regions of an engine (host only): rank engines the round's
// regions (rank_geometry), REF_STRIPES the P independent stripes, GLOBAL the
// field; with the load/store row mappings.
gol_status raw_regions(gol_engine* e, uint64_t h, const gol_config* cfg, const RankGeom* geom,
                       std::vector<std::vector<SegDesc>>& raw)
{
    if (e->nranks > 1) {
        e->buf_rows = geom->buf_rows;
        e->overlap = geom->overlap;
        e->band_plans = geom->band;
        e->xchg_tune = geom->tune;
        raw = geom->raw;
        e->user_regions.push_back({e->Hx, e->row0, 0, e->R});
        e->load_regions = e->user_regions;
    } else if (e->sem == GOL_SEM_REF_STRIPES) {
        e->P = cfg->ref_ranks ? cfg->ref_ranks : 1;
        if (h / e->P == 0) return fail(GOL_EINVAL, "REF_STRIPES needs h >= ref_ranks");
        std::vector<SegDesc> segs;
        uint64_t base = 0;
        const uint64_t c = h / e->P;
        for (uint32_t r = 0; r < e->P; ++r) {
            uint64_t s0, n;
            ref_stripe(h, e->P, r, &s0, &n);
            SegDesc s{};
            s.base_row = (int64_t)base;
            s.in_rows = (int64_t)n;
            s.glob0 = 0;
            s.field_h = (int64_t)n;
            s.out_lo = 0;
            s.out_hi = (int64_t)n;
            segs.push_back(s);
            e->load_regions.push_back({base, s0, s0, n});
            // writeDataToFile (:149-175): own rows [r*c, (r+1)*c), last rank to h
            const uint64_t lo = r * c, hi = (r == e->P - 1) ? h : (r + 1) * c;
            e->user_regions.push_back({base + (lo - s0), lo, lo, hi - lo});
            base += n;
        }
        e->buf_rows = base;
        raw.push_back(segs);
    } else {
        e->buf_rows = h;
        SegDesc s{};
        s.base_row = 0;
        s.in_rows = (int64_t)h;
        s.glob0 = 0;
        s.field_h = (int64_t)h;
        s.out_lo = 0;
        s.out_hi = (int64_t)h;
        raw.push_back({s});
        e->user_regions.push_back({0, 0, 0, h});
        e->load_regions = e->user_regions;
    }
    return GOL_OK;
}

// Common construction; geometry (row0, R, Hx, rank) already set.
gol_status init_common(gol_engine* e, uint64_t h, uint64_t w, const gol_config* cfg,
                       const RankGeom* geom)
{
    GOL_TRY(host_layout(e, h, w, cfg));
    if (cfg->device >= 0) HIP_TRY(hipSetDevice(cfg->device));
    HIP_TRY(hipGetDevice(&e->device));
    HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    if (e->nranks > 1) {
        HIP_TRY(hipStreamCreateWithFlags(&e->comm_stream, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&e->band_stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_band, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_xdone, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
    }

    std::vector<std::vector<SegDesc>> raw;
    GOL_TRY(raw_regions(e, h, cfg, geom, raw));

    const size_t words = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    decide_passes(e, words);
    // (r06 dev A/B) GOL_DEV_XCD_SHIFT = "c0c1...c7:m": speed class 0-3 of the
    // workgroups with blockIdx mod 8 == x, and the strip modulus m (life_stencil.h)
    if (const char* v = gol::kDevKernels ? std::getenv("GOL_DEV_XCD_SHIFT") : nullptr) {
        uint32_t code = 0;
        int i = 0;
        for (; i < 8 && v[i] >= '0' && v[i] <= '3'; ++i) code |= (uint32_t)(v[i] - '0') << (2 * i);
        const int m = (i == 8 && v[8] == ':') ? std::atoi(v + 9) : 0;
        if (m >= 1 && m <= 255) e->xcd_shift = code | ((uint32_t)m << 16);
    }
    const size_t halves = e->npass > 1 ? 2 : 1;
    e->nbuf = e->npass > 1 ? 4 : 2;
    e->shadow_off = e->npass > 1 ? (uint32_t)(words * sizeof(uint64_t)) : 0u;
    for (int b = 0; b < e->nbuf; ++b) {
        HIP_TRY(hipMalloc(&e->alloc[b], halves * words * sizeof(uint64_t)));
        HIP_TRY(hipMemsetAsync(e->alloc[b], 0, halves * words * sizeof(uint64_t), e->stream));
        e->buf[b] = e->alloc[b] + (size_t)gol::kGuardRows * e->stride;
    }
    HIP_TRY(hipMalloc(&e->d_acc, 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc(&e->d_flag, sizeof(int)));
    gol_status st = GOL_OK;
    {
        // plan and register under the lock, so that engines created by several
        // threads see each other (wait_release).  The registry entry covers every
        // candidate the autotuner may pick; the timing itself runs after the lock
        // is released (it takes tens of ms), and the entry is narrowed to the pick.
        std::lock_guard<std::mutex> lock(g_wait_mu);
        const bool off = wait_registry_off();
        const WaitReg reg = g_wait_reg[e->device];
        gol_config c = *cfg;
        if (!off && (reg.hand || reg.resident)) e->handoff = 1;
        if (!off && reg.hand) c.resident = 1;
        st = build_plans(e, raw);
        if (st == GOL_OK) st = plan_resident(e, &c);
        if (st == GOL_OK && !off) {
            WaitReg& r = g_wait_reg[e->device];
            if (e->res.on) {
                e->reg_res = true;
                r.resident++;
            } else {
                bool hand = false;
                for (const auto& pl : e->plans) hand |= (pl.hand && pl.multi_blk) || pl.npass > 1;
                for (const auto& alts : e->plan_alts)
                    for (const auto& pl : alts) hand |= (pl.hand && pl.multi_blk) || pl.npass > 1;
                if (hand && e->side[0]) {
                    e->reg_hand = true;
                    r.hand = e;
                }
            }
        }
    }
    if (st == GOL_OK) st = autotune_plans(e);
    if (st != GOL_OK) return st;
    resolve_aliases(e);
    if (e->reg_hand) {
        bool hand = false;
        for (const auto& pl : e->plans) hand |= (pl.hand && pl.multi_blk) || pl.npass > 1;
        if (!hand) {  // the autotuner picked classic blocks: free the device's entry
            std::lock_guard<std::mutex> lock(g_wait_mu);
            WaitReg& r = g_wait_reg[e->device];
            if (r.hand == e) r.hand = nullptr;
            e->reg_hand = false;
        }
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    return GOL_OK;
}

gol_status flush_timing(gol_engine* e)
{
    for (size_t i = 0; i < e->ev_pending.size(); ++i) {
        auto& p = e->ev_pending[i];
        HIP_TRY(hipEventSynchronize(p.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.first, p.second));
        e->tm.launches += 1;
        e->tm.kernel_ms += ms;
        e->tm.cell_gens += e->pending_cells[i];
        e->tm.cell_gens_computed += e->pending_cells_comp[i];
        e->tm.launch_rows += e->pending_rows[i];
        e->ev_free.push_back(p.first);
        e->ev_free.push_back(p.second);
    }
    // an overlapped exchange is exposed for the part that ends after its round's
    // compute span (the next round's launches wait for it); a blocking one sits
    // between two rounds on the compute stream, all of it exposed
    std::map<hipEvent_t, float> round_end_to_xend;
    for (auto& r : e->ev_rpending) {
        HIP_TRY(hipEventSynchronize(r.end));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, r.start, r.end));
        e->tm.rounds += 1;
        e->tm.round_ms += ms;
        if (r.xend) {
            HIP_TRY(hipEventSynchronize(r.xend));
            float tail = 0.f;
            HIP_TRY(hipEventElapsedTime(&tail, r.end, r.xend));
            round_end_to_xend[r.xend] = tail;
        }
        e->ev_free.push_back(r.start);
        e->ev_free.push_back(r.end);
    }
    for (size_t i = 0; i < e->ev_xpending.size(); ++i) {
        auto& p = e->ev_xpending[i];
        HIP_TRY(hipEventSynchronize(p.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.first, p.second));
        e->tm.exchanges += 1;
        e->tm.exchange_ms += ms;
        float exposed = ms;
        if (!e->xpending_blocking[i]) {
            auto it = round_end_to_xend.find(p.second);
            exposed = it == round_end_to_xend.end() ? ms : std::min(ms, std::max(0.f, it->second));
        }
        e->tm.exchange_exposed_ms += exposed;
        e->ev_free.push_back(p.first);
        e->ev_free.push_back(p.second);
    }
    e->ev_pending.clear();
    e->ev_xpending.clear();
    e->xpending_blocking.clear();
    e->ev_rpending.clear();
    e->pending_cells.clear();
    e->pending_cells_comp.clear();
    e->pending_rows.clear();
    return GOL_OK;
}

gol_status get_event(gol_engine* e, hipEvent_t* ev)
{
    if (e->ev_free.empty()) {
        HIP_TRY(hipEventCreate(ev));
        return GOL_OK;
    }
    *ev = e->ev_free.back();
    e->ev_free.pop_back();
    return GOL_OK;
}

// HIP events around every `timing_every`-th kernel launch (gol_set_timing).
gol_status timing_begin(gol_engine* e, hipStream_t s, hipEvent_t* e0, hipEvent_t* e1)
{
    *e0 = *e1 = nullptr;
    if (e->timing_every) e->tm.launches_issued += 1;
    if (!e->timing_every || (e->launch_count++ % e->timing_every) != 0) return GOL_OK;
    GOL_TRY(get_event(e, e0));
    GOL_TRY(get_event(e, e1));
    HIP_TRY(hipEventRecord(*e0, s));
    return GOL_OK;
}

gol_status timing_end(gol_engine* e, hipStream_t s, hipEvent_t e0, hipEvent_t e1, double own,
                      double computed, double rows = 0)
{
    if (!e0) return GOL_OK;
    HIP_TRY(hipEventRecord(e1, s));
    e->ev_pending.push_back({e0, e1});
    e->pending_cells.push_back(own);
    e->pending_cells_comp.push_back(computed);
    e->pending_rows.push_back(rows);
    return GOL_OK;
}

// Resident plan: tiles of `band_rows` rows x one 64-lane strip, one 1024-thread
// workgroup each (at most one per CU: every workgroup of the launch must be
// resident at once, since tiles wait for their neighbours), each wavefront
// holding `rows` rows, so a tile holds 16 rows >= band + 2K halo rows.  Cost per
// generation, in us, fitted to 12 (rows, K, band) shapes at 4096^2
// (profiles/r02/c2_resident_sweep.jsonl, within 8%): 0.17 + 0.046 (B + K) / 16
// (the rows still exact, averaged over an epoch, per wavefront) + 0.068 rows
// (barrier, LDS edge exchange, per-row fixed work) + 3.3 / K (the epoch hand-off:
// publish, flag, neighbour wait, halo reload).
gol_status plan_resident(gol_engine* e, const gol_config* cfg)
{
    if (cfg->resident == 1 || e->nranks > 1 || e->sem != GOL_SEM_GLOBAL || e->planes != 2)
        return GOL_OK;
    const bool knobs = cfg->tb_depth || cfg->rows_per_wave || cfg->handoff || cfg->strip_lanes ||
                       cfg->word_planes;
    if (cfg->resident == 0 && knobs) return GOL_OK;
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device));
    const int64_t strips = e->ng <= 64 ? 1 : ((int64_t)e->ng + 61) / 62;
    if (strips > cus) return GOL_OK;
    const int64_t h = (int64_t)e->H;
    double best = 1e300;
    for (int M : gol::kResRowsList) {
        if (cfg->resident == 2 && cfg->rows_per_wave && (uint32_t)M != cfg->rows_per_wave) continue;
        if (gol::resident_blocks_per_cu(M, e->rule) < 1) continue;
        // the generic-mask rule keeps 8 rows per wavefront only with spills
        if (e->rule == gol::RULE_GENERIC && M > 6 && cfg->rows_per_wave != (uint32_t)M) continue;
        const int64_t NR = (int64_t)gol::kResWaves * M;
        const int64_t max_bands = std::min<int64_t>(cus / strips, h);
        for (int64_t nb = 1; nb <= max_bands; ++nb) {
            const int64_t B = (h + nb - 1) / nb;
            const int64_t bands = (h + B - 1) / B;
            int64_t kmax = (NR - B) / 2;
            if (strips > 1) kmax = std::min<int64_t>(kmax, 63);
            int64_t K = (cfg->resident == 2 && cfg->tb_depth) ? (int64_t)cfg->tb_depth : kmax;
            if (K < 1 || K > kmax || (cfg->resident == 0 && K < 8)) continue;
            const int64_t span = (K + B - 1) / B;  // bands a K-row halo reaches
            if ((2 * span + 1) * (strips > 1 ? 3 : 1) - 1 > 64) continue;
            const double cost = 0.17 + 0.046 * (double)(B + K) / gol::kResWaves + 0.068 * M +
                                3.3 / (double)K;
            if (cost < best * 0.999) {
                best = cost;
                e->res.rows = M;
                e->res.strips = (int32_t)strips;
                e->res.bands = (int32_t)bands;
                e->res.band_rows = (int32_t)B;
                e->res.K = (int32_t)K;
            }
        }
    }
    if (best >= 1e300) {
        if (cfg->resident == 2 && (cfg->tb_depth || cfg->rows_per_wave))
            return fail(GOL_EINVAL, "resident: the field does not fit with this tb_depth / rows_per_wave");
        return GOL_OK;
    }
    const size_t tiles = (size_t)e->res.bands * (size_t)e->res.strips;
    HIP_TRY(hipMalloc(&e->res.flags, tiles * sizeof(uint32_t)));
    HIP_TRY(hipMemset(e->res.flags, 0, tiles * sizeof(uint32_t)));
    HIP_TRY(hipEventCreateWithFlags(&e->res.ev_in, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&e->res.ev_out, hipEventDisableTiming));
    e->res.on = true;
    {
        const char* v = std::getenv("GOL_DEV_RES_COOP");
        e->res.coop = v && std::atoi(v) == 1;
    }
#if GOL_DEV_KERNELS
    // dev build: the wave-level temporal blocking of life_resident_mb.hip (r06,
    // measured slower at every MB: DESIGN §4)
    if (const char* v = std::getenv("GOL_DEV_RES_MB")) {
        const int mb = std::atoi(v);
        if (mb >= 2 && gol::resident_mb_exists(e->res.rows, mb, e->rule) &&
            gol::resident_mb_blocks_per_cu(e->res.rows, mb, e->rule) >= 1)
            e->res.mb = mb;
    }
#endif
    e->K = (uint32_t)e->res.K;
    return GOL_OK;
}

// The resident launches of every engine of this process on one device run on one
// shared stream, in order: each needs all its tiles resident at once, one per CU,
// so two side by side could each hold CUs the other's tiles wait for.  (Engines
// of different processes on one GPU are not ordered: their resident waits are
// bounded and a timeout is reported by gol_sync.)
hipStream_t resident_stream(int device)
{
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    std::lock_guard<std::mutex> lock(mu);
    auto it = streams.find(device);
    if (it != streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    streams[device] = s;
    return s;
}

// gol_step on a resident engine: one launch (per 2^30 generations).
gol_status step_resident(gol_engine* e, uint64_t generations)
{
    auto& r = e->res;
    hipStream_t rs = resident_stream(e->device);
    if (!rs) return fail(GOL_EHIP, "resident launch stream");
    HIP_TRY(hipEventRecord(r.ev_in, e->stream));
    HIP_TRY(hipStreamWaitEvent(rs, r.ev_in, 0));
    uint64_t left = generations;
    while (left > 0) {
        const int32_t g = (int32_t)std::min<uint64_t>(left, 1u << 30);
        gol::ResArgs a{};
        a.buf0 = e->buf[e->cur];
        a.buf1 = e->buf[e->cur ^ 1];
        a.flags = r.flags;
        a.err = e->d_err;
        a.stride = (int64_t)e->stride;
        a.h = (int64_t)e->H;
        a.ng = (int64_t)e->ng;
        a.lastmask = e->lastmask_split[0];
        a.strips = r.strips;
        a.bands = r.bands;
        a.band_rows = r.band_rows;
        a.K = r.K;
        a.span = (r.K + r.band_rows - 1) / r.band_rows;
        a.gens = g;
        a.flag_base = r.flag_base;
        a.birth = e->birth;
        a.survive = e->survive;
#if GOL_EXP
        a.wlog = g_dev_wave_log;
#endif
        hipEvent_t e0, e1;
        GOL_TRY(timing_begin(e, rs, &e0, &e1));
#if GOL_DEV_KERNELS
        if (r.mb > 1)
            HIP_TRY(gol::launch_resident_mb(a, r.rows, r.mb, e->rule, r.bands * r.strips, rs));
        else
#endif
            HIP_TRY(gol::launch_resident(a, r.rows, e->rule, r.bands * r.strips, rs, r.coop));
        // lanes process every held row of every tile, every generation (wave-level
        // blocking: rows + mb - 1 per generation on average over a super-step)
        const double comp = (double)g * r.bands * r.strips * gol::kResWaves * (r.rows + r.mb - 1) *
                            64.0 * 64.0;
        GOL_TRY(timing_end(e, rs, e0, e1, (double)e->H * (double)e->W * g, comp));
        const uint32_t epochs = (uint32_t)((g + r.K - 1) / r.K);
        r.flag_base += epochs;
        if (epochs & 1) e->cur ^= 1;
        left -= (uint64_t)g;
    }
    HIP_TRY(hipEventRecord(r.ev_out, rs));
    HIP_TRY(hipStreamWaitEvent(e->stream, r.ev_out, 0));
    return GOL_OK;
}

// `passes` > 1: a multi-pass launch of that many depth-K passes (plans with npass
// >= passes), reading buf[cur] and writing buf[cur + 1 .. cur + passes]
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

gol_status launch(gol_engine* e, int plan, uint32_t depth, bool swap = true,
                  hipStream_t stream = nullptr, int passes = 1)
{
    hipStream_t s = stream ? stream : e->stream;
    const int region = (e->band_stream && s == e->band_stream) ? 1 : 0;
    const auto& p = e->plans[plan];
    if (passes < 1 || (passes > 1 && (passes > p.npass || depth != e->K || !e->mpflags)))
        return fail(GOL_ESTATE, "multi-pass launch of a plan without passes");
    StepArgs a{};
    for (int i = 0; i <= passes; ++i) a.pbuf[i] = e->buf[(e->cur + i) % e->nbuf];
    a.npass = passes;
#if GOL_EXP
    // (timing-only switches that invalidate the field: experimental builds only)
    if (passes > 1)
        if (const char* v = std::getenv("GOL_DEV_MP_FLAGS")) a.mp_dev = (uint32_t)std::atoi(v);
#endif
    a.shadow_off = e->shadow_off;
    a.mpflags = e->mpflags;
    a.err = e->d_err;
    a.segs = p.dev;
    a.nseg = (int32_t)p.segs.size() + (p.pair_units ? 1 : 0);
    if (p.segs.size() == 1) {
        a.seg0_only = 1;
        a.seg0 = p.segs[0];
    }
    a.strips = p.groups;
    a.lane_shift = p.lane_shift;
    a.stride = (int64_t)e->stride;
    a.ng = (int64_t)e->ng;
    a.lastmask[0] = e->lastmask_split[0];  // the kernel works on stored (split) words
    a.lastmask[1] = e->lastmask_split[1];
    a.rows_per_wave = p.rpw;
    a.total_units = p.total_units;
    a.birth = e->birth;
    a.survive = e->survive;
    const bool hand = p.hand && p.multi_blk && e->side[region] &&
                      handoff_fits(p.rpw, (int)depth, e->planes) &&
                      gol::handoff_kernel_exists((int)depth, e->rule);
    if (hand) {
        a.side = e->side[region];
        a.flags = e->flags[region];
        a.side_slot = (int64_t)2 * (depth - 1) * 64 * (e->planes / 2);
        a.tail_off = gol::handoff_toff(p.rpw, (int)depth, e->planes);
        // The pair forms (life_stencil.h stage_rm) take a step's pair parity from
        // its unrolled index, which holds only while a consumer's tail starts at an
        // even step t_side = R + 2: every hand-off block length must be even.
        if ((p.rpw & 1) || (p.rows_old && ((p.rows_old | p.rows_young) & 1)))
            return fail(GOL_ESTATE, "hand-off plan with an odd block length");
    }
    if (p.rows_old) {
        a.rows_per_wave = p.rows_young;
        a.rows_old = p.rows_old;
        a.units_old = p.units_old;
    }
    // (r06 dev A/B, GOL_DEV_XCD_SHIFT) per-XCD row shift between paired blocks:
    // blocks keep >= the length their closure needs after giving up 8 rows
    if (e->xcd_shift && p.segs.size() == 1) {
        const int64_t shortest = p.rows_old ? std::min<int64_t>(p.rows_old, p.rows_young) : p.rpw;
        const bool fits = hand ? handoff_fits(shortest - 8, (int)depth, e->planes) : shortest - 8 >= 2;
        if (fits) a.xcd_shift = e->xcd_shift;
    }
    a.edge = p.edge;
    a.right_q0 = p.right_q0;
    a.half_q0 = p.half_q0;
    a.half_hi = p.half_hi;
    a.pair_units = p.pair_units;
    a.pair0 = p.total_units - p.pair_units;
    a.pairs = p.dpairs;
#if GOL_EXP
    a.wlog = g_dev_wave_log;
    a.prog = g_dev_prog;
#endif
    hipEvent_t e0, e1;
    GOL_TRY(timing_begin(e, s, &e0, &e1));
    HIP_TRY(gol::launch_life(a, (int)depth, e->rule, e->planes, hand, s));
    if (e0) {
        // cell-generations the lanes actually process: every stage of a block
        // computes its rows, a classic block (and the last block of a hand-off
        // segment) also d(d-1) stage-rows of vertical halo, and every strip also
        // its 2 halo lanes
        double comp = 0;
        for (const auto& sg : p.segs) {
            const double n = (double)std::max<int64_t>(0, sg.out_hi - sg.out_lo);
            const double classic = hand ? (double)std::min<int64_t>(1, sg.nblk) : (double)sg.nblk;
            comp += depth * n + classic * depth * (depth - 1.0);
        }
        // (the half strip's units: 64 lanes over one block's rows each, classic)
        double comp_half = 0;
        for (size_t i = 0; i + 2 < p.pairs.size(); i += 3)
            comp_half += depth * (double)p.pairs[i + 2] + depth * (depth - 1.0);
        const double cols = 64.0 * 32.0 * e->planes;  // per strip or unit
        double rows = 0;
        for (const auto& sg : p.segs) rows += (double)std::max<int64_t>(0, sg.out_hi - sg.out_lo);
        GOL_TRY(timing_end(e, s, e0, e1, p.own_rows * (double)e->W * depth * passes,
                           (comp * p.groups + comp_half) * cols * passes, rows * passes));
    }
    if (swap) e->cur = (e->cur + passes) % e->nbuf;
    return GOL_OK;
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

// Order everything the side streams of a stripe engine have enqueued (band
// launches, overlapped exchanges) before the next work on its compute stream, so
// reads of the field on `stream` (store, digest) see the band rows.
gol_status join_side_streams(gol_engine* e)
{
    if (e->band_stream) {
        HIP_TRY(hipEventRecord(e->ev_join, e->band_stream));
        HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_join, 0));
    }
    if (e->comm_stream) {
        HIP_TRY(hipEventRecord(e->ev_join, e->comm_stream));
        HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_join, 0));
    }
    return GOL_OK;
}

// Before a load replaces the field: finish every stream of this engine and the
// neighbours' exchange streams that may still be copying from its buffers.
gol_status quiesce(gol_engine* e)
{
    HIP_TRY(hipSetDevice(e->device));
    if (e->comm_stream) HIP_TRY(hipStreamSynchronize(e->comm_stream));
    if (e->band_stream) HIP_TRY(hipStreamSynchronize(e->band_stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (gol_engine* n : {e->up, e->down})
        if (n && n->comm_stream) HIP_TRY(hipStreamSynchronize(n->comm_stream));
    e->halo_fresh = false;
    return GOL_OK;
}

// The kernel's hand-off wait gives up after a bounded time and flags it: report.
gol_status check_err(gol_engine* e)
{
    if (!e->d_err) return GOL_OK;
    int err = 0;
    HIP_TRY(hipMemcpy(&err, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (!err) return GOL_OK;
    HIP_TRY(hipMemset(e->d_err, 0, sizeof(int)));
    for (int r = 0; r < 2; ++r)
        if (e->flags[r]) {
            const int64_t n = [&] {
                int64_t m = 0;
                for (const auto& p : e->plans) m = std::max(m, p.total_units);
                return m;
            }();
            HIP_TRY(hipMemset(e->flags[r], 0, (size_t)n * sizeof(uint32_t)));
        }
    return fail(GOL_EHIP, "a wait for a neighbour's rows timed out in the stencil kernel; "
                          "the field is not valid");
}

// Halo exchange (replaces exchangeGridData, Parallel_Life_MPI.cpp:104-145, whose
// receives land in copies): Hx rows each way with the up/down neighbour, over
// RCCL or through the caller's host transport.
gol_status exchange_body(gol_engine* e, hipStream_t st);

// An exchange, timed with HIP events on its stream while timing is on (every
// exchange: a few per 1000 generations).
gol_status exchange(gol_engine* e, hipStream_t st)
{
    if (!e->timing_every) return exchange_body(e, st);
    hipEvent_t e0, e1;
    GOL_TRY(get_event(e, &e0));
    GOL_TRY(get_event(e, &e1));
    HIP_TRY(hipEventRecord(e0, st));
    GOL_TRY(exchange_body(e, st));
    HIP_TRY(hipEventRecord(e1, st));
    e->ev_xpending.push_back({e0, e1});
    e->xpending_blocking.push_back(st == e->stream ? 1 : 0);
    return GOL_OK;
}

gol_status exchange_body(gol_engine* e, hipStream_t st)
{
    uint64_t* b = e->buf[e->cur];
    const size_t n = (size_t)e->Hx * e->stride;
    const size_t S = e->stride;
    const bool has_up = e->rank > 0, has_dn = e->rank < e->nranks - 1;
    if (e->xfer == XFER_RCCL) {
        // p2p operations to one peer inside a group are matched in issue order, so
        // the self-loop communicator delivers the up rows to the up halo and the
        // down rows to the down halo
        NCCL_TRY(ncclGroupStart());
        if (has_up) {
            NCCL_TRY(ncclSend(b + e->Hx * S, n, ncclUint64, e->peer_up, e->comm, st));
            NCCL_TRY(ncclRecv(b, n, ncclUint64, e->peer_up, e->comm, st));
        }
        if (has_dn) {
            NCCL_TRY(ncclSend(b + e->R * S, n, ncclUint64, e->peer_dn, e->comm, st));
            NCCL_TRY(ncclRecv(b + (e->R + e->Hx) * S, n, ncclUint64, e->peer_dn, e->comm, st));
        }
        NCCL_TRY(ncclGroupEnd());
        return GOL_OK;
    }
    if (e->xfer != XFER_HOST) return fail(GOL_ESTATE, "engine has no halo transport");
    // host transport: stage the boundary rows, let the caller move them, copy back
    uint64_t* send_up = e->host_xfer;
    uint64_t* recv_up = send_up + n;
    uint64_t* send_dn = recv_up + n;
    uint64_t* recv_dn = send_dn + n;
    if (has_up) HIP_TRY(hipMemcpyAsync(send_up, b + e->Hx * S, n * 8, hipMemcpyDeviceToHost, st));
    if (has_dn) HIP_TRY(hipMemcpyAsync(send_dn, b + e->R * S, n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int rc = e->tp.exchange(e->tp.ctx, has_up ? send_up : nullptr, has_up ? recv_up : nullptr,
                                  has_dn ? send_dn : nullptr, has_dn ? recv_dn : nullptr,
                                  (uint64_t)(n * 8));
    if (rc != 0)
        return fail(GOL_EXFER, "halo transport callback returned " + std::to_string(rc));
    if (has_up) HIP_TRY(hipMemcpyAsync(b, recv_up, n * 8, hipMemcpyHostToDevice, st));
    if (has_dn)
        HIP_TRY(hipMemcpyAsync(b + (e->R + e->Hx) * S, recv_dn, n * 8, hipMemcpyHostToDevice, st));
    // the staging buffers are reused by the next exchange, on either stream
    HIP_TRY(hipStreamSynchronize(st));
    return GOL_OK;
}

}  // namespace

extern "C" {

void gol_config_init(gol_config* cfg)
{
    if (!cfg) return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->birth_mask = GOL_REF_BIRTH;
    cfg->survive_mask = GOL_REF_SURVIVE;
    cfg->device = -1;
    cfg->semantics = GOL_SEM_GLOBAL;
    cfg->ref_ranks = 1;
}

const char* gol_last_error(void) { return g_last_error.c_str(); }

gol_status gol_create(uint64_t h, uint64_t w, const gol_config* cfg, gol_engine** out)
{
    if (!out) return fail(GOL_EINVAL, "null out");
    *out = nullptr;
    gol_status st = check_cfg(cfg);
    if (st != GOL_OK) return st;
    if (h == 0 || w == 0) return fail(GOL_EINVAL, "h and w must be >= 1");
    if (h > (1ull << 40) || w > (1ull << 40)) return fail(GOL_EINVAL, "field too large");
    gol_engine* e = new (std::nothrow) gol_engine();
    if (!e) return fail(GOL_ENOMEM, "host allocation");
    e->R = h;
    uint32_t S = cfg->streams;
    if (S == 0)
        S = (cfg->semantics == GOL_SEM_GLOBAL && h >= kCompositeMinRows && !single_stream_skews(h, w, cfg))
                ? 2
                : 1;
    if (S > 1 && cfg->semantics == GOL_SEM_GLOBAL && h / S >= 256) {
        // composite: S same-device stripes with deep halos, advanced together
        gol_config c = *cfg;
        c.streams = 1;
        // the stripes run side by side on one device, so at most one of them could
        // keep hand-off blocks (gol_create_group); unbalanced stripes lose more than
        // that one gains (profiles/r02/ab_handoff_policy.jsonl): classic blocks
        if (c.handoff == 0) c.handoff = 1;
        const Layout lay = auto_layout(h / S, cfg);
        c.tb_depth = lay.K;
        c.word_planes = (uint32_t)lay.planes;
        if (!c.halo_depth) c.halo_depth = 16 * c.tb_depth;
        int dev = cfg->device;
        if (dev < 0) {
            hipError_t he = hipGetDevice(&dev);
            if (he != hipSuccess) {
                delete e;
                return fail(GOL_EHIP, std::string("hipGetDevice: ") + hipGetErrorString(he));
            }
        }
        std::vector<int> devs(S, dev);
        e->parts.assign(S, nullptr);
        st = gol_create_group(h, w, &c, (int)S, devs.data(), e->parts.data());
        if (st != GOL_OK) {
            e->parts.clear();
            delete e;
            return st;
        }
        e->H = h;
        e->W = w;
        e->wq = (w + 63) / 64;
        e->device = dev;
        e->K = e->parts[0]->K;
        *out = e;
        return GOL_OK;
    }
    st = init_common(e, h, w, cfg, nullptr);
    if (st != GOL_OK) {
        std::string msg = g_last_error;
        gol_destroy(e);
        g_last_error = msg;
        return st;
    }
    *out = e;
    return GOL_OK;
}

gol_status gol_rank_rows(uint64_t h, int nranks, int rank, uint64_t* row0, uint64_t* rows)
{
    if (nranks <= 0 || rank < 0 || rank >= nranks || !row0 || !rows)
        return fail(GOL_EINVAL, "bad rank/nranks");
    const uint64_t base = h / (uint64_t)nranks, extra = h % (uint64_t)nranks;
    const uint64_t r = (uint64_t)rank;
    *rows = base + (r < extra ? 1 : 0);
    *row0 = r * base + std::min(r, extra);
    return GOL_OK;
}

gol_status gol_comm_unique_id(uint8_t id[128])
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
    return GOL_OK;
}

gol_status gol_round_schedule(uint64_t h, uint64_t w, const gol_config* cfg, int rank, int nranks,
                              uint64_t generations, int halo_fresh, gol_sched_op* ops,
                              uint64_t cap, uint64_t* nops, uint32_t* tb_depth,
                              uint32_t* halo_depth)
{
    if (!nops) return fail(GOL_EINVAL, "null nops");
    gol_status st = check_cfg(cfg);
    if (st != GOL_OK) return st;
    if (h == 0 || w == 0) return fail(GOL_EINVAL, "h and w must be >= 1");
    if (cfg->semantics != GOL_SEM_GLOBAL)
        return fail(GOL_EINVAL, "rank engines implement GLOBAL semantics only");
    RankGeom g;
    st = rank_geometry(h, cfg, rank, nranks, &g);
    if (st != GOL_OK) return st;
    if (tb_depth) *tb_depth = g.K;
    if (halo_depth) *halo_depth = (uint32_t)g.Hx;
    std::vector<SchedOp> v;
    if (nranks > 1) {
        step_schedule(g.K, g.Hx, g.overlap, halo_fresh != 0 && g.overlap, generations, v);
    } else {
        for (uint64_t left = generations; left > 0;) {
            const uint32_t d = pick_depth(g.K, left);
            v.push_back({GOL_OP_LAUNCH, d, -1});
            left -= d;
        }
    }
    *nops = v.size();
    if (ops) {
        if (cap < v.size()) return fail(GOL_EINVAL, "schedule needs " + std::to_string(v.size()) + " ops");
        uint32_t shrink = 0;
        for (size_t i = 0; i < v.size(); ++i) {
            gol_sched_op o{};
            o.kind = v[i].kind;
            o.depth = v[i].depth;
            if (o.kind == GOL_OP_EXCHANGE || o.kind == GOL_OP_WAIT_EXCHANGE) shrink = 0;
            if (o.kind == GOL_OP_LAUNCH || o.kind == GOL_OP_BAND) shrink += o.depth;
            o.shrink = o.kind == GOL_OP_EXCHANGE_ASYNC ? 0 : shrink;
            if (v[i].plan >= 0) {
                const auto& segs = g.raw[(size_t)v[i].plan];
                o.nseg = (uint32_t)std::min<size_t>(2, segs.size());
                for (uint32_t k = 0; k < o.nseg; ++k) {
                    o.out_lo[k] = segs[k].out_lo;
                    o.out_hi[k] = segs[k].out_hi;
                }
            } else if (o.kind == GOL_OP_LAUNCH) {  // single stripe: the whole field
                o.nseg = 1;
                o.out_lo[0] = 0;
                o.out_hi[0] = (int64_t)h;
            }
            ops[i] = o;
        }
    }
    return GOL_OK;
}

gol_status gol_plan_model(uint64_t h, uint64_t w, const gol_config* cfg, int rank, int nranks,
                          int cus, int occ_classic, int occ_hand, gol_plan_summary* out)
{
    if (!out) return fail(GOL_EINVAL, "null out");
    *out = gol_plan_summary{};
    gol_status st = check_cfg(cfg);
    if (st != GOL_OK) return st;
    if (h == 0 || w == 0) return fail(GOL_EINVAL, "h and w must be >= 1");
    if (h > (1ull << 40) || w > (1ull << 40)) return fail(GOL_EINVAL, "field too large");
    if (cus <= 0 || occ_classic <= 0 || occ_hand < 0)
        return fail(GOL_EINVAL, "cus and occ_classic must be >= 1, occ_hand >= 0");
    if (nranks > 1 && cfg->semantics != GOL_SEM_GLOBAL)
        return fail(GOL_EINVAL, "rank engines implement GLOBAL semantics only");
    RankGeom g;
    gol_config c = *cfg;
    if (nranks > 1) {
        st = rank_geometry(h, cfg, rank, nranks, &g);
        if (st != GOL_OK) return st;
        c.resident = 1;
        c.tb_depth = g.K;
    } else if (nranks != 1 || rank != 0) {
        return fail(GOL_EINVAL, "rank must be 0 of 1, or 0 <= rank < nranks");
    }
    std::unique_ptr<gol_engine> e(new (std::nothrow) gol_engine());
    if (!e) return fail(GOL_ENOMEM, "host allocation");
    e->model.on = true;
    e->model.cus = cus;
    e->model.occ_c = occ_classic;
    e->model.occ_h = occ_hand;
    if (nranks > 1) {
        e->rank = rank;
        e->nranks = nranks;
        e->row0 = g.row0;
        e->R = g.R;
        e->Hx = g.Hx;
    } else {
        e->R = h;
    }
    GOL_TRY(host_layout(e.get(), h, w, &c));
    std::vector<std::vector<SegDesc>> raw;
    GOL_TRY(raw_regions(e.get(), h, &c, nranks > 1 ? &g : nullptr, raw));
    decide_passes(e.get(), (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride);
    GOL_TRY(build_plans(e.get(), raw));
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const size_t pi = nranks > 1 ? std::min<size_t>(e->plans.size() - 1, e->K - 1) : 0;
    const auto& p = e->plans[pi];
    out->tb_depth = e->K;
    out->halo_depth = (uint32_t)e->Hx;
    out->plans = (uint32_t)e->plans.size();
    for (int a : e->plan_alias) out->distinct_plans += a < 0 ? 1u : 0u;
    out->rows_lo = p.segs.empty() ? 0 : p.segs[0].out_lo;
    out->rows_hi = p.segs.empty() ? 0 : p.segs.back().out_hi;
    out->rows_per_wave = p.rows_old ? p.rows_young : p.rpw;
    out->rows_old = p.rows_old;
    out->units_old = p.units_old;
    out->strips = p.groups;
    out->lane_shift = p.lane_shift;
    out->total_units = p.total_units;
    out->half_units = p.pair_units;
    for (const auto& sg : p.segs) out->blocks += sg.nblk;
    out->handoff = (p.hand && p.multi_blk) ? 1 : 0;
    out->tail_off = out->handoff ? gol::handoff_toff(p.rpw, (int)e->K, e->planes) : -1;
    out->passes = (uint32_t)p.npass;
    out->candidates = pi < e->plan_alts.size() ? (uint32_t)e->plan_alts[pi].size() : 0u;
    return GOL_OK;
}

}  // extern "C"

namespace {

// Geometry + device state of stripe `rank` of `nranks` (no transport yet).
gol_status make_rank_engine(uint64_t h, uint64_t w, const gol_config* cfg, int rank, int nranks,
                            gol_engine** out, bool shared_device = false, bool group = false,
                            bool tune_ok = false)
{
    *out = nullptr;
    gol_status st = check_cfg(cfg);
    if (st != GOL_OK) return st;
    if (cfg->semantics != GOL_SEM_GLOBAL)
        return fail(GOL_EINVAL, "rank engines implement GLOBAL semantics only");
    if (h == 0 || w == 0) return fail(GOL_EINVAL, "h and w must be >= 1");
    RankGeom g;
    st = rank_geometry(h, cfg, rank, nranks, &g, group, tune_ok);
    if (st != GOL_OK) return st;
    gol_engine* e = new (std::nothrow) gol_engine();
    if (!e) return fail(GOL_ENOMEM, "host allocation");
    e->rank = rank;
    e->nranks = nranks;
    e->row0 = g.row0;
    e->R = g.R;
    e->Hx = g.Hx;
    e->shared_device = shared_device;
    e->grouped = group && nranks > 1;  // (decide_passes reads it in init_common)
    // stripe engines run the streaming kernel even as the only rank, so that
    // gol_round_schedule (host-only: no occupancy query for the resident plan)
    // lists exactly the launches gol_step runs
    gol_config c = *cfg;
    c.resident = 1;
    c.tb_depth = g.K;  // (a resident-only epoch length maps to the auto depth)
    st = init_common(e, h, w, &c, &g);
    if (st != GOL_OK) {
        std::string msg = g_last_error;
        gol_destroy(e);
        g_last_error = msg;
        return st;
    }
    *out = e;
    return GOL_OK;
}

// (r07) gol_config.exchange_overlap = 0 on a rank engine over RCCL: time both
// exchange modes on this communicator -- blocking (after the round's last launch)
// and overlapped (band launch, then the exchange on the comm stream beside the
// interior launch) -- and keep the faster.  Both schedules are bit-exact (the
// parity tests run each one); only the time differs, and that depends on what an
// exchange costs: a device-local copy on the RCCL self-loop of a one-GPU box, an
// xGMI transfer plus RCCL's kernels between two MI355X.  Every rank runs the same
// sequence (the same geometry, generations and modes, so its exchanges pair up),
// and the max over ranks of each mode's best sample decides (ncclAllReduce), so all
// ranks keep one mode.  Overlapped must be kXchgMargin faster (samples scatter by
// ~1%).  Like the plan autotuner: on a p = 0.5 field, zeroed again afterwards.
constexpr float kXchgMargin = 0.99f;

gol_status tune_exchange(gol_engine* e)
{
    if (!e->xchg_tune || !e->band_plans || e->xfer != XFER_RCCL) return GOL_OK;
    HIP_TRY(hipSetDevice(e->device));
    const size_t words_all = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    HIP_TRY(gol::launch_init_random(e->buf[e->cur], (int64_t)e->stride, (int64_t)e->wq,
                                    e->lastmask, 0, 0, (int64_t)e->buf_rows, 0x5eedull,
                                    e->planes, e->stream));
    hipEvent_t t0 = nullptr, t1 = nullptr;
    HIP_TRY(hipEventCreate(&t0));
    HIP_TRY(hipEventCreate(&t1));
    // samples of 4 rounds (the last overlapped exchange of a sample is exposed by
    // the join, as at the end of a caller's step); one untimed pass of both modes
    constexpr int kReps = 2, kRounds = 4;
    float best[2] = {1e30f, 1e30f};
    gol_status st = GOL_OK;
    for (int rep = 0; rep <= kReps && st == GOL_OK; ++rep)
        for (int m = 0; m < 2 && st == GOL_OK; ++m) {
            e->overlap = m == 1;  // (a pending overlapped exchange is waited for first)
            float ms = 0;
            if (hipEventRecord(t0, e->stream) != hipSuccess) st = fail(GOL_EHIP, "exchange tuning event");
            if (st == GOL_OK) st = gol_step(e, (uint64_t)kRounds * e->Hx);
            if (st == GOL_OK) st = join_side_streams(e);
            if (st == GOL_OK && (hipEventRecord(t1, e->stream) != hipSuccess ||
                                 hipEventSynchronize(t1) != hipSuccess ||
                                 hipEventElapsedTime(&ms, t0, t1) != hipSuccess))
                st = fail(GOL_EHIP, "exchange tuning timing");
            if (rep > 0) best[m] = std::min(best[m], ms);
        }
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    e->overlap = false;
    if (st == GOL_OK) st = quiesce(e);
    if (st == GOL_OK) st = check_err(e);
    if (st != GOL_OK) return st;
    float agreed[2] = {best[0], best[1]};
    HIP_TRY(hipMemcpy(e->d_acc, agreed, sizeof agreed, hipMemcpyHostToDevice));
    NCCL_TRY(ncclAllReduce(e->d_acc, e->d_acc, 2, ncclFloat32, ncclMax, e->comm, e->stream));
    HIP_TRY(hipMemcpyAsync(agreed, e->d_acc, sizeof agreed, hipMemcpyDeviceToHost, e->stream));
    for (int b = 0; b < e->nbuf; ++b)
        HIP_TRY(hipMemsetAsync(e->alloc[b], 0, words_all * sizeof(uint64_t), e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->xchg_ms[0] = agreed[0] / kRounds;
    e->xchg_ms[1] = agreed[1] / kRounds;
    e->overlap = agreed[1] < kXchgMargin * agreed[0];
    e->halo_fresh = false;
    if (std::getenv("GOL_DEV_PLANS"))
        std::fprintf(stderr, "exchange mode: %s (blocking %.3f ms, overlapped %.3f ms per round)\n",
                     e->overlap ? "overlapped" : "blocking", e->xchg_ms[0], e->xchg_ms[1]);
    return GOL_OK;
}

}  // namespace

extern "C" {

gol_status gol_create_rank(uint64_t h, uint64_t w, const gol_config* cfg, int rank, int nranks,
                           const uint8_t id[128], gol_engine** out)
{
    if (!out || !id) return fail(GOL_EINVAL, "null argument");
    gol_engine* e = nullptr;
    gol_status st = make_rank_engine(h, w, cfg, rank, nranks, &e, false, false, true);
    if (st != GOL_OK) return st;
    if (nranks > 1) {
        ncclUniqueId u;
        std::memcpy(&u, id, 128);
        // the communicator binds to the calling thread's current device
        hipError_t he = hipSetDevice(e->device);
        if (he != hipSuccess) {
            gol_destroy(e);
            return fail(GOL_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
        }
        // GOL_DEV_RCCL_SELF=1 (test hook, tests/test_gpu_rccl.py): RCCL refuses two
        // ranks on one device, so a one-GPU box runs this rank's byte mover against
        // a 1-rank communicator whose up and down peers are the rank itself -- each
        // exchange sends the boundary rows to itself and its halos receive them
        // (a caller's host transport that returns what it is sent does the same)
        // (with an id of its own: every rank of the caller's job is rank 0 of its
        // own communicator)
        const char* selfv = std::getenv("GOL_DEV_RCCL_SELF");
        const bool self_loop = selfv && selfv[0] == '1';
        if (self_loop) {
            ncclResult_t r = ncclGetUniqueId(&u);
            if (r != ncclSuccess) {
                gol_destroy(e);
                return fail(GOL_ERCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
            }
        }
        e->peer_up = self_loop ? 0 : rank - 1;
        e->peer_dn = self_loop ? 0 : rank + 1;
        ncclResult_t r = self_loop ? ncclCommInitRank(&e->comm, 1, u, 0)
                                   : ncclCommInitRank(&e->comm, nranks, u, rank);
        if (r != ncclSuccess) {
            gol_destroy(e);
            return fail(GOL_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        e->xfer = XFER_RCCL;
        st = tune_exchange(e);
        if (st != GOL_OK) {
            std::string msg = g_last_error;
            gol_destroy(e);
            g_last_error = msg;
            return st;
        }
    }
    *out = e;
    return GOL_OK;
}

gol_status gol_create_rank_transport(uint64_t h, uint64_t w, const gol_config* cfg, int rank,
                                     int nranks, const gol_transport* tp, gol_engine** out)
{
    if (!out || !tp || !tp->exchange) return fail(GOL_EINVAL, "null argument");
    *out = nullptr;
    gol_engine* e = nullptr;
    gol_status st = make_rank_engine(h, w, cfg, rank, nranks, &e);
    if (st != GOL_OK) return st;
    if (nranks > 1) {
        e->tp = *tp;
        e->xfer = XFER_HOST;
        const size_t bytes = 4 * (size_t)e->Hx * e->stride * sizeof(uint64_t);
        hipError_t he = hipHostMalloc((void**)&e->host_xfer, bytes, hipHostMallocDefault);
        if (he != hipSuccess) {
            gol_destroy(e);
            return fail(GOL_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(he));
        }
    }
    *out = e;
    return GOL_OK;
}

gol_status gol_create_group(uint64_t h, uint64_t w, const gol_config* cfg, int nranks,
                            const int* devices, gol_engine** engines)
{
    if (!engines || nranks <= 0) return fail(GOL_EINVAL, "bad group arguments");
    for (int r = 0; r < nranks; ++r) engines[r] = nullptr;
    gol_status st = GOL_OK;
    // Hand-off row blocks wait for other wavefronts of their own launch, which
    // is safe when only one such launch runs on a device at a time (a launch's
    // blocks start in order on each XCD; two waiting launches side by side could
    // hold each other's slots).  Members sharing a device run concurrently, so
    // only the first member on each device keeps hand-off blocks.
    std::vector<int> devs;
    for (int r = 0; r < nranks; ++r) {
        int d = devices ? devices[r] : (cfg->device >= 0 ? cfg->device : -1);
        if (d < 0 && hipGetDevice(&d) != hipSuccess) d = -1;
        devs.push_back(d);
    }
    for (int r = 0; r < nranks && st == GOL_OK; ++r) {
        gol_config c = *cfg;
        c.device = devices ? devices[r] : (cfg->device >= 0 ? cfg->device : -1);
        if (std::find(devs.begin(), devs.begin() + r, devs[r]) != devs.begin() + r) c.handoff = 1;
        st = make_rank_engine(h, w, &c, r, nranks, &engines[r],
                              std::count(devs.begin(), devs.end(), devs[r]) > 1, true);
    }
    for (int r = 0; r < nranks && st == GOL_OK; ++r) {
        gol_engine* e = engines[r];
        e->grouped = nranks > 1;
        e->xfer = nranks > 1 ? XFER_GROUP : XFER_NONE;
        e->up = r > 0 ? engines[r - 1] : nullptr;
        e->down = r + 1 < nranks ? engines[r + 1] : nullptr;
        hipError_t he = hipSetDevice(e->device);
        if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_ready, hipEventDisableTiming);
        if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_copied, hipEventDisableTiming);
        for (gol_engine* n : {e->up, e->down}) {
            if (he != hipSuccess || !n || n->device == e->device) continue;
            int can = 0;
            he = hipDeviceCanAccessPeer(&can, e->device, n->device);
            if (he == hipSuccess && can) {
                he = hipDeviceEnablePeerAccess(n->device, 0);
                if (he == hipErrorPeerAccessAlreadyEnabled) {
                    (void)hipGetLastError();
                    he = hipSuccess;
                }
            }
        }
        if (he != hipSuccess) st = fail(GOL_EHIP, std::string("group setup: ") + hipGetErrorString(he));
    }
    if (st != GOL_OK) {
        std::string msg = g_last_error;
        for (int r = 0; r < nranks; ++r) {
            gol_destroy(engines[r]);
            engines[r] = nullptr;
        }
        g_last_error = msg;
    }
    return st;
}

void gol_destroy(gol_engine* e)
{
    if (!e) return;
    if (!e->parts.empty()) {
        for (auto* p : e->parts) (void)hipStreamSynchronize(p->stream);
        for (auto* p : e->parts) gol_destroy(p);
        delete e;
        return;
    }
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->comm_stream) (void)hipStreamSynchronize(e->comm_stream);
    if (e->band_stream) (void)hipStreamSynchronize(e->band_stream);
    // group neighbours may still be copying from this engine's buffers
    for (gol_engine* n : {e->up, e->down}) {
        if (!n) continue;
        if (n->stream) (void)hipStreamSynchronize(n->stream);
        if (n->comm_stream) (void)hipStreamSynchronize(n->comm_stream);
        if (n->band_stream) (void)hipStreamSynchronize(n->band_stream);
    }
    wait_release(e);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    if (e->host_xfer) (void)hipHostFree(e->host_xfer);
    if (e->up) e->up->down = nullptr;
    if (e->down) e->down->up = nullptr;
    if (e->ev_ready) (void)hipEventDestroy(e->ev_ready);
    if (e->ev_copied) (void)hipEventDestroy(e->ev_copied);
    for (hipEvent_t ev : {e->ev_band, e->ev_in, e->ev_xdone, e->ev_join})
        if (ev) (void)hipEventDestroy(ev);
    if (e->band_stream) (void)hipStreamDestroy(e->band_stream);
    if (e->comm_stream) (void)hipStreamDestroy(e->comm_stream);
    for (auto& p : e->plans) free_plan(p);
    for (auto& alts : e->plan_alts)
        for (auto& p : alts) free_plan(p);
    for (int b = 0; b < 4; ++b)
        if (e->alloc[b]) (void)hipFree(e->alloc[b]);
    for (int b = 0; b < 2; ++b) {
        if (e->side[b]) (void)hipFree(e->side[b]);
        if (e->flags[b]) (void)hipFree(e->flags[b]);
    }
    if (e->mpflags) (void)hipFree(e->mpflags);
    if (e->d_err) (void)hipFree(e->d_err);
    if (e->res.flags) (void)hipFree(e->res.flags);
    for (hipEvent_t ev : {e->res.ev_in, e->res.ev_out})
        if (ev) (void)hipEventDestroy(ev);
    for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second.exec);
    if (e->d_acc) (void)hipFree(e->d_acc);
    if (e->d_flag) (void)hipFree(e->d_flag);
    for (const auto* pend : {&e->ev_pending, &e->ev_xpending})
        for (auto& p : *pend) {
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
    for (auto& r : e->ev_rpending) {  // (xend belongs to ev_xpending)
        (void)hipEventDestroy(r.start);
        (void)hipEventDestroy(r.end);
    }
    for (auto ev : e->ev_free) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

static uint64_t user_rows(const gol_engine* e)
{
    uint64_t n = 0;
    for (const auto& r : e->user_regions) n += r.rows;
    return n;
}

static uint64_t load_rows_needed(const gol_engine* e)
{
    // rows of the caller's buffer that a load reads: the whole field for
    // GLOBAL/REF_STRIPES, own rows for a rank engine
    return e->nranks > 1 ? e->R : e->H;
}

}  // extern "C"

// Host <-> device transfer of the load/store regions.  The caller's words use the
// public bit order (bit j = column 64q+j) and are converted to/from the
// engine's lane groups (bitlayout.h).
static gol_status upload(gol_engine* e, const uint64_t* words, uint64_t rs)
{
    GOL_TRY(quiesce(e));
    // clear everything (halos, unused rows) then copy each region, masking pad bits
    const size_t words_all = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    HIP_TRY(hipMemsetAsync(e->alloc[e->cur], 0, words_all * 8, e->stream));
    std::vector<uint64_t> tmp;
    for (const auto& r : e->load_regions) {
        tmp.assign((size_t)r.rows * e->stride, 0);
        const uint64_t urow = e->nranks > 1 ? 0 : r.user_row;
        for (uint64_t i = 0; i < r.rows; ++i) {
            const uint64_t* src = words + (urow + i) * rs;
            uint64_t* dst = tmp.data() + i * e->stride;
            const uint64_t G = (uint64_t)e->planes / 2;
            for (uint64_t gq = 0; gq < e->ng; ++gq) {
                uint64_t c[2] = {0, 0};
                for (uint64_t j = 0; j < G; ++j) {
                    const uint64_t q = gq * G + j;
                    if (q < e->wq) c[j] = q == e->wq - 1 ? (src[q] & e->lastmask) : src[q];
                }
                gol_split_group(c, dst + gq * G, e->planes);
            }
        }
        HIP_TRY(hipMemcpyAsync(e->buf[e->cur] + r.buf_row * e->stride, tmp.data(),
                               tmp.size() * 8, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    return GOL_OK;
}

static gol_status download(gol_engine* e, uint64_t* words, uint64_t rs)
{
    HIP_TRY(hipSetDevice(e->device));
    GOL_TRY(join_side_streams(e));
    std::vector<uint64_t> tmp;
    for (const auto& r : e->user_regions) {
        tmp.resize((size_t)r.rows * e->stride);
        HIP_TRY(hipMemcpyAsync(tmp.data(), e->buf[e->cur] + r.buf_row * e->stride,
                               tmp.size() * 8, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        const uint64_t urow = e->nranks > 1 ? 0 : r.user_row;
        for (uint64_t i = 0; i < r.rows; ++i) {
            uint64_t* dst = words + (urow + i) * rs;
            const uint64_t* src = tmp.data() + i * e->stride;
            const uint64_t G = (uint64_t)e->planes / 2;
            for (uint64_t gq = 0; gq < e->ng; ++gq) {
                uint64_t c[2];
                gol_join_group(src + gq * G, c, e->planes);
                for (uint64_t j = 0; j < G; ++j)
                    if (gq * G + j < e->wq) dst[gq * G + j] = c[j];
            }
        }
    }
    return check_err(e);
}

// composite engines: part r holds field rows [row0_r, row0_r + rows_r)
static void part_rows(const gol_engine* e, size_t r, uint64_t* row0, uint64_t* rows)
{
    gol_rank_rows(e->H, (int)e->parts.size(), (int)r, row0, rows);
}

extern "C" {

gol_status gol_load_packed(gol_engine* e, const uint64_t* words, uint64_t rs)
{
    if (!e || !words) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        for (size_t r = 0; r < e->parts.size(); ++r) {
            uint64_t r0, n;
            part_rows(e, r, &r0, &n);
            gol_status st = gol_load_packed(e->parts[r], words + r0 * rs, rs);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    if (rs < e->wq) return fail(GOL_EINVAL, "row stride smaller than ceil(w/64)");
    return upload(e, words, rs);
}

gol_status gol_load_ascii(gol_engine* e, const char* buf, size_t len)
{
    if (!e || !buf) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        if (len != e->H * (e->W + 1))
            return fail(GOL_EINVAL, "ASCII length must be rows*(w+1) = " +
                                        std::to_string(e->H * (e->W + 1)));
        for (size_t r = 0; r < e->parts.size(); ++r) {
            uint64_t r0, n;
            part_rows(e, r, &r0, &n);
            gol_status st = gol_load_ascii(e->parts[r], buf + r0 * (e->W + 1), n * (e->W + 1));
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    const uint64_t rows = load_rows_needed(e);
    if (len != rows * (e->W + 1))
        return fail(GOL_EINVAL, "ASCII length must be rows*(w+1) = " +
                                    std::to_string(rows * (e->W + 1)) + ", got " +
                                    std::to_string(len));
    // raw bytes to the device, packed there by the ASCII codec kernel
    GOL_TRY(quiesce(e));
    DeviceBytes bytes;
    HIP_TRY(hipMalloc(&bytes.p, len));
    HIP_TRY(hipMemcpyAsync(bytes.p, buf, len, hipMemcpyHostToDevice, e->stream));
    const size_t words_all = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    HIP_TRY(hipMemsetAsync(e->alloc[e->cur], 0, words_all * 8, e->stream));
    HIP_TRY(hipMemsetAsync(e->d_flag, 0, sizeof(int), e->stream));
    for (const auto& r : e->load_regions) {
        const uint64_t urow = e->nranks > 1 ? 0 : r.user_row;
        HIP_TRY(gol::launch_ascii_pack(bytes.p + urow * (e->W + 1), (int64_t)r.rows,
                                       (int64_t)e->W, (int64_t)e->ng,
                                       e->buf[e->cur] + r.buf_row * e->stride,
                                       (int64_t)e->stride, e->d_flag, e->planes, e->stream));
    }
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, e->d_flag, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (bad) return fail(GOL_EINVAL, "malformed ASCII: a line is not w cells followed by '\\n'");
    return GOL_OK;
}

gol_status gol_store_packed(gol_engine* e, uint64_t* words, uint64_t rs)
{
    if (!e || !words) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        for (size_t r = 0; r < e->parts.size(); ++r) {
            uint64_t r0, n;
            part_rows(e, r, &r0, &n);
            gol_status st = gol_store_packed(e->parts[r], words + r0 * rs, rs);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    if (rs < e->wq) return fail(GOL_EINVAL, "row stride smaller than ceil(w/64)");
    return download(e, words, rs);
}

gol_status gol_store_ascii(gol_engine* e, char* buf, size_t len)
{
    if (!e || !buf) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        if (len != e->H * (e->W + 1))
            return fail(GOL_EINVAL, "ASCII length must be rows*(w+1) = " +
                                        std::to_string(e->H * (e->W + 1)));
        for (size_t r = 0; r < e->parts.size(); ++r) {
            uint64_t r0, n;
            part_rows(e, r, &r0, &n);
            gol_status st = gol_store_ascii(e->parts[r], buf + r0 * (e->W + 1), n * (e->W + 1));
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    const uint64_t rows = user_rows(e);
    if (len != rows * (e->W + 1))
        return fail(GOL_EINVAL, "ASCII length must be rows*(w+1) = " +
                                    std::to_string(rows * (e->W + 1)));
    HIP_TRY(hipSetDevice(e->device));
    GOL_TRY(join_side_streams(e));
    DeviceBytes bytes;
    HIP_TRY(hipMalloc(&bytes.p, len));
    for (const auto& r : e->user_regions) {
        const uint64_t urow = e->nranks > 1 ? 0 : r.user_row;
        HIP_TRY(gol::launch_ascii_unpack(e->buf[e->cur] + r.buf_row * e->stride,
                                         (int64_t)e->stride, (int64_t)r.rows, (int64_t)e->W,
                                         (int64_t)e->ng, bytes.p + urow * (e->W + 1), e->planes,
                                         e->stream));
    }
    HIP_TRY(hipMemcpyAsync(buf, bytes.p, len, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return check_err(e);
}

gol_status gol_init_random(gol_engine* e, uint64_t seed)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) {
        for (auto* p : e->parts) {
            gol_status st = gol_init_random(p, seed);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    GOL_TRY(quiesce(e));
    const size_t words_all = (size_t)(e->buf_rows + 2 * gol::kGuardRows) * e->stride;
    HIP_TRY(hipMemsetAsync(e->alloc[e->cur], 0, words_all * 8, e->stream));
    for (const auto& r : e->load_regions)
        HIP_TRY(gol::launch_init_random(e->buf[e->cur], (int64_t)e->stride, (int64_t)e->wq,
                                        e->lastmask, (int64_t)r.buf_row, (int64_t)r.glob_row,
                                        (int64_t)r.rows, seed, e->planes, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return GOL_OK;
}

}  // extern "C"

namespace {

// Loopback exchange of a group member on stream `st`: pull the neighbours'
// boundary rows into this engine's halo rows (same layout as the RCCL exchange).
// `ready` names the neighbour event after which those rows are final.
gol_status pull_halos(gol_engine* e, hipStream_t st, hipEvent_t gol_engine::*ready)
{
    const size_t S = e->stride, n = (size_t)e->Hx * S * sizeof(uint64_t);
    uint64_t* b = e->buf[e->cur];
    if (gol_engine* u = e->up) {
        HIP_TRY(hipStreamWaitEvent(st, u->*ready, 0));
        const uint64_t* src = u->buf[u->cur] + u->R * S;  // its last Hx own rows
        if (u->device == e->device)
            HIP_TRY(hipMemcpyAsync(b, src, n, hipMemcpyDeviceToDevice, st));
        else
            HIP_TRY(hipMemcpyPeerAsync(b, e->device, src, u->device, n, st));
    }
    if (gol_engine* d = e->down) {
        HIP_TRY(hipStreamWaitEvent(st, d->*ready, 0));
        const uint64_t* src = d->buf[d->cur] + d->Hx * S;  // its first Hx own rows
        uint64_t* dst = b + (e->R + e->Hx) * S;
        if (d->device == e->device)
            HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st));
        else
            HIP_TRY(hipMemcpyPeerAsync(dst, e->device, src, d->device, n, st));
    }
    return GOL_OK;
}

// Make the compute stream wait for an overlapped exchange issued at the end of
// the previous round (own halo rows received; for groups also the neighbours'
// pulls of my band rows, which my next launches overwrite).
gol_status wait_fresh_halos(gol_engine* e)
{
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_xdone, 0));
    if (e->grouped) {
        if (e->up) HIP_TRY(hipStreamWaitEvent(e->stream, e->up->ev_xdone, 0));
        if (e->down) HIP_TRY(hipStreamWaitEvent(e->stream, e->down->ev_xdone, 0));
    }
    e->halo_fresh = false;
    return GOL_OK;
}

// Run one launch op of a stripe engine's schedule.  `xchg` starts the
// overlapped exchange after a band launch (on comm_stream after ev_band).
template <class Xchg>
gol_status run_launch_op(gol_engine* e, const SchedOp& op, Xchg&& xchg)
{
    switch (op.kind) {
    case GOL_OP_LAUNCH: return launch(e, op.plan, op.depth);
    case GOL_OP_BAND:
        // band rows on the band stream, concurrent with the interior launch
        HIP_TRY(hipEventRecord(e->ev_in, e->stream));
        HIP_TRY(hipStreamWaitEvent(e->band_stream, e->ev_in, 0));
        GOL_TRY(launch(e, op.plan, op.depth, false, e->band_stream));
        HIP_TRY(hipEventRecord(e->ev_band, e->band_stream));
        return GOL_OK;
    case GOL_OP_INTERIOR:
        GOL_TRY(launch(e, op.plan, op.depth, false));  // interior, overlaps the exchange
        e->cur = (e->cur + 1) % e->nbuf;
        return GOL_OK;
    case GOL_OP_EXCHANGE_ASYNC:
        GOL_TRY(xchg());
        e->halo_fresh = true;
        return GOL_OK;
    default: return fail(GOL_ESTATE, "bad schedule op");
    }
}

// Passes of the next launch of plan `plan` at depth d with `left` generations to
// go: multi-pass plans run up to npass full-depth passes per launch.
int passes_for(const gol_engine* e, int plan, uint32_t d, uint64_t left)
{
    const int np = e->plans[(size_t)plan].npass;
    if (np <= 1 || d != e->K) return 1;
    return (int)std::min<uint64_t>((uint64_t)np, left / d);
}

// Single-stream engines: the launch sequence of gol_step(gens) as a captured
// hipGraph, replayed from the second call on (LRU cache keyed by gens and the
// starting buffer).
gol_status step_single(gol_engine* e, uint64_t generations)
{
    if (e->res.on) return step_resident(e, generations);
    uint64_t left = generations;
    const bool graphable = e->timing_every == 0 && generations >= 4 * (uint64_t)e->K;
    if (graphable) {
        const auto key = std::make_pair(generations, e->cur);
        auto it = e->graphs.find(key);
        if (it == e->graphs.end()) {
            if (e->graphs.size() >= kGraphCache) {
                auto lru = e->graphs.begin();
                for (auto j = e->graphs.begin(); j != e->graphs.end(); ++j)
                    if (j->second.used < lru->second.used) lru = j;
                HIP_TRY(hipStreamSynchronize(e->stream));
                (void)hipGraphExecDestroy(lru->second.exec);
                e->graphs.erase(lru);
            }
            hipGraph_t g = nullptr;
            HIP_TRY(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
            const int cur0 = e->cur;
            gol_status st = GOL_OK;
            while (left > 0 && st == GOL_OK) {
                const uint32_t d = pick_depth(e->K, left);
                const int np = passes_for(e, 0, d, left);
                st = launch(e, 0, d, true, nullptr, np);
                left -= (uint64_t)d * np;
            }
            const hipError_t ce = hipStreamEndCapture(e->stream, &g);
            if (st != GOL_OK) {
                if (g) (void)hipGraphDestroy(g);
                e->cur = cur0;
                return st;
            }
            if (ce != hipSuccess) {
                e->cur = cur0;
                return fail(GOL_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
            }
            hipGraphExec_t x = nullptr;
            const hipError_t ie = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ie != hipSuccess) {
                e->cur = cur0;
                return fail(GOL_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
            }
            it = e->graphs.emplace(key, gol_engine::GraphEntry{x, e->cur, 0}).first;
            e->cur = cur0;
        }
        it->second.used = ++e->graph_clock;
        HIP_TRY(hipGraphLaunch(it->second.exec, e->stream));
        e->cur = it->second.cur_after;
        return GOL_OK;
    }
    while (left > 0) {
        const uint32_t d = pick_depth(e->K, left);
        const int np = passes_for(e, 0, d, left);
        GOL_TRY(launch(e, 0, d, true, nullptr, np));
        left -= (uint64_t)d * np;
    }
    return GOL_OK;
}

}  // namespace

extern "C" {

gol_status gol_step(gol_engine* e, uint64_t generations)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) return gol_group_step(e->parts.data(), (int)e->parts.size(), generations);
    if (e->grouped) return fail(GOL_ESTATE, "group members advance with gol_group_step");
    HIP_TRY(hipSetDevice(e->device));
    if (e->nranks <= 1) return step_single(e, generations);
    auto xchg = [e]() -> gol_status {  // overlapped: on comm after the band launch
        HIP_TRY(hipStreamWaitEvent(e->comm_stream, e->ev_band, 0));
        GOL_TRY(exchange(e, e->comm_stream));
        HIP_TRY(hipEventRecord(e->ev_xdone, e->comm_stream));
        return GOL_OK;
    };
    std::vector<SchedOp> ops;
    step_schedule(e->K, e->Hx, e->overlap, e->halo_fresh, generations, ops);
    // consecutive full-depth launch ops of one block plan (the shared region of a
    // round, rank_geometry) run as one multi-pass launch when the plan has passes
    auto root = [e](int pi) { return e->plan_alias[(size_t)pi] >= 0 ? e->plan_alias[(size_t)pi] : pi; };
    // timing on: each round's compute span (after its exchange op, to after its
    // last launch with the band stream joined) for the per-rank breakdown
    gol_engine::RoundEv rev{nullptr, nullptr, nullptr};
    auto close_round = [e, &rev]() -> gol_status {
        if (!rev.start) return GOL_OK;
        if (e->band_stream) {
            HIP_TRY(hipEventRecord(e->ev_join, e->band_stream));
            HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_join, 0));
        }
        GOL_TRY(get_event(e, &rev.end));
        HIP_TRY(hipEventRecord(rev.end, e->stream));
        e->ev_rpending.push_back(rev);
        rev = {nullptr, nullptr, nullptr};
        return GOL_OK;
    };
    for (size_t i = 0; i < ops.size(); ++i) {
        const SchedOp& op = ops[i];
        if (e->timing_every && (op.kind == GOL_OP_EXCHANGE || op.kind == GOL_OP_WAIT_EXCHANGE))
            GOL_TRY(close_round());
        if (e->timing_every && op.kind == GOL_OP_EXCHANGE_ASYNC && rev.start) {
            // the round's overlapped exchange: its end event is the one exchange() records
            GOL_TRY(run_launch_op(e, op, xchg));
            rev.xend = e->ev_xpending.empty() ? nullptr : e->ev_xpending.back().second;
            continue;
        }
        if (op.kind == GOL_OP_LAUNCH && op.depth == e->K && e->plans[(size_t)op.plan].npass > 1) {
            int n = 1;
            while (n < e->plans[(size_t)op.plan].npass && i + n < ops.size() &&
                   ops[i + n].kind == GOL_OP_LAUNCH && ops[i + n].depth == e->K &&
                   root(ops[i + n].plan) == root(op.plan))
                ++n;
            GOL_TRY(launch(e, op.plan, op.depth, true, nullptr, n));
            i += (size_t)n - 1;
            continue;
        }
        if (op.kind == GOL_OP_EXCHANGE) {
            GOL_TRY(exchange(e, e->stream));
        } else if (op.kind == GOL_OP_WAIT_EXCHANGE) {
            GOL_TRY(wait_fresh_halos(e));
        } else {
            GOL_TRY(run_launch_op(e, op, xchg));
            continue;
        }
        if (e->timing_every) {  // the round's launches start here
            GOL_TRY(get_event(e, &rev.start));
            HIP_TRY(hipEventRecord(rev.start, e->stream));
        }
    }
    return close_round();
}

gol_status gol_group_step(gol_engine** engines, int nranks, uint64_t generations)
{
    if (!engines || nranks <= 0) return fail(GOL_EINVAL, "bad group arguments");
    for (int r = 0; r < nranks; ++r) {
        gol_engine* e = engines[r];
        if (!e || e->rank != r || e->nranks != nranks)
            return fail(GOL_EINVAL, "engines must be the members of one group, in rank order");
    }
    if (nranks == 1) return gol_step(engines[0], generations);
    // every member runs the same schedule (same K, Hx and overlap decision); a
    // member whose halos are not fresh (a reload) makes the round exchange block
    bool fresh = true;
    for (int r = 0; r < nranks; ++r) fresh &= engines[r]->halo_fresh;
    if (!fresh)
        for (int r = 0; r < nranks; ++r) {
            gol_engine* e = engines[r];
            if (e->halo_fresh) {  // its overlapped pulls must land before the new ones
                HIP_TRY(hipSetDevice(e->device));
                GOL_TRY(wait_fresh_halos(e));
            }
            e->halo_fresh = false;
        }
    std::vector<SchedOp> ops;
    step_schedule(engines[0]->K, engines[0]->Hx, engines[0]->overlap, fresh, generations, ops);
    size_t i = 0;
    while (i < ops.size()) {
        // one round: its exchange op, then the launches up to the next exchange
        const SchedOp& x = ops[i++];
        if (x.kind == GOL_OP_EXCHANGE) {
            // blocking exchange on the compute streams (first round after a load)
            for (int r = 0; r < nranks; ++r) {  // every member's state is final
                gol_engine* e = engines[r];
                HIP_TRY(hipSetDevice(e->device));
                HIP_TRY(hipEventRecord(e->ev_ready, e->stream));
            }
            for (int r = 0; r < nranks; ++r) {
                gol_engine* e = engines[r];
                HIP_TRY(hipSetDevice(e->device));
                GOL_TRY(pull_halos(e, e->stream, &gol_engine::ev_ready));
                HIP_TRY(hipEventRecord(e->ev_copied, e->stream));
            }
            for (int r = 0; r < nranks; ++r) {  // neighbours done reading my rows
                gol_engine* e = engines[r];
                HIP_TRY(hipSetDevice(e->device));
                if (e->up) HIP_TRY(hipStreamWaitEvent(e->stream, e->up->ev_copied, 0));
                if (e->down) HIP_TRY(hipStreamWaitEvent(e->stream, e->down->ev_copied, 0));
            }
        } else {
            for (int r = 0; r < nranks; ++r) {
                HIP_TRY(hipSetDevice(engines[r]->device));
                GOL_TRY(wait_fresh_halos(engines[r]));
            }
        }
        size_t j = i;
        while (j < ops.size() && ops[j].kind != GOL_OP_EXCHANGE &&
               ops[j].kind != GOL_OP_WAIT_EXCHANGE)
            ++j;
        // launches; the overlapped pulls are issued once every member has
        // recorded its band event (the callback only marks the round)
        bool pulls_due = false;
        for (int r = 0; r < nranks; ++r) {
            gol_engine* e = engines[r];
            HIP_TRY(hipSetDevice(e->device));
            for (size_t k = i; k < j; ++k)
                GOL_TRY(run_launch_op(e, ops[k], [&pulls_due]() -> gol_status {
                    pulls_due = true;
                    return GOL_OK;
                }));
        }
        if (pulls_due) {
            for (int r = 0; r < nranks; ++r) {
                gol_engine* e = engines[r];
                HIP_TRY(hipSetDevice(e->device));
                HIP_TRY(hipStreamWaitEvent(e->comm_stream, e->ev_band, 0));
                GOL_TRY(pull_halos(e, e->comm_stream, &gol_engine::ev_band));
                HIP_TRY(hipEventRecord(e->ev_xdone, e->comm_stream));
            }
        }
        i = j;
    }
    return GOL_OK;
}

gol_status gol_sync(gol_engine* e)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) {
        for (auto* p : e->parts) {
            gol_status st = gol_sync(p);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->band_stream) HIP_TRY(hipStreamSynchronize(e->band_stream));
    if (e->comm_stream) HIP_TRY(hipStreamSynchronize(e->comm_stream));
    return check_err(e);
}

gol_status gol_digest(gol_engine* e, uint64_t* live, uint64_t* hash)
{
    if (!e || !live || !hash) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        uint64_t L = 0, Hs = 0;
        for (auto* p : e->parts) {
            uint64_t l, h;
            gol_status st = gol_digest(p, &l, &h);
            if (st != GOL_OK) return st;
            L += l;
            Hs += h;
        }
        *live = L;
        *hash = Hs;
        return GOL_OK;
    }
    HIP_TRY(hipSetDevice(e->device));
    GOL_TRY(join_side_streams(e));
    HIP_TRY(hipMemsetAsync(e->d_acc, 0, 2 * sizeof(unsigned long long), e->stream));
    for (const auto& r : e->user_regions)
        HIP_TRY(gol::launch_digest(e->buf[e->cur], (int64_t)e->stride, (int64_t)e->wq,
                                   (int64_t)e->ng, (int64_t)r.buf_row, (int64_t)r.glob_row,
                                   (int64_t)r.rows, e->d_acc, e->planes, e->stream));
    unsigned long long acc[2];
    HIP_TRY(hipMemcpyAsync(acc, e->d_acc, sizeof(acc), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    *live = acc[0];
    *hash = acc[1];
    return check_err(e);
}

gol_status gol_digest_rows(gol_engine* e, uint64_t row0, uint64_t rows, uint64_t* live,
                           uint64_t* hash)
{
    if (!e || !live || !hash) return fail(GOL_EINVAL, "null argument");
    if (row0 > e->H || rows > e->H - row0) return fail(GOL_EINVAL, "rows outside the field");
    if (!e->parts.empty()) {
        uint64_t L = 0, Hs = 0;
        for (auto* p : e->parts) {
            uint64_t l, h;
            gol_status st = gol_digest_rows(p, row0, rows, &l, &h);
            if (st != GOL_OK) return st;
            L += l;
            Hs += h;
        }
        *live = L;
        *hash = Hs;
        return GOL_OK;
    }
    HIP_TRY(hipSetDevice(e->device));
    GOL_TRY(join_side_streams(e));
    HIP_TRY(hipMemsetAsync(e->d_acc, 0, 2 * sizeof(unsigned long long), e->stream));
    for (const auto& r : e->user_regions) {
        // the field rows of this region inside [row0, row0 + rows)
        const uint64_t lo = std::max<uint64_t>(r.glob_row, row0);
        const uint64_t hi = std::min<uint64_t>(r.glob_row + r.rows, row0 + rows);
        if (hi <= lo) continue;
        HIP_TRY(gol::launch_digest(e->buf[e->cur], (int64_t)e->stride, (int64_t)e->wq,
                                   (int64_t)e->ng, (int64_t)(r.buf_row + (lo - r.glob_row)),
                                   (int64_t)lo, (int64_t)(hi - lo), e->d_acc, e->planes,
                                   e->stream));
    }
    unsigned long long acc[2];
    HIP_TRY(hipMemcpyAsync(acc, e->d_acc, sizeof(acc), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    *live = acc[0];
    *hash = acc[1];
    return check_err(e);
}

gol_status gol_comm_info(gol_engine* e, int* count, int* rank, int* peer_up, int* peer_down,
                         int* device)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->comm) return fail(GOL_ESTATE, "engine has no RCCL communicator");
    int n = 0, r = -1, d = -1;
    NCCL_TRY(ncclCommCount(e->comm, &n));
    NCCL_TRY(ncclCommUserRank(e->comm, &r));
    NCCL_TRY(ncclCommCuDevice(e->comm, &d));
    if (count) *count = n;
    if (rank) *rank = r;
    if (peer_up) *peer_up = e->rank > 0 ? e->peer_up : -1;
    if (peer_down) *peer_down = e->rank < e->nranks - 1 ? e->peer_dn : -1;
    if (device) *device = d;
    return GOL_OK;
}

gol_status gol_plan_tuning(gol_engine* e, uint32_t* variant, float* tuned_us, float* model_us)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) return gol_plan_tuning(e->parts[0], variant, tuned_us, model_us);
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const bool rk = e->nranks > 1 && e->Hx >= e->K;
    const auto& p = rk ? e->plans[e->K - 1] : e->plans[0];
    const bool on = !e->res.on;
    if (variant) *variant = on ? (uint32_t)p.tuned : 0u;
    if (tuned_us) *tuned_us = on ? 1e3f * p.tune_ms : 0.f;
    if (model_us) *model_us = on ? 1e3f * p.tune_ms_model : 0.f;
    return GOL_OK;
}

gol_status gol_plan_exchange(gol_engine* e, uint32_t* mode, float* blocking_ms, float* overlapped_ms)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    const gol_engine* s = e->parts.empty() ? e : e->parts[0];
    if (mode) *mode = s->nranks > 1 ? (s->overlap ? 2u : 1u) : 0u;
    if (blocking_ms) *blocking_ms = s->xchg_ms[0];
    if (overlapped_ms) *overlapped_ms = s->xchg_ms[1];
    return GOL_OK;
}

gol_status gol_plan_passes(gol_engine* e, uint32_t* passes)
{
    if (!e || !passes) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) return gol_plan_passes(e->parts[0], passes);
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const bool rk = e->nranks > 1 && e->Hx >= e->K;
    const auto& p = rk ? e->plans[e->K - 1] : e->plans[0];
    *passes = e->res.on ? 1u : (uint32_t)p.npass;
    return GOL_OK;
}

gol_status gol_set_timing(gol_engine* e, int every)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) {
        for (auto* p : e->parts) {
            gol_status st = gol_set_timing(p, every);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    if (every < 0) return fail(GOL_EINVAL, "timing sample interval must be >= 0");
    e->timing_every = (uint32_t)every;
    e->launch_count = 0;
    return GOL_OK;
}

// Copy a timing record into the caller's struct: all of it when the caller says it
// has this header's layout (struct_size), else the r04 prefix only.
static void put_timing(gol_timing* out, const gol_timing& t)
{
    if (out->struct_size == (uint32_t)sizeof(gol_timing)) {
        *out = t;
        out->struct_size = (uint32_t)sizeof(gol_timing);
    } else {
        static_assert(offsetof(gol_timing, struct_size) + sizeof(uint32_t) == GOL_TIMING_R04_BYTES,
                      "r04 gol_timing prefix");
        std::memcpy(out, &t, offsetof(gol_timing, struct_size));
        out->struct_size = GOL_TIMING_R04_BYTES;
    }
}

gol_status gol_get_timing(gol_engine* e, gol_timing* out)
{
    if (!e || !out) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        gol_timing t{};
        for (auto* p : e->parts) {
            gol_timing pt{};
            pt.struct_size = (uint32_t)sizeof(gol_timing);
            gol_status st = gol_get_timing(p, &pt);
            if (st != GOL_OK) return st;
            t.launches += pt.launches;
            t.kernel_ms += pt.kernel_ms;
            t.cell_gens += pt.cell_gens;
            t.cell_gens_computed += pt.cell_gens_computed;
            t.launches_issued += pt.launches_issued;
            t.launch_rows += pt.launch_rows;
            t.exchanges += pt.exchanges;
            t.exchange_ms += pt.exchange_ms;
            t.rounds += pt.rounds;
            t.round_ms += pt.round_ms;
            t.exchange_exposed_ms += pt.exchange_exposed_ms;
        }
        t.streams = (uint32_t)e->parts.size();
        put_timing(out, t);
        return GOL_OK;
    }
    gol_status st = flush_timing(e);
    if (st != GOL_OK) return st;
    gol_timing t = e->tm;
    t.streams = 1;
    put_timing(out, t);
    return GOL_OK;
}

gol_status gol_reset_timing(gol_engine* e)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) {
        for (auto* p : e->parts) {
            gol_status st = gol_reset_timing(p);
            if (st != GOL_OK) return st;
        }
        return GOL_OK;
    }
    gol_status st = flush_timing(e);
    if (st != GOL_OK) return st;
    e->tm = gol_timing{};
    return GOL_OK;
}

gol_status gol_info(gol_engine* e, uint64_t* h, uint64_t* w, uint64_t* row0, uint64_t* rows,
                    uint32_t* tb_depth, uint32_t* halo_depth, uint32_t* rows_per_wave)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) {
        gol_status st = gol_info(e->parts[0], nullptr, nullptr, nullptr, nullptr, tb_depth,
                                 halo_depth, rows_per_wave);
        if (st != GOL_OK) return st;
        if (h) *h = e->H;
        if (w) *w = e->W;
        if (row0) *row0 = 0;
        if (rows) *rows = e->H;
        return GOL_OK;
    }
    // (rank engines: plans[Hx-1], the round's full-depth launch; the band and
    // interior plans come after it)
    const size_t full = (e->nranks > 1 && e->Hx >= 1 && e->plans.size() >= e->Hx) ? e->Hx - 1
                                                                                   : e->plans.size() - 1;
    if (rows_per_wave)
        *rows_per_wave = e->res.on ? (uint32_t)e->res.rows
                                   : e->plans.empty() ? 0 : (uint32_t)e->plans[full].rpw;
    if (h) *h = e->H;
    if (w) *w = e->W;
    if (row0) *row0 = e->row0;
    if (rows) *rows = e->nranks > 1 ? e->R : e->H;
    if (tb_depth) *tb_depth = e->K;
    if (halo_depth) *halo_depth = (uint32_t)e->Hx;
    return GOL_OK;
}

gol_status gol_plan_info(gol_engine* e, uint32_t* strip_lanes, uint32_t* rows_per_wave,
                         uint32_t* word_planes)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty())
        return gol_plan_info(e->parts[0], strip_lanes, rows_per_wave, word_planes);
    if (word_planes) *word_planes = (uint32_t)e->planes;
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    // rank engines: plans[Hx-1] is the full-round launch over own rows; else plans[0]
    const auto& p = e->nranks > 1 ? e->plans[e->Hx - 1] : e->plans[0];
    if (strip_lanes) *strip_lanes = e->res.on ? 64u : (uint32_t)(64 >> p.lane_shift);
    if (rows_per_wave) *rows_per_wave = e->res.on ? (uint32_t)e->res.rows : (uint32_t)p.rpw;
    return GOL_OK;
}

gol_status gol_plan_skew(gol_engine* e, uint32_t* rows_old, uint32_t* rows_young,
                         uint32_t* units_old)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) return gol_plan_skew(e->parts[0], rows_old, rows_young, units_old);
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const auto& p = e->nranks > 1 ? e->plans[e->Hx - 1] : e->plans[0];
    const bool on = !e->res.on && p.rows_old;
    if (rows_old) *rows_old = on ? (uint32_t)p.rows_old : 0u;
    if (rows_young) *rows_young = on ? (uint32_t)p.rows_young : 0u;
    if (units_old) *units_old = on ? (uint32_t)p.units_old : 0u;
    return GOL_OK;
}
gol_status gol_plan_columns(gol_engine* e, uint32_t* strips, uint32_t* half_units,
                            uint32_t* half_groups)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) return gol_plan_columns(e->parts[0], strips, half_units, half_groups);
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const auto& p = e->nranks > 1 ? e->plans[e->Hx - 1] : e->plans[0];
    const bool on = !e->res.on;
    if (strips) *strips = on ? (uint32_t)p.groups : (uint32_t)e->res.strips;
    if (half_units) *half_units = on ? (uint32_t)p.pair_units : 0u;
    if (half_groups)
        *half_groups = on && p.pair_units ? (uint32_t)(p.half_hi - p.half_q0) : 0u;
    return GOL_OK;
}

gol_status gol_plan_resident(gol_engine* e, uint32_t* on, uint32_t* bands, uint32_t* strips)
{
    if (!e || !on) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) {
        *on = 0;
        if (bands) *bands = 0;
        if (strips) *strips = 0;
        return GOL_OK;
    }
    *on = e->res.on ? 1u : 0u;
    if (bands) *bands = (uint32_t)e->res.bands;
    if (strips) *strips = (uint32_t)e->res.strips;
    return GOL_OK;
}

gol_status gol_plan_resident_rows(gol_engine* e, uint32_t* rows, uint32_t* band_rows,
                                  uint32_t* epoch, uint32_t* swap_every)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    const bool on = e->parts.empty() && e->res.on;
    if (rows) *rows = on ? (uint32_t)e->res.rows : 0u;
    if (band_rows) *band_rows = on ? (uint32_t)e->res.band_rows : 0u;
    if (epoch) *epoch = on ? (uint32_t)e->res.K : 0u;
    if (swap_every) *swap_every = on ? (uint32_t)e->res.mb : 0u;
    return GOL_OK;
}

gol_status gol_plan_handoff(gol_engine* e, uint32_t* handoff)
{
    if (!e || !handoff) return fail(GOL_EINVAL, "null argument");
    if (!e->parts.empty()) return gol_plan_handoff(e->parts[0], handoff);
    if (e->plans.empty()) return fail(GOL_ESTATE, "no launch plan");
    const auto& p = e->nranks > 1 ? e->plans[e->Hx - 1] : e->plans[0];
    *handoff = (!e->res.on && p.hand && p.multi_blk && e->side[0] && handoff_fits(p.rpw, (int)e->K, e->planes))
                   ? 1u
                   : 0u;
    return GOL_OK;
}

}  // extern "C"

#if GOL_EXP
// Dev timing builds only: log every stencil wavefront's (start, end) s_memrealtime
// stamps, HW_ID | XCC_ID << 32 and unit into `dev` (4 words per wavefront; null
// turns the log off).  Not part of include/gol.h.
extern "C" __attribute__((visibility("default"))) void gol_dev_set_wave_log(void* dev)
{
    g_dev_wave_log = static_cast<uint64_t*>(dev);
}
#endif
