// engine_internal.h -- what the host side of libgol.so shares between its
// translation units: the engine struct, the stripe geometry, the error macros and
// the internal functions each unit exports to the others.
//   engine.cpp   C ABI lifecycle, load/store, single-field and resident steps,
//                launches and timing, digests, plan queries
//   plan.cpp     launch planning: column layout, rows per wavefront, age-skewed
//                blocks, hand-off vs classic, the plan autotuner
//   stripes.cpp  multi-GPU stripes: rank geometry and halo rounds, the exchange
//                (RCCL, host transport, device copies) and its mode, rank and
//                group engines
// Mirrors main()'s flow in Parallel_Life_MPI.cpp:190-240: create
// (readGridFromFile's allocation :88-89) -> load (:91-99) -> step (the epoch loop
// :215-221 with the halo exchange :104-145) -> store (:157-164).
#pragma once

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

namespace golh __attribute__((visibility("hidden"))) {

using gol::SegDesc;
using gol::StepArgs;

extern thread_local std::string g_last_error;

#if GOL_EXP
// Dev timing builds (tools/exp_build.sh): device buffer the stencil kernel logs
// per-wavefront (start, end, hardware id, unit) into; set by gol_dev_set_wave_log.
extern uint64_t* g_dev_wave_log;
extern uint32_t* g_dev_prog;  // GOL_EXP & 1024: per-SIMD progress words
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

inline Layout auto_layout(uint64_t rows, const gol_config* cfg)
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

inline gol_status fail(gol_status st, const std::string& msg)
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

inline uint64_t last_mask(uint64_t w)
{
    const unsigned rem = (unsigned)(w & 63);
    return rem ? ((1ull << rem) - 1ull) : ~0ull;
}

// Parallel_Life_MPI.cpp:70-81 -- rank r's extended stripe [start, start+rows).
inline bool ref_stripe(uint64_t h, uint64_t P, uint64_t r, uint64_t* start, uint64_t* rows)
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

}  // namespace golh

using namespace golh;  // (internal header: the library's own units only)

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
    // (late r06) exchange_overlap = 0 on a rank engine over RCCL: both modes timed at
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

namespace golh __attribute__((visibility("hidden"))) {

// One operation of a stripe engine's step (gol_sched_op without the rows).
struct SchedOp {
    uint32_t kind, depth;
    int plan;  // launch ops: index into the plans (RankGeom)
};

// ---- engine.cpp
gol_status check_cfg(const gol_config* cfg);
gol_status host_layout(gol_engine* e, uint64_t h, uint64_t w, const gol_config* cfg);
gol_status init_common(gol_engine* e, uint64_t h, uint64_t w, const gol_config* cfg,
                       const RankGeom* geom);
gol_status plan_resident(gol_engine* e, const gol_config* cfg);
gol_status launch(gol_engine* e, int plan, uint32_t depth, bool swap = true,
                  hipStream_t stream = nullptr, int passes = 1);
gol_status get_event(gol_engine* e, hipEvent_t* ev);
gol_status join_side_streams(gol_engine* e);
gol_status quiesce(gol_engine* e);
gol_status check_err(gol_engine* e);

// ---- plan.cpp
bool handoff_fits(int64_t R, int d, int planes);
bool single_stream_skews(uint64_t h, uint64_t w, const gol_config* cfg);
void free_plan(gol_engine::Plan& q);
gol_status build_plans(gol_engine* e, const std::vector<std::vector<SegDesc>>& raw);
void decide_passes(gol_engine* e, size_t words);
gol_status autotune_plans(gol_engine* e);
void resolve_aliases(gol_engine* e);

// ---- stripes.cpp
uint32_t pick_depth(uint32_t K, uint64_t remaining);
void step_schedule(uint32_t K, uint64_t Hx, bool overlap, bool halo_fresh, uint64_t gens,
                   std::vector<SchedOp>& ops);
gol_status step_stripe(gol_engine* e, uint64_t generations);

}  // namespace golh
