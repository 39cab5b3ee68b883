// engine.cpp -- host side of libgol.so: the C ABI of include/gol.h.  This unit:
// engine lifecycle, load/store, single-field and resident steps, launches and
// timing, digests and plan queries; planning is plan.cpp, multi-GPU stripes
// stripes.cpp (engine_internal.h).
//
// Owns device memory, the HIP streams, the halo transport (RCCL communicator,
// a caller's host transport, or device copies inside a group) and the launch
// plans.  Mirrors main()'s flow in Parallel_Life_MPI.cpp:190-240: create
// (readGridFromFile's allocation :88-89) -> load (:91-99) -> step (the epoch loop
// :215-221 with the halo exchange :104-145) -> store (:157-164).
#include "engine_internal.h"

namespace golh __attribute__((visibility("hidden"))) {

thread_local std::string g_last_error;

#if GOL_EXP
// Dev timing builds (tools/exp_build.sh): device buffer the stencil kernel logs
// per-wavefront (start, end, hardware id, unit) into; set by gol_dev_set_wave_log.
uint64_t* g_dev_wave_log = nullptr;
uint32_t* g_dev_prog = nullptr;  // GOL_EXP & 1024: per-SIMD progress words
#endif

}  // namespace golh

namespace golh __attribute__((visibility("hidden"))) {


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

gol_status launch(gol_engine* e, int plan, uint32_t depth, bool swap, hipStream_t stream,
                  int passes)
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


}  // namespace golh

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


extern "C" {

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

namespace golh __attribute__((visibility("hidden"))) {


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

}  // namespace golh

extern "C" {

gol_status gol_step(gol_engine* e, uint64_t generations)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    if (!e->parts.empty()) return gol_group_step(e->parts.data(), (int)e->parts.size(), generations);
    if (e->grouped) return fail(GOL_ESTATE, "group members advance with gol_group_step");
    HIP_TRY(hipSetDevice(e->device));
    if (e->nranks <= 1) return step_single(e, generations);
    return step_stripe(e, generations);
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
