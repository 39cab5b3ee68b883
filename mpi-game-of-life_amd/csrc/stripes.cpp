// stripes.cpp -- the multi-GPU stripe path of libgol.so (engine_internal.h):
// balanced row stripes with Hx-deep halo rounds (replacing the reference's stripe
// split, Parallel_Life_MPI.cpp:70-81, and its exchangeGridData, :104-145), the
// exchange over RCCL, a caller's host transport or device copies, the exchange
// mode (blocking or overlapped, chosen at create by timing on the communicator),
// rank engines (one process per GPU) and in-process groups.
#include "engine_internal.h"

namespace golh __attribute__((visibility("hidden"))) {

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
    // than its neighbours, whose exchanges then move different row counts (late-r06 fix;
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
    // exchange costs more and may be worth hiding, so (late r06) with
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

// A stripe engine's gol_step (rank engines; group members go through
// gol_group_step): the schedule step_schedule exports, run op by op.
gol_status step_stripe(gol_engine* e, uint64_t generations)
{
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

}  // namespace golh

extern "C" {

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

}  // extern "C"

namespace golh __attribute__((visibility("hidden"))) {

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

// (late r06) gol_config.exchange_overlap = 0 on a rank engine over RCCL: time both
// exchange modes on this communicator -- blocking (after the round's last launch)
// and overlapped (band launch, then the exchange on the comm stream beside the
// interior launch) -- and keep the faster.  Both schedules are bit-exact (the
// parity tests run each one); only the time differs, and that depends on what an
// exchange costs: a device-local copy on the RCCL self-loop of a one-GPU box, an
// xGMI transfer plus RCCL's kernels between two MI355X.  Every rank runs the same
// sequence (the same geometry, generations and modes, so its exchanges pair up),
// and the max over ranks of each mode's best sample decides (ncclAllReduce), so all
// ranks keep one mode.  Overlapped must be 2% faster (kXchgMargin): samples scatter
// by ~1%, and blocking is the mode the one-GPU measurements favoured (3-6% at the
// 2/4/8-way rank shapes over the self-loop, profiles/r06/rank_proxy_exchange_auto.jsonl).  Like the plan autotuner: on a p = 0.5 field, zeroed again afterwards.
constexpr float kXchgMargin = 0.98f;

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
    // the join, as at the end of a caller's step); one untimed pass of both modes,
    // then the best of 3 samples per mode
    constexpr int kReps = 3, kRounds = 4;
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

}  // namespace golh

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

gol_status gol_plan_exchange(gol_engine* e, uint32_t* mode, float* blocking_ms, float* overlapped_ms)
{
    if (!e) return fail(GOL_EINVAL, "null engine");
    const gol_engine* s = e->parts.empty() ? e : e->parts[0];
    if (mode) *mode = s->nranks > 1 ? (s->overlap ? 2u : 1u) : 0u;
    if (blocking_ms) *blocking_ms = s->xchg_ms[0];
    if (overlapped_ms) *overlapped_ms = s->xchg_ms[1];
    return GOL_OK;
}

}  // extern "C"
