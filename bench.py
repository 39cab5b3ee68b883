#!/usr/bin/env python3
"""Benchmark: Game of Life cell updates per second (GCUPS) on MI355X.

BASELINE.json metric: "cell updates/sec (GCUPS) at 65536^2, 1/2/4/8 GPUs; % of HBM
roofline".  Workload (configs[2]/[3]): a 65536 x 65536 bit-packed random field
(splitmix64, p = 0.5, seed 1), dead border, the reference's effective rule B/S2;
one "step" = 1000 generations over the whole field (the C3 job).  At N > 1 the
same field is split into N row stripes, one per GPU and process, with k-deep
RCCL halo exchanges (strong scaling: total work fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Timed region: W untimed steps, then barrier + device sync, K steps, device sync
+ barrier; max over ranks.  No HIP events are recorded inside it (r06); K more
steps with sampled launch events follow it and give the launch durations
(`roofline`) and the per-rank breakdown.  The field is resident in HBM
throughout.  Rank 0 prints one JSON line.

`roofline` names the bound that binds.  The stencil kernel is temporally blocked
(K = 16 generations per launch) and VALU-issue bound, not HBM bound (DESIGN.md
§4), so:
  * bound "valu": achieved = the VALU issue slots the stage logic actually
    issues per second of the timed launches -- cell-generations per launch /
    4096 cells per wave-instruction x the slots the kernel issues per lane group
    and generation (ISSUED_SLOTS: B/S2 21 = 13 v_bitop3 + 2 DPP moves and 2
    v_alignbit at two slots each; B3/S23 24; the pair features of
    life_stencil.h, static count of the steady loop, tools/valu_mix.py) / the
    mean HIP-event launch time x concurrent streams; peak = the spec issue rate,
    1024 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction = 1228.8 G/s
    (MI355X_MICROARCH.md), with the best measured rate beside it
    (profiles/r01/valu_rate.json, 1067 G/s: peak_measured, frac_vs_measured).
    Up to r04 `frac` was priced in the r01-r03 stage logic's slot count (24 / 28,
    STAGE_SLOTS), i.e. normalised throughput; that number stays under
    frac_vs_r03_slot_unit;
  * valu.issue_frac: ALL VALU instructions per launch (rocprofv3 SQ_INSTS_VALU
    of this configuration, committed in profiles/r0N/counters.json: warm-up,
    masks and halo work included) at the same peak;
  * hbm_equiv_frac: SURVEY §8(d)'s 0.25 B per cell-generation x GCUPS / 8 TB/s
    (> 1 is what temporal blocking buys); hbm_measured_frac: the measured HBM
    bytes per launch (FETCH_SIZE/WRITE_SIZE, calibrated; `traffic`) x launches/s.
`cpu_baseline` times the oracle's scalar port of the reference algorithm
(oracle/gol_oracle.c: int per cell, per-cell neighbour loop, Parallel_Life_MPI.cpp
:16-54) on this host's allowed cores, on the benchmark's own field; the reference
binary itself cannot be built here (it includes <windows.h>, :6).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import __graft_entry__ as entry  # noqa: E402

METRIC = "cell updates/sec (GCUPS) at 65536^2, 1/2/4/8 GPUs; % of HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_CELL_GEN = 0.25
SIMDS = 1024  # 256 CUs x 4
# MI355X_MICROARCH.md: each SIMD-32 issues one wave64 VALU instruction per 2 cycles
# at the 2.4 GHz engine clock -> 1.2 G wave-instruction slots per SIMD per second
SPEC_SLOT_RATE = 2.4e9 / 2
CELLS_PER_WAVE_INSTR = 64 * 64  # 64 lanes x one 64-column lane group (2 planes)
# VALU issue slots per lane group and generation of the stage logic (v_bitop3 = 1,
# DPP move and v_alignbit = 2 each): tools/valu_mix.py, profiles/r02/valu_mix.json
STAGE_SLOTS = {"ref": 24, "conway": 28}
# ... and the slots the kernel actually issues for them (r04: both rules reduce the
# pair of rows two outputs share once, life_stencil.h GOL_PAIR_SUM: B/S2 13 v_bitop3,
# B3/S23 16, + 2 DPP moves + 2 v_alignbit per lane group and generation on average)
ISSUED_SLOTS = {"ref": 21, "conway": 24}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--size", type=int, default=65536, help="field is size x size")
    p.add_argument("--gens", type=int, default=1000, help="generations per step")
    p.add_argument("--tb-depth", type=int, default=0)
    p.add_argument("--rows-per-wave", type=int, default=0)
    p.add_argument("--halo-depth", type=int, default=0)
    p.add_argument("--handoff", type=int, default=0)
    p.add_argument("--streams", type=int, default=0)
    p.add_argument("--rule", default="ref", choices=["ref", "conway"])
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-sub-records", action="store_true",
                   help="skip the B3/S23 65536^2 and C2 4096^2 lines after the headline")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = the allowed CPUs")
    return p.parse_args()


def load_json(rel):
    try:
        return json.load(open(os.path.join(ROOT, rel)))
    except Exception:
        return None


def valu_peak_rate():
    """Best measured full-rate VALU issue rate per SIMD (wave-instructions/s)."""
    r = load_json("profiles/r01/valu_rate.json") or {}
    return max(r.get("v_bitop3_b32_at_0mod8_2waves", 0.0), r.get("v_xor_b32", 0.0), 9.0e8)


def valu_mix_rate():
    """Measured issue-slot rate per SIMD of the stage's own instruction mix (1 DPP
    move, 1 v_alignbit, 6 v_bitop3 per chain = 10 slots per 8 instructions; 2 waves
    per SIMD, placed at 4 mod 8 like the kernel's loop): the ceiling the steady loop
    can reach with this mix."""
    r = load_json("profiles/r01/valu_rate.json") or {}
    v = r.get("mix_at_4mod8_2w")
    return v * 10.0 / 8.0 if v else None


# revision of the stage logic whose counters a record holds (per rule): 2 = the
# binary pair sum (r04), 3 = the pair features (r04); records without the field are
# revision 1
STAGE_REV = {"ref": 3, "conway": 3}


def counters_for(cfg):
    """Per-launch PMC record (SQ_INSTS_VALU, HBM bytes) of this configuration: the
    record of the same stage-logic revision, field, rule, depth, streams, GPUs and
    block kind whose rows per wavefront is the same or within 5% (the autotuner's
    skew variants move it by ~3%; at the same work ratio the counters move by well
    under 1%)."""
    recs = []
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # newest first
        recs += (load_json(f"profiles/{rnd}/counters.json") or {}).get("records", [])
    keys = ("size", "rule", "tb_depth", "streams", "n_gpus", "handoff")
    best = None
    for r in recs:
        if not all(r.get(k) == cfg.get(k) for k in keys):
            continue
        if r.get("stage_rev", 1) != STAGE_REV.get(cfg.get("rule"), 1):
            continue
        d = abs(r.get("rows_per_wave", 0) - cfg.get("rows_per_wave", 0))
        if d <= 0.05 * max(1, cfg.get("rows_per_wave", 0)) and (best is None or d < best[0]):  # noqa: E501
            best = (d, r)
    return best[1] if best else None


def host_info():
    """CPU model, the CPUs this process may run on, their physical cores, compiler."""
    import platform
    import subprocess
    allowed = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in allowed:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(),
                       open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    model = platform.processor()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        cc = subprocess.run(["gcc", "--version"], capture_output=True,
                            text=True).stdout.split("\n")[0]
    except Exception:
        cc = "gcc"
    return {"cpu_model": model, "cpus_allowed": len(allowed), "physical_cores": len(cores),
            "compiler": cc + ", -O3 -fPIC (oracle/Makefile)"}


def cpu_baseline(w, seed, threads=0):
    """Oracle port of the reference algorithm (int per cell, per-cell neighbour
    loop) on the benchmark's own field: `threads` stripes of 512 rows x w columns
    (rows [0, threads*512) of the splitmix64 field), each evolved alone like one
    `mpirun -np threads` rank (Parallel_Life_MPI.cpp:199, :215-221, :233-237).
    Two samples, GCUPS from T(E) - T(0) so building the field is not counted:
    E = 160 generations of B/S2 (`value`: the field is p = 0.5 for ~3 generations,
    then sparse, like the GPU run's 1000) and E = 3 on stripes of 2048 rows
    (`dense`: the p = 0.5 regime only)."""
    info = host_info()
    capped = None
    if not threads:
        threads = info["physical_cores"]
        omp = os.environ.get("OMP_NUM_THREADS")
        if omp and omp.isdigit() and int(omp) < threads:
            # the GPU pool gives one GPU's job a CPU share of OMP_NUM_THREADS
            # threads (16) of the host's cores and asks worker pools to stay in it
            capped = (f"{int(omp)} of {threads} physical cores: the GPU box's CPU share for "
                      f"a one-GPU job (OMP_NUM_THREADS={omp}; the pool asks worker pools to "
                      f"stay within it)")
            threads = int(omp)
    orc = entry.load_oracle()
    rows = 512

    def rate(rows, gens):
        t0 = time.perf_counter()
        orc.ref_baseline(rows, w, 0, threads, seed)
        t_init = time.perf_counter() - t0
        t0 = time.perf_counter()
        orc.ref_baseline(rows, w, gens, threads, seed)
        t = time.perf_counter() - t0 - t_init
        return threads * rows * w * gens / t / 1e9, t

    # about 13 s and 3 s of CPU work on the box (16 EPYC 9575F cores)
    sparse_gens, dense_rows = 160, 2048
    gcups, t = rate(rows, sparse_gens)
    dense, td = rate(dense_rows, 3)
    rec = {
        "value": round(gcups, 4),
        "unit": "GCUPS",
        "cores": threads,
        "kind": "port",
        "why_port": "the reference binary is unbuildable here: Parallel_Life_MPI.cpp:6 "
                    "includes <windows.h>",
        "sample": f"{threads} stripes x {rows} rows x {w} cols of the bench field (splitmix64 "
                  f"seed {seed}), E = {sparse_gens} generations of B/S2 (dense for ~3 generations, "
                  f"then sparse), T(E) - T(0) = {t:.2f} s",
        "per_core_mcups": round(gcups * 1e3 / threads, 1),
        "dense": {"value": round(dense, 4), "unit": "GCUPS",
                  "per_core_mcups": round(dense * 1e3 / threads, 1),
                  "sample": f"{threads} stripes x {dense_rows} rows x {w} cols of the same field, "
                            f"E = 3 generations (p = 0.5 throughout), "
                            f"T(E) - T(0) = {td:.2f} s"},
        "cores_capped": capped,
    }
    rec.update(info)
    return rec


def ctl_device(dist):
    """Device of the control-plane tensors (timing max, digest sums)."""
    return "cpu" if dist.get_backend() == "gloo" else "cuda"


def rccl_selfcheck(pkg, dist, torch, world, rank, local, handoff=0):
    """N > 1: the RCCL halo path end to end on a small field before the timed run.
    Every rank advances its stripe of a 4096^2 B3/S23 field (rounds of Hx
    generations with ncclSend/Recv exchanges); rank 0 evolves the whole field
    alone on its GPU and compares, per rank, that rank's stripe digest with the
    single engine's digest of the same rows (gol_digest_rows), and the sum of all
    of them with the single engine's whole-field digest.  Each rank also reports
    its communicator as RCCL sees it (gol_comm_info: ncclCommCount, user rank,
    device, up/down peers), so that a first multi-GPU failure is diagnosable from
    the record alone.  Not part of the timed region."""
    n, gens, seed = 4096, 3 * 64 + 21, 5
    uid = [pkg.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    with pkg.Engine(n, n, rule=pkg.CONWAY, device=local, rank=rank, nranks=world,
                    uid=uid[0], handoff=handoff) as e:
        hx = e.halo_depth
        row0, rows = e.row0, e.rows
        try:
            comm = e.comm_info()
        except Exception as ex:  # noqa: BLE001 -- reported, not fatal here
            comm = {"error": str(ex)}
        e.init_random(seed)
        e.step(gens)
        mine = e.digest()
    per = [None] * world
    dist.all_gather_object(per, {"rank": rank, "row0": row0, "rows": rows,
                                 "digest": list(mine), "comm": comm,
                                 "device": local})
    mask = (1 << 64) - 1
    got = (sum(p["digest"][0] for p in per) & mask, sum(p["digest"][1] for p in per) & mask)
    rec = {"field": f"{n}x{n}", "rule": "B3/S23", "generations": gens, "halo_depth": hx,
           "ranks": world}
    if rank == 0:
        with pkg.Engine(n, n, rule=pkg.CONWAY, device=local, handoff=handoff) as ref:
            ref.init_random(seed)
            ref.step(gens)
            want = ref.digest()
            for p in per:
                w = ref.digest_rows(p["row0"], p["rows"])
                p["want"] = list(w)
                p["ok"] = tuple(p["digest"]) == w
        rec["ok"] = got == want and all(p["ok"] for p in per)
        rec["digest"] = list(got)
        rec["want"] = list(want)
        rec["per_rank"] = per
    return rec


def timed_steps(eng, gens, steps, warmup, world, dist, torch, timing_every=8):
    """W untimed steps, then K steps between barrier + device sync brackets with
    no events on the streams (single-stream engines replay their hipGraph): the
    measured time.  Then K more steps with HIP events around every
    `timing_every`-th launch (and, on rank engines, every halo round and
    exchange): the launch durations and the per-rank breakdown.  Returns
    (seconds, seconds of the event pass, timing of the event pass)."""
    def barrier():
        if world > 1:
            dist.barrier()

    def region():
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.step(gens)
        eng.sync()
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0
    for _ in range(warmup):
        eng.step(gens)
    eng.sync()
    eng.set_timing(0)
    dt = region()
    eng.set_timing(timing_every)
    eng.reset_timing()
    dt_ev = region()
    tm = eng.timing()
    eng.set_timing(0)
    return dt, dt_ev, tm


def rank_breakdown(eng, tm, dt, steps, rank):
    """Where one rank's step time goes, from its own HIP events (N > 1), as
    measured spans that add up to ms_per_step in both exchange modes (r06):
      kernel_span: each halo round's compute-stream span, from before its first
        launch to after its last (band stream joined), summed (launch gaps
        inside a round included);
      exchange: the halo exchanges' own stream time (RCCL's includes waiting for
        the peers), split into exchange_exposed (outside the round spans: all of
        a blocking exchange, the tail of an overlapped one past its round's end)
        and exchange_hidden (the rest, under the interior launch);
      other = ms_per_step - kernel_span - exchange_exposed: host work and gaps
        between rounds (the max-over-ranks barrier is not in it).
    avg_launch_ms: the mean sampled launch (overlapped band and interior launches
    run concurrently, so launches x mean is not a time share).  Rows per launch =
    the buffer rows a full-depth launch computes (stripes.cpp rank_geometry)."""
    launches = max(tm["launches"], 1)
    avg = tm["kernel_ms"] / launches
    span = tm["round_ms"] / steps
    xch = tm["exchange_ms"] / steps
    exposed = tm["exchange_exposed_ms"] / steps
    ms = dt / steps * 1e3
    return {
        "rank": rank, "own_rows": eng.rows, "row0": eng.row0, "halo_depth": eng.halo_depth,
        "tb_depth": eng.tb_depth, "rows_per_wave": eng.rows_per_wave, "handoff": eng.handoff,
        "age_skew": eng.age_skew, "autotune": list(eng.tuning),
        "ms_per_step": round(ms, 3),
        "launches_per_step": round(tm["launches_issued"] / steps, 2),
        "rows_per_launch": round(tm["launch_rows"] / launches, 1),
        "avg_launch_ms": round(avg, 4),
        "own_tcups_per_launch": round(eng.rows * eng.w * eng.tb_depth / (avg * 1e-3) / 1e12, 2)
        if avg > 0 else None,
        "rounds_per_step": round(tm["rounds"] / steps, 2),
        "kernel_span_ms_per_step": round(span, 3),
        "exchanges_per_step": round(tm["exchanges"] / steps, 2),
        "exchange_ms_per_step": round(xch, 3),
        "exchange_exposed_ms_per_step": round(exposed, 3),
        "exchange_hidden_ms_per_step": round(xch - exposed, 3),
        "other_ms_per_step": round(ms - span - exposed, 3),
    }


def valu_frac(tm, rule):
    """The VALU issue slots the stage logic issues per second of the sampled
    launches over the spec issue rate (module docstring), and the work ratio."""
    launches = max(tm["launches"], 1)
    launch_s = tm["kernel_ms"] / launches / 1e3
    cg = tm["cell_gens"] / launches
    streams = max(1, tm.get("streams", 1))
    achieved = cg / CELLS_PER_WAVE_INSTR * ISSUED_SLOTS[rule] * streams / max(launch_s, 1e-12)
    return (round(achieved / (SIMDS * SPEC_SLOT_RATE), 4),
            round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1), 4))


def sub_record(pkg, torch, local, size, rule, gens, steps, warmup, seed):
    """One more N = 1 configuration, timed like the headline (its own engine):
    north_star's literal rule B3/S23 at 65536^2, or the C2 field 4096^2 (resident
    kernel)."""
    r = pkg.REF_RULE if rule == "ref" else pkg.CONWAY
    with pkg.Engine(size, size, rule=r, device=local) as eng:
        eng.init_random(seed)
        dt, _, tm = timed_steps(eng, gens, steps, warmup, 1, None, torch)
        frac, work = valu_frac(tm, rule)
        return {
            "workload": f"{size}x{size}, {gens} generations per step, "
                        f"{'B/S2' if rule == 'ref' else 'B3/S23'}",
            "value": round(float(size) * size * gens * steps / dt / 1e9, 2),
            "unit": "GCUPS",
            "steps": steps, "warmup": warmup,
            "ms_per_step": round(dt / steps * 1e3, 3),
            "kernel": "life_res_kernel" if eng.resident else "life_tb_kernel",
            "avg_launch_ms": round(tm["kernel_ms"] / max(tm["launches"], 1), 4),
            "valu_frac": frac,
            "work_ratio": work,
            "tb_depth": eng.tb_depth, "resident": eng.resident, "age_skew": eng.age_skew,
            "autotune": list(eng.tuning),
        }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GOL_DEV_RCCL_SELF=1 (rehearsal of the N > 1 path on a one-GPU box): every
    # rank's engine talks RCCL to itself (stripes.cpp gol_create_rank), ranks share
    # the GPUs there are, torch.distributed runs over gloo (RCCL refuses two ranks
    # of one communicator on one device), and rccl_selfcheck is expected to fail
    # (a self-looped stripe is not the field's stripe).  Such a record carries
    # "rehearsal": true, the physical GPU count, and `value` null (the rate is
    # under "rehearsal_value"): it is never an N-GPU result.
    rehearsal = os.environ.get("GOL_DEV_RCCL_SELF") == "1"
    if world != a.gpus:
        if not (world == 1 and a.gpus == 1):
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch with torchrun")

    import torch
    import torch.distributed as dist

    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    n = a.size
    if rehearsal:
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    kw = dict(rule=rule, device=local, tb_depth=a.tb_depth, rows_per_wave=a.rows_per_wave,
              handoff=a.handoff)
    # ranks sharing a GPU (the one-GPU rehearsal) must not run kernels that wait for
    # other wavefronts of their own launch: two such launches from two processes can
    # hold each other's slots (the per-process registry cannot see the other
    # process).  Classic blocks there, as gol-mpi does when ranks share a GPU.
    shared_gpu = rehearsal and world > max(1, torch.cuda.device_count())
    if shared_gpu and not a.handoff:
        kw["handoff"] = 1

    def barrier():
        if world > 1:
            dist.barrier()

    def rank_engine(overlap):
        uid = [pkg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        return pkg.Engine(n, n, halo_depth=a.halo_depth, rank=rank, nranks=world, uid=uid[0],
                          exchange_overlap=overlap, **kw)

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=ctl_device(dist))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    modes = None
    if world > 1:
        dist.init_process_group("gloo" if rehearsal else "nccl")
        selfcheck = rccl_selfcheck(pkg, dist, torch, world, rank, local, kw["handoff"])
        # each exchange mode forced -- overlapped (band launch + RCCL exchange on a
        # side stream beside the interior launch, exchange_overlap = 2) and blocking
        # (after the round's last launch, 1) -- over the same K steps, reported beside
        # `value`, which is the default engine's: exchange_overlap = 0, the mode the
        # engine chose at create by timing both on this communicator (late r06)
        modes = {}
        for name, ov in (("overlapped", 2), ("blocking", 1)):
            eng = rank_engine(ov)
            eng.init_random(a.seed)
            m_dt, m_dt_ev, m_tm = timed_steps(eng, a.gens, a.steps, a.warmup, world, dist, torch, 8)
            m_per = [None] * world
            dist.all_gather_object(m_per, rank_breakdown(eng, m_tm, m_dt_ev, a.steps, rank))
            m_dt = max_over_ranks(m_dt)
            modes[name] = {"value": round(float(n) * n * a.gens * a.steps / m_dt / 1e9, 2),
                           "ms_per_step": round(m_dt / a.steps * 1e3, 3),
                           "halo_depth": eng.halo_depth, "per_rank": m_per}
            eng.close()
        eng = rank_engine(0)
    else:
        eng = pkg.Engine(n, n, streams=a.streams, **kw)
        selfcheck = None
    eng.init_random(a.seed)

    # the timed region runs without events; a second pass of K steps with HIP
    # events around every 8th launch (representative launch durations without the
    # per-event stream cost, ~6 us, on every launch) gives the launch times, the
    # roofline and the per-rank breakdown
    dt, dt_ev, tm = timed_steps(eng, a.gens, a.steps, a.warmup, world, dist, torch, 8)
    per_rank = None
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, rank_breakdown(eng, tm, dt_ev, a.steps, rank))
    dt_ev = max_over_ranks(dt_ev)
    dt = max_over_ranks(dt)
    avg_launch_ms = max_over_ranks(tm["kernel_ms"] / max(tm["launches"], 1))

    cell_gens = float(n) * n * a.gens * a.steps
    gcups = cell_gens / dt / 1e9
    if modes is not None:
        mode, tb, to = eng.exchange
        modes["auto"] = {"value": round(gcups, 2), "ms_per_step": round(dt / a.steps * 1e3, 3),
                         "halo_depth": eng.halo_depth, "default": True, "mode": mode,
                         # the create-time rounds both modes ran (max over ranks)
                         "tuned_ms_per_round": {"blocking": tb, "overlapped": to},
                         "per_rank": per_rank}
    ok = selfcheck is None or selfcheck.get("ok", True)
    # dominant kernel: the fused stencil (HIP events on each stripe's stream)
    cg_per_launch = tm["cell_gens"] / max(tm["launches"], 1)
    # a composite engine (gol_config.streams > 1) runs that many stripe launches
    # concurrently, each timed on its own stream: per-launch rate x streams
    streams = max(1, tm.get("streams", 1))
    launch_s = avg_launch_ms / 1e3
    peak_slot_rate = SIMDS * SPEC_SLOT_RATE  # wave-instruction slots / s (spec)
    meas_slot_rate = SIMDS * valu_peak_rate()  # best measured issue rate
    slots_per_launch = cg_per_launch / CELLS_PER_WAVE_INSTR * ISSUED_SLOTS[a.rule]
    valu_achieved = slots_per_launch * streams / launch_s
    cfg_key = {"size": n, "rule": a.rule, "tb_depth": eng.tb_depth, "streams": streams,
               "n_gpus": world, "rows_per_wave": eng.rows_per_wave, "handoff": eng.handoff}
    ctr = counters_for(cfg_key) or {}
    insts = ctr.get("insts_valu_per_launch")
    traffic = ctr.get("hbm_bytes_per_launch")
    tuning = eng.tuning
    eng.close()

    # north_star's literal rule (B3/S23) at 65536^2 and the C2 field (4096^2,
    # resident kernel), timed after the headline on rank 0 at N = 1
    subs = None
    if world == 1 and not a.no_sub_records and n == 65536 and a.gens == 1000:
        subs = {
            ("conway_65536" if a.rule == "ref" else "ref_65536"): sub_record(pkg, torch, local, 65536,
                                       "conway" if a.rule == "ref" else "ref", 1000, 3, 1, a.seed),
            "c2_4096": sub_record(pkg, torch, local, 4096, a.rule, 1000, 3, 1, a.seed),
        }

    if rank == 0:
        rec = {
            "metric": METRIC,
            # a failed RCCL self-check voids the multi-GPU number; a rehearsal on
            # one GPU (self-looped RCCL) is never the N-GPU number
            "value": round(gcups, 2) if (ok and not rehearsal) else None,
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            # the same K steps with HIP events on the streams (the launch timing pass)
            "ms_per_step_event_pass": round(dt_ev / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": f"synthetic: splitmix64 p=0.5 field, seed {a.seed}, generated on device",
            "config": {
                "workload": f"{n}x{n} bit-packed random grid, {a.gens} generations per step",
                "h": n, "w": n, "gens_per_step": a.gens,
                "rule": "B/S2 (reference effective rule)" if a.rule == "ref" else "B3/S23",
                "tb_depth": eng.tb_depth, "word_planes": eng.word_planes,
                "halo_depth": eng.halo_depth, "rows_per_wave": eng.rows_per_wave,
                "handoff": eng.handoff, "resident": eng.resident,
                # N > 1: the exchange mode the rank engines chose at create (late r06)
                "exchange": eng.exchange[0] if world > 1 else None,
                "age_skew": eng.age_skew,
                # (strips per row block, half-strip wavefronts, half-strip lane groups)
                "columns": list(eng.columns),
                # the plan the timed launches ran: the cost models' plan or the
                # autotuner's variant, with the create-time best launch (us) of
                # each (plan.cpp autotune_plans; rank 0's first full-depth plan)
                "autotune": {"variant": tuning[0], "launch_us": tuning[1],
                             "models_launch_us": tuning[2],
                             "gain": (round(tuning[2] / tuning[1] - 1, 4)
                                      if tuning[1] and tuning[2] else None)},
                "parallelism": f"row-stripes x{world}" if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(valu_achieved / 1e9, 1),
                "peak": round(peak_slot_rate / 1e9, 1),
                "unit": "G VALU issue slots/s (the slots the stage logic issues: v_bitop3 "
                        "1 slot, DPP move and v_alignbit 2 slots)",
                "frac": round(valu_achieved / peak_slot_rate, 4),
                # the same rate in the r01-r03 slot unit (24 / 28 per lane group and
                # generation): normalised throughput, the r04 headline `frac`
                "frac_vs_r03_slot_unit": round(valu_achieved / peak_slot_rate * STAGE_SLOTS[a.rule]
                                               / ISSUED_SLOTS[a.rule], 4),
                "peak_from": "MI355X_MICROARCH.md: 1024 SIMD-32 x 2.4 GHz / 2 cycles per wave64 "
                             "VALU instruction",
                "peak_measured": round(meas_slot_rate / 1e9, 1),
                "frac_vs_measured": round(valu_achieved / meas_slot_rate, 4),
                "peak_measured_from": "profiles/r01/valu_rate.json (v_bitop3, 2 waves/SIMD, best "
                                      "code placement) x 1024 SIMDs",
                # the stage's instruction mix in a microbenchmark at 2 waves/SIMD
                "peak_mix_measured": (round(SIMDS * valu_mix_rate() / 1e9, 1)
                                      if valu_mix_rate() else None),
                "frac_vs_mix": (round(valu_achieved / (SIMDS * valu_mix_rate()), 4)
                                if valu_mix_rate() else None),
                "traffic": traffic,
                "kernel": "life_res_kernel" if eng.resident else "life_tb_kernel",
                "avg_launch_ms": round(avg_launch_ms, 4),
                "launches": tm["launches"],
                "concurrent_streams": streams,
                "cell_gens_per_launch": cg_per_launch,
                "work_ratio": round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1), 4),
                "valu": {
                    "slots_per_word_gen": ISSUED_SLOTS[a.rule],
                    "r03_unit_slots_per_word_gen": STAGE_SLOTS[a.rule],
                    "insts_per_launch": insts,
                    "issue_frac": (round(insts * streams / launch_s / peak_slot_rate, 4)
                                   if insts else None),
                    "issue_frac_vs_measured": (round(insts * streams / launch_s / meas_slot_rate, 4)
                                               if insts else None),
                    "counters_from": (f"profiles/{ctr.get('source_round', 'r02')}/counters.json "
                                      f"(record {ctr.get('source')}, rows_per_wave "
                                      f"{ctr.get('rows_per_wave')})" if insts else None),
                },
                "hbm_equiv_frac": round(BYTES_PER_CELL_GEN * gcups / HBM_PEAK_GBPS, 4),
                "hbm_measured_frac": (round(traffic * streams / launch_s
                                            / (HBM_PEAK_GBPS * 1e9), 4) if traffic else None),
            },
            "sub_records": subs,
            "cpu_baseline": None,
            "rccl_selfcheck": selfcheck,
            "exchange_modes": modes,
        }
        if rehearsal:
            rec["rehearsal"] = True
            rec["rehearsal_classic_blocks"] = shared_gpu
            rec["rehearsal_value"] = round(gcups, 2)
            rec["physical_gpus"] = torch.cuda.device_count()
        if world == 1 and not a.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(n, a.seed, a.cpu_threads)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and not ok and not rehearsal:
        print("rccl_selfcheck failed: the RCCL halo path does not reproduce the single "
              "field", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
