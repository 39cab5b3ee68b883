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
+ barrier; max over ranks.  The field is resident in HBM throughout.  Rank 0
prints one JSON line.  `roofline` prices the stencil kernel at SURVEY §8(d)'s
0.25 algorithmic bytes per cell-generation (1 bit read + 1 bit written) against
8 TB/s, using HIP events recorded around every launch on the engine's stream;
`cpu_baseline` times the oracle's scalar port of the reference algorithm
(oracle/gol_oracle.c, int per cell, per-cell neighbour loop) on a bounded
sample on this host's cores.
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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--size", type=int, default=65536, help="field is size x size")
    p.add_argument("--gens", type=int, default=1000, help="generations per step")
    p.add_argument("--tb-depth", type=int, default=0)
    p.add_argument("--word-planes", type=int, default=0)
    p.add_argument("--rows-per-wave", type=int, default=0)
    p.add_argument("--halo-depth", type=int, default=0)
    p.add_argument("--rule", default="ref", choices=["ref", "conway"])
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16)
    return p.parse_args()


def cpu_baseline(threads, w):
    """Oracle port of the reference algorithm, bounded sample: `threads` stripes of
    512 rows x w columns (like mpirun -np threads), 16 generations."""
    orc = entry.load_oracle()
    rows, gens = 512, 64
    t0 = time.perf_counter()
    orc.ref_baseline(rows, w, 0, threads)
    t_init = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc.ref_baseline(rows, w, gens, threads)
    t = time.perf_counter() - t0 - t_init
    cells = threads * rows * w * gens
    return {
        "value": round(cells / t / 1e9, 4),
        "unit": "GCUPS",
        "cores": threads,
        "kind": "port",
        "sample": f"{threads} stripes x {rows} rows x {w} cols, {gens} gens, int32 per cell, "
                  f"per-cell countNeighbours loop (Parallel_Life_MPI.cpp:16-54), "
                  f"{t:.1f} s, init subtracted",
    }


def traffic_for(cfg):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        rec = json.load(open(path))
    except Exception:
        return None
    for r in rec.get("records", []):
        defaults = {"word_planes": 2}
        if all(r.get(k, defaults.get(k, 1)) == cfg.get(k)
               for k in ("size", "tb_depth", "rows_per_wave", "n_gpus", "streams", "word_planes")):
            return r.get("hbm_bytes_per_launch")
    return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if not (world == 1 and a.gpus == 1):
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch with torchrun")

    import torch
    import torch.distributed as dist

    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    n = a.size
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl")
        uid = [pkg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng = pkg.Engine(n, n, rule=rule, device=local, tb_depth=a.tb_depth,
                         rows_per_wave=a.rows_per_wave, halo_depth=a.halo_depth,
                         word_planes=a.word_planes,
                         rank=rank, nranks=world, uid=uid[0])
    else:
        eng = pkg.Engine(n, n, rule=rule, device=local, tb_depth=a.tb_depth,
                         rows_per_wave=a.rows_per_wave, word_planes=a.word_planes)
    eng.init_random(a.seed)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        eng.step(a.gens)
    eng.sync()
    # HIP events around every 8th launch: representative launch durations without
    # the per-event stream cost (~6 us) landing on every launch of the timed region
    eng.set_timing(8)
    eng.reset_timing()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step(a.gens)
    eng.sync()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    tm = eng.timing()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        k = torch.tensor([tm["kernel_ms"] / max(tm["launches"], 1)], dtype=torch.float64,
                         device="cuda")
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        avg_launch_ms = float(k.item())
    else:
        avg_launch_ms = tm["kernel_ms"] / max(tm["launches"], 1)

    cell_gens = float(n) * n * a.gens * a.steps
    gcups = cell_gens / dt / 1e9
    # dominant kernel: the fused stencil; algorithmic bytes per launch =
    # 0.25 B x (own cell-generations one launch produces)
    cg_per_launch = tm["cell_gens"] / max(tm["launches"], 1)
    # a composite engine (gol_config.streams > 1) runs that many stripe launches
    # concurrently, each timed on its own stream: per-launch rate x streams
    streams = max(1, tm.get("streams", 1))
    achieved = BYTES_PER_CELL_GEN * cg_per_launch * streams / (avg_launch_ms / 1e3) / 1e9
    cfg_key = {"size": n, "tb_depth": eng.tb_depth, "rows_per_wave": a.rows_per_wave,
               "n_gpus": world, "streams": streams, "word_planes": eng.word_planes}
    traffic = traffic_for(cfg_key)

    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
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
                "halo_depth": eng.halo_depth,
                "rows_per_wave": eng.rows_per_wave,
                "parallelism": f"row-stripes x{world}" if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": "life_tb_kernel",
                "avg_launch_ms": round(avg_launch_ms, 4),
                "launches": tm["launches"],
                "concurrent_streams": streams,
                "achieved_wall": round(BYTES_PER_CELL_GEN * gcups, 1),
                "cell_gens_per_launch": cg_per_launch,
                "bytes_per_cell_gen": BYTES_PER_CELL_GEN,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not a.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(a.cpu_threads, n)
        print(json.dumps(rec), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
