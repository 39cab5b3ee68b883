#!/usr/bin/env python3
"""Dev tool: per-rank rate of the N-GPU strong-scaling bench, on ONE GPU.

bench.py --gpus N runs one rank engine per GPU over RCCL.  Here one rank engine
of that split (the slowest kind: a middle rank, halos on both sides) runs alone on
the GPU with a host transport that moves no rows (the B/S2 stencil's cost does not
depend on the data), through the
same schedule: Hx-generation rounds, shrinking launches, band + interior split
with the exchange on its own stream.  Transports (--transports):
  * noop: a native host transport that moves nothing: the engine still stages
    the halo rows through pinned host memory and waits for the band launch on the
    host each round (which RCCL does not);
  * rccl: the RCCL byte mover itself against a self-loop communicator
    (GOL_DEV_RCCL_SELF=1): RCCL's kernels and stream ordering are paid, the
    1 MiB per neighbour and round move as device-local copies instead of over xGMI.
Prints per-rank TCUPS (own rows) and the aggregate N x rate a perfectly balanced
job would report.

    python tools/rank_proxy.py [--size 65536] [--ranks 2,4,8] [--skews auto,0] \
        [--transports noop,rccl] [--overlaps 1,2]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

# engines of this tool are stepped one at a time: no waiting-kernel registry
os.environ.setdefault("GOL_DEV_SHARED_WAITS", "1")


NOOP_C = """#include <stdint.h>
int gol_noop_exchange(void* ctx, const void* su, void* ru, const void* sd, void* rd, uint64_t n)
{ (void)ctx; (void)su; (void)ru; (void)sd; (void)rd; (void)n; return 0; }
"""


def noop_transport(pkg):
    """A native transport that moves nothing (the halo rows keep whatever the
    pinned staging buffers hold): the engine's D2H/H2D staging and stream
    synchronisation stay, the caller's byte mover costs nothing."""
    import ctypes
    import subprocess
    import tempfile
    d = tempfile.mkdtemp()
    src, so = os.path.join(d, "noop.c"), os.path.join(d, "libnoop.so")
    open(src, "w").write(NOOP_C)
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    fn = pkg.HALO_EXCHANGE_FN(ctypes.cast(lib.gol_noop_exchange, ctypes.c_void_p).value)
    return pkg.Transport(fn, None), (lib, fn)


def rank_engine(pkg, n, rank, nranks, tp, handoff=0, overlap=0, transport="noop", hx=0):
    import ctypes
    if transport == "rccl":
        os.environ["GOL_DEV_RCCL_SELF"] = "1"
        try:
            return pkg.Engine(n, n, device=0, rank=rank, nranks=nranks, uid=pkg.unique_id(),
                              handoff=handoff, exchange_overlap=overlap, halo_depth=hx)
        finally:
            os.environ.pop("GOL_DEV_RCCL_SELF", None)
    cfg = pkg.make_config(pkg.REF_RULE, 0, pkg.SEM_GLOBAL, 1, 0, hx, 0, handoff, 0, 0, 0, 0,
                          exchange_overlap=overlap)
    h = ctypes.c_void_p()
    pkg._check(pkg.lib().gol_create_rank_transport(n, n, ctypes.byref(cfg), rank, nranks,
                                                   ctypes.byref(tp), ctypes.byref(h)))
    return pkg.Engine(n, n, _handle=h)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--ranks", default="2,4,8")
    p.add_argument("--skews", default="auto,0", help="GOL_DEV_AGE_SKEW values (auto = unset)")
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--handoff", type=int, default=0, help="gol_config.handoff")
    p.add_argument("--overlaps", default="0", help="gol_config.exchange_overlap values "
                   "(0 auto = blocking for rank engines, 1 blocking, 2 overlapped)")
    p.add_argument("--lib", default="", help="library build to load (GOL_LIB), dev A/B")
    p.add_argument("--transports", default="noop", help="noop and/or rccl (self-loop)")
    p.add_argument("--halo-depths", default="0", help="gol_config.halo_depth values (0 = auto)")
    p.add_argument("--passes", default="1", help="GOL_DEV_PASSES values: passes per "
                   "full-depth launch (1 = single-pass launches, 2-3 multi-pass)")
    p.add_argument("--shrinks", default="0", help="GOL_DEV_RANK_SHRINK values: 0 = one region "
                   "for the full-depth launches of a round (default), 1 = shrinking regions")
    p.add_argument("--env-var", default="", help="another create-time switch to A/B "
                   "(e.g. GOL_DEV_XCD_SHIFT)")
    p.add_argument("--env-values", default="", help="its values, ';'-separated (auto = unset)")
    a = p.parse_args()
    if a.lib:
        os.environ["GOL_LIB"] = os.path.abspath(a.lib)
    pkg = entry.load_package()
    n = a.size
    tp, keep = noop_transport(pkg)  # noqa: F841 (keeps the library and callback alive)
    for N in (int(x) for x in a.ranks.split(",")):
        rank = N // 2
        engines = []
        for trn in a.transports.split(","):
            for ov in (int(x) for x in a.overlaps.split(",")):
                for hx in (int(x) for x in a.halo_depths.split(",")):
                    for shr in a.shrinks.split(","):
                        os.environ["GOL_DEV_RANK_SHRINK"] = shr
                        for npass in a.passes.split(","):
                            os.environ["GOL_DEV_PASSES"] = npass
                            for sk in a.skews.split(","):
                                if sk == "auto":
                                    os.environ.pop("GOL_DEV_AGE_SKEW", None)
                                else:
                                    os.environ["GOL_DEV_AGE_SKEW"] = sk
                                for ev in (a.env_values.split(";") if a.env_var else [None]):
                                    if a.env_var:
                                        if ev == "auto":
                                            os.environ.pop(a.env_var, None)
                                        else:
                                            os.environ[a.env_var] = ev
                                    e = rank_engine(pkg, n, rank, N, tp, a.handoff, ov, trn, hx)
                                    e.init_random(1)
                                    e.step(a.gens)
                                    e.sync()
                                    engines.append(((sk, ov, trn, shr, ev), e, []))
                                if a.env_var:
                                    os.environ.pop(a.env_var, None)
        os.environ.pop("GOL_DEV_AGE_SKEW", None)
        os.environ.pop("GOL_DEV_PASSES", None)
        os.environ.pop("GOL_DEV_RANK_SHRINK", None)
        for _ in range(a.rounds):
            for sk, e, ts in engines:
                t0 = time.perf_counter()
                e.step(a.gens)
                e.sync()
                ts.append(time.perf_counter() - t0)
        for sk, e, ts in engines:
            t = statistics.median(ts)
            rate = e.rows * n * a.gens / t / 1e12
            print(json.dumps({"lib": os.path.basename(os.environ.get("GOL_LIB", "libgol.so")), "size": n, "nranks": N, "rank": rank, "own_rows": e.rows,
                              "halo_depth": e.halo_depth, "tb_depth": e.tb_depth,
                              "rows_per_wave": e.rows_per_wave, "handoff": e.handoff,
                              "age_skew": e.age_skew, "skew_cfg": sk[0], "overlap_cfg": sk[1], "exchange": list(e.exchange),
                              "transport": sk[2], "shrink_cfg": sk[3], "passes": e.passes,
                              **({a.env_var: sk[4]} if a.env_var else {}),
                              "autotune": list(e.tuning),
                              "rank_tcups": round(rate, 2),
                              "aggregate_tcups_if_balanced": round(rate * N, 1),
                              "ms_per_1000_gens": round(t * 1e3 * 1000 / a.gens, 2)}), flush=True)
            e.close()


if __name__ == "__main__":
    main()
