#!/usr/bin/env python3
"""A/B of engine configurations (gol_config fields as Engine keyword arguments) in
ONE process, interleaved rounds: wall-clock TCUPS (median of the rounds), kernel
time per launch, work ratio, and whether every variant's digest agrees.

    GOL_LIB=mpi-game-of-life_amd/libgol_dev.so python tools/ab_cfg.py \
        --cfgs '[{}, {"tb_depth": 8, "word_planes": 4}]' --shapes 65536,8448
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

os.environ.setdefault("GOL_DEV_SHARED_WAITS", "1")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cfgs", default='[{}]')
    p.add_argument("--shapes", default="65536")
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--gens", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--rule", default="ref")
    a = p.parse_args()
    pkg = entry.load_package()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    cfgs = json.loads(a.cfgs)
    for sh in a.shapes.split(","):
        h, w = (int(x) for x in sh.split("x")) if "x" in sh else (int(sh), a.width)
        engines = []
        for c in cfgs:
            kw = dict(rule=rule, device=0, streams=1, resident=1)
            kw.update({k: v for k, v in c.items() if k != "env"})
            env = c.get("env", {})  # environment at create (dev knobs)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update({k: str(v) for k, v in env.items()})
            e = pkg.Engine(h, w, **kw)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            e.init_random(1)
            e.step(a.gens)
            e.sync()
            engines.append((c, e, []))
        for _ in range(a.rounds):
            for c, e, ts in engines:
                t0 = time.perf_counter()
                e.step(a.gens)
                e.sync()
                ts.append(time.perf_counter() - t0)
        digests = {e.digest() for _, e, _ in engines}
        for c, e, ts in engines:
            e.set_timing(1)
            e.reset_timing()
            e.step(a.gens)
            e.sync()
            tm = e.timing()
            e.set_timing(0)
            cells = float(h) * w * a.gens
            print(json.dumps({
                "shape": f"{h}x{w}", "rule": a.rule, "cfg": c,
                "handoff": e.handoff, "tb_depth": e.tb_depth, "word_planes": e.word_planes,
                "rows_per_wave": e.rows_per_wave, "age_skew": e.age_skew, "columns": e.columns,
                "gens": a.gens,
                "tcups_wall_median": round(cells / statistics.median(ts) / 1e12, 2),
                "tcups_wall_best": round(cells / min(ts) / 1e12, 2),
                "kernel_us_avg": round(tm["kernel_ms"] / max(tm["launches"], 1) * 1e3, 2),
                "work_ratio": round(tm["cell_gens_computed"] / max(tm["cell_gens"], 1), 4),
                "digests_equal": len(digests) == 1}), flush=True)
            e.close()


if __name__ == "__main__":
    main()
