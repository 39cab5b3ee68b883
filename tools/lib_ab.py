#!/usr/bin/env python3
"""Dev A/B of library builds (tools/variant_build.sh): runs bench.py once per
library per repetition, alternating, each in its own process (GOL_LIB), and
prints one JSON line per run with the rate and the mean stencil launch.

    python tools/lib_ab.py --libs libgol.so,libgol_xlds.so [--reps 2] -- [bench args]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi-game-of-life_amd")


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    p = argparse.ArgumentParser()
    p.add_argument("--libs", required=True)
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args(argv)
    for rep in range(a.reps):
        for lib in a.libs.split(","):
            env = dict(os.environ, GOL_LIB=os.path.join(PKG, lib))
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline",
                                "--no-sub-records"] + extra, env=env, capture_output=True,
                               text=True, timeout=600)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rf = rec["roofline"]
            print(json.dumps({"lib": lib, "rep": rep, "args": " ".join(extra),
                              "value": rec["value"], "ms_per_step": rec["ms_per_step"],
                              "avg_launch_ms": rf["avg_launch_ms"], "frac": rf["frac"],
                              "work_ratio": rf["work_ratio"],
                              "autotune": rec["config"].get("autotune")}), flush=True)


if __name__ == "__main__":
    main()
