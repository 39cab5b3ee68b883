#!/usr/bin/env python3
"""Dev tool: the reference program's full surface at a large size -- write a
random data.txt (n x n) + grid_size_data.txt into DIR, run the `gol` CLI, and
report wall times (the reference prints only its own "Total time").

    python tools/cli_e2e.py --n 65536 --gens 1000 --dir /tmp/gol_e2e
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=65536)
p.add_argument("--gens", type=int, default=1000)
p.add_argument("--dir", default="/tmp/gol_e2e")
p.add_argument("--extra", default="")
a = p.parse_args()
os.makedirs(a.dir, exist_ok=True)
t0 = time.perf_counter()
rng = np.random.default_rng(1)
with open(os.path.join(a.dir, "data.txt"), "wb") as f:
    for r0 in range(0, a.n, 1024):
        rows = min(1024, a.n - r0)
        block = np.empty((rows, a.n + 1), dtype=np.uint8)
        block[:, :a.n] = 48 + rng.integers(0, 2, size=(rows, a.n), dtype=np.uint8)
        block[:, a.n] = 10
        f.write(block.tobytes())
with open(os.path.join(a.dir, "grid_size_data.txt"), "w") as f:
    f.write(f"{a.n} {a.n} {a.gens}")
t_gen = time.perf_counter() - t0
out = os.path.join(a.dir, "output.txt")
if os.path.exists(out):
    os.remove(out)
t0 = time.perf_counter()
r = subprocess.run([os.path.join(ROOT, "mpi-game-of-life_amd", "gol"), "--dir", a.dir]
                   + a.extra.split(), capture_output=True, text=True)
t_run = time.perf_counter() - t0
print(json.dumps({"n": a.n, "gens": a.gens, "rc": r.returncode, "generate_s": round(t_gen, 2),
                  "cli_wall_s": round(t_run, 3), "stdout": r.stdout.strip().splitlines()[-1:],
                  "stderr": r.stderr.strip()[-300:],
                  "output_bytes": os.path.getsize(out) if os.path.exists(out) else 0}))
sys.exit(r.returncode)
