#!/usr/bin/env python3
"""Dev tool: per-plan launch durations of a rank engine (tools/rank_plans.py run
under rocprofv3 --kernel-trace).  Launch j of every round runs the plan of its cumulative shrink,
plans[(j+1) K - 1] (stripes.cpp round_ops); prints
per plan: rows, blocks kind and lengths, mean duration, and the rate per row.

    python tools/plan_trace.py gpurun_out/r03n/t256 gpurun_out/r03n/plans256.err gpurun_out/r03n/plans256.json
"""
import csv
import glob
import json
import re
import statistics
import sys


def main():
    tdir, err, js = sys.argv[1:4]
    info = [json.loads(l) for l in open(js) if l.startswith("{")][-1]
    L = info["launches_per_round"]
    plans = []
    for line in open(err):
        m = re.match(r"plan (\d+): rows \[(-?\d+), (-?\d+)\) x (\d+) segs, R (\d+), strips (\d+), "
                     r"units (\d+), hand (\d), skew (\d+)/(\d+)", line)
        if m:
            plans.append([int(x) for x in m.groups()])
    trace = glob.glob(f"{tdir}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(trace)) if "life_tb_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    # the last `rounds - 1` full rounds (the first round follows the warm-up step)
    nr = info["rounds"] - 1
    durs = durs[-nr * L:]
    total = 0.0
    for j in range(L):
        d = statistics.mean(durs[j::L])
        pi = (j + 1) * info["tb_depth"] - 1
        p = plans[pi] if pi < len(plans) else None
        total += d
        if p:
            nrows = p[2] - p[1]
            print(f"launch {j:2d}: rows {nrows:5d} R {p[4]:4d} units {p[6]:5d} hand {p[7]} "
                  f"skew {p[8]}/{p[9]}  {d:7.1f} us  {nrows / d:6.1f} rows/us")
    print(json.dumps({**info, "round_us": round(total, 1),
                      "own_rows_per_us": round(info["rows"] * info["halo_depth"] / 16 / total, 1)}))


if __name__ == "__main__":
    main()
