#!/usr/bin/env python3
"""Per-stream timeline of the stencil launches in a rocprofv3 kernel trace: how
much of the time two stripe streams' launches run concurrently (the composite
engine's overlap), per-stream busy fraction and inter-launch gaps.

    python tools/trace_overlap.py gpurun_out/prof_r02c/trace/bench_kernel_trace.csv [--json out]
"""
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    rows = [r for r in csv.DictReader(open(path)) if "life_tb_kernel" in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows)
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    # sweep: time with >= 1 and >= 2 stencil launches running
    ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
    level, last, busy1, busy2 = 0, t0, 0, 0
    for t, d in ev:
        if level >= 1:
            busy1 += t - last
        if level >= 2:
            busy2 += t - last
        level += d
        last = t
    per = {}
    for s, e, sid in iv:
        per.setdefault(sid, []).append((s, e))
    streams = {}
    for sid, v in per.items():
        v.sort()
        gaps = [b[0] - a[1] for a, b in zip(v, v[1:])]
        streams[sid] = {"launches": len(v), "busy_frac": round(sum(e - s for s, e in v) / (t1 - t0), 4),
                        "mean_launch_us": round(statistics.mean(e - s for s, e in v) / 1e3, 2),
                        "median_gap_us": round(statistics.median(gaps) / 1e3, 2) if gaps else None}
    out = {"source": path, "span_ms": round((t1 - t0) / 1e6, 3), "launches": len(iv),
           "any_running_frac": round(busy1 / (t1 - t0), 4),
           "two_or_more_running_frac": round(busy2 / (t1 - t0), 4), "streams": streams}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
