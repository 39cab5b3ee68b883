#!/usr/bin/env python3
"""Dev tool: per-wavefront timing of one stencil launch (exp builds with
GOL_EXP & 128, tools/exp_build.sh), and the wall-clock rate of the same shape.

Each wavefront logs its s_memrealtime start/end stamps (100 MHz), HW_ID and
XCC_ID, and (r05) the stamps where its warm-up and its steady blocks end.  Wavefronts sharing a SIMD (same XCC, SE, SH, CU, SIMD) are paired, and
the tool reports how long the first-finishing wave of a pair ends before the
second (the time its partner runs alone on the SIMD), the spread of start and
end stamps, and the launch span.

    GOL_LIB=mpi-game-of-life_amd/libgol_exp128.so python tools/wave_log.py --rows 8448
"""
import argparse
import collections
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=8448)
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--handoff", type=int, default=0)
    p.add_argument("--streams", type=int, default=1)
    p.add_argument("--gens", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--tag", default="")
    p.add_argument("--cus", type=int, default=256)
    p.add_argument("--probe", action="store_true",
                   help="GOL_EXP & 16384 builds: words 4/5 are the start probe (initial loads "
                        "issued / landed) instead of the warm-up / steady ends")
    a = p.parse_args()
    import torch
    pkg = entry.load_package()
    L = pkg.lib()
    e = pkg.Engine(a.rows, a.width, device=0, handoff=a.handoff, streams=a.streams)
    e.init_random(1)
    e.step(a.gens)
    e.sync()
    ts = []
    for _ in range(a.rounds):
        t0 = time.perf_counter()
        e.step(a.gens)
        e.sync()
        ts.append(time.perf_counter() - t0)
    tcups = a.rows * a.width * a.gens / statistics.median(ts) / 1e12
    log = torch.zeros(8 * 65536, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    L.gol_dev_set_wave_log(ctypes.c_void_p(log.data_ptr()))
    e.step(e.tb_depth)  # one full-depth launch
    e.sync()
    L.gol_dev_set_wave_log(ctypes.c_void_p(0))
    w = log.view(-1, 8).cpu().numpy().astype("uint64")
    w = w[w[:, 0] != 0]
    start, end = w[:, 0].astype("int64"), w[:, 1].astype("int64")
    hw = [int(x) for x in w[:, 2]]
    t0 = start.min()
    dur_us = (end - start) / 100.0  # s_memrealtime: 100 MHz
    # xcc | se, sh, cu, simd (HW_ID bits 15:4 without the pipe id)
    simd_key = [((x >> 32) << 16) | (((x & 0xFFFF) >> 4) & ~0xC) for x in hw]
    pairs = collections.defaultdict(list)
    for i, k in enumerate(simd_key):
        pairs[int(k)].append(i)
    solo, lead_share = [], []
    occ = collections.Counter(len(v) for v in pairs.values())
    for v in pairs.values():
        if len(v) != 2:
            continue
        i, j = v
        first, second = sorted((end[i], end[j]))
        span = max(end[i], end[j]) - min(start[i], start[j])
        solo.append((second - first) / 100.0)
        lead_share.append((second - first) / span)
    # per SIMD, the share of the launch span with 2, 1 and 0 of its waves running
    # (the issue model: full rate needs both; r04)
    span_all = float(end.max() - t0)
    conc = collections.Counter()
    for v in pairs.values():
        ev = sorted([(int(start[i]), 1) for i in v] + [(int(end[i]), -1) for i in v])
        cur, last = 0, int(t0)
        for t, d in ev:
            conc[min(cur, 2)] += t - last
            cur += d
            last = t
        conc[0] += int(end.max()) - last
    tot = sum(conc.values()) or 1
    concurrency = {str(k): round(conc[k] / tot, 4) for k in (2, 1, 0)}
    rec = {
        "simd_time_share_by_waves_running": concurrency,
        "tag": a.tag, "lib": os.path.basename(os.environ.get("GOL_LIB", "libgol.so")),
        "shape": f"{a.rows}x{a.width}", "tb_depth": e.tb_depth, "rows_per_wave": e.rows_per_wave,
        "handoff": e.handoff, "tcups_wall_median": round(tcups, 2),
        "waves": int(len(w)), "simds_by_waves": {str(k): n for k, n in sorted(occ.items())},
        "launch_span_us": round((end.max() - t0) / 100.0, 2),
        "start_spread_us": round((start.max() - t0) / 100.0, 2),
        "wave_us": {"min": round(float(dur_us.min()), 2), "median": round(float(statistics.median(dur_us)), 2),
                    "max": round(float(dur_us.max()), 2)},
        "end_us_quantiles": [round(float(x), 2) for x in
                             ((sorted(end - t0)[int(q * (len(end) - 1))]) / 100.0
                              for q in (0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0))],
        "pair_solo_us": ({"median": round(statistics.median(solo), 2), "max": round(max(solo), 2),
                          "mean": round(statistics.mean(solo), 2)} if solo else None),
        "pair_solo_share_median": round(statistics.median(lead_share), 3) if lead_share else None,
        "wave_slot_ids": dict(collections.Counter(int(x) & 15 for x in hw)),
    }
    # dispatch order vs wave slot: which workgroups got slot 0 (the older wave of a
    # pair), and the median end stamp of each slot
    wg = w[:, 3].astype("int64") >> 32
    slot = [x & 15 for x in hw]
    ncu = int(a.cus)
    rec["slot0_wg_lt_ncu"] = round(sum(1 for i, s in enumerate(slot) if s == 0 and wg[i] < ncu)
                                   / max(1, sum(1 for s in slot if s == 0)), 4)
    rec["slot1_wg_ge_ncu"] = round(sum(1 for i, s in enumerate(slot) if s == 1 and wg[i] >= ncu)
                                   / max(1, sum(1 for s in slot if s == 1)), 4)
    for sl in (0, 1):
        ends = [float(end[i] - t0) / 100.0 for i, s in enumerate(slot) if s == sl]
        if ends:
            rec[f"slot{sl}_end_us_median"] = round(statistics.median(ends), 2)
    # (r05) phases of each wavefront: warm-up (the unrolled first 2K steps), steady
    # blocks, tail (hand-off side rows / classic drain), by block length
    tw, tsd = w[:, 4].astype("int64"), w[:, 5].astype("int64")
    nrows = (w[:, 6] & 0xFFFFFFFF).astype("int64")
    tb1 = (w[:, 6] >> 32).astype("int64")  # second warm-up block's end, from the start
    tb0 = w[:, 7].astype("int64")
    by_len = collections.defaultdict(list)
    for i in range(len(w)):
        if tw[i] and tsd[i]:
            by_len[int(nrows[i])].append(((tw[i] - start[i]) / 100.0, (tsd[i] - tw[i]) / 100.0,
                                          (end[i] - tsd[i]) / 100.0,
                                          (tb0[i] - start[i]) / 100.0 if tb0[i] else 0.0,
                                          (start[i] - t0) / 100.0, tb1[i] / 100.0))
    names = ("to_loads_issued", "loads_landed", "to_end") if a.probe else ("warm", "steady", "tail")
    rec["phases_us_by_rows"] = {
        str(k): {"waves": len(v),
                 names[0]: round(statistics.median(x[0] for x in v), 2),
                 names[1]: round(statistics.median(x[1] for x in v), 2),
                 names[2]: round(statistics.median(x[2] for x in v), 2),
                 "first_block": round(statistics.median(x[3] for x in v), 2),
                 "second_block": round(statistics.median(x[5] for x in v), 2),
                 "start_offset": round(statistics.median(x[4] for x in v), 2)}
        for k, v in sorted(by_len.items(), key=lambda kv: -len(kv[1]))[:6]}
    # (r05) the last-finishing waves, which set the launch's end: their age class
    # (slot), block index from the bottom, strip, row count, XCC, and start offset
    order = sorted(range(len(w)), key=lambda i: -int(end[i]))
    blkv = (w[:, 3] & 0xFFFFFFFF).astype("int64")
    n_last = max(1, len(w) // 50)
    last = order[:n_last]
    rec["last_2pct"] = {
        "end_us_min": round(float(end[last[-1]] - t0) / 100.0, 2),
        "slot": dict(collections.Counter(int(hw[i]) & 15 for i in last)),
        "xcc": dict(collections.Counter(int(hw[i]) >> 32 for i in last)),
        "rows": dict(collections.Counter(int(nrows[i]) for i in last)),
        "blk": dict(collections.Counter(int(blkv[i]) for i in last).most_common(8)),
        "start_us_median": round(statistics.median(float(start[i] - t0) / 100.0 for i in last), 2),
        "dur_us_median": round(statistics.median(float(dur_us[i]) for i in last), 2),
        "wg": sorted(int(wg[i]) for i in last)[:24],
    }
    # (r05) per XCC (HW_REG_XCC_ID): wavefronts, median / max end and median duration
    # of the old (slot 0) and young (slot 1) waves
    by_x = collections.defaultdict(list)
    for i in range(len(w)):
        by_x[int(hw[i]) >> 32].append(i)
    rec["per_xcc"] = {
        str(x): {"waves": len(v),
                 "end_med": round(statistics.median(float(end[i] - t0) for i in v) / 100.0, 2),
                 "end_max": round(max(float(end[i] - t0) for i in v) / 100.0, 2),
                 "dur_old": round(statistics.median([float(dur_us[i]) for i in v if int(hw[i]) & 15 == 0] or [0]), 2),
                 "dur_young": round(statistics.median([float(dur_us[i]) for i in v if int(hw[i]) & 15 == 1] or [0]), 2)}
        for x, v in sorted(by_x.items())}
    # (r06) does the workgroup -> XCC mapping follow round-robin (XCC = wg mod 8)?
    # (the per-XCD row shift, GOL_DEV_XCD_SHIFT, assumes it for speed only)
    rec["xcc_is_wg_mod8"] = round(sum(1 for i in range(len(w)) if int(hw[i]) >> 32 == int(wg[i]) % 8)
                                  / max(1, len(w)), 4)
    rec["xcc_of_wg_mod8"] = {str(m): dict(collections.Counter(int(hw[i]) >> 32 for i in range(len(w))
                                                              if int(wg[i]) % 8 == m))
                             for m in range(8)}
    print(json.dumps(rec), flush=True)
    e.close()


if __name__ == "__main__":
    main()
