#!/usr/bin/env python3
"""Turn tools/gpu_profile_r02.sh output into profiles/r02/counters.json records
(read by bench.py's roofline):

  insts_valu_per_launch  SQ_INSTS_VALU per life_tb_kernel launch (mean)
  hbm_bytes_per_launch   FETCH_SIZE x f_read + WRITE_SIZE x f_write, the factors
                         calibrated in the same run on kernels whose byte counts
                         are known exactly (MI355X_MICROARCH.md §HBM):
                           digest_kernel      reads  rows*wq*8 B, 8 B per lane
                           init_random_kernel writes rows*stride*8 B, 8 B per lane
  plus SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY, GRBM_GUI_ACTIVE means, and the mean
  launch time of the dominant stencil instantiation in the bench's kernel trace.

    python tools/pmc_counters.py gpurun_out/prof_r03_c3 --out profiles/r03/counters.json
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_kernel(path, counter):
    """Counter values per kernel name, in dispatch order."""
    out = {}
    rows = list(csv.DictReader(open(path)))
    if rows and "Dispatch_Id" in rows[0]:
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        name = "life_tb_kernel" if "life_tb_kernel" in k else (
            "life_res_kernel" if "life_res_kernel" in k else (
                "digest_kernel" if "digest_kernel" in k else (
                    "init_random_kernel" if "init_random_kernel" in k else k)))
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


def config_of(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"rows_per_wave"' in line:
            return json.loads(line)
    raise SystemExit(f"no configuration line in {log}")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof_dir")
    p.add_argument("--out", default="profiles/r05/counters.json")
    p.add_argument("--stage-rev", type=int, default=0,
                   help="stage-logic revision of the profiled build (bench.py STAGE_REV; "
                        "0 = the current one of the profiled rule)")
    a = p.parse_args()
    d = a.prof_dir
    cfg = config_of(os.path.join(d, "pmc_FETCH_SIZE.log"))
    n, S = cfg["size"], cfg["streams"]
    # rows the digest reads and init_random writes: the field, or a rank engine's
    # own rows (profile_run.py --ranks)
    own = cfg.get("own_rows", n)
    # (r05) only the profiled step's launches (the last `launches` of the stencil
    # kernel): the autotuner's candidates at create are other plans
    last = int(cfg.get("launches", 0)) or None
    kern = cfg.get("kernel", "life_tb_kernel")
    gpl = cfg.get("gens_per_launch", cfg["tb_depth"])
    fetch = per_kernel(os.path.join(d, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE")
    wq = (n + 63) // 64
    stride = (wq + 7) // 8 * 8
    # a composite engine runs digest / init per part, over 1/S of the rows each
    f_read = own * wq * 8 / S / (statistics.mean(fetch["digest_kernel"]) * 1024)
    # (the user's init_random, the last one: the autotuner's fills the whole buffer)
    f_write = own * stride * 8 / S / (statistics.mean(write["init_random_kernel"][-S:]) * 1024)
    rd = statistics.mean(fetch[kern][-last:] if last else fetch[kern]) * 1024 * f_read
    wr = statistics.mean(write[kern][-last:] if last else write[kern]) * 1024 * f_write
    sq = os.path.join(d, "pmc_sq", "pmc_counter_collection.csv")
    rec = dict(cfg)
    for k in ("launches", "digest0", "digest", "gens_per_launch"):
        rec.pop(k, None)
    rec.update({
        "hbm_bytes_per_launch": round(rd + wr), "read_bytes_per_launch": round(rd),
        "write_bytes_per_launch": round(wr),
        "bytes_per_cell_gen_measured": round((rd + wr) * S / (own * n * gpl), 5),
        "gens_per_launch": gpl,
        "fetch_size_calibration": round(f_read, 4), "write_size_calibration": round(f_write, 4),
    })
    if os.path.exists(sq):
        for c in ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "GRBM_GUI_ACTIVE", "SQ_INSTS_SALU"):
            v = per_kernel(sq, c).get(kern)
            if v and last:
                v = v[-last:]
            if v:
                rec[c.lower() + "_per_launch"] = round(statistics.mean(v))
        rec["insts_valu_per_launch"] = rec.get("sq_insts_valu_per_launch")
        rec["launches_profiled"] = min(len(per_kernel(sq, "SQ_INSTS_VALU").get(kern, [])),
                                       last or 1 << 30)
    stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
    if stats:  # the bench command's kernel trace: the dominant stencil instantiation
        rows = [r for r in csv.DictReader(open(stats[0])) if kern in r["Name"]]
        if rows:
            top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            rec["trace_kernel"] = top["Name"]
            rec["trace_avg_launch_ns"] = float(top["AverageNs"])
            rec["trace_calls"] = int(top["Calls"])
    rec["stage_rev"] = a.stage_rev or {"ref": 3, "conway": 3}.get(cfg.get("rule"), 1)
    rec["source"] = os.path.basename(os.path.normpath(d))
    rec["source_round"] = os.path.basename(os.path.dirname(os.path.abspath(a.out)))
    doc = {"records": []}
    if os.path.exists(a.out):
        doc = json.load(open(a.out))
    keys = ("stage_rev", "size", "rule", "tb_depth", "streams", "n_gpus", "rows_per_wave", "handoff")
    doc["records"] = [r for r in doc["records"] if not all(r.get(k) == rec.get(k) for k in keys)]
    doc["records"].append(rec)
    doc["_doc"] = ("Per-launch counters of the stencil kernel (life_tb_kernel, or life_res_kernel "
                   "for resident fields) by configuration: rocprofv3 --pmc "
                   "passes (FETCH_SIZE, WRITE_SIZE and the SQ set each in its own run) over "
                   "tools/profile_run.py; see tools/pmc_counters.py")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(doc, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
