#!/usr/bin/env python3
"""Turn tools/gpu_profile.sh output into profiles/traffic.json records.

HBM bytes per stencil launch = FETCH_SIZE x f_read + WRITE_SIZE x f_write, with
the two factors calibrated in the same run on kernels whose byte counts are
known exactly (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only for some
access widths):
  digest_kernel       reads  size*size/8 bytes with 8-byte-per-lane loads
  init_random_kernel  writes rows*stride*8 bytes with 8-byte-per-lane stores

    python tools/pmc_traffic.py gpurun_out/prof_r01 --size 65536 --tb-depth 8 \
        --rows-per-wave 0 --out profiles/traffic.json
"""
import argparse
import csv
import json
import os
import statistics


def per_kernel(path, counter):
    rows = list(csv.DictReader(open(path)))
    out = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof_dir")
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--tb-depth", type=int, default=8)
    p.add_argument("--rows-per-wave", type=int, default=0)
    p.add_argument("--out", default="profiles/traffic.json")
    p.add_argument("--tag", default="")
    p.add_argument("--streams", type=int, default=2, help="engine stripe streams when profiled")
    p.add_argument("--word-planes", type=int, default=2)
    a = p.parse_args()
    fetch = per_kernel(os.path.join(a.prof_dir, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"),
                       "FETCH_SIZE")
    write = per_kernel(os.path.join(a.prof_dir, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"),
                       "WRITE_SIZE")
    n = a.size
    wq = (n + 63) // 64
    stride = (wq + 7) // 8 * 8
    # with a composite engine every part runs its own digest / init over 1/streams
    # of the rows (the tool profiles the default engine of tools/profile_run.py)
    digest_bytes = n * wq * 8 / a.streams
    init_bytes = n * stride * 8 / a.streams
    f_read = digest_bytes / statistics.mean(fetch["digest_kernel"])
    f_write = init_bytes / statistics.mean(write["init_random_kernel"])
    rd = statistics.mean(fetch["life_tb_kernel"]) * f_read
    wr = statistics.mean(write["life_tb_kernel"]) * f_write
    cells = n * n
    launches = len(fetch["life_tb_kernel"])
    rec = {
        "size": n, "tb_depth": a.tb_depth, "rows_per_wave": a.rows_per_wave, "n_gpus": 1,
        "streams": a.streams, "word_planes": a.word_planes,
        "hbm_bytes_per_launch": round(rd + wr),
        "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
        "field_bytes": cells // 8,
        # each launch covers 1/streams of the field
        "bytes_per_cell_gen_measured": round((rd + wr) * a.streams / (cells * a.tb_depth), 5),
        "fetch_size_calibration": round(f_read, 4), "write_size_calibration": round(f_write, 4),
        "launches_profiled": launches,
        "source": os.path.basename(os.path.normpath(a.prof_dir)) + (f" {a.tag}" if a.tag else ""),
    }
    doc = {"records": []}
    if os.path.exists(a.out):
        doc = json.load(open(a.out))
    doc["records"] = [r for r in doc["records"]
                      if not all(r.get(k, 2 if k == "word_planes" else None) == rec[k]
                                 for k in ("size", "tb_depth", "rows_per_wave", "n_gpus",
                                           "streams", "word_planes"))]
    doc["records"].append(rec)
    doc["_doc"] = ("HBM bytes per life_tb_kernel launch from rocprofv3 FETCH_SIZE / WRITE_SIZE "
                   "(separate passes), calibrated on digest_kernel / init_random_kernel in the "
                   "same run; see tools/pmc_traffic.py")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(doc, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
