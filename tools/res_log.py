#!/usr/bin/env python3
"""Dev tool: per-wavefront timing of the resident kernel (exp build with
GOL_EXP & 2048, tools/exp_build.sh 2048): shader cycles in all, waiting for the
upper neighbour wave's edge (progress-word reads issued -> edge values in
registers), and in the epoch hand-offs (gen loop done -> halo reload landed; of
it: band publish + workgroup barrier, neighbour-tile flag wait + barrier).

    GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so python tools/res_log.py --size 4096
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--rows-per-wave", type=int, default=0)
    p.add_argument("--tb-depth", type=int, default=0)
    a = p.parse_args()
    import torch
    pkg = entry.load_package()
    L = pkg.lib()
    kw = dict(resident=2, rows_per_wave=a.rows_per_wave, tb_depth=a.tb_depth) \
        if (a.rows_per_wave or a.tb_depth) else {}
    e = pkg.Engine(a.size, a.size, device=0, **kw)
    e.init_random(1)
    e.step(a.gens)
    e.sync()
    log = torch.zeros(8 * 65536, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    L.gol_dev_set_wave_log(ctypes.c_void_p(log.data_ptr()))
    e.step(a.gens)
    e.sync()
    L.gol_dev_set_wave_log(ctypes.c_void_p(0))
    w = log.view(-1, 8).cpu().numpy()
    w = w[w[:, 0] != 0]
    tot, wait, ep = w[:, 0].astype(float), w[:, 1].astype(float), w[:, 2].astype(float)
    gmax = (w[:, 3] & 0xFFFFFFFF).astype(int)
    pub, flag = w[:, 4].astype(float), w[:, 5].astype(float)
    by_g = {}
    for i, g in enumerate(gmax):
        by_g.setdefault(int(g), []).append((wait[i] / tot[i], ep[i] / tot[i], pub[i] / tot[i],
                                            flag[i] / tot[i]))
    print(json.dumps({
        "size": a.size, "gens": a.gens, "resident": e.resident, "tb_depth": e.tb_depth,
        "rows_per_wave": e.rows_per_wave, "waves": len(w),
        "cycles_total_median": statistics.median(tot),
        "wait_frac_median": round(statistics.median(wait / tot), 4),
        "epoch_frac_median": round(statistics.median(ep / tot), 4),
        "compute_frac_median": round(statistics.median((tot - wait - ep) / tot), 4),
        "cycles_per_gen": round(statistics.median(tot) / a.gens, 1),
        "by_gmax (wait, epoch, of which publish+barrier, flag wait+barrier)": {
            g: [round(statistics.median(x[j] for x in v), 3) for j in range(4)]
            for g, v in sorted(by_g.items())},
    }))
    e.close()


if __name__ == "__main__":
    main()
