#!/usr/bin/env python3
"""Dev tool: per-generation timeline of the resident kernel's middle tile (exp
build with GOL_EXP & 4096, tools/exp_build.sh 4096): for generations 32..95 and
every wavefront, shader-clock stamps at generation start (A), upper edge in
registers (B), top edge + word published (C), lower edge in registers (D),
bottom edge + word published (E).  Prints medians of the pieces and of the
cross-wave hops (upper neighbour's E -> this wave's B; lower neighbour's C ->
this wave's D), for the waves that compute the whole epoch.

    GOL_LIB=mpi-game-of-life_amd/libgol_exp4096.so python tools/res_trace.py
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--rule", default="ref")
    a = p.parse_args()
    import torch
    pkg = entry.load_package()
    L = pkg.lib()
    rule = pkg.REF_RULE if a.rule == "ref" else pkg.CONWAY
    e = pkg.Engine(a.size, a.size, device=0, rule=rule)
    e.init_random(1)
    e.step(a.gens)
    e.sync()
    log = torch.zeros(8 * 65536, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    L.gol_dev_set_wave_log(ctypes.c_void_p(log.data_ptr()))
    e.step(a.gens)
    e.sync()
    L.gol_dev_set_wave_log(ctypes.c_void_p(0))
    t = log[262144:262144 + 16 * 64 * 8].view(16, 64, 8).cpu().numpy().astype(np.int64)
    W, G = 16, 64
    gmax = t[:, :, 5].max(axis=1)
    full = [w for w in range(W) if gmax[w] >= 16 and (t[w, :, 0] != 0).all()]
    pieces = {"up_wait(A->B)": (0, 1), "top(B->C)": (1, 2), "dn_wait(C->D)": (2, 3),
              "bottom(D->E)": (3, 4)}
    out = {"size": a.size, "rule": a.rule, "full_waves": full, "gmax": gmax.tolist()}
    for name, (i, j) in pieces.items():
        v = [int(t[w, g, j] - t[w, g, i]) for w in full for g in range(G)]
        out[name] = statistics.median(v)
    v = [int(t[w, g + 1, 0] - t[w, g, 4]) for w in full for g in range(G - 1)
         if (g + 33) % 16 != 0]  # not across an epoch hand-off
    out["tail(E->next A)"] = statistics.median(v)
    per = [int(t[w, g + 1, 0] - t[w, g, 0]) for w in full for g in range(G - 1)
           if (g + 33) % 16 != 0]
    out["period(A->next A)"] = statistics.median(per)
    up = [int(t[w, g, 1] - t[w - 1, g - 1, 4]) for w in full if w - 1 in full
          for g in range(1, G) if (g + 32) % 16 != 0]
    dn = [int(t[w, g, 3] - t[w + 1, g - 1, 2]) for w in full if w + 1 in full
          for g in range(1, G) if (g + 32) % 16 != 0]
    out["hop_up(E[w-1] -> B[w])"] = statistics.median(up) if up else None
    out["hop_dn(C[w+1] -> D[w])"] = statistics.median(dn) if dn else None
    # one wave's generation skew against its neighbours: A[w] - A[w-1]
    sk = [int(t[w, g, 0] - t[w - 1, g, 0]) for w in full if w - 1 in full for g in range(G)]
    out["skew(A[w]-A[w-1])"] = statistics.median(sk) if sk else None
    ep = [int(t[w, g + 1, 0] - t[w, g, 4]) for w in full for g in range(G - 1)
          if (g + 33) % 16 == 0]
    out["epoch(E->next A across hand-off)"] = statistics.median(ep) if ep else None
    print(json.dumps(out), flush=True)
    # raw rows of the middle wave, first 20 generations (relative to its first A)
    w = full[len(full) // 2]
    base = t[w, 0, 0]
    for g in range(20):
        print(w, g + 32, (t[w, g, :5] - base).tolist())


if __name__ == "__main__":
    main()
