#!/usr/bin/env python3
"""Dev A/B of the per-XCD row shift (GOL_DEV_XCD_SHIFT, life_stencil.h; VERDICT r05
item 2(ii)) on THIS box, in two steps:

1. the per-XCC wave timing of the 8-way rank launch shape (tools/wave_log.py on
   the GOL_EXP & 128 build, libgol_exp128.so, in a child process): which XCCs end
   last, and whether workgroup w lands on XCC w mod 8 (the shift assumes it);
2. the RCCL per-rank proxy (tools/rank_proxy.py, shipped library) with the shift
   off, with a table built from step 1 (the XCCs that end first take rows from
   the ones that end last), the same table at half the strips, and its reverse
   (a control that should lose).

    python tools/ab_xcd_shift.py [--ranks 8] [--rounds 5]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", default="8")
    p.add_argument("--rows", type=int, default=8416)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    env = dict(os.environ, GOL_LIB=os.path.join(ROOT, "mpi-game-of-life_amd", "libgol_exp128.so"))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "wave_log.py"), "--rows",
                          str(a.rows), "--handoff", "2"], env=env, capture_output=True, text=True,
                         timeout=300)
    if out.returncode != 0:
        print(out.stderr[-2000:], file=sys.stderr)
        raise SystemExit(out.returncode)
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    per = rec["per_xcc"]
    print(json.dumps({"wave_log": {k: rec.get(k) for k in
                                   ("launch_span_us", "per_xcc", "xcc_is_wg_mod8", "last_2pct")}}),
          flush=True)
    ends = sorted((v["end_med"], int(x)) for x, v in per.items())
    code = [1] * 8
    for _, x in ends[:2]:
        code[x] = 2  # the two XCCs that end first take rows
    for _, x in ends[-2:]:
        code[x] = 0  # from the two that end last
    table = "".join(str(c) for c in code)
    rev = "".join(str(2 - c) for c in code)
    values = ";".join(["auto", f"{table}:1", f"{table}:2", f"{rev}:1"])
    cmd = [sys.executable, os.path.join(ROOT, "tools", "rank_proxy.py"), "--transports", "rccl",
           "--ranks", a.ranks, "--skews", "auto", "--rounds", str(a.rounds),
           "--env-var", "GOL_DEV_XCD_SHIFT", "--env-values", values]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    sys.stdout.write(res.stdout)
    if res.returncode != 0:
        print(res.stderr[-2000:], file=sys.stderr)
        raise SystemExit(res.returncode)


if __name__ == "__main__":
    main()
