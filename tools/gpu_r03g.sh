#!/bin/bash
# r03: resident (M, K) sweep at 4096^2 x 1000 with the current kernel.
set -o pipefail
OUT=gpurun_out/r03g2
mkdir -p $OUT
timeout -k 10 300 python3 tools/sweep.py --size 4096 --gens 1000 --resident 2 \
   --rpw 3,4,6 --depths 16,18,20,22,24,28,32,40 --rounds 3 2>/dev/null | grep -v error > $OUT/sweep.log || exit 5
python3 - <<'PY'
import json
for line in open("gpurun_out/r03g2/sweep.log"):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print(d["tb_depth"], d["rows_per_wave"], d["resident"], d["gcups_wall_median"], d["kernel_us_avg"])
PY
