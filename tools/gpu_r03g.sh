#!/bin/bash
# r03: resident tiles per CU 1 vs 2 at 4096^2 x 1000 (M, K sweep); parity of 2/CU.
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
GOL_DEV_RES_PER_CU=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 200 --timeout-method thread > $OUT/tests2.log 2>&1 || { tail -20 $OUT/tests2.log; exit 2; }
tail -1 $OUT/tests2.log
for pc in 1 2; do
GOL_DEV_RES_PER_CU=$pc timeout -k 10 200 python3 tools/sweep.py --size 4096 --gens 1000 --resident 2 \
   --rpw 2,3,4 --depths 8,12,16,20,24 --rounds 3 2>/dev/null | grep -v error | sed "s/^/pc$pc /" >> $OUT/sweep.log || exit 5
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r03g/sweep.log"):
    tag, js = line.split(" ", 1)
    d = json.loads(js)
    print(tag, d["tb_depth"], d["rows_per_wave"], d["resident"], d["gcups_wall_median"], d["kernel_us_avg"])
PY
for pc in 1 2; do
GOL_DEV_RES_PER_CU=$pc GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py 2>/dev/null | tail -1
done
