#!/bin/bash
# r03: resident kernel without per-generation barriers -- parity, then A/B vs r02.
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -k "resident or c2" -v -rf --timeout 200 --timeout-method thread \
    > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/tests.log | head -20; exit $rc; fi
for i in 1 2; do
  for lib in libgol_r02.so libgol.so; do
    GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 60 python3 tools/profile_resident.py --steps 5 | sed "s/^/$lib /" >> $OUT/ab.log || exit 5
  done
done
cat $OUT/ab.log
