#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03am
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_autotune.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
