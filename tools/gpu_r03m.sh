#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_fullsize.py tests/test_gpu_transport.py -k "rccl or c4 or rank_engines" -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" $OUT/tests.log | tail -8
exit $rc
