#!/bin/bash
# r03: resident kernel through hipLaunchCooperativeKernel -- resident tests, C2 bench
set -o pipefail
OUT=gpurun_out/r03ac
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --size 4096 --no-cpu-baseline > $OUT/bench_c2_$i.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_c2_$i.json')); print(d['value'], d['ms_per_step'])"
done
