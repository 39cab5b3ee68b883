#!/bin/bash
# r03: resident launch default back to plain; cooperative opt-in test; C2 bench
set -o pipefail
OUT=gpurun_out/r03ae
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --size 4096 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_c2.json')); print(d['value'], d['ms_per_step'])"
