#!/bin/bash
# r03: hand-off tail offset 2 at depth 16 (VGPR-capped) -- parity, rank-shape A/B
# (autotuned), rank proxy
set -o pipefail
OUT=gpurun_out/r03aj
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_halfstrip.py tests/test_gpu_skew.py tests/test_gpu_autotune.py tests/test_gpu_rccl.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
GOL_DEV_AUTOTUNE=1 timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values auto \
    --shapes 8224,8288,8352,8416,8480,8544,8608,8672 --gens 512 --rounds 5 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); print(d['shape'], d['tcups_wall_median'], d['age_skew'], d['rows_per_wave'])
"
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
grep '^{' $OUT/rank_proxy.jsonl | cut -c1-330
