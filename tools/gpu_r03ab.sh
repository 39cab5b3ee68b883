#!/bin/bash
# r03: hand-off tail offset 6 -- parity (half strip, skew, full-size), A/B at the
# rank launch shapes, per-rank RCCL proxy
set -o pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_halfstrip.py tests/test_gpu_skew.py tests/test_gpu_fullsize.py tests/test_gpu_rccl.py \
    -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto \
    --shapes 8224,8448,8544,8704,12288,16640 --gens 512 --rounds 5 > $OUT/ab_default.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_default.jsonl
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
grep '^{' $OUT/rank_proxy.jsonl
