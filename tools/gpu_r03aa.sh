#!/bin/bash
# r03: hand-off + half strip default -- GPU suite, A/B of the defaults vs no half
# strip, per-rank RCCL proxy, bench.
set -o pipefail
OUT=gpurun_out/r03aa
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto \
    --shapes 8448,8704,12288,16640,33024 --gens 512 --rounds 5 > $OUT/ab_default.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_default.jsonl
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1,2 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
grep '^{' $OUT/rank_proxy.jsonl
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 4; }
cat $OUT/bench_c3.json
