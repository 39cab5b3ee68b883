#!/bin/bash
# r03: plan autotuner -- autotune + full GPU suite, A/B autotuned vs models' plans
# at the rank shapes, rank proxy, C3 bench
set -o pipefail
OUT=gpurun_out/r03ag
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
GOL_DEV_PLANS=1 timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_AUTOTUNE --values 0,1 \
    --shapes 8224,8448,8608,8672,16640,65536 --gens 512 --rounds 5 > $OUT/ab_autotune.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_autotune.jsonl
grep "autotune plan" $OUT/ab.err | head -20
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
grep '^{' $OUT/rank_proxy.jsonl
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_c3.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
