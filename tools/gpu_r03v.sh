#!/bin/bash
# r03: half strip + planner policy -- full GPU suite, smoke, bench (C3, C2),
# in-process A/B vs GOL_DEV_PAIRS=0 at the rank shapes, per-rank RCCL proxy.
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 4; }
cat $OUT/bench_c3.json
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto \
    --shapes 8448,12288,16640,33024,65536 --gens 512 --rounds 5 > $OUT/ab_default.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_default.jsonl
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
cat $OUT/rank_proxy.jsonl
