#!/bin/bash
# r03 final tree: GPU suite, smoke, C3 and C2 bench lines, the N = 2 bench path
# rehearsed on one GPU (RCCL self-loops).
set -o pipefail
OUT=gpurun_out/r03final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 4; }
cat $OUT/bench_c3.json
timeout -k 10 300 python -u bench.py --size 4096 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 4; }
cat $OUT/bench_c2.json
GOL_DEV_RCCL_SELF=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --handoff 1 \
    > $OUT/bench_rehearsal2.json 2> $OUT/bench_rehearsal2.err || { grep -A3 Error $OUT/bench_rehearsal2.err | head -30; exit 5; }
cat $OUT/bench_rehearsal2.json
