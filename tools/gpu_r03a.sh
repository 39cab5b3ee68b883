#!/bin/bash
# r03: RCCL self-loop tests, the N>1 bench path rehearsed on one GPU, N=1 bench.
set -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -v -rf --timeout 300 --timeout-method thread \
    > $OUT/rccl_tests.log 2>&1
rc=$?
tail -15 $OUT/rccl_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
GOL_DEV_RCCL_SELF=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --handoff 1 \
    > $OUT/bench_rehearsal2.json 2> $OUT/bench_rehearsal2.err || { tail -30 $OUT/bench_rehearsal2.err; exit 4; }
cat $OUT/bench_rehearsal2.json
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 5; }
cat $OUT/bench.json
exit $rc
