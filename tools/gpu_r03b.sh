#!/bin/bash
# r03: the N>1 bench path rehearsed on one GPU (RCCL self-loops), N=1 bench.
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
GOL_DEV_RCCL_SELF=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --handoff 1 \
    > $OUT/bench_rehearsal2.json 2> $OUT/bench_rehearsal2.err || { grep -A3 Error $OUT/bench_rehearsal2.err | head -30; exit 4; }
cat $OUT/bench_rehearsal2.json
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 5; }
cat $OUT/bench.json
