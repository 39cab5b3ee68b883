#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03an
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_c3.json')); print(d['value'], d['config']['columns'])"
GOL_DEV_RCCL_SELF=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --handoff 1 \
    > $OUT/bench_rehearsal2.json 2> $OUT/bench_rehearsal2.err || { grep -A3 Error $OUT/bench_rehearsal2.err | head -30; exit 5; }
tail -1 $OUT/bench_rehearsal2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['columns'])"
