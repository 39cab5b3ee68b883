#!/bin/bash
# r03: HIP_FORCE_DEV_KERNARG unset vs 1, alternating, rank proxy 4/8-way and C3 bench
set -o pipefail
OUT=gpurun_out/r03at
mkdir -p $OUT
for rep in 1 2 3; do
for kv in unset 1; do
  if [ $kv = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=1; fi
  timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 4,8 --rounds 2 > $OUT/rp.jsonl 2> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
  grep '^{' $OUT/rp.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('kernarg=$kv', d['nranks'], d['rank_tcups'], flush=True)
" | tee -a $OUT/summary.txt
done
done
unset HIP_FORCE_DEV_KERNARG
