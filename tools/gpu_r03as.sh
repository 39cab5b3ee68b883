#!/bin/bash
# r03: rank proxy with device-side kernel arguments forced (HIP_FORCE_DEV_KERNARG)
set -o pipefail
OUT=gpurun_out/r03as
mkdir -p $OUT
for kv in 0 1; do
HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 4,8 > $OUT/rp_$kv.jsonl 2> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
grep '^{' $OUT/rp_$kv.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('devkernarg=$kv', d['nranks'], d['rank_tcups'])
"
done
