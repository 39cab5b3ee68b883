#!/bin/bash
# r03: halo depth 128 vs 256 at the 2- and 4-way rank shapes (RCCL self-loop proxy), twice
set -o pipefail
OUT=gpurun_out/r03ao
mkdir -p $OUT
for rep in 1 2; do
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 2,4 --halo-depths 128,256 >> $OUT/rp.jsonl 2>> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
done
grep '^{' $OUT/rp.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['nranks'], d['halo_depth'], d['rank_tcups'])
"
