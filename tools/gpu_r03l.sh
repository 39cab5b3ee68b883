#!/bin/bash
# r03: rank proxy over the RCCL self-loop: halo depth sweep at 4 and 8 ranks.
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 500 python3 tools/rank_proxy.py --ranks 8,4 --skews auto --transports rccl --overlaps 1,2 \
    --halo-depths 64,128,192,256 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail -20 $OUT/rank_proxy.err; exit 3; }
grep '^{' $OUT/rank_proxy.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['nranks'], d['transport'], d['overlap_cfg'], d['halo_depth'], d['rank_tcups'], d['aggregate_tcups_if_balanced'], d['handoff'], d['age_skew'])
"
