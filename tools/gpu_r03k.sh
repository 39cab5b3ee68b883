#!/bin/bash
# r03: per-rank proxy of the N-GPU split on one GPU: host no-op vs RCCL self-loop
# transport, blocking vs overlapped exchange; per-GPU shapes (skew A/B).
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 400 python3 tools/rank_proxy.py --ranks 2,4,8 --skews auto --transports noop,rccl --overlaps 1,2 \
    > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail -20 $OUT/rank_proxy.err; exit 3; }
python3 -c "
import json
for l in open('$OUT/rank_proxy.jsonl'):
    d=json.loads(l); print(d['nranks'], d['transport'], d['overlap_cfg'], d['rank_tcups'], d['aggregate_tcups_if_balanced'], d['handoff'], d['age_skew'])
"
timeout -k 10 300 python3 tools/ab_skew.py --shapes 8448,12288,16640 --rhos auto --handoffs 0,1 > $OUT/ab_skew.jsonl 2>&1 || { tail -5 $OUT/ab_skew.jsonl; exit 4; }
python3 -c "
import json
for l in open('$OUT/ab_skew.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['handoff_cfg'], d['handoff'], d['age_skew'], d['tcups_wall_median'], d['kernel_us_avg'], d['digests_equal'])
"
