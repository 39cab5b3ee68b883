#!/bin/bash
# r03: half-strip block length under classic plans (scale of the young length)
set -o pipefail
OUT=gpurun_out/r03al
mkdir -p $OUT
GOL_DEV_AUTOTUNE=0 timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_HALF_SCALE_CLASSIC --values auto,0.85,0.93,1.07 \
    --shapes 65536,33024 --gens 512 --rounds 7 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); print(d['shape'], d['GOL_DEV_HALF_SCALE_CLASSIC'], d['tcups_wall_median'], d['age_skew'], d['digests_equal'])
"
