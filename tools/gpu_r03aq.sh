#!/bin/bash
# r03: the 4-way rank's launch shapes run alone (autotuned): per-launch time
set -o pipefail
OUT=gpurun_out/r03aq
mkdir -p $OUT
GOL_DEV_AUTOTUNE=1 timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values auto \
    --shapes 16384,16448,16512,16576,16608,16640 --gens 512 --rounds 5 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); print(d['shape'], d['tcups_wall_median'], d['kernel_us_avg'], d['age_skew'], d['handoff'])
"
