#!/bin/bash
# r03: hand-off skew rate rho at the 8-way rank (per-launch trace) and the per-GPU
# shapes (in-process A/B).
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
for rho in auto 0.82 0.86 0.9; do
  if [ $rho = auto ]; then unset GOL_DEV_AGE_SKEW; else export GOL_DEV_AGE_SKEW=$rho; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/t$rho -o t --output-format csv -- python3 tools/rank_plans.py --nranks 8 > $OUT/plans$rho.json 2> $OUT/plans$rho.err || { tail -5 $OUT/plans$rho.err; exit 3; }
  python3 tools/plan_trace.py $OUT/t$rho $OUT/plans$rho.err $OUT/plans$rho.json | tail -1
done
unset GOL_DEV_AGE_SKEW
timeout -k 10 400 python3 tools/ab_skew.py --shapes 8448,8704,16896 --rhos auto,0.82,0.86,0.9 --handoffs 0 > $OUT/ab_skew.jsonl 2>&1 || { tail -5 $OUT/ab_skew.jsonl; exit 4; }
grep '^{' $OUT/ab_skew.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], d['rho'], d['handoff'], d['age_skew'], d['tcups_wall_median'], d['kernel_us_avg'], d['digests_equal'])
"
