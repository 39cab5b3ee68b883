#!/bin/bash
# r03: packed half strip at the rank shapes -- hand-off vs classic plans, with and
# without the half strip, in one process per shape set.
set -o pipefail
OUT=gpurun_out/r03u
mkdir -p $OUT
for ho in 1 2; do
  timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto --handoff $ho \
      --shapes 8448,8416,12288,16640 --gens 512 --rounds 5 >> $OUT/ab_pairs_handoff.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
done
cat $OUT/ab_pairs_handoff.jsonl
