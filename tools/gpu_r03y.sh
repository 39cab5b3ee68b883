#!/bin/bash
# r03: hand-off plans with the half strip, its blocks scaled (GOL_DEV_HALF_SCALE)
set -o pipefail
OUT=gpurun_out/r03y
mkdir -p $OUT
for sc in 1.0 0.8 0.6; do
  GOL_DEV_HALF_SCALE=$sc timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,2 --handoff 2 \
      --shapes 8448,12288 --gens 512 --rounds 5 | sed "s/^/{\"scale\": $sc, \"r\": /; s/\$/}/" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
done
cat $OUT/ab.jsonl
