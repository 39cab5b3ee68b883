#!/bin/bash
# r03: hand-off blocks with the half strip (GOL_DEV_PAIRS=2) vs without, and vs the
# classic default, at long-block shapes.
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,2 --handoff 2 \
    --shapes 65536,33024,32768x262144 --gens 512 --rounds 5 > $OUT/ab_hand.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values auto --handoff 0 \
    --shapes 65536,33024,32768x262144 --gens 512 --rounds 5 >> $OUT/ab_hand.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_hand.jsonl
