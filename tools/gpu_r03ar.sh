#!/bin/bash
# r03: rocprof of a standalone 16608-row stripe (same measurement as the rank trace)
set -o pipefail
OUT=gpurun_out/r03ar
mkdir -p $OUT
export TMPDIR=/tmp
GOL_DEV_AUTOTUNE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o sa --output-format csv -- \
    python3 tools/ab_env.py --var GOL_DEV_PAIRS --values auto --shapes 16608 --gens 512 --rounds 3 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab.jsonl | cut -c1-250
head -6 $OUT/trace/sa_kernel_stats.csv | cut -c1-160
