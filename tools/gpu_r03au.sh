#!/bin/bash
# r03: 4-way rank with Hx = 16 (one plan, one launch per round) under rocprof: do its
# launches run like the stripe alone?
set -o pipefail
OUT=gpurun_out/r03au
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o rp --output-format csv -- \
    python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 4 --rounds 2 --halo-depths 16 > $OUT/rp.jsonl 2> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
grep '^{' $OUT/rp.jsonl | cut -c1-260
head -6 $OUT/trace/rp_kernel_stats.csv | cut -c1-160
