#!/bin/bash
# r03: kernel trace of the 4-way rank proxy (RCCL self-loop): stencil launches vs
# RCCL exchange kernels per round
set -o pipefail
OUT=gpurun_out/r03ap
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o rp --output-format csv -- \
    python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 4 --rounds 2 > $OUT/rp.jsonl 2> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
grep '^{' $OUT/rp.jsonl | cut -c1-200
head -12 $OUT/trace/rp_kernel_stats.csv | cut -c1-180
