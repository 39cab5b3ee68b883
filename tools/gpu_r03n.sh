#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
for hx in 256 128; do
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/t$hx -o t --output-format csv -- python3 tools/rank_plans.py --nranks 8 --halo-depth $hx > $OUT/plans$hx.json 2> $OUT/plans$hx.err || { tail -5 $OUT/plans$hx.err; exit 3; }
done
echo ok
