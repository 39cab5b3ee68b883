#!/bin/bash
# Run on the GPU box (via gpurun): kernel-trace stats of the bench, then the PMC
# passes (FETCH_SIZE and WRITE_SIZE separately, never with sys/runtime traces).
# Usage: tools/gpu_profile.sh TAG [bench args...]
set -e
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o bench --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_traced.json 2> $OUT/trace.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_$C -o pmc --output-format csv -- \
      python3 tools/profile_run.py "$@" > $OUT/pmc_$C.log 2>&1
done
echo done > $OUT/DONE
