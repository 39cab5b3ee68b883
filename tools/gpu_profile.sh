#!/bin/bash
# Profile set (run on the GPU box via gpurun), for one configuration:
#   A  kernel trace + stats of the bench command (the stats average must match
#      bench.py's HIP-event average)
#   B  SQ counters (VALU issue, waits) of the same kernel
#   C/D FETCH_SIZE and WRITE_SIZE, each in its own pass (never with traces)
#   E  the bench line itself, without the profiler
# Each step has its own time limit; the first failure ends the script.
# Usage: bash tools/gpu_profile.sh TAG [--size N ...] (args shared by bench.py
# and tools/profile_run.py)
set -e -o pipefail
TAG=${1:?TAG}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records "$@" > $OUT/bench_traced.json 2> $OUT/trace.err
echo "A done"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o pmc \
    --output-format csv -- python3 tools/profile_run.py "$@" > $OUT/pmc_sq.log 2>&1
echo "B done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/pmc_$C -o pmc --output-format csv -- \
      python3 tools/profile_run.py "$@" > $OUT/pmc_$C.log 2>&1
  echo "$C done"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-sub-records "$@" > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo done > $OUT/DONE
