#!/bin/bash
# GPU-box A/B: parity suite, then in-process variant sweeps, then the bench.
# Usage (via gpurun): bash tools/gpu_ab.sh "<sweep args 1>" "<sweep args 2>" ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
i=0
for args in "$@"; do
  i=$((i+1))
  echo "== sweep $i: $args" | tee -a gpurun_out/sweeps.log
  timeout -k 10 300 python -u tools/sweep.py $args 2>&1 | tee -a gpurun_out/sweeps.log || exit 1
done
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
