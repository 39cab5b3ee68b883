#!/bin/bash
# GPU-box check (via gpurun): the -m gpu parity suite, smoke, then one default
# bench line.  A failing test does not stop the bench; a fault, abort, crash or
# time limit does (nothing more runs on the GPU after one).
# Usage: bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-check}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log | tail -20; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 4; }
cat $OUT/bench.json
exit $rc
