#!/bin/bash
# r03: full -m gpu suite + smoke + default bench (N=1) + C2 bench line.
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 400 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
grep -E "FAILED" $OUT/gpu_tests.log | head -20
timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 4; }
timeout -k 10 300 python -u bench.py --size 4096 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 4; }
cut -c1-400 $OUT/bench.json $OUT/bench_c2.json

GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py > $OUT/res_log.json 2>&1 || tail -5 $OUT/res_log.json
cat $OUT/res_log.json | tail -1
exit $rc
