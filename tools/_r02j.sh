set -o pipefail
O=gpurun_out/r02j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/res_tests.log 2>&1 || { tail -30 $O/res_tests.log; exit 3; }
tail -2 $O/res_tests.log
timeout -k 10 300 python3 bench.py > $O/bench_65536.json 2> $O/bench.err || exit 4
timeout -k 10 120 python3 bench.py --size 4096 --steps 20 --warmup 3 > $O/bench_4096.json 2>> $O/bench.err || exit 5
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 -- python3 bench.py --size 4096 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_4096_traced.json 2> $O/prof_c2.err || exit 6
for S in "1024 0" "2048 0" "8192 0" "16384 4096" "12288 4096" "8192 2048"; do
  set -- $S
  timeout -k 10 200 python3 tools/sweep.py --size $1 --width $2 --gens 1000 --depths 0 --rpw 0 --resident 0,1 >> $O/crossover.jsonl 2>> $O/cross.err || exit 7
done
