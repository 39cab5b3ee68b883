set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/res_tests.log 2>&1 || { tail -30 $O/res_tests.log; exit 3; }
tail -2 $O/res_tests.log
for L in libgol libgol_exp96; do
  echo "== $L" >> $O/exp.jsonl
  GOL_LIB=$PWD/mpi-game-of-life_amd/$L.so timeout -k 10 120 python3 tools/sweep.py --size 4096 --gens 1000 --depths 0,8,12,16 --rpw 2,3,4,6 --resident 2 >> $O/exp.jsonl 2>> $O/exp.err || exit 5
done
