set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for L in libgol libgol_prev libgol libgol_prev; do
  echo "== $L" >> $O/ab.jsonl
  GOL_LIB=$PWD/mpi-game-of-life_amd/$L.so timeout -k 10 300 python3 tools/ab_handoff.py --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || exit 5
done
