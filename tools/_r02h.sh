set -o pipefail
O=gpurun_out/r02h; mkdir -p $O
for L in libgol libgol_exp16 libgol_exp32 libgol_exp64 libgol_exp96; do
  echo "== $L" >> $O/exp.jsonl
  GOL_LIB=$PWD/mpi-game-of-life_amd/$L.so timeout -k 10 120 python3 tools/sweep.py --size 4096 --gens 1000 --depths 0,8 --rpw 2,4,8 --resident 2 >> $O/exp.jsonl 2>> $O/exp.err || exit 5
done
