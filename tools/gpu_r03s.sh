#!/bin/bash
# r03: per-wave epoch timing of the flag and granule hand-offs (GOL_EXP 2048 builds)
set -o pipefail
OUT=gpurun_out/r03s
mkdir -p $OUT
for lib in libgol_exp2048.so libgol_gran2048.so; do
  GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 60 python3 tools/res_log.py > $OUT/res_log_$lib.json 2>&1 || exit 5
  echo $lib; tail -1 $OUT/res_log_$lib.json
done
