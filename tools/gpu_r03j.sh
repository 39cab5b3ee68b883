#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py 2>/dev/null | tail -1
GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py --tb-depth 8 --rows-per-wave 2 2>/dev/null | tail -1
GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py --tb-depth 24 --rows-per-wave 4 2>/dev/null | tail -1
