#!/bin/bash
# Dev: build timing-experiment variants of libgol.so (GOL_EXP bits, see
# life_stencil.h: 1-8; life_resident.hip: 64 no epoch waits between tiles,
# 2048 per-wave cycle stamps of the resident kernel) as mpi-game-of-life_amd/libgol_exp<N>.so.  Results of these
# libraries are not valid fields; they exist to time pieces of the hand-off.
# Usage: [EXP_DEFS="-DX=Y" EXP_TAG=_y] tools/exp_build.sh N [N ...]
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
for N in "$@"; do
  D=/tmp/golexp$N
  rm -rf $D && mkdir -p $D && cp -r $ROOT/mpi-game-of-life_amd $D/ && cp -r $ROOT/include $D/
  rm -rf $D/mpi-game-of-life_amd/build $D/mpi-game-of-life_amd/*.so
  make -s -C $D/mpi-game-of-life_amd -j8 libgol.so KFLAGS="-mllvm -pragma-unroll-threshold=1000000 -DGOL_EXP=$N $EXP_DEFS" \
       CXXFLAGS="-O3 -std=c++17 -fPIC -DGOL_EXP=$N"
  cp $D/mpi-game-of-life_amd/libgol.so $ROOT/mpi-game-of-life_amd/libgol_exp$N$EXP_TAG.so
done
