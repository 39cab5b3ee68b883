#!/bin/bash
# Dev: build a variant of libgol.so with extra compile definitions (valid
# fields, unlike tools/exp_build.sh's timing probes) as
# mpi-game-of-life_amd/libgol_<NAME>.so, for in-process A/B through GOL_LIB.
# Usage: tools/variant_build.sh NAME "-DFOO=1 -DBAR=2"
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
NAME=$1; DEFS=$2
D=/tmp/golvar_$NAME
rm -rf $D && mkdir -p $D && cp -r $ROOT/mpi-game-of-life_amd $D/ && cp -r $ROOT/include $D/
rm -rf $D/mpi-game-of-life_amd/build $D/mpi-game-of-life_amd/*.so
make -s -C $D/mpi-game-of-life_amd -j8 libgol.so KFLAGS="-mllvm -pragma-unroll-threshold=1000000 $DEFS" \
     CXXFLAGS="-O3 -std=c++17 -fPIC $DEFS"
cp $D/mpi-game-of-life_amd/libgol.so $ROOT/mpi-game-of-life_amd/libgol_$NAME.so
mkdir -p $ROOT/mpi-game-of-life_amd/build_$NAME
cp $D/mpi-game-of-life_amd/build/life_tb_d16*.o $ROOT/mpi-game-of-life_amd/build_$NAME/ 2>/dev/null || true
