#!/bin/bash
# Dev A/B: build mpi-game-of-life_amd/libgol_<name>.so from the current sources
# with extra defines (e.g. -DGOL_RES_GRAN=1), for GOL_LIB=... comparisons.
# Usage: tools/build_alt.sh NAME [-DFOO=1 ...]
set -e
N=$1; shift
ROOT=$(cd $(dirname $0)/.. && pwd)
D=/tmp/golalt_$N
rm -rf $D && mkdir -p $D && cp -r $ROOT/mpi-game-of-life_amd $D/ && cp -r $ROOT/include $D/
rm -rf $D/mpi-game-of-life_amd/build $D/mpi-game-of-life_amd/*.so
make -s -C $D/mpi-game-of-life_amd -j8 libgol.so KFLAGS="-mllvm -pragma-unroll-threshold=1000000 $*" \
     CXXFLAGS="-O3 -std=c++17 -fPIC $*"
cp $D/mpi-game-of-life_amd/libgol.so $ROOT/mpi-game-of-life_amd/libgol_$N.so
ls -la $ROOT/mpi-game-of-life_amd/libgol_$N.so
