#!/bin/bash
# r03: resident (M, K) sweep at 4096^2 x 1000, new kernel and r02.
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
for lib in libgol.so libgol_r02.so; do
GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 200 python3 tools/sweep.py --size 4096 --gens 1000 --resident 2 \
   --rpw 2,3,4,6 --depths 8,12,16,24,32 --rounds 3 2>&1 | grep -v error | sed "s/^/$lib /" >> $OUT/sweep.log || exit 5
done
cat $OUT/sweep.log | cut -c1-330
