#!/bin/bash
# Dev A/B: build tools/libgol_<name>.so from the current sources with extra
# defines, K=16 kernels only (GOL_DEV_ONLY_DEPTH), for GOL_LIB=... sweeps.
# Usage: tools/build_alt.sh NAME [-DFOO=1 ...]
set -e
N=$1; shift
cd "$(dirname "$0")/../mpi-game-of-life_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -DGOL_DEV_ONLY_DEPTH=16 "$@" --offload-arch=gfx950 -shared \
  -o ../tools/libgol_$N.so csrc/life_kernels.hip csrc/engine.cpp -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib 2>&1 | grep -E "error" || true
ls -la ../tools/libgol_$N.so
