#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against the host sanitizer builds:
# libgol_asan.so (engine.cpp under ASan + UBSan, mpi-game-of-life_amd/asan.mk)
# and liboracle_asan.so (oracle/asan.mk), with the clang sanitizer runtime
# preloaded into the (uninstrumented) Python interpreter.  Leak checking is off:
# the interpreter itself never frees its arenas.  A report aborts the test
# process (halt_on_error, -fno-sanitize-recover=undefined).  CPU only.
#   bash tools/asan_cpu_suite.sh [LOG] [pytest args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$ROOT/profiles/r05/asan_cpu_suite.log}; shift || true
make -s -C "$ROOT/mpi-game-of-life_amd" -f asan.mk -j8 || exit 1
make -s -C "$ROOT/oracle" -f asan.mk || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
mkdir -p "$(dirname "$LOG")"
{
  echo "# libgol: $ROOT/mpi-game-of-life_amd/build/asan/libgol_asan.so"
  echo "# oracle: $ROOT/oracle/liboracle_asan.so"
  echo "# runtime: $RT"
  echo "# instrumented: $(nm -D "$ROOT/mpi-game-of-life_amd/build/asan/libgol_asan.so" | grep -c ' U __asan_report') asan report symbols, $(nm -D "$ROOT/mpi-game-of-life_amd/build/asan/libgol_asan.so" | grep -c ' U __ubsan_handle') ubsan handlers imported by libgol_asan.so"
  echo "# ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1"
} > "$LOG"
GOL_LIB="$ROOT/mpi-game-of-life_amd/build/asan/libgol_asan.so" \
GOL_ORACLE_LIB="$ROOT/oracle/liboracle_asan.so" \
GOL_ASAN_SUITE=1 \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
LD_PRELOAD="$RT" \
  python -u -m pytest "$ROOT/tests" -m "not gpu" -v -p no:cacheprovider "$@" 2>&1 | tee -a "$LOG"
