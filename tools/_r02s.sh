set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
export TMPDIR=/tmp
# hand-off kernels under the kernel-trace profiler: previous build, then this one
GOL_LIB=$PWD/mpi-game-of-life_amd/libgol_prev.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prev -o t --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --handoff 2 > $O/prev.json 2> $O/prev.err; echo "prev rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/cur -o t --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --handoff 2 > $O/cur.json 2> $O/cur.err; echo "cur rc=$?"
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --handoff 2 > $O/cur_noprof.json 2> $O/cur_noprof.err; echo "noprof rc=$?"
grep -h "GolError" $O/*.err | head
