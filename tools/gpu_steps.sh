#!/bin/bash
# The one GPU-box recipe (run via gpurun): a list of steps, each under its own
# time limit, output under gpurun_out/<OUT>/.  The first step that fails ends the
# script (nothing more runs on the GPU after a fault, abort, crash or timeout).
#
#   bash tools/gpu_steps.sh OUT STEP [STEP ...]
#
# Steps (arguments after ':' are split on spaces):
#   tests[:FILES]       the -m gpu suite (FILES: test files instead of all of tests/)
#   smoke               __graft_entry__.smoke()
#   bench:NAME[:ARGS]   python bench.py ARGS -> NAME.json
#   rehearse2:NAME[:ARGS]  bench.py --gpus 2 on ONE GPU with self-looped RCCL
#                       (GOL_DEV_RCCL_SELF=1, ranks over gloo) -> NAME.json
#   rehearse8:NAME[:ARGS]  the same with 8 ranks sharing the one GPU
#   proxy:NAME:ARGS     python tools/rank_proxy.py ARGS -> NAME.jsonl
#   py:NAME:ARGS        python ARGS (a tool script and its arguments) -> NAME.out
#   trace:NAME:CMD      rocprofv3 --kernel-trace --stats of python CMD -> NAME/
#   pmc:NAME:CTRS:CMD   one rocprofv3 --pmc pass (CTRS comma-separated, one pass's
#                       worth) of python CMD -> NAME/
# Example:
#   gpurun -- bash tools/gpu_steps.sh r04a tests smoke bench:c3 \
#       "proxy:rp:--transports rccl --ranks 4,8 --shrinks 0,1"
set -o pipefail
OUT=gpurun_out/${1:?OUT}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  name=${rest%%:*}
  args=${rest#*:}; [ "$args" = "$rest" ] && args=""
  echo "== $kind $name $args"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest ${rest:-tests} -m gpu -v -rf --timeout 300 \
          --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
      rc=$?
      grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -2
      if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" "$OUT/gpu_tests.log" | head -20; exit $rc; fi ;;
    smoke)
      timeout -k 10 120 python -u -c "import __graft_entry__ as e; e.smoke()" \
          > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 3; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err" \
          || { tail -30 "$OUT/$name.err"; exit 4; }
      cut -c1-600 "$OUT/$name.json" ;;
    rehearse2)
      GOL_DEV_RCCL_SELF=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
          $args > "$OUT/$name.json" 2> "$OUT/$name.err" \
          || { grep -A3 Error "$OUT/$name.err" | head -30; exit 5; }
      cut -c1-600 "$OUT/$name.json" ;;
    rehearse8)
      GOL_DEV_RCCL_SELF=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 \
          $args > "$OUT/$name.json" 2> "$OUT/$name.err" \
          || { grep -A3 Error "$OUT/$name.err" | head -30; exit 5; }
      cut -c1-600 "$OUT/$name.json" ;;
    proxy)
      timeout -k 10 600 python -u tools/rank_proxy.py $args > "$OUT/$name.jsonl" \
          2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 6; }
      cut -c1-400 "$OUT/$name.jsonl" ;;
    py)
      timeout -k 10 600 python -u $args > "$OUT/$name.out" 2> "$OUT/$name.err" \
          || { tail -20 "$OUT/$name.err"; exit 7; }
      tail -40 "$OUT/$name.out" | cut -c1-400 ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
          --output-format csv -- python3 $args > "$OUT/$name.out" 2> "$OUT/$name.err" \
          || { tail -20 "$OUT/$name.err"; exit 8; }
      head -6 "$OUT/$name/run_kernel_stats.csv" | cut -c1-200 ;;
    pmc)
      ctrs=${args%%:*}; cmd=${args#*:}
      timeout -s KILL 180 rocprofv3 --pmc ${ctrs//,/ } -d "$OUT/$name" -o pmc \
          --output-format csv -- python3 $cmd > "$OUT/$name.out" 2>&1 \
          || { tail -20 "$OUT/$name.out"; exit 9; }
      echo "pmc $name done" ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo done > "$OUT/DONE"
