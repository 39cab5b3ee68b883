#!/bin/bash
# Profile set of one N-way rank shape on ONE GPU (run via gpurun): the middle
# rank of the 65536^2 N-way split as a rank engine over an RCCL self-loop
# communicator (its launches are the N-GPU run's per-rank launches).
#   A  kernel trace + stats of tools/rank_proxy.py (the rank's steps)
#   B  SQ counters, C/D FETCH_SIZE and WRITE_SIZE (each pass its own run) of
#      tools/profile_run.py --ranks N
# tools/pmc_counters.py turns the directory into a counters.json record keyed by
# n_gpus = N and the rank's rows per wavefront (bench.py reads it at N > 1).
# Usage: bash tools/gpu_profile_rank.sh TAG N [--rule conway]
set -e -o pipefail
TAG=${1:?TAG}; N=${2:?N}; shift 2
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RULE=ref
[ "$1" = "--rule" ] && RULE=$2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o rank --output-format csv -- \
    python3 tools/rank_proxy.py --transports rccl --ranks $N --skews auto --rounds 3 \
    > $OUT/proxy_traced.jsonl 2> $OUT/trace.err
echo "A done"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o pmc \
    --output-format csv -- python3 tools/profile_run.py --ranks $N --rule $RULE > $OUT/pmc_sq.log 2>&1
echo "B done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/pmc_$C -o pmc --output-format csv -- \
      python3 tools/profile_run.py --ranks $N --rule $RULE > $OUT/pmc_$C.log 2>&1
  echo "$C done"
done
echo done > $OUT/DONE
