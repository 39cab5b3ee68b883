#!/bin/bash
# SQ/GRBM counters for the stencil kernel (separate pass from the HBM counters).
set -e
TAG=${1:-sq}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
   -T -d $OUT/pmc -o sq --output-format csv -- python3 tools/profile_run.py "$@" > $OUT/sq.log 2>&1
