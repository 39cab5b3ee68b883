#!/bin/bash
# r03: full -m gpu suite, then resident-kernel (C2) kernel stats + SQ counters.
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 400 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/gpu_tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o res --output-format csv -- \
    python3 tools/profile_resident.py > $OUT/res_trace.log 2>&1 || { tail -5 $OUT/res_trace.log; exit 5; }
tail -1 $OUT/res_trace.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS \
    -d $OUT/pmc1 -o sq --output-format csv -- python3 tools/profile_resident.py > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 6; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
    -d $OUT/pmc2 -o sq --output-format csv -- python3 tools/profile_resident.py > $OUT/pmc2.log 2>&1 || { tail -5 $OUT/pmc2.log; exit 7; }
echo done
exit $rc
