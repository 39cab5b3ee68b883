set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|WAIT_INST|INST_LEVEL|SQC_" $O/counters.txt | head -60 > $O/counters_sel.txt || true
for V in "--rows 8448 --handoff 1" "--rows 8448 --handoff 2" "--rows 33024 --handoff 1" "--rows 33024 --handoff 2"; do
  T=$(echo $V | tr -d ' -')
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_IFETCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$T -o pmc --output-format csv -- python3 tools/profile_shape.py $V > $O/pmc_$T.log 2>&1 || exit 5
  echo "$T done"
done
