set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "handoff or random_fields or row_blocking or generic" > $O/tests.log 2>&1
echo rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | head -40
