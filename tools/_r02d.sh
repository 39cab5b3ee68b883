set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/ab_handoff.py --rounds 3 > $O/ab.jsonl 2>> $O/ab.err || exit 5
cat $O/ab.jsonl
exit $rc
