set -o pipefail
O=gpurun_out/cw2; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --rule conway --no-cpu-baseline --steps 2 > $O/bench_conway.json 2> $O/err || { tail $O/err; exit 9; }
cut -c1-250 $O/bench_conway.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > $O/bench_ref.json 2>> $O/err || { tail $O/err; exit 9; }
cut -c1-250 $O/bench_ref.json
timeout -k 10 300 python -u tools/ab_skew.py --shapes 8448 --rhos auto --handoffs 0 --gens 256 --rounds 3 --rule conway > $O/ab.jsonl 2>> $O/err || { tail $O/err; exit 9; }
cat $O/ab.jsonl
