#!/bin/bash
# r03: autotuner with the 3% margin -- autotune tests, rank proxy, engine create
# time, C3 bench
set -o pipefail
OUT=gpurun_out/r03ah
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_autotune.py tests/test_gpu_rccl.py -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 120 python3 - > $OUT/create_time.txt 2>&1 <<'PY' || { cat $OUT/create_time.txt; exit 8; }
import os, time, sys
sys.path.insert(0, ".")
import __graft_entry__ as entry
pkg = entry.load_package()
for tune in ("0", "1"):
    os.environ["GOL_DEV_AUTOTUNE"] = tune
    for h in (65536, 8448):
        t0 = time.perf_counter()
        e = pkg.Engine(h, 65536, device=0, streams=1)
        t1 = time.perf_counter()
        e.close()
        print(f"autotune {tune} {h}x65536 create {1e3 * (t1 - t0):.1f} ms", flush=True)
PY
cat $OUT/create_time.txt
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 > $OUT/rank_proxy.jsonl 2> $OUT/rank_proxy.err || { tail $OUT/rank_proxy.err; exit 7; }
grep '^{' $OUT/rank_proxy.jsonl
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_c3.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['age_skew'])"
