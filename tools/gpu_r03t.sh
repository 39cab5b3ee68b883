#!/bin/bash
# r03: packed half strip -- plans, parity (half-strip, skew, full-size tests), the
# in-process A/B against GOL_DEV_PAIRS=0, then the default bench line.
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
GOL_DEV_PLANS=1 timeout -k 10 120 python3 -c "
import __graft_entry__ as e
pkg = e.load_package()
for h, w in [(65536, 65536), (8448, 65536), (16640, 65536), (32768, 262144)]:
    with pkg.Engine(h, w, device=0, streams=1) as g:
        print(h, w, g.columns, g.age_skew, g.handoff, flush=True)
" > $OUT/plans.log 2>&1 || { tail -20 $OUT/plans.log; exit 5; }
cat $OUT/plans.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_halfstrip.py tests/test_gpu_skew.py tests/test_gpu_fullsize.py \
    -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto \
    --shapes 65536,8448,16640,33024,32768x262144 --gens 512 --rounds 5 > $OUT/ab_pairs.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_pairs.jsonl
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 4; }
cat $OUT/bench.json
