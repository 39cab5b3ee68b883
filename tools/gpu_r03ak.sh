#!/bin/bash
# r03: bench lines beside the headline: B3/S23 at 65536^2, the whole 262144^2 field
set -o pipefail
OUT=gpurun_out/r03ak
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --rule conway --no-cpu-baseline > $OUT/bench_conway.json 2> $OUT/bench_conway.err || { tail -20 $OUT/bench_conway.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/bench_conway.json')); print('conway', d['value'], d['ms_per_step'], d['config']['age_skew'], d['config']['handoff'])"
timeout -k 10 300 python -u bench.py --size 262144 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_262144.json 2> $OUT/bench_262144.err || { tail -20 $OUT/bench_262144.err; exit 5; }
python3 -c "import json; d=json.load(open('$OUT/bench_262144.json')); print('262144', d['value'], d['ms_per_step'], d['config']['age_skew'], d['roofline']['frac'])"
