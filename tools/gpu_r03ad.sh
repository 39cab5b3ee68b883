#!/bin/bash
# r03: resident kernel, cooperative vs plain launch (one process, interleaved)
set -o pipefail
OUT=gpurun_out/r03ad
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_cfg.py --cfgs '[{"resident": 2}, {"resident": 2, "env": {"GOL_DEV_RES_COOP": 0}}, {"resident": 2}, {"resident": 2, "env": {"GOL_DEV_RES_COOP": 0}}]' \
    --shapes 4096x4096 --gens 1000 --rounds 9 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
timeout -k 10 300 python3 tools/ab_cfg.py --rule conway --cfgs '[{"resident": 2}, {"resident": 2, "env": {"GOL_DEV_RES_COOP": 0}}]' \
    --shapes 4096x4096,8192x8192 --gens 1000 --rounds 9 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab.jsonl
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_AGE_SKEW --values 0.66,0.69,auto,0.75,0.78 \
    --shapes 65536,33024 --gens 512 --rounds 5 > $OUT/ab_rho.jsonl 2> $OUT/ab_rho.err || { tail $OUT/ab_rho.err; exit 7; }
cat $OUT/ab_rho.jsonl
