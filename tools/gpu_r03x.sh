#!/bin/bash
# r03: 4-plane lane groups at K = 8 (dev build) vs the K = 16 2-plane default
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
GOL_LIB=mpi-game-of-life_amd/libgol_dev.so timeout -k 10 400 python3 tools/ab_cfg.py \
    --cfgs '[{}, {"tb_depth": 8, "word_planes": 4}, {"tb_depth": 8, "word_planes": 4, "handoff": 1}, {"tb_depth": 8}]' \
    --shapes 65536,8448,16640 --gens 512 --rounds 5 > $OUT/ab_np4.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
cat $OUT/ab_np4.jsonl
