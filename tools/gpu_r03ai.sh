#!/bin/bash
# r03: halo depth at the 4- and 8-way rank shapes (RCCL self-loop proxy, autotuned)
set -o pipefail
OUT=gpurun_out/r03ai
mkdir -p $OUT
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 4 --halo-depths 128,256 > $OUT/rp4.jsonl 2> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
timeout -k 10 300 python3 tools/rank_proxy.py --transports rccl --overlaps 1 --skews auto --ranks 8 --halo-depths 256,512 > $OUT/rp8.jsonl 2>> $OUT/rp.err || { tail $OUT/rp.err; exit 7; }
grep -h '^{' $OUT/rp4.jsonl $OUT/rp8.jsonl
