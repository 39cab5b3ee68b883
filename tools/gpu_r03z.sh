#!/bin/bash
# r03: half-strip block scale under hand-off plans (sweep), and classic + half strip
set -o pipefail
OUT=gpurun_out/r03z
mkdir -p $OUT
for sc in 0.7 0.75 0.8 0.85 0.9; do
  GOL_DEV_HALF_SCALE=$sc timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 2 --handoff 2 \
      --shapes 8448,8704,12288,16640,33024 --gens 512 --rounds 5 | sed "s/^/{\"scale\": $sc, \"r\": /; s/\$/}/" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
done
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0,auto --handoff 1 \
    --shapes 8448,8704,12288,16640,33024 --gens 512 --rounds 5 | sed "s/^/{\"scale\": \"classic\", \"r\": /; s/\$/}/" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
timeout -k 10 300 python3 tools/ab_env.py --var GOL_DEV_PAIRS --values 0 --handoff 2 \
    --shapes 8448,8704,12288,16640,33024 --gens 512 --rounds 5 | sed "s/^/{\"scale\": \"hand_nopairs\", \"r\": /; s/\$/}/" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
python3 - <<'PY'
import json, collections
t = collections.defaultdict(dict)
for l in open("gpurun_out/r03z/ab.jsonl"):
    d = json.loads(l); r = d["r"]
    key = f'{d["scale"]}/{r["GOL_DEV_PAIRS"]}'
    t[r["shape"]][key] = r["tcups_wall_median"]
for sh, v in t.items():
    print(sh, json.dumps(v))
PY
