#!/bin/bash
# r03: plan candidates at the 8-way rank launch shapes (block kind x half strip x
# skew rate), one process per shape set
set -o pipefail
OUT=gpurun_out/r03af
mkdir -p $OUT
CFGS='[{"handoff": 2}, {"handoff": 2, "env": {"GOL_DEV_PAIRS": 0}}, {"handoff": 2, "env": {"GOL_DEV_AGE_SKEW": 0.7}}, {"handoff": 2, "env": {"GOL_DEV_AGE_SKEW": 0.82}}, {"handoff": 2, "env": {"GOL_DEV_AGE_SKEW": 0}}, {"handoff": 1}, {"handoff": 1, "env": {"GOL_DEV_AGE_SKEW": 0.78}}]'
timeout -k 10 500 python3 tools/ab_cfg.py --cfgs "$CFGS" --shapes 8224,8288,8352,8416,8480,8544,8608,8672 --gens 512 --rounds 3 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 6; }
python3 - <<'PY'
import json, collections
t = collections.defaultdict(list)
for l in open("gpurun_out/r03af/ab.jsonl"):
    d = json.loads(l)
    t[d["shape"]].append((d["tcups_wall_median"], json.dumps(d["cfg"]), d["age_skew"]))
for sh, v in t.items():
    print(sh, " | ".join(f"{x[0]} {x[1]} {x[2]}" for x in v))
PY
