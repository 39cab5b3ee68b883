#!/bin/bash
# r03: resident kernel A/B -- priority for the edge rows (exp4096), per-row skip
# of the edge rows (exp8192), both (exp12288) vs the default; C2 and Conway.
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in libgol.so libgol_exp4096.so libgol_exp8192.so libgol_exp12288.so; do
    for rule in ref conway; do
      GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 60 python3 tools/profile_resident.py --steps 5 --rule $rule 2>/dev/null | sed "s/^/$lib /" >> $OUT/ab.log || exit 5
    done
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
dig = {}
for line in open("gpurun_out/r03h/ab.log"):
    lib, js = line.split(" ", 1)
    d = json.loads(js)
    r[(lib, d["rule"])].append(d["tcups_wall"])
    dig.setdefault(d["rule"], set()).add(tuple(d["digest"]))
for k, v in sorted(r.items()):
    print(k, sorted(v))
print({k: len(v) for k, v in dig.items()}, "distinct digests per rule (must be 1)")
PY
