#!/bin/bash
# r03: resident kernel -- parity of the split progress words, then A/B vs the
# priority variant and r02.
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -k "resident or c2" -q --timeout 200 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $OUT/tests.log | head -20; exit 2; }
tail -1 $OUT/tests.log
for rep in 1 2 3; do
  for lib in libgol.so libgol_split.so libgol_prio.so; do
    for rule in ref conway; do
      GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 60 python3 tools/profile_resident.py --steps 5 --rule $rule 2>/dev/null | sed "s/^/$lib /" >> $OUT/ab.log || exit 5
    done
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
dig = {}
for line in open("gpurun_out/r03i/ab.log"):
    lib, js = line.split(" ", 1)
    d = json.loads(js)
    r[(lib, d["rule"])].append(d["tcups_wall"])
    dig.setdefault(d["rule"], set()).add(tuple(d["digest"]))
for k, v in sorted(r.items()):
    print(k, sorted(v))
print({k: len(v) for k, v in dig.items()}, "distinct digests per rule (must be 1)")
PY
GOL_LIB=mpi-game-of-life_amd/libgol_exp2048.so timeout -k 10 60 python3 tools/res_log.py 2>/dev/null | tail -1
