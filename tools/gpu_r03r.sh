#!/bin/bash
# r03: resident epoch hand-off by tagged granules (libgol_gran.so, GOL_RES_GRAN=1)
# vs flags (libgol.so): resident parity tests with both, then the C2 A/B.
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
for lib in libgol.so libgol_gran.so; do
  GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q \
      --timeout 120 --timeout-method thread > $OUT/tests_$lib.log 2>&1
  rc=$?
  tail -2 $OUT/tests_$lib.log
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for lib in libgol.so libgol_gran.so; do
    for rule in ref conway; do
      GOL_LIB=mpi-game-of-life_amd/$lib timeout -k 10 60 python3 tools/profile_resident.py --steps 5 --rule $rule 2>/dev/null | sed "s/^/$lib /" >> $OUT/ab.log || exit 5
    done
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
dig = {}
for line in open("gpurun_out/r03r/ab.log"):
    lib, js = line.split(" ", 1)
    d = json.loads(js)
    r[(lib, d["rule"])].append(d["tcups_wall"])
    dig.setdefault(d["rule"], set()).add(tuple(d["digest"]))
for k, v in sorted(r.items()):
    print(k, sorted(v))
print({k: len(v) for k, v in dig.items()}, "distinct digests per rule (must be 1)")
PY
