set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
for HX in 128 256; do
timeout -k 10 300 python3 - <<PY >> $O/sub.jsonl 2>> $O/s.err || exit 4
import sys, time, json
sys.path.insert(0, '.')
import __graft_entry__ as entry
pkg = entry.load_package()
for ho in (1, 2):
    e = pkg.Group(8192, 65536, 2, devices=[0, 0], tb_depth=16, halo_depth=$HX, handoff=ho) if hasattr(pkg, 'Group') else None
    e.init_random(1); e.step(512); e.sync()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); e.step(512); e.sync(); ts.append(time.perf_counter() - t0)
    t = sorted(ts)[1]
    print(json.dumps({"shape": "8192x65536 as 2 stripes on 2 streams", "halo_depth": $HX, "handoff": ho, "tcups": round(8192*65536*512/t/1e12, 2)}), flush=True)
    e.close()
PY
done
