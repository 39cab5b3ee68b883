import sys, json, time
sys.path.insert(0, '.')
import __graft_entry__ as entry
pkg = entry.load_package()
N = 65536
R = pkg.CONWAY
with pkg.Engine(N, N, rule=R, device=0, streams=1, tb_depth=1) as e:
    e.init_random(1); e.step(16); ref16 = e.digest()
print(json.dumps({"ref16": ref16}), flush=True)
cfgs = [{}, {"handoff": 1}, {"streams": 1, "handoff": 2}]
bad = {str(c): 0 for c in cfgs}
for rep in range(8):
    for kw in cfgs:
        with pkg.Engine(N, N, rule=R, device=0, **kw) as e:
            e.init_random(1)
            e.step(16)
            d = e.digest()
            if d != ref16:
                bad[str(kw)] += 1
                print(json.dumps({"rep": rep, "cfg": kw, "bad": d}), flush=True)
print(json.dumps({"bad_counts": bad}), flush=True)
