import sys, json
sys.path.insert(0, '.')
import __graft_entry__ as entry
pkg = entry.load_package()
N = 65536
def dig(gens, **kw):
    with pkg.Engine(N, N, rule=pkg.CONWAY, device=0, **kw) as e:
        e.init_random(1)
        e.step(gens)
        return e.digest(), e.handoff
ref16 = dig(16, streams=1, tb_depth=1)[0]
print(json.dumps({"ref16": ref16}), flush=True)
for rep in range(3):
    for kw in ({}, {"handoff": 1}, {"streams": 1}, {"streams": 1, "handoff": 2}):
        d, ho = dig(16, **kw)
        print(json.dumps({"rep": rep, "cfg": kw, "handoff": ho, "ok": d == ref16, "d": d}), flush=True)
