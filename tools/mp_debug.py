#!/usr/bin/env python3
"""Dev tool: where a multi-pass launch (GOL_DEV_PASSES) differs from the oracle.
Prints, per configuration, the mismatching rows / 64-bit column words and the
plan's block length, so that a wrong row band (a block seam, a hand-off tail) or
column band (a strip's halo lanes) shows.

    python tools/mp_debug.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402

pkg = entry.load_package()


def run(h, w, passes, handoff, rpw, gens, rule, skew=None, K=16):
    os.environ["GOL_DEV_PASSES"] = str(passes)
    if skew is not None:
        os.environ["GOL_DEV_AGE_SKEW"] = str(skew)
    else:
        os.environ.pop("GOL_DEV_AGE_SKEW", None)
    g = oracle.bp_random(h, w, 7)
    kw = dict(rows_per_wave=rpw) if rpw else {}
    with pkg.Engine(h, w, rule=rule, device=0, tb_depth=K, handoff=handoff, **kw) as e:
        e.load_packed(g)
        e.step(gens)
        got = e.store_packed()
        info = dict(h=h, w=w, passes=passes, handoff=handoff, rpw_cfg=rpw, gens=gens, skew=skew,
                    plan_passes=e.passes, plan_handoff=e.handoff, rows_per_wave=e.rows_per_wave,
                    age_skew=e.age_skew, columns=e.columns)
    want = oracle.bp_run(g, w, gens, rule)
    bad = got != want
    rows = np.nonzero(bad.any(axis=1))[0]
    cols = np.nonzero(bad.any(axis=0))[0]
    info["bad_rows"] = len(rows)
    info["bad_row_list"] = rows[:40].tolist()
    info["bad_col_words"] = cols[:40].tolist()
    print(json.dumps(info), flush=True)


W = 62 * 64 * 2 + 100
for args in [
    (3007, W, 2, 2, 64, 32, pkg.REF_RULE, 0),
    (3007, W, 2, 2, 0, 32, pkg.REF_RULE, None),
    (3007, 4000, 2, 2, 64, 32, pkg.REF_RULE, 0),
    (1000, 4000, 2, 2, 100, 32, pkg.REF_RULE, 0),
    (3007, W, 1, 2, 64, 32, pkg.REF_RULE, 0),
    (3007, W, 2, 1, 64, 32, pkg.REF_RULE, 0),
]:
    run(*args)
