"""Host-side logic of bench.py (no GPU): the per-rank breakdown adds up, the
counters record lookup, and the JSON contract's timing passes.

rank_breakdown (r06) turns one rank's gol_timing into per-step spans:
kernel_span + exchange_exposed + other = ms_per_step, exchange_exposed +
exchange_hidden = exchange, none negative when the timing is self-consistent
(what the engine's disjoint compute-stream intervals guarantee).
"""
import importlib.util
import os
import types

import pytest

from conftest import ROOT


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def fake_engine():
    return types.SimpleNamespace(rows=8192, row0=24576, halo_depth=128, tb_depth=16,
                                 rows_per_wave=58, handoff=True, age_skew=(82, 58, 1024),
                                 tuning=("models", 75.8, 75.8), w=65536)


def timing(round_ms, xch_ms, exposed_ms, steps=3, launches=24, issued=189):
    return {"launches": launches, "kernel_ms": launches * 0.0704, "cell_gens": 0.0,
            "cell_gens_computed": 0.0, "streams": 1, "launches_issued": issued,
            "launch_rows": launches * 8416.0, "exchanges": 8 * steps, "exchange_ms": xch_ms,
            "rounds": 8 * steps, "round_ms": round_ms, "exchange_exposed_ms": exposed_ms}


@pytest.mark.parametrize("mode", ["blocking", "overlapped"])
def test_rank_breakdown_adds_up(mode):
    bench = load_bench()
    steps = 3
    # per step: 4.30 ms of round spans, 0.16 ms of exchanges; blocking: all of it
    # exposed, overlapped: 0.02 ms past the round ends
    exposed = 0.16 * steps if mode == "blocking" else 0.02 * steps
    tm = timing(4.30 * steps, 0.16 * steps, exposed, steps)
    dt = 4.55e-3 * steps
    r = bench.rank_breakdown(fake_engine(), tm, dt, steps, 3)
    total = r["kernel_span_ms_per_step"] + r["exchange_exposed_ms_per_step"] + r["other_ms_per_step"]
    assert total == pytest.approx(r["ms_per_step"], abs=2e-3)
    assert r["exchange_exposed_ms_per_step"] + r["exchange_hidden_ms_per_step"] == \
        pytest.approx(r["exchange_ms_per_step"], abs=2e-3)
    for k in ("kernel_span_ms_per_step", "exchange_exposed_ms_per_step",
              "exchange_hidden_ms_per_step", "other_ms_per_step"):
        assert r[k] >= 0, (k, r)
    assert r["rounds_per_step"] == 8 and r["exchanges_per_step"] == 8
    # the mean launch is reported, not multiplied into a time share
    assert r["avg_launch_ms"] == pytest.approx(0.0704)
    assert "kernel_ms_per_step" not in r


def test_counters_lookup_prefers_newest_round():
    bench = load_bench()
    cfg = {"size": 65536, "rule": "ref", "tb_depth": 16, "streams": 1, "n_gpus": 1,
           "rows_per_wave": 440, "handoff": False}
    rec = bench.counters_for(cfg)
    assert rec is not None and rec["source_round"] == "r06", rec and rec.get("source")
    assert rec["insts_valu_per_launch"] > 0 and rec["hbm_bytes_per_launch"] > 0
    # a rows-per-wave more than 5% away matches nothing
    assert bench.counters_for(dict(cfg, rows_per_wave=600)) is None


def test_timed_steps_has_no_events_in_the_timed_pass():
    """timed_steps: the measured pass runs with timing off (set_timing(0)), the
    event pass after it with sampling on; the returned timing is the event pass's."""
    bench = load_bench()
    calls = []

    class Eng:
        def step(self, g):
            calls.append(("step", self.every))

        def sync(self):
            pass

        def set_timing(self, every):
            self.every = every
            calls.append(("timing", every))

        def reset_timing(self):
            calls.append(("reset", None))

        def timing(self):
            return {"pass": "events"}

    e = Eng()
    e.every = None
    torch = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda: None))
    dt, dt_ev, tm = bench.timed_steps(e, 1000, 3, 1, 1, None, torch, 8)
    steps = [c for c in calls if c[0] == "step"]
    assert len(steps) == 1 + 3 + 3
    assert all(every == 0 for _, every in steps[1:4]), steps  # the measured pass
    assert all(every == 8 for _, every in steps[4:]), steps    # the event pass
    assert tm == {"pass": "events"} and dt > 0 and dt_ev > 0
    assert calls[-1] == ("timing", 0)
