"""bench.py's one JSON line on the GPU: the driver's contract keys, the roofline
and cpu_baseline objects, and a value consistent with ms_per_step (a small field,
so it runs in seconds; the headline 65536^2 line is the driver's own run)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_json_contract():
    n, gens, steps = 2048, 64, 2
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--size", str(n),
                        "--gens", str(gens), "--steps", str(steps), "--warmup", "1",
                        "--cpu-threads", "2"], capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == steps and rec["warmup"] == 1
    assert rec["higher_is_better"] is True and rec["unit"] == "GCUPS"
    # value is the whole job's cell updates over the measured time
    assert rec["value"] == pytest.approx(n * n * gens / (rec["ms_per_step"] * 1e-3) / 1e9,
                                         rel=0.01)
    assert "workload" in rec["config"]
    rf = rec["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert 0 < rf["frac"] < 1 and rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"], rel=0.01)
    cb = rec["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["cores"] == 2 and cb["kind"] == "port" and cb["value"] > 0


def test_bench_two_rank_rehearsal_exchange_modes():
    """bench.py --gpus 2 under torch.distributed.run on ONE GPU (GOL_DEV_RCCL_SELF=1:
    each rank's engine talks RCCL to itself, ranks over gloo): the N > 1 record
    carries both forced exchange modes and the default engine's own choice (late r06),
    and a rehearsal never reports an N-GPU value."""
    env = dict(os.environ, GOL_DEV_RCCL_SELF="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", "29561", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--size", "8192", "--gens", "256", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=280, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["rehearsal"] is True and rec["value"] is None
    modes = rec["exchange_modes"]
    assert set(modes) == {"overlapped", "blocking", "auto"}
    auto = modes["auto"]
    assert auto["default"] is True and auto["mode"] in ("blocking", "overlapped")
    assert rec["config"]["exchange"] == auto["mode"]
    assert all(v > 0 for v in auto["tuned_ms_per_round"].values())
    for m in modes.values():
        assert m["value"] > 0 and len(m["per_rank"]) == 2
