"""GPU parity of autotuned plans (plan.cpp build_plans variants +
autotune_plans).

At create, an engine alone on its device times the cost models' plan of every
full-depth launch against a few variants (no half strip, skew rate x 0.95 /
1.05, the other block kind) and keeps the fastest.  Every variant is a plan kind
the other tests pin; here the autotuned engines are checked bit-exact against
the oracle and against the models' plans at the rank launch shapes where the
variants differ most, and through the rank round schedule over RCCL.
"""
import pytest

pytestmark = pytest.mark.gpu

W = 65536
THREADS = 16


@pytest.fixture
def autotune(monkeypatch):
    monkeypatch.setenv("GOL_DEV_AUTOTUNE", "1")


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("h", [8224, 8608])
def test_autotuned_stripe_vs_oracle(pkg, oracle, autotune, h, rule):
    R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
    gens = 2 * 16 + 3
    with pkg.Engine(h, W, rule=R, device=0, streams=1) as e:
        e.init_random(9)
        e.step(gens)
        got = e.digest()
    g = oracle.bp_run(oracle.bp_random(h, W, 9), W, gens, R, threads=THREADS)
    assert got == oracle.bp_digest(g, W)


def test_autotuned_equals_model_plans_c3(pkg, autotune, monkeypatch):
    """65536^2, Conway over several launches: autotuned vs the models' plan."""
    gens = 3 * 16 + 5
    with pkg.Engine(W, W, rule=pkg.CONWAY, device=0) as e:
        e.init_random(4)
        e.step(gens)
        got = e.digest()
    monkeypatch.setenv("GOL_DEV_AUTOTUNE", "0")
    with pkg.Engine(W, W, rule=pkg.CONWAY, device=0) as e:
        e.init_random(4)
        e.step(gens)
        assert e.digest() == got


def test_autotuned_rank_shape(pkg, monkeypatch):
    """The 8-way C4 rank (8192 own rows + 2 x 128 halo rows, one shared full-depth plan
    autotuned) over RCCL self-loops, against the models' plans (same field after
    four rounds and a partial one)."""
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    n, world, rank, gens = 65536, 8, 3, 2 * 256 + 40
    out = []
    for tune in ("1", "0"):
        monkeypatch.setenv("GOL_DEV_AUTOTUNE", tune)
        with pkg.Engine(n, n, rule=pkg.CONWAY, device=0, rank=rank, nranks=world,
                        uid=pkg.unique_id()) as e:
            e.init_random(3)
            e.step(gens)
            out.append((e.digest(), e.store_packed()))
    assert out[0][0] == out[1][0]
    assert (out[0][1] == out[1][1]).all()


def test_autotune_respects_waiting_kernel_registry(pkg, oracle, autotune):
    """Two default engines at a hand-off shape on one GPU, both autotuned: the
    second (device's hand-off slot taken) gets no hand-off variant, and both fields
    stay exact when stepped without syncs in between."""
    h, gens = 8448, 40
    want = oracle.bp_digest(oracle.bp_run(oracle.bp_random(h, W, 5), W, gens, oracle.CONWAY,
                                          threads=THREADS), W)
    a = pkg.Engine(h, W, rule=pkg.CONWAY, device=0)
    b = pkg.Engine(h, W, rule=pkg.CONWAY, device=0)
    try:
        assert not b.handoff
        for e in (a, b):
            e.init_random(5)
        for _ in range(2):
            a.step(gens // 2)
            b.step(gens // 2)
        assert a.digest() == want and b.digest() == want
    finally:
        a.close()
        b.close()


# ---- every variant the autotuner can pick, forced (GOL_DEV_PLAN_VARIANT) ----
# build_plans makes the named variant of every full-depth plan and runs it in
# place of the models' plan, untimed.  A variant that equals the models' plan at
# a shape is dropped there by the autotuner too (tuning reports "models").
VARIANTS = ["no_half_strip", "skew_0.95", "skew_1.05", "other_block_kind"]
_C3_WANT = {}


def _c3_want(oracle, rule, gens):
    """Oracle digest of the 65536^2 bench field after `gens` generations."""
    key = (rule, gens)
    if key not in _C3_WANT:
        R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
        g = oracle.bp_run(oracle.bp_random(W, W, 4), W, gens, R, threads=THREADS)
        _C3_WANT[key] = oracle.bp_digest(g, W)
    return _C3_WANT[key]


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_forced_variant_c3_vs_oracle(pkg, oracle, monkeypatch, variant, rule):
    """65536^2 (the C3 headline field) with the variant forced: one K = 16 launch
    and one more plus a remainder, against the oracle."""
    monkeypatch.setenv("GOL_DEV_PLAN_VARIANT", variant)
    R = pkg.REF_RULE if rule == "ref" else pkg.CONWAY
    with pkg.Engine(W, W, rule=R, device=0) as e:
        ran = e.tuning[0]
        e.init_random(4)
        e.step(16)
        d16 = e.digest()
        e.step(16 + 5)
        d37 = e.digest()
    assert ran in (variant, "models"), ran
    assert d16 == _c3_want(oracle, rule, 16), f"{variant} ({ran}) after one launch"
    assert d37 == _c3_want(oracle, rule, 37), f"{variant} ({ran}) after 37 generations"


@pytest.mark.parametrize("rule", ["ref", "conway"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_forced_variant_rank8_vs_oracle(pkg, oracle, monkeypatch, variant, rule):
    """The 8-way C4 rank shape (8192 own rows + 2 x 128 halo rows, its round's
    full-depth launches sharing one plan) with the variant forced, over an RCCL
    self-loop: against the oracle of the mirrored stripe (test_gpu_rccl.py)."""
    from test_gpu_rccl import mirrored_steps
    monkeypatch.setenv("GOL_DEV_RCCL_SELF", "1")
    monkeypatch.setenv("GOL_DEV_PLAN_VARIANT", variant)
    R = oracle.REF_RULE if rule == "ref" else oracle.CONWAY
    n, world, rank, gens = 65536, 8, 3, 2 * 16 + 5
    with pkg.Engine(n, n, rule=R, device=0, rank=rank, nranks=world,
                    uid=pkg.unique_id()) as e:
        ran, hx = e.tuning[0], e.halo_depth
        e.init_random(3)
        own = e.store_packed()
        e.step(gens)
        got = e.store_packed()
    assert ran in (variant, "models"), ran
    want = mirrored_steps(oracle, own, n, [gens], R, hx, True, True)[0]
    assert (got == want).all(), f"{variant} ({ran})"


def test_tuning_report(pkg, monkeypatch):
    """gol_plan_tuning: the models' plan untimed with the autotuner off; a forced
    variant is reported by name; an autotuned engine reports both timings."""
    monkeypatch.setenv("GOL_DEV_AUTOTUNE", "0")
    with pkg.Engine(W, W, device=0) as e:
        assert e.tuning == ("models", 0.0, 0.0)
    monkeypatch.setenv("GOL_DEV_PLAN_VARIANT", "no_half_strip")
    with pkg.Engine(W, W, device=0) as e:
        assert e.tuning[0] == "no_half_strip" and e.columns[1] == 0
    monkeypatch.delenv("GOL_DEV_PLAN_VARIANT")
    monkeypatch.setenv("GOL_DEV_AUTOTUNE", "1")
    with pkg.Engine(W, W, device=0) as e:
        v, t, m = e.tuning
        assert v in pkg.TUNE_VARIANTS and t > 0 and m > 0 and t <= m
