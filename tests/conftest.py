import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as entry  # noqa: E402

# The engine's autotuner (plan.cpp autotune_plans) times a few variants of the
# cost models' plan at create and may pick another, equally exact one.  Parity
# tests run with it on (the shipped default); tests that pin plan properties (the
# skew lengths, the half strip's layout, the waiting-kernel registry's block
# kinds) take the `model_plans` fixture.  test_gpu_autotune.py forces each variant.

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgol.so on the GPU)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def model_plans(monkeypatch):
    """The cost models' plans (GOL_DEV_AUTOTUNE=0) for tests that assert them."""
    monkeypatch.setenv("GOL_DEV_AUTOTUNE", "0")


@pytest.fixture(scope="session")
def oracle():
    return entry.load_oracle()


@pytest.fixture(scope="session")
def pkg():
    return entry.load_package()


@pytest.fixture(scope="session")
def ref_data():
    with open(os.path.join(GOLDEN, "data.txt"), "rb") as f:
        return f.read()
