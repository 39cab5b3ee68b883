import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as entry  # noqa: E402

# Plans as the cost models choose them: the engine's autotuner (engine.cpp
# autotune_plans) times variants at create and may pick another, equally exact
# one; tests that pin plan properties need the models' choice.  The autotuner
# itself is covered in test_gpu_autotune.py.
os.environ.setdefault("GOL_DEV_AUTOTUNE", "0")

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgol.so on the GPU)")
    config.addinivalue_line("markers", "slow: long-running")


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
