import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gym-so100-c_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def model():
    from gym_so100.model import build_model
    return build_model()


@pytest.fixture(scope="session")
def oracle64():
    from oracle.oracle import Oracle
    return Oracle(64)


@pytest.fixture(scope="session")
def oracle32():
    from oracle.oracle import Oracle
    return Oracle(32)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_task.npz")))
