import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        O.build()
    return O


@pytest.fixture(scope="session")
def mp():
    import mpfft_loader
    return mpfft_loader.load()
