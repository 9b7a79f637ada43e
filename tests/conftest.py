import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    if not os.path.exists(oracle.LIB):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    import prt
    return prt.Context(0)
