import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libp2v's HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from support import ensure_built
    ensure_built()
