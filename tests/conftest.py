import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU-side checks")


@pytest.fixture(scope="session")
def golden_cases():
    import goldens
    return goldens.load_cases()
