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


@pytest.fixture(autouse=True, scope="session")
def _torch_hip_first(request):
    """GPU sessions: torch's HIP runtime is initialised before any library context.  torch ships its
    own HIP runtime beside the system one that libsccg links; when a library context opens the
    device first, torch can report "No HIP GPUs are available" later in the same process (seen
    when a test that uses torch ran after library-only tests)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.zeros(1, device="cuda:0")
        except Exception:
            pass
    yield
