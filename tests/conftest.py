import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ggml-cuda-experiments_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU visible (torch.cuda.is_available() is False)")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _reset_planner_options():
    """fattn_set_option state is process-wide: whatever a test sets (and however
    it ends), the next test starts from the defaults."""
    yield
    try:
        import fattn
        fattn.reset_options()
    except Exception:
        pass  # library not built / not loadable: nothing was set
