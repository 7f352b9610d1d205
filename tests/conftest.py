import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "speedy-ml-1_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (tests marked gpu must run on the MI355X box)")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return dict(np.load(os.path.join(REPO, "tests", "golden", "spectral_ref.npz")))


@pytest.fixture(scope="session")
def dyn_golden():
    """Reference `step` outputs (tests/golden/make_dyn_golden.py)."""
    import numpy as np

    return dict(np.load(os.path.join(REPO, "tests", "golden", "dyn_ref.npz")))


DYN_CASES = ("fwd", "lf0", "lf", "expl")
