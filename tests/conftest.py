import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "montecarlo-gated-mil_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def hip_lib():
    """The built libmcgmil.so (built on demand)."""
    from mcgmil import _build, _lib
    _build.build()
    return _lib.load()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    from mcgmil import _build
    _build.build()
    return torch.device("cuda", 0)
