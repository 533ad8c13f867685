import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """GPU tests run on the GPU box only.  The HIP library must load there:
    a missing extension is a failure, never a skip."""
    if not gpu_available():
        pytest.skip("no GPU visible")
    from stencil_amd import _lib
    _lib.load()
    return 0
