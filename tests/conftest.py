"""Test configuration: `-m "not gpu"` runs on CPU (oracle, host logic, C-ABI exports, gloo
multi-process plan); `-m gpu` runs the HIP parity tests on an MI355X."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels); run with -m gpu")


@pytest.fixture(scope="session")
def native():
    """The product library (built in-tree by __graft_entry__.build() / make)."""
    from shadow_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


@pytest.fixture(scope="session")
def gpu():
    """Fails loudly (never skips to a fallback) when a gpu-marked test has no device."""
    import torch  # import first: one HIP runtime for torch and the library
    assert torch.cuda.is_available(), "gpu test needs a HIP device"
    from shadow_amd import _lib
    L = _lib.lib()
    assert L.srt_device_count() >= 1
    return L
