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


# SRT_FORM keys: forcing of internal forms for tests, one environment variable
def set_form(monkeypatch, **kv):
    """Merge key=value pairs into SRT_FORM for this test (monkeypatch restores it)."""
    cur = {}
    for item in os.environ.get("SRT_FORM", "").split(","):
        if "=" in item:
            k, v = item.split("=", 1)
            cur[k.strip()] = v
    cur.update({k: str(v) for k, v in kv.items()})
    monkeypatch.setenv("SRT_FORM", ",".join(f"{k}={v}" for k, v in cur.items()))


class form_env:
    """Context manager: SRT_FORM with key=value pairs merged in, restored on exit (for a part of
    a test; set_form covers a whole test)."""

    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = os.environ.get("SRT_FORM")
        cur = {}
        for item in (self.old or "").split(","):
            if "=" in item:
                k, v = item.split("=", 1)
                cur[k.strip()] = v
        cur.update(self.kv)
        os.environ["SRT_FORM"] = ",".join(f"{k}={v}" for k, v in cur.items())
        return self

    def __exit__(self, *exc):
        if self.old is None:
            os.environ.pop("SRT_FORM", None)
        else:
            os.environ["SRT_FORM"] = self.old
        return False
