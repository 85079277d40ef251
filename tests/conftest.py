"""Shared pytest setup.

-m "not gpu": oracle vs the reference's own golden data, host logic, C-ABI
              exports, multi-process (gloo) sharding -- runs without a GPU.
-m gpu:       parity of the HIP path against the oracle, through the C ABI.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rust-raytrace_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def _ensure_built():
    need = [(os.path.join(ROOT, "oracle", "libref64.so"), ["make", "-s", "-C", os.path.join(ROOT, "oracle")]),
            (os.path.join(PKG, "librtamd.so"), ["make", "-s", "-j8", "-C", PKG])]
    for path, cmd in need:
        if not os.path.exists(path):
            subprocess.run(cmd, check=True)


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds on CPU")


@pytest.fixture(scope="session")
def gpu_ctx():
    import libraytrace as lr
    if lr.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X (no CPU fallback exists)")
    ctx = lr.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(autouse=True)
def _native_fault_trace():
    """RT_SEGV_BT=1: print the native stack of a SIGSEGV / SIGBUS (tools/segv_bt.c;
    diagnostic).  Installed before every test, after pytest's faulthandler and after
    whatever the HIP runtime installs when it starts."""
    if os.environ.get("RT_SEGV_BT") == "1":
        import ctypes
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libsegv_bt.so"))
        assert lib.segv_bt_install() == 0
    yield
