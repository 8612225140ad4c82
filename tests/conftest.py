import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "robust-object-detection_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _segv_bt():
    """MX_SEGV_BT=1: native backtrace on a host crash (tools/native/segv_bt.c), installed after the HIP
    runtime is up (run pytest with -p no:faulthandler)."""
    if os.environ.get("MX_SEGV_BT") == "1":
        import ctypes
        ctypes.CDLL(os.path.join(ROOT, "tools", "native", "libsegvbt.so")).mx_segv_bt_install()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.zeros(1, device="cuda:0")
    _segv_bt()
    return torch.device("cuda:0")
