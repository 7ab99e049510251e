import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def gpu_present() -> bool:
    """True if a HIP device is visible (without initialising torch)."""
    try:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


@pytest.fixture(scope="session")
def fixtures():
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_lib():
    """The C oracle (built by __graft_entry__.build() / make -C oracle)."""
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    from oracle import coracle
    return coracle


def pytest_collection_finish(session):
    """GPU sessions: bring up torch's HIP runtime before libmerklekv_hip.so's. torch ships its own
    libamdhip64; when the in-tree library (linked to /opt/rocm's) initialises the device first, torch's
    later init reports no device. Tests that stage device buffers with torch need it the other way round."""
    if any(item.get_closest_marker("gpu") for item in session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
