"""Runs the C++ ports of merkle.rs's 56 tests (tests/cpp/test_merkle_ref.cpp, built by
__graft_entry__.build()) against the HIP library through include/mkv_merkle.hpp."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tests", "cpp", "test_merkle_ref")


def test_cpp_reference_ports():
    if not os.path.exists(BIN):
        import __graft_entry__
        __graft_entry__.build_cpp_tests()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "56 tests, 0 failed" in r.stdout


def test_cpp_boundary_const_call_sites():
    """sync.rs:61-67 / server.rs:661-675 shapes: get_root_hash / diff_keys on const MerkleTree&."""
    b = os.path.join(ROOT, "tests", "cpp", "test_boundary")
    if not os.path.exists(b):
        import __graft_entry__
        __graft_entry__.build_cpp_tests()
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    print(r.stdout[-4000:])
    assert r.returncode == 0 and "boundary: ok" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]


def test_cpp_sharded_comm():
    """mkv_comm_* / mkv_sharded_* from C++: RCCL at world 1 and the host form at world 3 (threads) vs an
    OpenSSL restatement of rebuild() / diff_keys() (tests/cpp/test_sharded.cpp)."""
    b = os.path.join(ROOT, "tests", "cpp", "test_sharded")
    if not os.path.exists(b):
        import __graft_entry__
        __graft_entry__.build_cpp_tests()
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    print(r.stdout[-4000:])
    assert r.returncode == 0 and "sharded: ok" in r.stdout, r.stdout[-4000:] + r.stderr[-2000:]
