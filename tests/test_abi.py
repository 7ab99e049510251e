"""CPU tests of the C-ABI boundary: the gfx950 library is built, loads, and exports every symbol that
include/mkv_merkle.h declares; without a GPU it fails loudly (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT, gpu_present


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mkv_merkle.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mkv_[a-z0-9_]+)\s*\(", src)))


def test_library_built_for_gfx950():
    from merklekv_amd._lib import LIB_PATH
    assert os.path.exists(LIB_PATH), "run __graft_entry__.build()"
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob  # embedded code object targets MI355X


def test_exports_every_header_symbol():
    from merklekv_amd._lib import EXPORTS, LIB_PATH
    lib = ctypes.CDLL(LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in mkv_merkle.h but not exported"
    assert sorted(EXPORTS) == syms, "merklekv_amd._lib.EXPORTS out of sync with the header"


def test_version_string():
    from merklekv_amd import version
    assert "gfx950" in version()


@pytest.mark.skipif(gpu_present(), reason="a GPU is present")
def test_no_gpu_fails_loudly():
    from merklekv_amd import MerkleError, MerkleTree
    from merklekv_amd._lib import MKV_EHIP
    with pytest.raises(MerkleError) as ei:
        MerkleTree()
    assert ei.value.status == MKV_EHIP


def test_product_path_does_not_import_oracle():
    """The product package never references oracle/ (it is test infrastructure only)."""
    pkg = os.path.join(ROOT, "merklekv_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".hpp")):
                txt = open(os.path.join(dp, f), encoding="utf-8").read()
                assert "import oracle" not in txt and "from oracle" not in txt and "liboracle" not in txt, f
