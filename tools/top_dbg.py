"""Per-level timestamps of k_reduce_top (s_memrealtime, 100 MHz) from the instrumented variant library
(bash scripts/mkvariant.sh topdbg scripts/variants/topdbg.py): where the top launch's time goes. Run with MKV_LIB_PATH set to it."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd._lib import lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
t = MerkleTree(0)
f = lib().mkv_dbg_top
f.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
for rep in range(4):
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    torch.cuda.synchronize()
    a = (ctypes.c_uint64 * 64)()
    assert f(a) == 0
    nf, nl, nt = a[60], a[61], a[62]
    t0 = a[0]
    p1 = [round((a[k] - t0) / 100, 1) for k in range(1, nf + 1)]
    p2 = [round((a[20 + k] - t0) / 100, 1) for k in range(0, nl - nf + 1)]
    print(f"nf={nf} nl={nl} tiles={nt} last_wg={a[19]}  phase1 (us from start, WG 0): {p1}  phase2: {p2}", flush=True)
