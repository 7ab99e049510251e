"""A/B driver for the 100M value-only top-down diff (diagnostic): median wall time per diff_keys_view call
and the mean device time of the call's queued work (the library's "diff" HIP-event pair), for the library
MKV_LIB_PATH points at (default: the in-tree one)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
A = MerkleTree(0)
A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
v = vb[: n * 100].view(n, 100)
v[torch.arange(0, n, 1000, device="cuda"), 0] ^= 1
torch.cuda.synchronize()
B = MerkleTree(0)
B.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
d = None
for _ in range(8):
    d = A.diff_keys_view(B)
ts = []
for _ in range(200):
    t0 = time.perf_counter()
    d = A.diff_keys_view(B)
    ts.append(time.perf_counter() - t0)
A.prof_enable(True)
A.prof_reset()
for _ in range(200):
    d = A.diff_keys_view(B)
A.prof_enable(False)
dms, dc = A.prof_read("diff")
ts.sort()
print(f"{tag} vo-diff {n // 1_000_000}M: wall median {1e3 * ts[100]:.4f} p10 {1e3 * ts[20]:.4f} ms  device {dms / max(dc, 1):.4f} ms"
      f"  keys {len(d)}", flush=True)
