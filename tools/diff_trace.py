"""Host phase trace (mkv_debug_trace) of value-only top-down diffs at n keys (default 100M): where the
wall time of diff_keys_view goes between the device phases."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import debug_trace, pool_stats  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
A = MerkleTree(0)
A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
v = vb[: n * 100].view(n, 100)
idx = torch.arange(0, n, 1000, device="cuda")
v[idx, 0] ^= 1
torch.cuda.synchronize()
B = MerkleTree(0)
B.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
keep = len(sys.argv) > 2 and sys.argv[2] == "keep"  # the bench's loop: the previous result stays alive
d = None
for rep in range(12):
    if not keep:
        d = None
    t0 = time.perf_counter()
    d2 = A.diff_keys_view(B)
    t1 = time.perf_counter()
    d = d2
    t2 = time.perf_counter()
    print(f"{1e3 * (t1 - t0):.3f} ms (+{1e3 * (t2 - t1):.3f} ms drop)  keys={len(d)}  {debug_trace()}  "
          f"pool={pool_stats()}", flush=True)
    del d2
ts = []
for rep in range(50):  # tight loop, as bench.py times it
    t0 = time.perf_counter()
    d = A.diff_keys_view(B)
    ts.append(time.perf_counter() - t0)
print("tight loop per call (ms):", [round(1e3 * x, 3) for x in ts[:12]], "median", round(1e3 * sorted(ts)[25], 3))
