"""Host phase trace (mkv_debug_trace) of value-only top-down diffs at n keys (default 100M): where the
wall time of diff_keys_view goes between the device phases."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import debug_trace  # noqa: E402

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
for rep in range(12):
    t0 = time.perf_counter()
    d = A.diff_keys_view(B)
    t1 = time.perf_counter()
    print(f"{1e3 * (t1 - t0):.3f} ms  keys={len(d)}  {debug_trace()}", flush=True)
    del d
