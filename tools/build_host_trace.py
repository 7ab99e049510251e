"""Host phase trace of the 10M build loop (diagnostic): per call, the library's host marks (mkv_debug_trace)
and the Python-level time of build_device + get_root_hash."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import debug_trace  # noqa: E402

n = 10_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
t = MerkleTree(0)
for _ in range(5):
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    t.get_root_hash()
torch.cuda.synchronize()
rows = []
for i in range(30):
    a = time.perf_counter()
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    b = time.perf_counter()
    tr = debug_trace()
    c = time.perf_counter()
    t.get_root_hash()
    d = time.perf_counter()
    rows.append((1e3 * (b - a), 1e3 * (d - c), 1e3 * (d - a), tr))
for r in rows[-8:]:
    print(f"build {r[0]:.4f} ms  root {r[1] * 1e3:.1f} us  step {r[2]:.4f} ms  {r[3]}")
ts = []
for i in range(50):
    a = time.perf_counter()
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    t.get_root_hash()
    ts.append(time.perf_counter() - a)
ts.sort()
print("tight loop median", round(1e3 * ts[25], 4), "ms; min", round(1e3 * ts[0], 4))
