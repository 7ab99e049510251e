"""Diagnostic: 10M records with 32-B keys and EMPTY values (every record an edge one, k_leaf_edges) — ms per
build from device blobs, for the library MKV_LIB_PATH points at."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402

n = 10_000_000
ctx = bench.Ctx()
kb, ko, _, _ = ctx.records(n)
vb = torch.zeros(16, dtype=torch.uint8, device="cuda")
vo = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
t = MerkleTree(0)
for _ in range(2):
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    r = t.get_root_hash()
print(f"empty-values 10M build: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms/step root {r.hex()[:16]}", flush=True)
