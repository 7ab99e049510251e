"""Top-down diff timing at 100M value-only (diagnostic; MKV_TD_SORT experiment)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from merklekv_amd import MerkleTree
import bench
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
A = MerkleTree(0); A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
vv = vb[: n * 100].view(n, 100)
idx = torch.randperm(n, device="cuda")[: n // 1000]
vv[idx, 3] ^= 1
torch.cuda.synchronize()
B = MerkleTree(0); B.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
for rep in range(4):
    t0 = time.perf_counter(); d = A.diff_keys_packed(B); t1 = time.perf_counter()
    print(f"rep {rep}: {1e3*(t1-t0):.3f} ms, {len(d[1])-1} keys", flush=True)
