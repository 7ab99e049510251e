"""Per-call wall-time distribution of diff_keys_view at 10M value-only (diagnostic for the bimodal
'diff.ms' of the build bench's secondary line)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from merklekv_amd import MerkleTree
import bench
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
vb2 = vb.clone()
v2 = vb2[: n * 100].view(n, 100)
idx = torch.arange(0, n, 1000, device="cuda")
v2[idx, 0] ^= 1
torch.cuda.synchronize()
A = MerkleTree(0); A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
B = MerkleTree(0); B.build_device(kb.data_ptr(), ko.data_ptr(), vb2.data_ptr(), vo.data_ptr(), n)
ts = []
for rep in range(60):
    t0 = time.perf_counter(); d = A.diff_keys_view(B); t1 = time.perf_counter()
    ts.append(1e3 * (t1 - t0))
print("ms per call:", " ".join(f"{t:.3f}" for t in ts), flush=True)
ts.sort()
print(f"min {ts[0]:.3f} median {ts[len(ts)//2]:.3f} max {ts[-1]:.3f} n_slow(>1ms) {sum(t > 1 for t in ts)}", flush=True)

# bench.py order: rebuild A after B, one warm call, then 5 timed calls; repeated
for it in range(8):
    B.build_device(kb.data_ptr(), ko.data_ptr(), vb2.data_ptr(), vo.data_ptr(), n)
    A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    d = A.diff_keys_view(B)
    torch.cuda.synchronize()
    ts = []
    for rep in range(5):
        t0 = time.perf_counter(); d = A.diff_keys_view(B); t1 = time.perf_counter()
        ts.append(1e3 * (t1 - t0))
    print(f"iter {it}:", " ".join(f"{t:.3f}" for t in ts), flush=True)
