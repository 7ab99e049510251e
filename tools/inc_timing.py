"""Host-side timing breakdown of the incremental workload's step (diagnostic)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from merklekv_amd import MerkleTree
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 125_000
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
base = MerkleTree(0)
base.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
v = base.clone()
g = torch.Generator(device="cuda"); g.manual_seed(1)
sel = torch.randint(0, n, (m,), device="cuda", generator=g)
ukb = kb[: n * 32].view(n, 32)[sel].contiguous().view(-1)
uvb = bench.random_values(torch, m, ctx.dev, g).contiguous().view(-1)
uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 32
uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 100
torch.cuda.synchronize()
v.prof_enable(True); base.prof_enable(True)
for rep in range(4):
    t0 = time.perf_counter()
    v.upsert_device(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m)
    t1 = time.perf_counter()
    d = base.diff_keys_packed(v)
    t2 = time.perf_counter()
    print(f"rep {rep}: upsert {1e3*(t1-t0):.3f} ms  diff {1e3*(t2-t1):.3f} ms  ndiff {len(d[1])-1}", flush=True)
print("prof update", v.prof_read("update"), "diff", base.prof_read("diff"))
