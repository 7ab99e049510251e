"""Host/device timing of diff_keys_many_packed vs pairwise diffs on 125M-key replicas (diagnostic)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from merklekv_amd import MerkleTree
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 125_000
R = 7
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
base = MerkleTree(0)
base.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
del vb, vo
vs = []
for r in range(R):
    v = base.clone()
    g = torch.Generator(device="cuda"); g.manual_seed(r)
    sel = torch.randint(0, n, (m,), device="cuda", generator=g)
    ukb = kb[: n * 32].view(n, 32)[sel].contiguous().view(-1)
    uvb = bench.random_values(torch, m, ctx.dev, g).contiguous().view(-1)
    uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 32
    uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 100
    torch.cuda.synchronize()
    v.upsert_device(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m)
    vs.append(v)
base.prof_enable(True)
for rep in range(3):
    base.prof_reset()
    t0 = time.perf_counter()
    d = base.diff_keys_many_packed(vs)
    t1 = time.perf_counter()
    dm = base.prof_read("diff")
    base.prof_reset()
    t2 = time.perf_counter()
    p = [base.diff_keys_packed(v) for v in vs]
    t3 = time.perf_counter()
    dp = base.prof_read("diff")
    print(f"rep {rep}: many {1e3*(t1-t0):.2f} ms (dev {dm[0]:.2f}/{dm[1]})  pairwise {1e3*(t3-t2):.2f} ms (dev {dp[0]:.2f}/{dp[1]})", flush=True)
