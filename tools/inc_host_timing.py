"""Host-side phase timing of the configs[4] incremental step (bench.py wl_incremental at n keys):
wall ms of upsert_device_many, of diff_keys_many_view and of releasing the previous step's key lists,
next to the device ms the library's profiling events report."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import debug_trace  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
m, R = 125_000, 8
ctx = bench.Ctx()
kb, ko, vb, vo = ctx.records(n)
base = MerkleTree(0)
base.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
del vb, vo
torch.cuda.empty_cache()
variants = [base.clone() for _ in range(R - 1)]
keep, ptrs = [], []
for r in range(R - 1):
    g = torch.Generator(device="cuda")
    g.manual_seed(1000 * r)
    sel = torch.randint(0, n, (m,), device="cuda", generator=g)
    ukb = kb[: n * 32].view(n, 32)[sel].contiguous().view(-1)
    uvb = bench.random_values(torch, m, "cuda", g).contiguous().view(-1)
    uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 32
    uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * 100
    keep.append((ukb, uko, uvb, uvo))
    ptrs.append((ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m))
torch.cuda.synchronize()
diffs = None
for t in [base] + variants:
    t.prof_enable(True)
for it in range(8):
    for t in [base] + variants:
        t.prof_reset()
    t0 = time.perf_counter()
    MerkleTree.upsert_device_many(variants, ptrs)
    t1 = time.perf_counter()
    tr_u = debug_trace()
    t1b = time.perf_counter()
    new = base.diff_keys_many_view(variants)
    t2 = time.perf_counter()
    tr_d = debug_trace()
    diffs = new  # releases the previous step's views
    t3 = time.perf_counter()
    upd = variants[0].prof_read("update")[0]
    dif = base.prof_read("diff")[0]
    print(f"step {it}: upsert {1e3 * (t1 - t0):.3f} ms (device {upd:.3f})  diff_many {1e3 * (t2 - t1b):.3f} ms "
          f"(device {dif:.3f})  release {1e3 * (t3 - t2):.3f} ms  total {1e3 * (t3 - t0):.3f}\n"
          f"   upsert trace: {tr_u}\n   diff trace: {tr_d}", flush=True)
