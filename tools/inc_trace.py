"""Host-side timeline of configs[4] steps (bench.py --workload incremental): when each call returns and
the host phase trace (mkv_debug_trace) of the batched update and the batched diff, to see which host wait
holds the next step's update behind the previous step's key-list copies."""
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
variants = [base.clone() for _ in range(R - 1)]
batches = []
for r in range(R - 1):
    g = torch.Generator(device="cuda")
    g.manual_seed(1000 * r)
    sel = torch.randint(0, n, (m,), device="cuda", generator=g)
    ukb = kb[: n * bench.KLEN].view(n, bench.KLEN)[sel].contiguous().view(-1)
    uvb = bench.random_values(torch, m, "cuda", g).contiguous().view(-1)
    batches.append((ukb, torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * bench.KLEN,
                    uvb, torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * bench.VLEN))
torch.cuda.synchronize()
ptrs = [(a.data_ptr(), b.data_ptr(), c.data_ptr(), d.data_ptr(), m) for a, b, c, d in batches]
diffs = None
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
upd, dif, slow = [], [], []
for step in range(steps):
    t0 = time.perf_counter()
    MerkleTree.upsert_device_many(variants, ptrs)
    t1 = time.perf_counter()
    tu = debug_trace()
    new = base.diff_keys_many_view(variants)
    t2 = time.perf_counter()
    td = debug_trace()
    diffs = new
    t3 = time.perf_counter()
    upd.append(t1 - t0)
    dif.append(t2 - t1)
    if t1 - t0 > 2.5e-3:
        slow.append(f"step {step}: {1e3 * (t1 - t0):.2f} ms {tu}")
    if step >= 10:
        continue
    print(f"step {step}: update {1e3 * (t1 - t0):.3f} ms | diff {1e3 * (t2 - t1):.3f} ms | drop {1e3 * (t3 - t2):.3f} ms"
          f"\n   upd: {tu}\n   diff: {td}", flush=True)
upd, dif = sorted(upd[2:]), sorted(dif[2:])
print(f"{len(upd)} steps: update median {1e3 * upd[len(upd) // 2]:.3f} max {1e3 * upd[-1]:.3f} ms | "
      f"diff median {1e3 * dif[len(dif) // 2]:.3f} max {1e3 * dif[-1]:.3f} ms")
print("  slowest updates (ms):", [round(1e3 * x, 2) for x in upd[-6:]], " > 2.5 ms:", sum(x > 2.5e-3 for x in upd))
print("  slowest diffs (ms):", [round(1e3 * x, 2) for x in dif[-6:]])
print("  slow update traces:", *slow[:4], sep="\n    ")
