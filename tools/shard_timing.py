"""Per-phase host timing of the sharded build protocol with 4 in-process shards (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from merklekv_amd import MerkleTree
import bench

W, n = 4, 2_500_000
ctx = bench.Ctx()
recs, trees = [], []
for g in range(W):
    kb = torch.empty(n * 32 + 64, dtype=torch.uint8, device="cuda"); vb = torch.empty(n * 100 + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(n + 1, dtype=torch.int64, device="cuda"); vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    from merklekv_amd.merkle import gen_records_device
    gen_records_device(0, bench.SEED, g * n, n, 32, 100, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), shard=g, nshards=W)
    recs.append((kb, ko, vb, vo)); trees.append(MerkleTree(0))
torch.cuda.synchronize()
for rep in range(4):
    t = {}
    t0 = time.perf_counter()
    counts = [tr.shard_prepare((kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), None, on_device=True) for tr, (kb, ko, vb, vo) in zip(trees, recs)]
    t1 = time.perf_counter()
    N = sum(counts)
    for r, tr in enumerate(trees): tr.shard_reduce(sum(counts[:r]), N)
    t2 = time.perf_counter()
    fr = b"".join(tr.shard_fringe() for tr in trees)
    t3 = time.perf_counter()
    roots = [tr.shard_combine(fr, W, N) for tr in trees]
    t4 = time.perf_counter()
    assert len(set(roots)) == 1
    print(f"rep {rep}: prepare {1e3*(t1-t0)/W:.3f} reduce {1e3*(t2-t1)/W:.3f} fringe {1e3*(t3-t2)/W:.3f} combine {1e3*(t4-t3)/W:.3f} ms per shard", flush=True)
