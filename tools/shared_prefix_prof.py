"""Kernel-trace target: 10M-key builds whose keys share 'tenant/0001/object/' (bench shared_prefix_10m)."""
import sys
import time

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import KLEN, SEED, VLEN  # noqa: E402
from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import gen_records_device  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
prefix = b"tenant/0001/object/"
kb = torch.empty(n * KLEN + 64, dtype=torch.uint8, device="cuda")
vb = torch.empty(n * VLEN + 64, dtype=torch.uint8, device="cuda")
ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
gen_records_device(0, SEED, 0, n, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr())
kb[: n * KLEN].view(n, KLEN)[:, : len(prefix)] = torch.frombuffer(bytearray(prefix), dtype=torch.uint8).cuda()
torch.cuda.synchronize()
t = MerkleTree()
for i in range(6):
    t0 = time.perf_counter()
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    r = t.get_root_hash()
    print(i, round((time.perf_counter() - t0) * 1e3, 3), "ms", r.hex()[:16], flush=True)
