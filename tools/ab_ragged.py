"""A/B driver for the leaf stage (diagnostic): 10M store-like ragged records (keys 8-64 B, values 16-256 B)
and 10M fixed 32/100-B records, built from device blobs. Prints ms/step and the stage split (HIP events)
for the library MKV_LIB_PATH points at (default: the in-tree one)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import gen_records_device, gen_records_ragged_device  # noqa: E402

SEED = 0x4D65726B6C654B56
N = 10_000_000


def blobs(ragged):
    kl, vl = (64, 256) if ragged else (32, 100)
    kb = torch.empty(N * kl + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(N * vl + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(N + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(N + 1, dtype=torch.int64, device="cuda")
    gen = gen_records_ragged_device if ragged else gen_records_device
    gen(0, SEED, 0, N, kl, vl, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr())
    torch.cuda.synchronize()
    return kb, ko, vb, vo


def run(tag, ragged, steps):
    kb, ko, vb, vo = blobs(ragged)
    comp = None
    if ragged:
        L = 8 + (ko[1:] - ko[:-1]) + (vo[1:] - vo[:-1])
        comp = int(((L + 9 + 63) // 64).sum().item())
    t = MerkleTree()
    f = lambda: t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), N)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        f()
        t.get_root_hash()
    ms = (time.perf_counter() - t0) / steps * 1e3
    t.prof_enable(True)
    t.prof_reset()
    for _ in range(steps):
        f()
    g = {k: t.prof_read(k) for k in ("leaf_hash", "sort", "reduce", "total_build")}
    t.prof_enable(False)
    leaf = g["leaf_hash"][0] / max(g["leaf_hash"][1], 1)
    line = f"{tag} {'ragged' if ragged else 'fixed '} {ms:.3f} ms/step  leaf {leaf:.3f}  sort {g['sort'][0] / steps:.3f}" \
           f"  reduce {g['reduce'][0] / steps:.3f}"
    if comp:
        line += f"  {comp / (leaf * 1e-3) / 1e9:.2f} G compressions/s"
    print(line, flush=True)
    del t, kb, vb, ko, vo
    torch.cuda.empty_cache()


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
    steps = int(os.environ.get("STEPS", "20"))
    modes = os.environ.get("MODES", "ragged,fixed").split(",")
    for m in modes:
        run(tag, m == "ragged", steps)
