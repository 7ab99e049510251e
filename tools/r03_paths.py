"""Focused driver for kernel traces of the round-3 paths (rocprofv3 --kernel-trace): MODE=build (10M fixed
build), ragged (10M store-like ragged build), mixed (100M mixed-divergence merge-join diff). Prints one
timing line per mode."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import gen_records_device, gen_records_ragged_device  # noqa: E402

SEED = 0x4D65726B6C654B56
K, V = 32, 100


def recs(n, idx0=0):
    kb = torch.empty(n * K + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(n * V + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    gen_records_device(0, SEED, idx0, n, K, V, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr())
    torch.cuda.synchronize()
    return kb, ko, vb, vo


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    modes = sys.argv[1:] or ["build", "ragged", "mixed"]
    steps = int(os.environ.get("STEPS", "5"))
    for mode in modes:
        if mode == "build":
            n = 10_000_000
            kb, ko, vb, vo = recs(n)
            t = MerkleTree()
            ms = timed(lambda: t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), steps)
            print(f"build 10M: {ms:.3f} ms/step", flush=True)
        elif mode == "ragged":
            n = 10_000_000
            kb = torch.empty(n * 64 + 64, dtype=torch.uint8, device="cuda")
            vb = torch.empty(n * 256 + 64, dtype=torch.uint8, device="cuda")
            ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
            vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
            gen_records_ragged_device(0, SEED, 0, n, 64, 256, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr())
            torch.cuda.synchronize()
            t = MerkleTree()
            ms = timed(lambda: t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), steps)
            print(f"ragged build 10M: {ms:.3f} ms/step", flush=True)
        elif mode in ("vo", "ident"):
            # merge-join over equal key sets (run with MKV_DIFF_TOPDOWN=0): "vo" = 0.1 % changed values
            # (aligned tiles + digest mismatches), "ident" = identical replicas (pure streaming)
            n = 100_000_000
            kb, ko, vb, vo = recs(n)
            A = MerkleTree()
            A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            if mode == "vo":
                g = torch.Generator(device="cuda")
                g.manual_seed(12)
                idx = torch.randperm(n, device="cuda", generator=g)[: n // 1000]
                vv = vb[: n * V].view(n, V)
                vv[idx, 0] ^= 1
            torch.cuda.synchronize()
            B = MerkleTree()
            B.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            del kb, vb
            torch.cuda.empty_cache()
            ms = timed(lambda: A.diff_keys_view(B), steps)
            print(f"{mode} merge diff 100M: {ms:.3f} ms/step ({len(A.diff_keys_view(B))} keys)", flush=True)
        elif mode == "mixed":
            n = 100_000_000
            kb, ko, vb, vo = recs(n)
            A = MerkleTree()
            A.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            nd = n // 1000
            g = torch.Generator(device="cuda")
            g.manual_seed(11)
            perm = torch.randperm(n, device="cuda", generator=g)
            kv, vv = kb[: n * K].view(n, K), vb[: n * V].view(n, V)
            c, r = nd * 8 // 10, nd // 10
            new = nd - c - r
            v2 = vv.clone()
            v2[perm[:c], 0] ^= 1
            keep = torch.ones(n, dtype=torch.bool, device="cuda")
            keep[perm[c:c + r]] = False
            nk, _, nv, _ = recs(new, idx0=10**12)
            kB = torch.cat([kv[keep], nk[: new * K].view(new, K)]).contiguous().view(-1)
            vB = torch.cat([v2[keep], nv[: new * V].view(new, V)]).contiguous().view(-1)
            del v2, keep
            nB = n - r + new
            koB = torch.arange(0, nB + 1, device="cuda", dtype=torch.int64) * K
            voB = torch.arange(0, nB + 1, device="cuda", dtype=torch.int64) * V
            torch.cuda.synchronize()
            B = MerkleTree()
            B.build_device(kB.data_ptr(), koB.data_ptr(), vB.data_ptr(), voB.data_ptr(), nB)
            del kB, vB
            torch.cuda.empty_cache()
            ms = timed(lambda: A.diff_keys_view(B), steps)
            print(f"mixed diff 100M: {ms:.3f} ms/step ({len(A.diff_keys_view(B))} keys)", flush=True)


if __name__ == "__main__":
    main()
