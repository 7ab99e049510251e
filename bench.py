#!/usr/bin/env python3
"""Benchmark: Merkle build leaves/s (+ diff keys/s) on MI355X — BASELINE.json configs[1] (10M keys, 1 GPU).

A step = one full tree build (leaf hashing + key ordering + dedup + gathers + level reduction) over
n synthetic records (32-B keys, 100-B values, generated on the device, already resident in HBM when
the timed region starts). With N>1 ranks (torch.distributed.run, one process per GPU) each rank owns
a contiguous key range of n records (weak scaling); the step adds the RCCL all-gathers of shard leaf
counts and seam fringes and the on-device seam combine that yields the global root on every rank.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x4D65726B6C654B56
KLEN, VLEN = 32, 100
LEAF_BYTES = 8 + KLEN + VLEN + 32   # algorithmic bytes per leaf for Kernel A: 140-B record read + 32-B digest
HBM_PEAK_GBS = 8000.0                # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # int32 lane-ops/s: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
SHA_OPS_PER_LEAF = 3 * 1450          # model: 3 compressions x ~1450 VALU lane-ops


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10_000_000, help="records per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample time")
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(local)

    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import sharded_root

    n = args.n
    kb = torch.empty(n * KLEN + 64, dtype=torch.uint8, device=dev)
    vb = torch.empty(n * VLEN + 64, dtype=torch.uint8, device=dev)
    ko = torch.empty(n + 1, dtype=torch.int64, device=dev)
    vo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    gen_records_device(local, SEED, rank * n, n, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                       vo.data_ptr(), shard=rank, nshards=world)
    torch.cuda.synchronize()

    tree = MerkleTree(local)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def step():
        if world == 1:
            tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            return tree.get_root_hash()
        root, _ = sharded_root(tree, (kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), None,
                               dist, device=dev, on_device=True)
        return root

    for _ in range(args.warmup):
        root = step()
    tree.prof_enable(True)
    tree.prof_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        root = step()
    barrier()
    t1 = time.perf_counter()
    tree.prof_enable(False)
    elapsed = t1 - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        rt = torch.frombuffer(bytearray(root), dtype=torch.uint8).to(dev)
        allr = torch.empty(world * 32, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(allr, rt)
        roots = allr.cpu().numpy().reshape(world, 32)
        assert (roots == roots[0]).all(), "ranks disagree on the global root"

    ms_per_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed
    leaf_ms, leaf_cnt = tree.prof_read("leaf_hash")
    groups = {g: tree.prof_read(g) for g in ("leaf_hash", "sort", "keycopy", "gather", "reduce", "total_build")}
    leaf_avg_ms = leaf_ms / max(leaf_cnt, 1)
    achieved = LEAF_BYTES * n / (leaf_avg_ms * 1e-3) / 1e9
    hashed_gbs = (8 + KLEN + VLEN) * n / (leaf_avg_ms * 1e-3) / 1e9
    valu_frac = SHA_OPS_PER_LEAF * n / (leaf_avg_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_leaf_hash.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("n") == n:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---------------- diff (secondary: keys/s over the union, value-only 0.1% divergence) -------------
    diff_info = None
    if not args.no_diff and world == 1:
        # replica B: same keys, value byte 0 flipped in every 1000th record (0.1 % value-only divergence)
        vb2 = vb.clone()
        v2 = vb2[: n * VLEN].view(n, VLEN)
        idx = torch.arange(0, n, 1000, device=dev)
        v2[idx, 0] = v2[idx, 0] ^ 1
        torch.cuda.synchronize()
        treeB = MerkleTree(local)
        treeB.build_device(kb.data_ptr(), ko.data_ptr(), vb2.data_ptr(), vo.data_ptr(), n)
        tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        d = tree.diff_keys_bytes(treeB)  # warm
        reps = 5
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d = tree.diff_keys_bytes(treeB)
        dt = (time.perf_counter() - t0) / reps
        diff_info = {"union_keys": n, "divergent": len(d), "expected_divergent": int(idx.numel()),
                     "ms": dt * 1e3, "keys_per_s": n / dt, "mode": "merge-join, value-only 0.1%"}
        del treeB, vb2

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "Merkle build leaves/s (10M keys, full tree: hash+sort+reduce)",
            "value": value,
            "unit": "leaves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (on-device splitmix64 generator, seed 0x4D65726B6C654B56)",
            "config": {"workload": "configs[1]: 10M keys x 1 MI355X per rank, 32-B keys / 100-B values",
                       "keys_per_gpu": n, "key_bytes": KLEN, "value_bytes": VLEN,
                       "parallelism": f"key-range shards x{world}" if world > 1 else "single GPU"},
            "root": root.hex() if root else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_leaf_hash", "bytes_per_leaf": LEAF_BYTES,
                         "avg_launch_ms": leaf_avg_ms, "launches": leaf_cnt,
                         "gb_per_s_hashed": hashed_gbs,
                         "valu_frac_model": valu_frac,
                         "note": "SHA-256 is VALU-bound (~22.7 ops/B vs 9.8 balance): HBM frac ceiling ~0.39"},
            "stage_ms_per_step": {g: (v[0] / max(v[1], 1) if g == "leaf_hash" else v[0] / args.steps)
                                  for g, v in groups.items()},
            "diff": diff_info,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(target_s: float):
    """Oracle (C restatement of merkle.rs, single thread, SHA-NI like sha2 0.10.9) on a bounded sample."""
    import ctypes

    from oracle import coracle as co
    shani = co.set_backend(1)
    try:
        buf = (ctypes.c_uint8 * 32)()
        n0 = 100_000
        kb, ko, vb, vo = co.gen_records(SEED, 0, n0)
        secs = co.lib().orc_bench_build(kb.ctypes.data, ko.ctypes.data, vb.ctypes.data, vo.ctypes.data, n0, buf)
        n = int(min(8_000_000, max(n0, n0 / secs * target_s)))
        kb, ko, vb, vo = co.gen_records(SEED, 0, n)
        secs = co.lib().orc_bench_build(kb.ctypes.data, ko.ctypes.data, vb.ctypes.data, vo.ctypes.data, n, buf)
        return {"value": n / secs, "unit": "leaves/s", "cores": 1, "kind": "port",
                "sample": f"one bulk build (= one merkle.rs rebuild) of {n} synthetic 32B/100B records, "
                          f"{secs:.1f} s, sha={'SHA-NI' if shani else 'portable'}",
                "cpu_model": _cpu_model()}
    finally:
        co.set_backend(0)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
