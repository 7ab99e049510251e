#!/usr/bin/env python3
"""Benchmark: Merkle build leaves/s (+ diff keys/s) on MI355X — BASELINE.json configs[1] (10M keys, 1 GPU).

Default workload (`--workload build`, what the driver runs): a step = one full tree build (leaf hashing
+ key ordering + dedup + gathers + level reduction + root readback) over n synthetic records (32-B
keys, 100-B values, generated on the device, already resident in HBM when the timed region starts).
With N>1 ranks (torch.distributed.run, one process per GPU) each rank owns a contiguous key range of n
records (weak scaling); the step adds the RCCL all-gathers of shard leaf counts and seam fringes and
the on-device seam combine that yields the global root on every rank. `--records 125000000` at N=8 is
configs[3] (1B keys over 8 GPUs); at N=1 it is one shard of it.

Other BASELINE configs (run explicitly; their JSON lines are committed under profiles/):
  --workload diff         configs[2]: two 100M-key replicas, (a) 0.1 % value-only divergence (top-down
                          walk) and (b) 0.1 % mixed 80/10/10 change/delete/insert (merge-join); a step =
                          one diff_keys incl. compaction and the D2H of the divergent key list.
  --workload incremental  configs[4]: a 1B-key tree (125M keys per GPU at N=8; --records per GPU), 8 replicas
                          = base + 7 variants; a step = each variant applies its own 1M-key value-update
                          batch (125K per GPU; dirty-path rehash + fringe/seam recombine) and the base is
                          diffed against all 7 (top-down).

Prints ONE JSON line on rank 0 (see DESIGN.md §5 for every field).
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
DIFF_BYTES_PER_KEY = 2 * (8 + 32)    # top-down/merge: prefix + digest per side, per union key
ALPHA = b"-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"  # sorted URL-safe base64


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Ctx:
    """Process-group + device plumbing shared by the workloads."""

    def __init__(self):
        import torch
        self.torch = torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        # Rehearsal knobs for a one-GPU box (never set by the driver): MKV_BENCH_SAME_GPU=1 puts every
        # rank on device 0, MKV_DIST_BACKEND=gloo runs the collectives on the host.
        if os.environ.get("MKV_BENCH_SAME_GPU") == "1":
            self.local = 0
        backend = os.environ.get("MKV_DIST_BACKEND", "nccl")  # "nccl" is RCCL over xGMI on ROCm
        self.dev = torch.device("cuda", self.local)
        self.coll = self.dev if backend == "nccl" else torch.device("cpu")
        if self.world > 1:
            import torch.distributed as dist_mod
            self.dist = dist_mod
            torch.cuda.set_device(self.local)
            if backend == "nccl":
                dist_mod.init_process_group("nccl", device_id=self.dev)
            else:
                dist_mod.init_process_group(backend)
        torch.cuda.set_device(self.local)

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max_over_ranks(self, x: float) -> float:
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.coll)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: int) -> int:
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.int64, device=self.coll)
        self.dist.all_reduce(t)
        return int(t.item())

    def records(self, n, idx0=None, vfield=1):
        """n records of this rank's key range, generated on the device (same generator as the oracle)."""
        torch = self.torch
        from merklekv_amd.merkle import gen_records_device
        kb = torch.empty(n * KLEN + 64, dtype=torch.uint8, device=self.dev)
        vb = torch.empty(n * VLEN + 64, dtype=torch.uint8, device=self.dev)
        ko = torch.empty(n + 1, dtype=torch.int64, device=self.dev)
        vo = torch.empty(n + 1, dtype=torch.int64, device=self.dev)
        gen_records_device(self.local, SEED, self.rank * n if idx0 is None else idx0, n, KLEN, VLEN,
                           kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), shard=self.rank,
                           nshards=self.world, vfield=vfield)
        torch.cuda.synchronize()
        return kb, ko, vb, vo

    def build(self, tree, kb, ko, vb, vo, n):
        """Full build of this rank's records; returns the global root (all ranks agree)."""
        if self.world == 1:
            tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            return tree.get_root_hash(), n
        from merklekv_amd.shard import sharded_root
        root, counts = sharded_root(tree, (kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), None,
                                    self.dist, device=self.coll, on_device=True)
        return root, sum(counts)

    def check_roots_agree(self, root: bytes):
        if self.dist is None or root is None:
            return
        torch = self.torch
        rt = torch.frombuffer(bytearray(root), dtype=torch.uint8).to(self.coll)
        allr = torch.empty(self.world * 32, dtype=torch.uint8, device=self.coll)
        self.dist.all_gather_into_tensor(allr, rt)
        roots = allr.cpu().numpy().reshape(self.world, 32)
        assert (roots == roots[0]).all(), "ranks disagree on the global root"

    def finish(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def base_line(ctx, args, metric, value, unit, ms_per_step, workload, dtype="u32", higher=True, scaling="weak"):
    return {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": ctx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": higher,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (on-device splitmix64 generator, seed 0x4D65726B6C654B56)",
        "config": {"workload": workload, "keys_per_gpu": args.n, "key_bytes": KLEN, "value_bytes": VLEN,
                   "parallelism": f"key-range shards x{ctx.world}" if ctx.world > 1 else "single GPU"},
    }


def random_values(torch, m, dev, gen):
    """m x VLEN value bytes from the base64 alphabet (device)."""
    alpha = torch.frombuffer(bytearray(ALPHA), dtype=torch.uint8).to(dev)
    return alpha[torch.randint(0, 64, (m, VLEN), device=dev, generator=gen)]


# ============================================================================================ build
def wl_build(ctx, args):
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    n = args.n
    kb, ko, vb, vo = ctx.records(n)
    tree = MerkleTree(ctx.local)

    for _ in range(args.warmup):
        root, N = ctx.build(tree, kb, ko, vb, vo, n)
    tree.prof_enable(True)
    tree.prof_reset()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        root, N = ctx.build(tree, kb, ko, vb, vo, n)
    ctx.barrier()
    t1 = time.perf_counter()
    tree.prof_enable(False)
    elapsed = ctx.max_over_ranks(t1 - t0)
    ctx.check_roots_agree(root)

    ms_per_step = elapsed / args.steps * 1e3
    value = ctx.world * n * args.steps / elapsed
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

    # ---------------- secondary, 1 GPU only: diff and incremental update on the same tree -------------
    diff_info = upd_info = None
    if not args.no_diff and ctx.world == 1:
        # replica B: same keys, value byte 0 flipped in every 1000th record (0.1 % value-only divergence)
        vb2 = vb.clone()
        v2 = vb2[: n * VLEN].view(n, VLEN)
        idx = torch.arange(0, n, 1000, device=ctx.dev)
        v2[idx, 0] = v2[idx, 0] ^ 1
        torch.cuda.synchronize()
        treeB = MerkleTree(ctx.local)
        treeB.build_device(kb.data_ptr(), ko.data_ptr(), vb2.data_ptr(), vo.data_ptr(), n)
        tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        d = tree.diff_keys_view(treeB)  # warm
        reps = 5
        torch.cuda.synchronize()
        rep_ms = []
        for _ in range(reps):
            t0 = time.perf_counter()
            d = tree.diff_keys_view(treeB)
            rep_ms.append((time.perf_counter() - t0) * 1e3)
        dt = sum(rep_ms) / reps / 1e3
        diff_info = {"union_keys": n, "divergent": len(d), "expected_divergent": int(idx.numel()),
                     "ms": dt * 1e3, "ms_per_rep": [round(x, 4) for x in rep_ms], "ms_median": sorted(rep_ms)[reps // 2], "keys_per_s": n / dt,
                     "mode": "top-down (equal key sets), value-only 0.1%, incl. key-list D2H"}
        # incremental: 0.1 % value-update batch of existing keys (dirty path), configs[4]'s ratio
        m = max(1, n // 1000)
        g = torch.Generator(device=ctx.dev)
        g.manual_seed(7)
        sel = torch.randint(0, n, (m,), device=ctx.dev, generator=g)
        ukb = kb[: n * KLEN].view(n, KLEN)[sel].contiguous().view(-1)
        uvb = random_values(torch, m, ctx.dev, g).contiguous().view(-1)
        uko = torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * KLEN
        uvo = torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * VLEN
        torch.cuda.synchronize()
        tree.upsert_device(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m)  # warm
        tree.prof_enable(True)
        tree.prof_reset()
        t0 = time.perf_counter()
        for _ in range(reps):
            tree.upsert_device(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m)
        dt = (time.perf_counter() - t0) / reps
        tree.prof_enable(False)
        ums, ucnt = tree.prof_read("update")
        upd_info = {"tree_keys": n, "batch": m, "ms": dt * 1e3, "device_ms": ums / max(ucnt, 1),
                    "update_keys_per_s": m / dt, "mode": "dirty-path rehash (value-only batch)"}
        # key-set change: 0.1 % mixed batch (80 % value updates, 10 % removes, 10 % new keys) through the
        # host API (mkv_tree_apply: batch sort + merge into the sorted leaves + reduction)
        import numpy as np
        sel_h = sel.cpu().numpy()
        kv_h = kb[: n * KLEN].view(n, KLEN)[sel].cpu().numpy()
        nnew = m // 10
        nk, _, _, _ = ctx.records(nnew, idx0=10**12)
        keys_h = np.concatenate([kv_h[: m - nnew], nk[: nnew * KLEN].view(nnew, KLEN).cpu().numpy()])
        rm_h = np.zeros(m, np.uint8)
        rm_h[int(m * 0.8): m - nnew] = 1
        vals_h = np.frombuffer(bytes(ALPHA * 2)[:VLEN] * m, np.uint8).reshape(m, VLEN)
        koff_h = np.arange(0, m + 1, dtype=np.uint64) * KLEN
        voff_h = np.arange(0, m + 1, dtype=np.uint64) * VLEN
        del sel_h
        ks_times = []
        for _ in range(3):
            tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tree.apply((keys_h.reshape(-1), koff_h), (vals_h.reshape(-1), voff_h), rm_h)
            ks_times.append(time.perf_counter() - t0)
        dt = min(ks_times)
        upd_info["keyset_batch"] = {"batch": m, "new": nnew, "removed": int(rm_h.sum()), "ms": dt * 1e3,
                                    "keys_per_s": m / dt, "leaves_after": len(tree),
                                    "mode": "batch sort + merge into sorted leaves + reduction (host blobs)"}
        del treeB, vb2

    cpu = None
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_build(args.cpu_seconds)

    if ctx.rank == 0:
        wl = ("configs[1]: 10M keys x 1 MI355X per rank, 32-B keys / 100-B values" if n == 10_000_000
              else f"{n} keys per rank (configs[3] = 125M x 8 ranks), 32-B keys / 100-B values")
        out = base_line(ctx, args, "Merkle build leaves/s (10M keys, full tree: hash+sort+reduce)", value,
                        "leaves/s", ms_per_step, wl)
        out["root"] = root.hex() if root else None
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                           "kernel": "k_leaf_hash", "bytes_per_leaf": LEAF_BYTES,
                           "avg_launch_ms": leaf_avg_ms, "launches": leaf_cnt,
                           "gb_per_s_hashed": hashed_gbs,
                           "valu_frac_model": valu_frac,
                           "note": "SHA-256 is VALU-bound (~22.7 ops/B vs 9.8 balance): HBM frac ceiling ~0.39; "
                                   "avg_launch_ms is measured while the sort co-runs on the aux stream"}
        out["stage_ms_per_step"] = {g: (v[0] / max(v[1], 1) if g == "leaf_hash" else v[0] / args.steps)
                                    for g, v in groups.items()}
        out["diff"] = diff_info
        out["incremental"] = upd_info
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)


# ============================================================================================= diff
def wl_diff(ctx, args):
    """configs[2]: two replicas with 0.1 % divergence; diff keys/s over the union of keys."""
    torch = ctx.torch
    import numpy as np
    from merklekv_amd import MerkleTree
    n = args.n
    kb, ko, vb, vo = ctx.records(n)
    A = MerkleTree(ctx.local)
    ctx.build(A, kb, ko, vb, vo, n)
    ndiv = max(1, n // 1000)
    g = torch.Generator(device=ctx.dev)
    g.manual_seed(11 + ctx.rank)
    perm = torch.randperm(n, device=ctx.dev, generator=g)
    res = {}
    for mode in ("value_only", "mixed"):
        kv, vv = kb[: n * KLEN].view(n, KLEN), vb[: n * VLEN].view(n, VLEN)
        vb2 = vv.clone()
        if mode == "value_only":
            chg, rm, new = perm[:ndiv], perm[:0], 0
        else:  # 80 % value changes, 10 % deletions, 10 % new keys (SURVEY §8d configs[2b])
            c, r = ndiv * 8 // 10, ndiv // 10
            chg, rm, new = perm[:c], perm[c:c + r], ndiv - c - r
        vb2[chg, 0] ^= 1
        keep = torch.ones(n, dtype=torch.bool, device=ctx.dev)
        keep[rm] = False
        kB, vB = kv[keep], vb2[keep]
        if new:
            nk, _, nv, _ = ctx.records(new, idx0=10**12 + ctx.rank * new)
            kB = torch.cat([kB, nk[: new * KLEN].view(new, KLEN)])
            vB = torch.cat([vB, nv[: new * VLEN].view(new, VLEN)])
        nB = kB.shape[0]
        kBf, vBf = kB.contiguous().view(-1), vB.contiguous().view(-1)
        koB = torch.arange(0, nB + 1, device=ctx.dev, dtype=torch.int64) * KLEN
        voB = torch.arange(0, nB + 1, device=ctx.dev, dtype=torch.int64) * VLEN
        # expected divergent keys: changed + removed + new (keys are unique)
        exp = torch.cat([kv[chg], kv[rm]] + ([kB[-new:]] if new else []))
        exp_np = exp.cpu().numpy()
        exp_sorted = exp_np[np.lexsort(exp_np.T[::-1])]
        del vb2, kB, vB, exp
        B = MerkleTree(ctx.local)
        ctx.build(B, kBf, koB, vBf, voB, nB)
        torch.cuda.synchronize()
        for _ in range(args.warmup):
            d = A.diff_keys_view(B)
        A.prof_enable(True)
        A.prof_reset()
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            d = A.diff_keys_view(B)
        ctx.barrier()
        el = ctx.max_over_ranks(time.perf_counter() - t0)
        A.prof_enable(False)
        dms, dcnt = A.prof_read("diff")
        got = d.raw.reshape(-1, KLEN)
        exact = got.shape == exp_sorted.shape and bool((got == exp_sorted).all())
        union = ctx.sum_over_ranks(n + new)
        res[mode] = {"union_keys": union, "divergent": ctx.sum_over_ranks(len(d)),
                     "expected_divergent": ctx.sum_over_ranks(int(exp_sorted.shape[0])),
                     "exact_vs_construction": exact, "ms": el / args.steps * 1e3,
                     "device_ms": dms / max(args.steps, 1),
                     "keys_per_s": union * args.steps / el,
                     "path": "top-down" if mode == "value_only" else "merge-join"}
        del B, kBf, vBf
        torch.cuda.empty_cache()
    cpu = None
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_diff()
    if ctx.rank == 0:
        v = res["value_only"]
        wl = (f"configs[2]: {n // 1_000_000}M keys x 2 replicas per rank, 0.1% divergence; value = value-only "
              f"(top-down) union keys/s; 'mixed' = 80/10/10 change/delete/insert (merge-join)")
        out = base_line(ctx, args, "Merkle diff keys/s (union keys compared, 2 replicas, 0.1% divergence)",
                        v["keys_per_s"], "keys/s", v["ms"], wl)
        achieved = DIFF_BYTES_PER_KEY * res["mixed"]["union_keys"] / (res["mixed"]["device_ms"] * 1e-3) / 1e9
        # HBM bytes per merge-join diff from the PMC passes (scripts/prof_summary.py), same per-rank size only
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_diff_merge.json")
        if os.path.exists(pmc_path):
            try:
                pm = json.load(open(pmc_path))
                if pm.get("union_keys") == res["mixed"]["union_keys"] // ctx.world:
                    traffic = pm.get("hbm_bytes_per_diff")
            except Exception:
                traffic = None
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "merge-join diff (mixed)",
                           "bytes_per_union_key": DIFF_BYTES_PER_KEY,
                           "note": "achieved = 80 B x union keys / device time of the whole diff call (partition, "
                                   "both passes, key gather); traffic = PMC HBM bytes of its merge-join kernels"}
        out["diff"] = res
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    del A


# ====================================================================================== incremental
def wl_incremental(ctx, args):
    """configs[4]: 8 replicas (base + 7 variants) of a 1B-key tree (per-GPU shard of n keys); a step =
    each variant applies its own value-update batch (dirty path + seam recombine) + base diffed vs all 7."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import shard_recombine
    n = args.n
    m = args.batch
    R = args.replicas
    kb, ko, vb, vo = ctx.records(n)
    base = MerkleTree(ctx.local)
    root, N = ctx.build(base, kb, ko, vb, vo, n)
    del vb, vo
    torch.cuda.empty_cache()
    variants = [base.clone() for _ in range(R - 1)]
    batches = []
    for r in range(R - 1):
        g = torch.Generator(device=ctx.dev)
        g.manual_seed(1000 * r + ctx.rank)
        sel = torch.randint(0, n, (m,), device=ctx.dev, generator=g)
        ukb = kb[: n * KLEN].view(n, KLEN)[sel].contiguous().view(-1)
        uvb = random_values(torch, m, ctx.dev, g).contiguous().view(-1)
        batches.append((ukb, torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * KLEN,
                        uvb, torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * VLEN,
                        int(torch.unique(sel).numel())))
    torch.cuda.synchronize()

    # The 7 value batches go through one mkv_tree_upsert_device_many call: per-replica locate/hash/sort
    # on each handle's own stream, then one shared dirty climb (one launch per level for all replicas).
    ptrs = [(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m) for ukb, uko, uvb, uvo, _ in batches]

    def step():
        MerkleTree.upsert_device_many(variants, ptrs)
        if ctx.world > 1:
            for t in variants:
                shard_recombine(t, ctx.dist, N, device=ctx.coll)
        return base.diff_keys_many_view(variants)  # one shared top-down walk (mkv_tree_diff_many)

    for _ in range(args.warmup):
        diffs = step()
    for t in [base] + variants:
        t.prof_enable(True)
        t.prof_reset()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        diffs = step()
    ctx.barrier()
    el = ctx.max_over_ranks(time.perf_counter() - t0)
    upd_ms = variants[0].prof_read("update")[0] / args.steps  # one batched call: all R-1 replicas
    diff_ms = base.prof_read("diff")[0] / (args.steps * (R - 1))  # batched walk: per-pair share
    ok = all(len(d) == b[4] for d, b in zip(diffs, batches))  # every updated key diverges, nothing else
    total_updates = ctx.sum_over_ranks(m) * (R - 1)
    roots = []
    if ctx.world == 1:
        roots = [t.get_root_hash().hex() for t in variants[:2]]
    if ctx.rank == 0:
        wl = (f"configs[4]: {N} keys ({n} per rank), {R} replicas (base + {R - 1} variants), "
              f"{m} value updates per variant per rank; step = {R - 1} dirty-path batches + 1-vs-{R - 1} diff")
        out = base_line(ctx, args, "Incremental anti-entropy: update keys/s (dirty-path rehash + 8-replica diff)",
                        total_updates * args.steps / el, "keys/s", el / args.steps * 1e3, wl)
        out["incremental"] = {"tree_keys": N, "batch_per_rank": m, "replicas": R,
                              "update_device_ms_all_replicas": upd_ms, "diff_device_ms_per_pair": diff_ms,
                              "diff_sizes_match_unique_updates": ok,
                              "divergent_per_pair_rank0": [len(d) for d in diffs], "variant_roots": roots}
        out["cpu_baseline"] = None if (args.no_cpu_baseline or ctx.world > 1) else cpu_baseline_update()
        print(json.dumps(out), flush=True)


# ===================================================================================== CPU baselines
def cpu_baseline_build(target_s: float):
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


def cpu_baseline_diff(n: int = 2_000_000):
    """Oracle diff_keys (merkle.rs:171-196 restated: merge of the sorted leaf lists) on two n-key trees."""
    from oracle import coracle as co
    kb, ko, vb, vo = co.gen_records(SEED, 0, n)
    vb2 = vb.copy()
    vb2[::100 * 1000] ^= 1  # 0.1 % value-only divergence (every 1000th record's value byte 0)
    a = co.OracleTree.build(kb, ko, vb, vo)
    b = co.OracleTree.build(kb, ko, vb2, vo)
    reps, t0 = 0, time.perf_counter()
    while True:  # repeat the (fast) diff for a stable figure
        d = a.diff(b)
        reps += 1
        secs = time.perf_counter() - t0
        if secs >= 3.0:
            break
    return {"value": n * reps / secs, "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": f"{reps} diffs of two {n}-key trees, 0.1% value-only ({len(d)} keys), {secs:.1f} s",
            "cpu_model": _cpu_model()}


def cpu_baseline_update(n: int = 2_000_000, m: int = 2_000):
    """The reference's way to apply a batch: upsert into the leaf map + full rebuild (merkle.rs:52-56),
    done once per batch (the reference does it once per insert)."""
    import numpy as np

    from oracle import coracle as co
    from oracle.merkle_oracle import pack, split_blob
    shani = co.set_backend(1)
    try:
        kb, ko, vb, vo = co.gen_records(SEED, 0, n)
        a = co.OracleTree.build(kb, ko, vb, vo)
        keys = split_blob(kb, ko)
        sel = np.random.default_rng(5).integers(0, n, size=m)
        ks = [keys[int(i)] for i in sel]
        vs = [b"u%099d" % j for j in range(m)]
        bk, bo = pack(ks)
        bv, bvo = pack(vs)
        t0 = time.perf_counter()
        a.upsert(bk, bo, bv, bvo)
        secs = time.perf_counter() - t0
        return {"value": m / secs, "unit": "keys/s", "cores": 1, "kind": "port",
                "sample": f"{m}-key value batch on a {n}-key tree: upsert + one full rebuild, {secs:.2f} s",
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("build", "diff", "incremental"), default="build")
    ap.add_argument("--records", dest="n", type=int, default=None,
                    help="records per GPU (default: 10M build, 100M diff, 125M incremental)")
    ap.add_argument("--batch", type=int, default=125_000, help="incremental: updates per variant per GPU")
    ap.add_argument("--replicas", type=int, default=8, help="incremental: base + variants")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample time")
    ap.add_argument("--no-diff", action="store_true")
    args = ap.parse_args()
    if args.n is None:
        args.n = {"build": 10_000_000, "diff": 100_000_000, "incremental": 125_000_000}[args.workload]
    ctx = Ctx()
    {"build": wl_build, "diff": wl_diff, "incremental": wl_incremental}[args.workload](ctx, args)
    ctx.finish()


if __name__ == "__main__":
    main()
