#!/usr/bin/env python3
"""Benchmark: Merkle build leaves/s (+ diff keys/s) on MI355X — BASELINE.json configs[1] (10M keys, 1 GPU).

Default workload (`--workload build`, what the driver runs): a step = one full tree build (leaf hashing
+ key ordering + dedup + gathers + level reduction + root readback) over n synthetic records (32-B
keys, 100-B values, generated on the device, already resident in HBM when the timed region starts).
N=1: n = 10M (configs[1]). N>1 ranks (torch.distributed.run, one process per GPU): each rank owns a
contiguous key range of the same 10M records per rank (weak scaling: equal work per GPU at every N, so
the driver's per-N values compare directly); the step adds the RCCL all-gathers of shard leaf counts
and seam fringes (device-resident buffers) and the on-device seam combine that yields the global root on
every rank. The N>1 line also carries `sharded_125m_per_rank` (the same sharded build at 125M records
per rank: configs[3] = 1B keys at N=8) and `diff_sharded`; the N=1 line carries `anchor_125m` (125M
keys on one GPU: the per-GPU anchor of the 125M-per-rank curve),
`diff_100m` (configs[2], both divergence modes, exactness vs construction), `configs0` (the 100K CPU
config on the GPU), `configs4` (configs[4]: 125M keys x 8 replicas, 125K-key value batches per variant —
the same measurement as `--workload incremental`, with the dirty climb's roofline), `configs3_1b_sequential`
(configs[3]'s 1B keys on ONE GPU: 8 key-range shards resident in HBM, built shard after shard and combined,
root checked against the CPU oracle's golden root), `configs3_1b_diff_sequential` (the diff of two 1B-key
replicas on ONE GPU, shard after shard: value-only through the top-down walk, mixed through the merge-join,
exact vs construction), `configs4_1b_sequential` (configs[4] at its full 1B keys on ONE GPU: 8 shards x
(base + 7 variants), 125K-key batches per shard, replica roots from their fringes) and the CPU baselines
(cpu_ref: the reference's data structures, single thread; cpu_mt: all host cores).

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
LEAF_BYTES = 8 + KLEN + VLEN + 32   # record model: 140-B record (k, v, 8 B of offsets) read + 32-B digest written
# (SURVEY §8(d)). The timed fixed-shape leaf kernel also WRITES the tree's own copy of each key and its offset
# (key ownership of a build from borrowed device buffers, csrc/k_leaf.hip: the key words it already holds in
# registers + koff): 40 more bytes per leaf, so it moves LEAF_BYTES_KERNEL = 212 B per leaf. `frac` keeps the
# §8(d) record model; `frac_kernel_bytes` uses the 212 B the kernel really moves (PMC traffic ~1.24x of 172).
LEAF_BYTES_KERNEL = LEAF_BYTES + KLEN + 8
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
        # MKV_BENCH_FORCE_DIST=1 (rehearsal knob, never set by the driver): take the sharded path and its
        # RCCL collectives even with one rank, so the device-resident fringe path runs on a one-GPU box.
        if self.world > 1 or os.environ.get("MKV_BENCH_FORCE_DIST") == "1":
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

    def build(self, tree, kb, ko, vb, vo, n, validate=False):
        """Full build of this rank's records; returns the global root (all ranks agree). validate: also
        check once that the shards hold contiguous key ranges ordered by rank (outside timed loops)."""
        if self.dist is None:
            tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            return tree.get_root_hash(), n
        from merklekv_amd.shard import sharded_root
        root, counts = sharded_root(tree, (kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n), None,
                                    self.dist, device=self.coll, on_device=True, validate=validate)
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
def leaf_roofline(n, leaf_avg_ms, launches):
    """roofline of the dominant kernel (the leaf hash, k_leaf_direct). achieved = §8(d)'s 172 B/leaf x n /
    live launch time (HIP events on the tree's stream, sort co-running); `frac_record_model` names the same
    figure. traffic and the VALU fractions come from the PMC file of the same tree
    (profiles/pmc_leaf_hash.json, written by scripts/prof_summary.py)."""
    achieved = LEAF_BYTES * n / (leaf_avg_ms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "k_leaf_direct",
           "bytes_per_leaf": LEAF_BYTES, "avg_launch_ms": leaf_avg_ms, "launches": launches,
           "frac_record_model": achieved / HBM_PEAK_GBS,
           "bytes_per_leaf_kernel": LEAF_BYTES_KERNEL,
           "frac_kernel_bytes": LEAF_BYTES_KERNEL * n / (leaf_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "gb_per_s_hashed": (8 + KLEN + VLEN) * n / (leaf_avg_ms * 1e-3) / 1e9,
           "note": "SHA-256 is VALU-bound (~22.7 ops/B vs 9.8 balance): the HBM frac ceiling is ~0.39; "
                   "avg_launch_ms is measured live while the ordering kernels co-run on the aux stream; frac = "
                   "172 B/leaf (SURVEY 8(d) record model), frac_kernel_bytes = 212 B/leaf (the kernel also stores "
                   "the tree's 32-B key copy + 8-B offset: the PMC traffic above 172 B/leaf is that copy)"}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_leaf_hash.json")
    try:
        pm = json.load(open(pmc_path))
    except (OSError, ValueError):
        pm = None
    if pm and pm.get("n") == n and pm.get("kernel") == out["kernel"]:
        out["traffic"] = pm.get("hbm_bytes_per_launch")
        out["traffic_source"] = pm.get("source")
        vi, gui, dur = pm.get("SQ_INSTS_VALU"), pm.get("GRBM_GUI_ACTIVE"), pm.get("avg_duration_us")
        if vi and gui and dur:
            # SQ_INSTS_VALU = wave64 VALU instructions per launch; capacity = 256 CU x 128 lanes per clock;
            # clock from GRBM_GUI_ACTIVE (summed over the 8 XCDs) over the PMC launch's duration
            f_clk = gui / 8 / (dur * 1e-6)
            lane_ops = vi * 64
            out["valu"] = {
                "SQ_INSTS_VALU": vi, "GRBM_GUI_ACTIVE": gui, "pmc_avg_duration_us": dur,
                "f_clk_ghz": f_clk / 1e9, "lane_ops_per_compression": lane_ops / (3 * n),
                "frac": lane_ops / (256 * 128 * gui / 8),
                "frac_live": lane_ops / (256 * 128 * f_clk * leaf_avg_ms * 1e-3),
                "frac_live_nominal_clk": lane_ops / (256 * 128 * 2.4e9 * leaf_avg_ms * 1e-3),
                "SQ_INSTS_SALU": pm.get("SQ_INSTS_SALU"), "source": pm.get("source"),
                "note": "frac = SQ_INSTS_VALU x 64 / (256 CU x 128 lanes x GRBM_GUI_ACTIVE/8) over the PMC "
                        "(serialised, standalone) launch; frac_live = the same instructions over the live "
                        "co-run launch time at the PMC clock"}
    return out


def diff_secondary(ctx, tree, kb, ko, vb, vo, n, reps=5):
    """10M value-only diff on the build's tree: per-rep host ms, device ms (HIP events) and pinned-pool
    activity (hipHostMalloc/Free counts and host ms) — a slow rep names its cause in the line."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import debug_trace, pool_stats
    vb2 = vb.clone()
    v2 = vb2[: n * VLEN].view(n, VLEN)
    idx = torch.arange(0, n, 1000, device=ctx.dev)
    v2[idx, 0] = v2[idx, 0] ^ 1
    torch.cuda.synchronize()
    treeB = MerkleTree(ctx.local)
    treeB.build_device(kb.data_ptr(), ko.data_ptr(), vb2.data_ptr(), vo.data_ptr(), n)
    tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    for _ in range(3):  # warm: the staging capacity settles and the pinned pool holds its blocks (the
        d = tree.diff_keys_view(treeB)  # first calls grow the capacity and pin new blocks, ~0.1-0.7 ms each)
        del d
    torch.cuda.synchronize()
    rep_ms, dev_ms, pool, traces, thr = [], [], [], [], []
    tree.prof_enable(True)
    for _ in range(reps):
        tree.prof_reset()
        p0, c0 = pool_stats(), _cgroup_cpu()
        t0 = time.perf_counter()
        d = tree.diff_keys_view(treeB)
        rep_ms.append((time.perf_counter() - t0) * 1e3)
        p1, c1 = pool_stats(), _cgroup_cpu()
        traces.append(debug_trace())
        dev_ms.append(tree.prof_read("diff")[0])
        pool.append({"mallocs": p1["host_mallocs"] - p0["host_mallocs"], "frees": p1["host_frees"] - p0["host_frees"],
                     "pin_ms": round(p1["pin_ms"] - p0["pin_ms"], 4)})
        thr.append({k: c1[k] - c0[k] for k in c0} if c0 and c1 else None)
        ndiv = len(d)
        del d  # the result's pinned block goes back to the pool before the next rep
    tree.prof_enable(False)
    dt = sum(rep_ms) / reps / 1e3
    del treeB, vb2
    return {"union_keys": n, "divergent": ndiv, "expected_divergent": int(idx.numel()),
            "ms": dt * 1e3, "ms_per_rep": [round(x, 4) for x in rep_ms],
            "device_ms_per_rep": [round(x, 4) for x in dev_ms], "pool_per_rep": pool,
            "host_trace_per_rep": traces, "cgroup_cpu_per_rep": thr,
            "ms_median": sorted(rep_ms)[reps // 2], "keys_per_s": n / dt,
            "mode": "top-down (equal key sets), value-only 0.1%, incl. key-list D2H"}


def incremental_secondary(ctx, tree, kb, ko, vb, vo, n, reps=5):
    torch = ctx.torch
    import numpy as np
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
    upd = {"tree_keys": n, "batch": m, "ms": dt * 1e3, "device_ms": ums / max(ucnt, 1),
           "update_keys_per_s": m / dt, "mode": "dirty-path rehash (value-only batch)"}
    # key-set change: 0.1 % mixed batch (80 % value updates, 10 % removes, 10 % new keys) through the host
    # API (mkv_tree_apply: batch sort + merge into the sorted leaves + reduction)
    kv_h = kb[: n * KLEN].view(n, KLEN)[sel].cpu().numpy()
    nnew = m // 10
    nk, _, _, _ = ctx.records(nnew, idx0=10**12)
    keys_h = np.concatenate([kv_h[: m - nnew], nk[: nnew * KLEN].view(nnew, KLEN).cpu().numpy()])
    rm_h = np.zeros(m, np.uint8)
    rm_h[int(m * 0.8): m - nnew] = 1
    vals_h = np.frombuffer(bytes(ALPHA * 2)[:VLEN] * m, np.uint8).reshape(m, VLEN)
    koff_h = np.arange(0, m + 1, dtype=np.uint64) * KLEN
    voff_h = np.arange(0, m + 1, dtype=np.uint64) * VLEN
    ks_times = []
    for _ in range(3):
        tree.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tree.apply((keys_h.reshape(-1), koff_h), (vals_h.reshape(-1), voff_h), rm_h)
        ks_times.append(time.perf_counter() - t0)
    dt = min(ks_times)
    upd["keyset_batch"] = {"batch": m, "new": nnew, "removed": int(rm_h.sum()), "ms": dt * 1e3,
                           "keys_per_s": m / dt, "leaves_after": len(tree),
                           "mode": "batch sort + merge into sorted leaves + reduction (host blobs)"}
    return upd


def _cgroup_cpu():
    """cgroup v2 CPU accounting of this container (nr_throttled / throttled_usec / usage_usec), or None."""
    try:
        d = {}
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k in ("usage_usec", "nr_throttled", "throttled_usec", "nr_periods"):
                d[k] = int(v)
        return d
    except (OSError, ValueError):
        return None


def anchor_block(ctx, n, steps=5, warmup=2):
    """The default build step at n keys on this one GPU (N=1 anchor of the 125M-per-rank SCALE curve)."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    kb, ko, vb, vo = ctx.records(n)
    t = MerkleTree(ctx.local)
    for _ in range(warmup):
        t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    t.prof_enable(True)
    t.prof_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        root = t.get_root_hash()
    el = time.perf_counter() - t0
    lm, lc = t.prof_read("leaf_hash")
    out = {"keys": n, "steps": steps, "ms_per_step": el / steps * 1e3, "leaves_per_s": n * steps / el,
           "leaf_hash_ms": lm / max(lc, 1), "root": root.hex()}
    del t, kb, vb
    torch.cuda.empty_cache()
    return out


def sharded_anchor_block(ctx, n, steps=5, warmup=2):
    """N>1: the sharded build at n keys per rank (125M: configs[3], 1B keys over 8 ranks), timed like the
    default step (barriers, max over ranks). The N=1 point of the same per-rank size is anchor_125m."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    kb, ko, vb, vo = ctx.records(n)
    t = MerkleTree(ctx.local)
    root, N = ctx.build(t, kb, ko, vb, vo, n, validate=True)
    for _ in range(warmup - 1):
        root, N = ctx.build(t, kb, ko, vb, vo, n, validate=False)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        root, N = ctx.build(t, kb, ko, vb, vo, n, validate=False)
    ctx.barrier()
    el = ctx.max_over_ranks(time.perf_counter() - t0)
    ctx.check_roots_agree(root)
    out = {"keys_per_rank": n, "global_keys": N, "ranks": ctx.world, "steps": steps,
           "ms_per_step": el / steps * 1e3, "leaves_per_s": N * steps / el, "root": root.hex() if root else None}
    del t, kb, vb
    torch.cuda.empty_cache()
    return out


def route_block(ctx, n, reps=2):
    """n unpartitioned records per rank (keys from the whole key space) -> sampled
    splitters -> one all-to-all -> key-range shards -> sharded build. Reports the redistribution time
    (max over ranks), bytes each rank sent to other ranks, the shard balance and the global root."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import redistribute, sharded_root
    kb = torch.empty(n * KLEN + 64, dtype=torch.uint8, device=ctx.dev)
    vb = torch.empty(n * VLEN + 64, dtype=torch.uint8, device=ctx.dev)
    ko = torch.empty(n + 1, dtype=torch.int64, device=ctx.dev)
    vo = torch.empty(n + 1, dtype=torch.int64, device=ctx.dev)
    gen_records_device(ctx.local, SEED, ctx.rank * n, n, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                       vo.data_ptr())  # nshards = 1: every rank's keys span the whole key space
    torch.cuda.synchronize()
    t = MerkleTree(ctx.local)
    times = []
    from merklekv_amd.shard import coll_stats, coll_stats_reset
    for i in range(reps + 1):
        if i == 1:
            coll_stats_reset()  # collective timings of the timed redistributions only
        ctx.barrier()
        t0 = time.perf_counter()
        routed = redistribute(t, kb, ko, vb, vo, n, ctx.dist, ctx.coll)
        ctx.barrier()
        times.append(ctx.max_over_ranks(time.perf_counter() - t0))
    ctx.barrier()
    t0 = time.perf_counter()
    root, counts = sharded_root(t, routed.blobs(), None, ctx.dist, device=ctx.coll, on_device=True, validate=True)
    ctx.barrier()
    build_s = ctx.max_over_ranks(time.perf_counter() - t0)
    ctx.check_roots_agree(root)
    me = ctx.rank
    moved = int(routed.sent[:, 1].sum() + routed.sent[:, 2].sum() - routed.sent[me, 1] - routed.sent[me, 2])
    moved_max = ctx.max_over_ranks(float(moved))
    red = sorted(times[1:])[len(times[1:]) // 2]
    coll = {k: {"ms_per_call": v[0] / max(v[1], 1) * 1e3, "calls": v[1],
                "bytes_per_rank_per_call": v[2] / max(v[1], 1)} for k, v in coll_stats.items()}
    out = {"records_per_rank": n, "global_keys": sum(counts), "redistribute_ms": red * 1e3,
           "build_after_ms": build_s * 1e3, "bytes_to_other_ranks_max": moved_max,
           "gb_per_s_per_rank": moved_max / red / 1e9, "shard_min": min(counts), "shard_max": max(counts),
           "root": root.hex() if root else None, "collectives": coll,
           "note": "median of %d redistributions after one warm-up; gb_per_s_per_rank = key+value bytes a "
                   "rank sends to other ranks / time (xGMI all-to-all incl. sampling, plan and pack)" % reps}
    del t, routed, kb, vb, ko, vo
    torch.cuda.empty_cache()
    return out


def shared_prefix_block(ctx, n, steps=5, warmup=2, prefix=b"tenant/0001/object/"):
    """Realistic keys that share their first bytes: the default build at n keys
    whose first len(prefix) bytes are common (the rest random base64), vs the same records unmodified."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    kb, ko, vb, vo = ctx.records(n)
    t = MerkleTree(ctx.local)

    def run():
        for _ in range(warmup):
            t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        t.prof_enable(True)
        t.prof_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
            root = t.get_root_hash()
        el = time.perf_counter() - t0
        sort_ms = t.prof_read("sort")[0] / steps
        t.prof_enable(False)
        return el / steps * 1e3, sort_ms, root

    base_ms, base_sort, _ = run()
    pre = torch.frombuffer(bytearray(prefix), dtype=torch.uint8).to(ctx.dev)
    kb[: n * KLEN].view(n, KLEN)[:, : len(prefix)] = pre  # every key now starts with `prefix`
    torch.cuda.synchronize()
    ms, sort_ms, root = run()
    out = {"keys": n, "shared_prefix": prefix.decode(), "shared_bytes": len(prefix),
           "ms_per_step": ms, "sort_ms_per_step": sort_ms, "random_keys_ms_per_step": base_ms,
           "random_keys_sort_ms_per_step": base_sort, "leaves_per_s": n / ms * 1e3, "root": root.hex()}
    del t, kb, vb, ko, vo
    torch.cuda.empty_cache()
    return out


def ragged_block(ctx, n, fixed_leaf_ms, steps=10, warmup=3, klen=64, vlen=256):
    """Store-like ragged records: keys 8-64 B, values 16-256 B, packed back to back (every
    record at an arbitrary byte offset), the oracle's gen_records(ragged=2). The default build over them
    (timed without the library's event pairs, like the headline loop); then the same number of profiled
    builds give the leaf-hash stage (k_leaf_direct hand-off + lane-refill k_leaf_ragged + k_leaf_edges) in
    SHA compressions/s next to the fixed 32/100-B shape's (3 compressions per leaf, same co-running sort)."""
    torch = ctx.torch
    import numpy as np
    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import gen_records_ragged_device
    kb = torch.empty(n * klen + 64, dtype=torch.uint8, device=ctx.dev)
    vb = torch.empty(n * vlen + 64, dtype=torch.uint8, device=ctx.dev)
    ko = torch.empty(n + 1, dtype=torch.int64, device=ctx.dev)
    vo = torch.empty(n + 1, dtype=torch.int64, device=ctx.dev)
    gen_records_ragged_device(ctx.local, SEED, 0, n, klen, vlen, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                              vo.data_ptr())
    torch.cuda.synchronize()
    L = 8 + (ko[1:] - ko[:-1]) + (vo[1:] - vo[:-1])
    comp = int(((L + 9 + 63) // 64).sum().item())
    lsum = int(L.sum().item())
    t = MerkleTree(ctx.local)
    for _ in range(warmup):
        t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        root = t.get_root_hash()
    el = time.perf_counter() - t0
    t.prof_enable(True)
    t.prof_reset()
    for _ in range(steps):
        t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    lm, lc = t.prof_read("leaf_hash")
    leaf_ms = lm / max(lc, 1)
    t.prof_enable(False)
    del t, kb, vb, ko, vo
    torch.cuda.empty_cache()
    # the fixed 32/100-B shape measured the same way right after (same clocks / thermal state as the ragged
    # builds: this block runs after the 100M / 125M sections, where the whole device runs warmer than at the
    # headline loop)
    fkb, fko, fvb, fvo = ctx.records(n)
    ft = MerkleTree(ctx.local)
    for _ in range(warmup):
        ft.build_device(fkb.data_ptr(), fko.data_ptr(), fvb.data_ptr(), fvo.data_ptr(), n)
    ft.prof_enable(True)
    ft.prof_reset()
    for _ in range(steps):
        ft.build_device(fkb.data_ptr(), fko.data_ptr(), fvb.data_ptr(), fvo.data_ptr(), n)
    fm, fc = ft.prof_read("leaf_hash")
    ft.prof_enable(False)
    fixed_adj_ms = fm / max(fc, 1)
    del ft, fkb, fko, fvb, fvo
    fixed_cps = 3 * n / (fixed_adj_ms * 1e-3)
    headline_cps = 3 * 10_000_000 / (fixed_leaf_ms * 1e-3) if fixed_leaf_ms else None
    cps = comp / (leaf_ms * 1e-3)
    out = {"keys": n, "key_bytes": f"{klen // 8}-{klen}", "value_bytes": f"{vlen // 16}-{vlen}",
           "mean_record_bytes": lsum / n - 8, "compressions": comp, "ms_per_step": el / steps * 1e3,
           "leaves_per_s": n * steps / el, "leaf_hash_ms": leaf_ms, "compressions_per_s": cps,
           "gb_per_s_hashed": lsum / (leaf_ms * 1e-3) / 1e9,
           "fixed_shape_compressions_per_s": fixed_cps, "fixed_shape_leaf_hash_ms": fixed_adj_ms,
           "ratio_vs_fixed": cps / fixed_cps, "root": root.hex(),
           "headline_fixed_compressions_per_s": headline_cps,
           "ratio_vs_headline_fixed": cps / headline_cps if headline_cps else None,
           "note": "leaf_hash_ms = the whole leaf stage of the build (k_leaf_direct hand-off, lane-refill k_leaf_ragged, "
                   "k_leaf_edges) while the ordering kernels co-run, HIP events on the tree's stream; ratio_vs_fixed "
                   "against the fixed 32/100-B shape's leaf stage measured the same way right after this block "
                   "(ratio_vs_headline_fixed: against the headline loop's, measured first in the run on a cooler device)"}
    torch.cuda.empty_cache()
    return out


def configs0_block(ctx, reps=5):
    """BASELINE configs[0] on the GPU: 100K-key tree A, replica B with 1 % 80/10/10 events, host blobs
    (what a server snapshot hands over): build A, build B, diff."""
    from merklekv_amd import MerkleTree
    a_rec, b_rec = _configs0_records()
    A, B = MerkleTree(ctx.local), MerkleTree(ctx.local)
    tb, td = [], []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        A.build((a_rec[0], a_rec[1]), (a_rec[2], a_rec[3]))
        B.build((b_rec[0], b_rec[1]), (b_rec[2], b_rec[3]))
        t1 = time.perf_counter()
        d = A.diff_keys_packed(B)
        t2 = time.perf_counter()
        tb.append(t1 - t0)
        td.append(t2 - t1)
    tb, td = sorted(tb[1:]), sorted(td[1:])
    return {"keys": len(a_rec[1]) - 1, "keys_b": len(b_rec[1]) - 1, "divergent": len(d[1]) - 1,
            "build_two_trees_ms": tb[len(tb) // 2] * 1e3, "diff_ms": td[len(td) // 2] * 1e3,
            "root_a": A.get_root_hash().hex(), "note": "host blobs incl. H2D; median of 5"}


def _configs0_records():
    """configs[0] records: 100K synthetic records and the 1 % 80/10/10 replica."""
    import numpy as np
    n, rate = 100_000, 10_000
    from merklekv_amd.merkle import pack_blob
    a = _gen_host(n)
    keys = [a[0][int(a[1][i]):int(a[1][i + 1])].tobytes() for i in range(n)]
    vals = [a[2][int(a[3][i]):int(a[3][i + 1])].tobytes() for i in range(n)]
    # replica B: the oracle generator's plan, restated with numpy here (bench.py must not need tests/)
    rng = np.random.default_rng(SEED & 0xFFFFFFFF)
    cls = rng.integers(0, 1_000_000, size=n)
    changed, deleted = cls < rate * 8 // 10, (cls >= rate * 8 // 10) & (cls < rate * 9 // 10)
    bk = [k for k, dl in zip(keys, deleted) if not dl]
    bv = [(b"#" + v[1:]) if ch else v for v, ch, dl in zip(vals, changed, deleted) if not dl]
    n_ins = n * rate // 10_000_000
    ins = _gen_host(n_ins, idx0=10**9)
    bk += [ins[0][int(ins[1][i]):int(ins[1][i + 1])].tobytes() for i in range(n_ins)]
    bv += [ins[2][int(ins[3][i]):int(ins[3][i + 1])].tobytes() for i in range(n_ins)]
    pk, pv = pack_blob(bk), pack_blob(bv)
    return a, (pk.bytes, pk.offsets, pv.bytes, pv.offsets)


def _gen_host(n, idx0=0):
    """Synthetic records generated on the device, copied to host numpy arrays (kb, koff, vb, voff)."""
    import torch
    from merklekv_amd.merkle import gen_records_device
    kb = torch.empty(n * KLEN + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(n * VLEN + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    gen_records_device(torch.cuda.current_device(), SEED, idx0, n, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(),
                       vb.data_ptr(), vo.data_ptr())
    torch.cuda.synchronize()
    return (kb[: n * KLEN].cpu().numpy(), ko.cpu().numpy().astype("uint64"), vb[: n * VLEN].cpu().numpy(),
            vo.cpu().numpy().astype("uint64"))


def wl_build(ctx, args):
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    n = args.n
    kb, ko, vb, vo = ctx.records(n)
    tree = MerkleTree(ctx.local)

    first = True
    for _ in range(args.warmup):
        root, N = ctx.build(tree, kb, ko, vb, vo, n, validate=first)
        first = False
    if first:  # no warmup: validate the shard ranges outside the timed region anyway
        ctx.build(tree, kb, ko, vb, vo, n, validate=True)
    if ctx.dist is not None:
        from merklekv_amd.shard import coll_stats_reset
        coll_stats_reset()  # per-collective timings of the timed steps only
    # the timed steps run without the library's HIP-event pairs (their records and readbacks add host
    # time to every step); the stage split and the leaf kernel's launch time come from as many
    # profiled steps right after
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        root, N = ctx.build(tree, kb, ko, vb, vo, n, validate=False)
    ctx.barrier()
    t1 = time.perf_counter()
    elapsed = ctx.max_over_ranks(t1 - t0)
    ctx.check_roots_agree(root)
    tree.prof_enable(True)
    tree.prof_reset()
    for _ in range(args.steps):
        ctx.build(tree, kb, ko, vb, vo, n, validate=False)
    tree.prof_enable(False)

    ms_per_step = elapsed / args.steps * 1e3
    value = ctx.world * n * args.steps / elapsed
    leaf_ms, leaf_cnt = tree.prof_read("leaf_hash")
    groups = {g: tree.prof_read(g) for g in ("leaf_hash", "sort", "keycopy", "gather", "reduce", "total_build")}
    leaf_avg_ms = leaf_ms / max(leaf_cnt, 1)
    roofline = leaf_roofline(n, leaf_avg_ms, leaf_cnt)

    coll = None
    if ctx.dist is not None:
        from merklekv_amd.shard import coll_stats
        coll = {k: {"ms_per_call": v[0] / max(v[1], 1) * 1e3, "calls": v[1], "bytes_per_rank_per_call":
                    v[2] / max(v[1], 1)} for k, v in coll_stats.items()}

    # ---------------- secondary, 1 GPU only ----------------
    diff_info = upd_info = d100 = anchor = c0 = shared = dN = ragged = None
    if not args.no_diff and ctx.world == 1:
        diff_info = diff_secondary(ctx, tree, kb, ko, vb, vo, n)
        upd_info = incremental_secondary(ctx, tree, kb, ko, vb, vo, n)
    del tree, kb, vb, ko, vo
    torch.cuda.empty_cache()
    if not args.no_diff and ctx.world == 1:  # right after the headline loop, like the fixed shape it is compared with
        ragged = ragged_block(ctx, n, leaf_avg_ms if n == 10_000_000 else None)
    if not args.no_diff and ctx.dist is not None:
        # N>1: configs[2]-style diff of two replicas of this rank's key range (both divergence modes),
        # exact vs construction on every rank, plus the global sorted list (all-gather-v) once
        dN = diff_modes(ctx, n, steps=5, warmup=2, gather=True)
    if not args.no_diff and ctx.world == 1:
        c0 = configs0_block(ctx)
        shared = shared_prefix_block(ctx, n)
        d100 = diff_modes(ctx, args.diff_records, steps=5, warmup=2)
        torch.cuda.empty_cache()
        if args.anchor_records:
            anchor = anchor_block(ctx, args.anchor_records)
    c4 = c3seq = c3diff = c4seq = None
    if not args.no_diff and ctx.world == 1 and not args.no_big:
        # configs[4] (125M x 8 replicas, 125K-key batches) and configs[3] (1B keys, 8 shards in sequence):
        # the 1B root, the 1B two-replica diff and the 1B incremental step on one GPU
        c4 = configs4_measure(ctx, 125_000_000, 125_000, 8, steps=10, warmup=3)
        c3seq = configs3_sequential_block(ctx)
        c3diff = configs3_diff_sequential_block(ctx)
        c4seq = configs4_sequential_block(ctx)
    c3 = None
    if not args.no_diff and ctx.dist is not None and args.anchor_records:
        c3 = sharded_anchor_block(ctx, args.anchor_records)

    route = None
    if args.route_records and ctx.dist is not None:
        route = route_block(ctx, args.route_records)

    cpu = None
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_build(args.cpu_seconds)

    if ctx.rank == 0:
        wl = ("configs[1]: 10M keys x 1 MI355X, 32-B keys / 100-B values" if n == 10_000_000 and ctx.world == 1
              else f"{n} keys per rank x {ctx.world} GPUs (configs[1] per rank, key-range shards; configs[3] = "
                   f"125M x 8 ranks in sharded_125m_per_rank), 32-B keys / 100-B values")
        out = base_line(ctx, args, "Merkle build leaves/s (full tree: hash+sort+reduce)", value,
                        "leaves/s", ms_per_step, wl)
        out["root"] = root.hex() if root else None
        out["global_keys"] = N
        out["roofline"] = roofline
        out["stage_ms_per_step"] = {g: (v[0] / max(v[1], 1) if g == "leaf_hash" else v[0] / args.steps)
                                    for g, v in groups.items()}
        out["diff"] = diff_info
        out["incremental"] = upd_info
        out["diff_100m"] = d100
        out["anchor_125m"] = anchor
        out["configs0_gpu"] = c0
        out["shared_prefix_10m"] = shared
        out["ragged_10m"] = ragged
        out["configs4"] = c4
        out["configs3_1b_sequential"] = c3seq
        out["configs3_1b_diff_sequential"] = c3diff
        out["configs4_1b_sequential"] = c4seq
        if ctx.dist is not None:
            out["diff_sharded"] = dN
            out["collectives_build"] = coll
            out["sharded_125m_per_rank"] = c3  # configs[3] at N = 8 (1B keys); N = 1 point: anchor_125m
        if route is not None:
            out["route"] = route
        out["cpu_baseline"] = cpu
        emit(out)


# ============================================================================================= diff
def _all_counts(ctx, x: int) -> list:
    """All-gather of one int per rank (host list)."""
    if ctx.dist is None:
        return [x]
    torch = ctx.torch
    t = torch.tensor([x], dtype=torch.int64, device=ctx.coll)
    out = torch.empty(ctx.world, dtype=torch.int64, device=ctx.coll)
    if ctx.coll.type == "cuda":
        ctx.dist.all_gather_into_tensor(out, t)
    else:
        ctx.dist.all_gather(list(out.chunk(ctx.world)), t)
    return [int(v) for v in out.tolist()]


def diff_modes(ctx, n, steps, warmup, gather=False):
    """configs[2]: two n-key replicas per rank, 0.1 % divergence, (a) value-only -> top-down walk,
    (b) mixed 80/10/10 change/delete/insert -> merge-join. Each output is checked against the constructed
    divergent set (exact_vs_construction). gather (N>1): also the global sorted list on every rank."""
    torch = ctx.torch
    import numpy as np
    from merklekv_amd import MerkleTree
    kb, ko, vb, vo = ctx.records(n)
    A = MerkleTree(ctx.local)
    ctx.build(A, kb, ko, vb, vo, n, validate=True)
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
        ctx.build(B, kBf, koB, vBf, voB, nB, validate=True)
        torch.cuda.synchronize()
        d = None
        for _ in range(max(warmup, 6)):  # like the timed loop, the previous result stays alive while the
            d = A.diff_keys_view(B)      # next call runs: the staging capacity settles (it halves towards
                                         # twice the result) and the pinned-block pool reaches its steady
                                         # state (with 2 warm calls one timed call still pinned a new block)
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):  # timed without the library's HIP-event pairs
            d = A.diff_keys_view(B)
        ctx.barrier()
        el = ctx.max_over_ranks(time.perf_counter() - t0)
        A.prof_enable(True)
        A.prof_reset()
        for _ in range(steps):  # device time: the same calls with event pairs
            d = A.diff_keys_view(B)
        A.prof_enable(False)
        dms, dcnt = A.prof_read("diff")
        got = d.raw.reshape(-1, KLEN)
        exact = got.shape == exp_sorted.shape and bool((got == exp_sorted).all())
        union = ctx.sum_over_ranks(n + new)
        res[mode] = {"union_keys": union, "union_keys_per_rank": n + new, "divergent": ctx.sum_over_ranks(len(d)),
                     "expected_divergent": ctx.sum_over_ranks(int(exp_sorted.shape[0])),
                     "exact_vs_construction": ctx.sum_over_ranks(int(exact)) == ctx.world,
                     "ms": el / steps * 1e3, "device_ms": dms / max(steps, 1),
                     "keys_per_s": union * steps / el,
                     "path": "top-down" if mode == "value_only" else "merge-join"}
        if mode == "value_only":
            res[mode]["roofline"] = topdown_roofline(A.walk_stats(), len(d), res[mode]["device_ms"])
        else:
            res[mode]["roofline"] = merge_roofline(n + new, res[mode]["device_ms"])
        if gather and ctx.dist is not None:
            # the global sorted list on every rank (sync.rs:67-83 consumes it whole): local diff +
            # all-gather-v of key lengths and bytes; this rank's slice must sit at its global offset
            from merklekv_amd.shard import coll_stats, sharded_diff_gather
            ctx.barrier()
            t0 = time.perf_counter()
            graw, goffs = sharded_diff_gather(A, B, ctx.dist, ctx.coll)
            ctx.barrier()
            gel = ctx.max_over_ranks(time.perf_counter() - t0)
            gk = graw.reshape(-1, KLEN)
            before = int(sum(_all_counts(ctx, len(d))[:ctx.rank]))
            mine_ok = bool((gk[before:before + len(d)] == got).all()) and len(goffs) - 1 == res[mode]["divergent"]
            sorted_ok = bool((np.lexsort(gk.T[::-1]) == np.arange(gk.shape[0])).all()) if gk.shape[0] else True
            res[mode]["global_list"] = {
                "ms": gel * 1e3, "keys": len(goffs) - 1, "bytes": int(goffs[-1]),
                "rank_slice_at_global_offset": ctx.sum_over_ranks(int(mine_ok)) == ctx.world,
                "sorted": sorted_ok,
                "all_gather_v_ms": coll_stats.get("diff_all_gather_v", [0, 1])[0]
                / max(coll_stats.get("diff_all_gather_v", [0, 1])[1], 1) * 1e3,
                "note": "local diff + one (count, bytes) all-gather + one all-gather of padded [u32 lengths | "
                        "key bytes] blocks; wall time max over ranks"}
        del d, B, kBf, vBf
        torch.cuda.empty_cache()
    del A, kb, vb
    torch.cuda.empty_cache()
    return res


def merge_roofline(union_keys_per_rank, device_ms):
    """The merge-join diff (mixed divergence): 80 B per union key (8-B prefix + 32-B leaf digest, both
    trees: SURVEY §8(d)) over the device time of the whole diff call; traffic = PMC HBM bytes of its
    kernels from profiles/pmc_diff_merge.json when that file describes a diff of this size."""
    achieved = DIFF_BYTES_PER_KEY * union_keys_per_rank / (device_ms * 1e-3) / 1e9
    traffic, src = None, None
    try:
        pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_diff_merge.json")))
        if pm.get("union_keys") == union_keys_per_rank:  # the PMC file is per rank
            traffic, src = pm.get("hbm_bytes_per_diff"), pm.get("source")
    except (OSError, ValueError):
        pass
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
            "kernel": "k_diff_pass1 + k_diff_pass2 (merge-join)", "bytes_per_union_key": DIFF_BYTES_PER_KEY,
            "algorithmic_bytes": DIFF_BYTES_PER_KEY * union_keys_per_rank, "device_ms": device_ms,
            "note": "achieved = 80 B x union keys / device time of the whole diff call (partition, passes, "
                    "verify, key gather)"}


def topdown_roofline(ws, m, device_ms):
    """The top-down walk (value-only divergence): the digest bytes the walk compared (mkv_tree_walk_stats:
    2^k descendants x 32 B x both trees per expanded frontier node) plus the divergent leaves' tail (the
    leaf-key check reads perm + two offsets + the key on both sides, the key gather reads the key and
    offsets and writes the list: ~184 B per divergent key), over the device time of the call. The walk
    is a chain of dependent launches, so it is latency- rather than bandwidth-bound."""
    walk_bytes = ws.get("bytes", 0) if ws else 0
    tail_bytes = 184 * m
    algo = walk_bytes + tail_bytes
    achieved = algo / (device_ms * 1e-3) / 1e9 if device_ms else None
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": None,
            "kernel": "k_topdown_jump chain + bitmap positions + key tail", "walk_bytes": walk_bytes,
            "walk_entries": ws.get("entries") if ws else None, "launches": ws.get("launches") if ws else None,
            "tail_bytes": tail_bytes, "algorithmic_bytes": algo, "device_ms": device_ms,
            "note": "latency-bound walk: %s dependent jump launches; frac reported against 8 TB/s anyway"
                    % (ws.get("launches") if ws else "?")}


def diff_roofline(res):
    m = res["mixed"]
    return merge_roofline(m["union_keys_per_rank"], m["device_ms"])


def wl_diff(ctx, args):
    """configs[2]: two replicas with 0.1 % divergence; diff keys/s over the union of keys."""
    res = diff_modes(ctx, args.n, args.steps, args.warmup)
    cpu = None
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_diff()
    if ctx.rank == 0:
        v = res["value_only"]
        n = args.n
        wl = (f"configs[2]: {n // 1_000_000}M keys x 2 replicas per rank, 0.1% divergence; value = value-only "
              f"(top-down) union keys/s; 'mixed' = 80/10/10 change/delete/insert (merge-join)")
        out = base_line(ctx, args, "Merkle diff keys/s (union keys compared, 2 replicas, 0.1% divergence)",
                        v["keys_per_s"], "keys/s", v["ms"], wl)
        out["roofline"] = diff_roofline(res)
        out["diff"] = res
        out["cpu_baseline"] = cpu
        emit(out)


# ====================================================================================== incremental
def configs4_measure(ctx, n, m, R, steps, warmup):
    """configs[4]: 8 replicas (base + 7 variants) of a 1B-key tree (per-GPU shard of n keys); a step =
    each variant applies its own value-update batch (dirty path + seam recombine) + base diffed vs all 7.
    Returns the measured dict (rank 0 fields valid on every rank)."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import shard_recombine_many
    kb, ko, vb, vo = ctx.records(n)
    base = MerkleTree(ctx.local)
    root, N = ctx.build(base, kb, ko, vb, vo, n, validate=True)
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

    # The 7 value batches go through one mkv_tree_upsert_device_many call: one locate / batch hash / sort
    # for all replicas, then ONE k_dirty_climb launch for every replica's whole climb.
    ptrs = [(ukb.data_ptr(), uko.data_ptr(), uvb.data_ptr(), uvo.data_ptr(), m) for ukb, uko, uvb, uvo, _ in batches]

    def step():
        MerkleTree.upsert_device_many(variants, ptrs)
        if ctx.dist is not None:  # all 7 variants' fringes in ONE all-gather, combined on the device
            shard_recombine_many(variants, ctx.dist, N, device=ctx.coll)
        return base.diff_keys_many_view(variants)  # one shared top-down walk (mkv_tree_diff_many)

    for _ in range(warmup):
        diffs = step()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):  # timed without the library's HIP-event pairs
        diffs = step()
    ctx.barrier()
    el = ctx.max_over_ranks(time.perf_counter() - t0)
    for t in [base] + variants:  # device-time split: the same steps with event pairs
        t.prof_enable(True)
        t.prof_reset()
    for _ in range(steps):
        diffs = step()
    upd_ms = variants[0].prof_read("update")[0] / steps  # one batched call: all R-1 replicas
    diff_ms = base.prof_read("diff")[0] / (steps * (R - 1))  # batched walk: per-pair share
    climb_ms = variants[0].prof_read("climb")[0] / steps      # the one climb launch, all replicas
    walk_ms = base.prof_read("walk")[0] / steps               # shared 1-vs-(R-1) walk launches
    d2h_ms = base.prof_read("d2h")[0] / (steps * (R - 1))     # key lists into pinned host memory
    for t in [base] + variants:
        t.prof_enable(False)
    # work of the last step (stats of the last update / walk; every step does the same amount)
    counts = [v.update_counts() for v in variants]
    rehashed = sum(sum(c[1:]) for c in counts)  # dirty internal nodes of the climb (promoted copies incl.)
    changed = sum(c[0] for c in counts if c)
    ws = base.walk_stats()
    ok = all(len(d) == b[4] for d, b in zip(diffs, batches))  # every updated key diverges, nothing else
    total_updates = ctx.sum_over_ranks(m) * (R - 1)
    roots = []
    if ctx.dist is None:
        roots = [t.get_root_hash().hex() for t in variants[:2]]
    climb_bytes = 96 * rehashed  # SURVEY §8(d) model: both children read (64 B) + the node written (32 B)
    try:  # PMC of the same workload (scripts/gpu_prof.sh BENCH_ARGS="--workload incremental")
        pmc_inc = json.load(open(os.path.join(ROOT, "profiles", "pmc_incremental.json")))
    except (OSError, ValueError):
        pmc_inc = {}
    pmc_ok = pmc_inc.get("tree_keys") == N and pmc_inc.get("replicas") == R and pmc_inc.get("batch") == m
    comp = 2 * rehashed          # one full + one constant-schedule compression per node
    roofline = {
        "bound": "hbm", "kernel": "k_dirty_climb + k_reduce_fused/top above its stop level (every replica per launch)",
        "achieved": climb_bytes / (climb_ms * 1e-3) / 1e9 if climb_ms else None, "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": climb_bytes / (climb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if climb_ms else None,
        "traffic": pmc_inc.get("climb_hbm_bytes_per_step") if pmc_ok else None,
        "traffic_source": pmc_inc.get("source") if pmc_ok else None,
        "bytes_per_rehashed_node": 96, "bytes_per_rehashed_node_kernel_min": 64,
        "rehashed_nodes_per_step": rehashed, "changed_leaves_per_step": changed, "climb_ms_per_step": climb_ms,
        "valu": {"compressions_per_step": comp, "lane_ops_model": comp * 1376,
                 "frac_of_78.6T": comp * 1376 / (climb_ms * 1e-3) / (VALU_PEAK_TOPS * 1e12) if climb_ms else None,
                 "note": "1,376 VALU lane-ops per compression (measured on the leaf kernel, PMC)"},
        "walk": {"ms_per_step": walk_ms, "ms_per_pair": walk_ms / (R - 1), "entries": ws["entries"],
                 "bytes_compared": ws["bytes"], "bytes_per_pair": ws["bytes"] / (R - 1),
                 "traffic": pmc_inc.get("walk_hbm_bytes_per_step") if pmc_ok else None,
                 "gb_per_s": ws["bytes"] / (walk_ms * 1e-3) / 1e9 if walk_ms else None,
                 "launches": ws["launches"], "divergent_positions": ws["divergent_positions"]},
        "note": "achieved = 96 B x rehashed nodes (SURVEY 8(d): both children + the node; read back from the trees) "
                "/ HIP-event time of the climb launch on the group's stream. The kernel itself moves ~64 B per "
                "rehashed node (the dirty child stays in registers; only the clean sibling is read). The climb "
                "is 2 SHA-256 compressions per node, so VALU binds (valu.frac_of_78.6T); walk = the shared "
                "top-down launches (digests compared in both trees) without the key gather / PCIe copy"}
    inc = {"tree_keys": N, "batch_per_rank": m, "replicas": R,
           "update_device_ms_all_replicas": upd_ms, "diff_device_ms_per_pair": diff_ms,
           "climb_device_ms": climb_ms, "walk_device_ms_per_pair": walk_ms / (R - 1),
           "keys_d2h_ms_per_pair": d2h_ms,  # on the copy stream, beside the next step's update (not in diff_device)
           "diff_sizes_match_unique_updates": ok,
           "divergent_per_pair_rank0": [len(d) for d in diffs], "variant_roots": roots}
    out = {"workload": (f"configs[4]: {N} keys ({n} per rank), {R} replicas (base + {R - 1} variants), "
                        f"{m} value updates per variant per rank; step = {R - 1} dirty-path batches + "
                        f"1-vs-{R - 1} diff"),
           "steps": steps, "warmup": warmup, "ms_per_step": el / steps * 1e3,
           "update_keys_per_s": total_updates * steps / el, "roofline": roofline, "incremental": inc}
    del base, variants, batches, kb, ko, diffs
    torch.cuda.empty_cache()
    return out


def wl_incremental(ctx, args):
    """configs[4] as its own line (value = update keys/s)."""
    r = configs4_measure(ctx, args.n, args.batch, args.replicas, args.steps, args.warmup)
    if ctx.rank == 0:
        out = base_line(ctx, args, "Incremental anti-entropy: update keys/s (dirty-path rehash + 8-replica diff)",
                        r["update_keys_per_s"], "keys/s", r["ms_per_step"], r["workload"])
        out["roofline"] = r["roofline"]
        out["incremental"] = r["incremental"]
        out["cpu_baseline"] = None if (args.no_cpu_baseline or ctx.world > 1) else cpu_baseline_update()
        emit(out)


def configs3_sequential_block(ctx, nshards=8, per_shard=125_000_000, steps=2, warmup=1):
    """configs[3] at its full size on ONE GPU: 1B keys = 8 key ranges x 125M records, all resident in HBM
    (140 GB of records + offsets), the global root built shard after shard (shard.sequential_root: prepare
    -> reduce at the shard's global offset -> fringe, then one seam combine). The 8-GPU form of the same
    config is the N=8 line's sharded_125m_per_rank. matches_golden: the root equals the CPU oracle's
    (tests/golden/roots_sharded.json, computed once by oracle/root_stream.c over the same records)."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import sequential_root
    blobs = []
    for g in range(nshards):
        kb = torch.empty(per_shard * KLEN + 64, dtype=torch.uint8, device=ctx.dev)
        vb = torch.empty(per_shard * VLEN + 64, dtype=torch.uint8, device=ctx.dev)
        ko = torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev)
        vo = torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev)
        gen_records_device(ctx.local, SEED, g * per_shard, per_shard, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(),
                           vb.data_ptr(), vo.data_ptr(), shard=g, nshards=nshards)
        blobs.append((kb, ko, vb, vo, per_shard))
    torch.cuda.synchronize()
    N = nshards * per_shard
    t = MerkleTree(ctx.local)
    for _ in range(warmup):
        root, counts = sequential_root(t, blobs, N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        root, counts = sequential_root(t, blobs, N)
    el = (time.perf_counter() - t0) / steps
    golden = None
    try:
        d = json.load(open(os.path.join(ROOT, "tests", "golden", "roots_sharded.json")))
        golden = next((c["root"] for c in d["cases"] if c["shards"] == nshards and c["per_shard"] == per_shard
                       and c["seed"] == SEED), None)
    except (OSError, ValueError):
        pass
    out = {"keys": N, "shards": nshards, "keys_per_shard": per_shard, "steps": steps,
           "ms_per_root": el * 1e3, "leaves_per_s": N / el, "root": root.hex() if root else None,
           "golden_root": golden, "matches_golden": (root.hex() == golden) if (root and golden) else None,
           "note": "records resident in HBM before timing; per shard hash + sort + dedup + reduction at its "
                   "global offset + fringe readback (<= 6 KiB), then the seam combine: 1B-key root on one GPU"}
    del t, blobs
    torch.cuda.empty_cache()
    return out


def _shard_blob(ctx, g, nshards, per_shard, bufs):
    """Generate key range g of nshards (records [g * per_shard, (g + 1) * per_shard)) into bufs."""
    from merklekv_amd.merkle import gen_records_device
    kb, ko, vb, vo = bufs
    gen_records_device(ctx.local, SEED, g * per_shard, per_shard, KLEN, VLEN, kb.data_ptr(), ko.data_ptr(),
                       vb.data_ptr(), vo.data_ptr(), shard=g, nshards=nshards)
    ctx.torch.cuda.synchronize()
    return (kb, ko, vb, vo, per_shard)


def configs3_diff_sequential_block(ctx, nshards=8, per_shard=125_000_000, steps=5, warmup=3):
    """configs[2] x configs[3] at full size on ONE GPU: the diff of two 1B-key replicas (8 key ranges x 125M,
    0.1 % divergence) shard after shard — what 8 ranks do in parallel. Per shard g: both replicas' shards
    prepared and reduced at their global offsets (shard_prepare + shard_reduce), then the shard-local
    diff_keys (value-only: top-down from the fringe roots; mixed, 90 % changed / 10 % replaced keys:
    merge-join), warmed, then timed `steps` times (HIP-event-free, like the 100M lines); the per-shard lists
    sit at the global offsets given by their counts. ms_per_1b_diff = the sum over the 8 shards of the mean
    diff call (list host-visible on return). exact: every shard's list equals the constructed divergent set
    (sorted), so the concatenation is the global list (merkle.rs:171-196, sync.rs:67-83)."""
    torch = ctx.torch
    import numpy as np
    from merklekv_amd import MerkleTree
    from merklekv_amd.merkle import gen_records_device
    bufs = (torch.empty(per_shard * KLEN + 64, dtype=torch.uint8, device=ctx.dev),
            torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev),
            torch.empty(per_shard * VLEN + 64, dtype=torch.uint8, device=ctx.dev),
            torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev))
    N = nshards * per_shard
    out = {"keys": N, "shards": nshards, "keys_per_shard": per_shard, "steps": steps}
    for mode in ("value_only", "mixed"):
        ta, tb = MerkleTree(ctx.local), MerkleTree(ctx.local)
        per_ms, counts, exact, fa, fb = [], [], True, [], []
        for g in range(nshards):
            kb, ko, vb, vo, ng = _shard_blob(ctx, g, nshards, per_shard, bufs)
            rows = torch.arange(3 + g, ng, 1000, device=ctx.dev)
            kv, v2 = kb[: ng * KLEN].view(ng, KLEN), vb[: ng * VLEN].view(ng, VLEN).clone()
            if mode == "value_only":
                v2[rows, 9] ^= 4
                blob_b = (kb, ko, v2.view(-1), vo, ng)
                exp = kv[rows]
            else:
                rm, chg = rows[(rows // 1000) % 10 == 0], rows[(rows // 1000) % 10 != 0]
                v2[chg, 9] ^= 4
                keep = torch.ones(ng, dtype=torch.bool, device=ctx.dev)
                keep[rm] = False
                new = rm.numel()
                nkb = torch.empty(new * KLEN + 64, dtype=torch.uint8, device=ctx.dev)
                nvb = torch.empty(new * VLEN + 64, dtype=torch.uint8, device=ctx.dev)
                nko = torch.empty(new + 1, dtype=torch.int64, device=ctx.dev)
                nvo = torch.empty(new + 1, dtype=torch.int64, device=ctx.dev)
                gen_records_device(ctx.local, SEED, 10**12 + g * new, new, KLEN, VLEN, nkb.data_ptr(), nko.data_ptr(),
                                   nvb.data_ptr(), nvo.data_ptr(), shard=g, nshards=nshards)
                torch.cuda.synchronize()
                nk = nkb[: new * KLEN].view(new, KLEN)
                kB = torch.cat([kv[keep], nk]).contiguous().view(-1)
                vB = torch.cat([v2[keep], nvb[: new * VLEN].view(new, VLEN)]).contiguous().view(-1)
                off = torch.arange(0, ng + 1, device=ctx.dev, dtype=torch.int64)
                blob_b = (kB, off * KLEN, vB, off * VLEN, ng)
                exp = torch.cat([kv[chg], kv[rm], nk])
                del nkb, nvb
            exp = exp.cpu().numpy()
            exp = exp[np.lexsort(exp.T[::-1])]
            torch.cuda.synchronize()
            o = sum(counts)
            counts.append(ta.shard_prepare((kb, ko, vb, vo, ng), None, on_device=True))
            ta.shard_reduce(o, N)
            nb = tb.shard_prepare(blob_b, None, on_device=True)
            tb.shard_reduce(o, N)  # equal leaf counts per shard in both modes
            del blob_b, v2
            if mode == "mixed":
                del kB, vB
            fa.append(ta.shard_fringe())
            fb.append(tb.shard_fringe())
            d = None
            for _ in range(warmup):
                d = ta.diff_keys_view(tb)
            t0 = time.perf_counter()
            for _ in range(steps):
                d = ta.diff_keys_view(tb)
            per_ms.append((time.perf_counter() - t0) / steps * 1e3)
            got = d.raw.reshape(-1, KLEN)
            exact = exact and nb == ng and got.shape == exp.shape and bool((got == exp).all())
            del d
        ra = ta.shard_combine(b"".join(fa), nshards, N)
        rb = tb.shard_combine(b"".join(fb), nshards, N)
        out[mode] = {"ms_per_1b_diff": sum(per_ms), "ms_per_shard_diff": per_ms,
                     "union_keys_per_s": N / (sum(per_ms) * 1e-3), "exact_vs_construction": exact,
                     "root_a": ra.hex() if ra else None, "roots_differ": ra != rb,
                     "path": "top-down from fringe roots" if mode == "value_only" else "merge-join"}
        del ta, tb
        torch.cuda.empty_cache()
    del bufs
    torch.cuda.empty_cache()
    return out


def configs4_sequential_block(ctx, nshards=8, per_shard=125_000_000, m=125_000, R=8, steps=5, warmup=2):
    """configs[4] at full size on ONE GPU: the 1B-key tree as 8 key ranges x 125M, base + 7 variants, every
    variant applying 125K value updates per shard (1M keys per variant), shard after shard. Per shard: the
    base shard built at its global offset and cloned per variant; a step = every variant's batch through
    one upsert_device_many (dirty path) + the base diffed against all 7 (diff_keys_many, one shared walk);
    warmed, then timed. ms_per_1b_step = the sum over shards of the mean step (what 8 ranks do in parallel,
    minus the fringe recombine). Afterwards every replica's global root from the seam combine of its 8
    fringes: the base's equals the golden 1B root."""
    torch = ctx.torch
    from merklekv_amd import MerkleTree
    bufs = (torch.empty(per_shard * KLEN + 64, dtype=torch.uint8, device=ctx.dev),
            torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev),
            torch.empty(per_shard * VLEN + 64, dtype=torch.uint8, device=ctx.dev),
            torch.empty(per_shard + 1, dtype=torch.int64, device=ctx.dev))
    N = nshards * per_shard
    fr = [[] for _ in range(R)]
    per_ms, ok, off = [], True, 0
    uko = torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * KLEN
    uvo = torch.arange(0, m + 1, device=ctx.dev, dtype=torch.int64) * VLEN
    for g in range(nshards):
        kb, ko, vb, vo, ng = _shard_blob(ctx, g, nshards, per_shard, bufs)
        base = MerkleTree(ctx.local)
        n_g = base.shard_prepare((kb, ko, vb, vo, ng), None, on_device=True)
        base.shard_reduce(off, N)
        off += n_g
        variants = [base.clone() for _ in range(R - 1)]
        batches, uniq = [], []
        for r in range(R - 1):
            gen = torch.Generator(device=ctx.dev)
            gen.manual_seed(1000 * r + g)
            sel = torch.randint(0, ng, (m,), device=ctx.dev, generator=gen)
            ukb = kb[: ng * KLEN].view(ng, KLEN)[sel].contiguous().view(-1)
            uvb = random_values(torch, m, ctx.dev, gen).contiguous().view(-1)
            batches.append((ukb, uvb))
            uniq.append(int(torch.unique(sel).numel()))
        torch.cuda.synchronize()
        ptrs = [(a.data_ptr(), uko.data_ptr(), b.data_ptr(), uvo.data_ptr(), m) for a, b in batches]

        def step():
            MerkleTree.upsert_device_many(variants, ptrs)
            return base.diff_keys_many_view(variants)

        for _ in range(warmup):
            diffs = step()
        t0 = time.perf_counter()
        for _ in range(steps):
            diffs = step()
        per_ms.append((time.perf_counter() - t0) / steps * 1e3)
        ok = ok and all(len(d) == u for d, u in zip(diffs, uniq))
        for i, t in enumerate([base] + variants):
            fr[i].append(t.shard_fringe())
        del diffs, base, variants, batches
        torch.cuda.empty_cache()
    holder = MerkleTree(ctx.local)
    roots = [holder.shard_combine(b"".join(f), nshards, N) for f in fr]
    golden = None
    try:
        d = json.load(open(os.path.join(ROOT, "tests", "golden", "roots_sharded.json")))
        golden = next((c["root"] for c in d["cases"] if c["shards"] == nshards and c["per_shard"] == per_shard
                       and c["seed"] == SEED), None)
    except (OSError, ValueError):
        pass
    total_updates = m * (R - 1) * nshards
    out = {"keys": N, "shards": nshards, "replicas": R, "batch_per_shard": m, "updates_per_variant": m * nshards,
           "steps": steps, "ms_per_1b_step": sum(per_ms), "ms_per_shard_step": per_ms,
           "update_keys_per_s": total_updates / (sum(per_ms) * 1e-3),
           "diff_sizes_match_unique_updates": ok, "base_root": roots[0].hex() if roots[0] else None,
           "base_matches_golden": (roots[0].hex() == golden) if (roots[0] and golden) else None,
           "distinct_replica_roots": len(set(roots)) == R,
           "note": "per shard: 7 value batches (dirty path, one call) + 1-vs-7 diff, key lists host-visible; the "
                   "1B step is the 8 shards in sequence; replica roots from the 8 fringes each"}
    del bufs
    torch.cuda.empty_cache()
    return out


# ===================================================================================== CPU baselines
def _host_threads() -> int:
    """Host threads this process may use: OMP_NUM_THREADS when set (the GPU box sets 16: its CPU share),
    else the affinity mask."""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "")))
    except ValueError:
        return max(1, len(os.sched_getaffinity(0)))


def cpu_baseline_build(target_s: float):
    """CPU baselines on the GPU box's host (oracle/: test infrastructure, never inside a timed GPU region).
    value = cpu_ref: the reference's own data structures (SipHash HashMap of heap Strings, node tree with
    the per-level deep clones of merkle.rs:107-108), single thread, SHA-NI like sha2 0.10.9 — one bulk
    build (= n x (compute_leaf_hash + map insert) + ONE rebuild). Beside it: the reference's real API
    cost (n x insert, a rebuild per insert, O(n^2 log n)) timed at 1K/2K and extrapolated; cpu_mt (all
    host threads); the lean single-thread port; and configs[0] (100K build + 1 % diff) per flavour."""
    import math

    from oracle import coracle as co
    shani = co.set_backend(1)
    try:
        thr = _host_threads()
        # ---- cpu_ref bulk build, sized to ~40 % of the budget
        kb, ko, vb, vo = co.gen_records(SEED, 0, 50_000)
        s0, _ = co.ref_bulk(kb, ko, vb, vo)
        n_ref = int(min(4_000_000, max(50_000, 50_000 / s0 * target_s * 0.4)))
        kb, ko, vb, vo = co.gen_records(SEED, 0, n_ref)
        s_ref, root_ref = co.ref_bulk(kb, ko, vb, vo)
        # ---- cpu_mt + the lean port on the same sample
        s_mt, root_mt = co.mt_build(kb, ko, vb, vo, thr)
        n_lean = min(n_ref, 2_000_000)
        buf = (__import__("ctypes").c_uint8 * 32)()
        s_lean = co.lib().orc_bench_build(kb.ctypes.data, ko.ctypes.data, vb.ctypes.data, vo.ctypes.data, n_lean, buf)
        assert root_mt == root_ref, "cpu_mt and cpu_ref disagree"
        del kb, vb
        # ---- the reference API: n x insert, each rebuilding (sync.rs:110-115, server.rs:664-667)
        loop = {}
        for m in (1000, 2000):
            a = co.gen_records(SEED, 0, m)
            loop[m] = co.ref_insert_loop(*a)[0]
        # sum_{i<=n} rebuild(i) ~ c * n^2 log2 n: fit c on 2K, extrapolate
        c = loop[2000] / (2000 ** 2 * math.log2(2000))
        est = {k: c * k * k * math.log2(k) for k in (100_000, 10_000_000)}
        # ---- configs[0]: 100K build of A and B + diff, per flavour
        (ak, ako, av, avo), (bk, bko, bv, bvo) = _configs0_records()
        ra, _ = co.ref_bulk(ak, ako, av, avo)
        rb, _ = co.ref_bulk(bk, bko, bv, bvo)
        rd, rcnt = co.ref_diff((ak, ako, av, avo), (bk, bko, bv, bvo))
        ma, _ = co.mt_build(ak, ako, av, avo, thr)
        mb, _ = co.mt_build(bk, bko, bv, bvo, thr)
        ta, tb = co.OracleTree.build(ak, ako, av, avo), co.OracleTree.build(bk, bko, bv, bvo)
        md, mcnt = co.mt_diff(ta, tb, thr)
        assert rcnt == mcnt == len(ta.diff(tb)), "configs[0] diff counts disagree"
        model = _cpu_model()
        return {"value": n_ref / s_ref, "unit": "leaves/s", "cores": 1, "kind": "port",
                "sample": f"cpu_ref: one bulk build of {n_ref} synthetic 32B/100B records with the reference's data "
                          f"structures (SipHash HashMap, per-level deep-cloned node tree), {s_ref:.1f} s, "
                          f"sha={'SHA-NI' if shani else 'portable'}",
                "cpu_model": model,
                "flavours": {
                    "cpu_ref": {"leaves_per_s": n_ref / s_ref, "cores": 1, "records": n_ref, "s": s_ref},
                    "cpu_mt": {"leaves_per_s": n_ref / s_mt, "cores": thr, "records": n_ref, "s": s_mt},
                    "lean_port_1t": {"leaves_per_s": n_lean / s_lean, "cores": 1, "records": n_lean, "s": s_lean,
                                     "note": "round-1 baseline: qsort index + flat levels, no node clones"}},
                "insert_loop": {"s_1k": loop[1000], "s_2k": loop[2000], "model": "c * n^2 log2 n fitted at 2K",
                                "est_s_100k": est[100_000], "est_s_10m": est[10_000_000],
                                "note": "the reference API as its callers use it (insert rebuilds every time)"},
                "configs0": {"keys": len(ako) - 1, "keys_b": len(bko) - 1, "divergent": rcnt,
                             "cpu_ref": {"build_two_trees_s": ra + rb, "diff_s": rd, "cores": 1},
                             "cpu_mt": {"build_two_trees_s": ma + mb, "diff_s": md, "cores": thr}}}
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


_RESULT_OUT = None


def emit(out):
    """The one JSON result line, on the process's original stdout (see main)."""
    f = _RESULT_OUT or sys.stdout
    f.write(json.dumps(out) + "\n")
    f.flush()


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes (one per GPU) through
    torch.distributed.run as a child process — this parent never touches the GPU — forward rank 0's
    JSON line and fail unless every rank succeeded and the line reports n_gpus == N."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "16")
    log(f"bench: launching {n} ranks: {' '.join(cmd)}")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)  # stderr streams through
    lines = []
    for line in p.stdout.splitlines():
        line = line.strip()
        if not line.startswith("{"):
            if line:
                log(line)
            continue
        try:
            d = json.loads(line)
        except ValueError:
            log(line)
            continue
        if isinstance(d, dict) and "metric" in d:
            lines.append(line)
    if p.returncode != 0:
        log(f"bench: rank launcher exited with {p.returncode}")
        return p.returncode or 1
    if len(lines) != 1:
        log(f"bench: expected one result line from rank 0, got {len(lines)}")
        return 1
    if json.loads(lines[0]).get("n_gpus") != n:
        log("bench: result line does not report n_gpus == --gpus")
        return 1
    sys.stdout.write(lines[0] + "\n")
    sys.stdout.flush()
    return 0


def main():
    global _RESULT_OUT
    # The result line is the only thing on stdout: fd 1 is pointed at stderr for the rest of the process,
    # so banners the communication libraries print (RCCL's version block, gloo's peer counts) land there.
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
    ap.add_argument("--no-diff", action="store_true", help="build workload: skip the secondary blocks")
    ap.add_argument("--no-big", action="store_true", help="build workload: skip the configs4 / 1B-key blocks")
    ap.add_argument("--diff-records", type=int, default=100_000_000, help="build workload: diff_100m keys")
    ap.add_argument("--anchor-records", type=int, default=125_000_000,
                    help="build workload: the 125M-per-GPU block (N=1 anchor_125m, N>1 sharded_125m_per_rank; "
                         "0 = skip)")
    ap.add_argument("--route-records", type=int, default=None,
                    help="build workload with a process group: also time the all-to-all redistribution of "
                         "this many unpartitioned records per rank (SURVEY 8f-3; default 10M at N>1; 0 = skip)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))  # before anything touches the GPU
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}")
    if args.route_records is None:
        args.route_records = 10_000_000 if int(os.environ.get("WORLD_SIZE", "1")) > 1 else 0
    if args.n is None:
        # the same work per rank at every N (weak scaling against the N = 1 line); the 125M-per-rank
        # sharded build (configs[3] at N = 8) is the sharded_125m_per_rank block of the N > 1 line
        args.n = {"build": 10_000_000, "diff": 100_000_000, "incremental": 125_000_000}[args.workload]
    ctx = Ctx()
    {"build": wl_build, "diff": wl_diff, "incremental": wl_incremental}[args.workload](ctx, args)
    ctx.finish()


if __name__ == "__main__":
    main()
