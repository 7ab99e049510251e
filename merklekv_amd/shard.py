"""Sharded (multi-GPU) trees: one process per GPU, contiguous key ranges ordered by rank.

SURVEY.md §8e. The protocol runs INSIDE the C library (csrc/comm.cpp; include/mkv_merkle.h
mkv_sharded_*): hash + sort + dedup of the rank's range, ONE all-gather of the 8-B leaf counts, the range
check, in-shard reduction, ONE all-gather of the <= 6 KiB seam fringes, device seam combine. Every rank
ends with the same global root, bit-exact with the single-tree root. This module is the thin caller: it
gets the communicator of a torch.distributed group (merklekv_amd.comm.Comm.from_dist: RCCL over xGMI
when the collective device is a GPU and the backend "nccl", else the host form over gloo) and calls
MerkleTree.sharded_build / sharded_root_many / sharded_diff. Collective timings are read back from the
communicator into `coll_stats`.

Range check: the seam protocol is exact only if rank r holds a contiguous key range below rank r+1's
(the reference keeps one leaf per key, last write wins). `validate=True` makes every rank check that
last(r) < first(next non-empty rank) and raise otherwise.

Trees without the C entry points (tests/shard_model.ModelShardTree: a pure-Python model of the shard_*
steps) run the same protocol here step by step over torch.distributed, so the CPU tests exercise the
orchestration and the seam math without a GPU.

Redistribution: `redistribute` moves records that sit on the ranks in no key order into
key-range shards with one all-to-all (route kernels in csrc/k_route.hip); `sharded_root_unpartitioned`
chains it with the sharded build.
"""
from __future__ import annotations

import numpy as np

from dataclasses import dataclass

from ._lib import FRINGE_BYTES

_bufs: dict = {}

# Wall time of each collective kind (host clock around the collective and the wait for its result):
# name -> [seconds, calls, payload bytes per rank]. Read by bench.py (per-collective timings).
coll_stats: dict = {}
# Library communicator only: name -> [host-staged payload bytes, meta bytes] (mkv_comm_traffic).
coll_traffic: dict = {}


def _coll_add(name: str, secs: float, nbytes: int) -> None:
    s = coll_stats.setdefault(name, [0.0, 0, 0])
    s[0] += secs
    s[1] += 1
    s[2] += int(nbytes)


def coll_stats_reset() -> None:
    coll_stats.clear()
    coll_traffic.clear()


def _is_gpu(device) -> bool:
    import torch
    return device is not None and torch.device(device).type == "cuda"


def _buf(device, tag: str, nbytes: int):
    """Cached device byte buffer (stable across steps: no allocator churn inside the timed loop)."""
    import torch
    key = (str(device), tag)
    b = _bufs.get(key)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
        _bufs[key] = b
    return b


def _all_gather_bytes(dist, payload: bytes, device, group=None) -> list[bytes]:
    """All-gather of equal-size host byte payloads (host path: gloo / CPU tests, one-off metadata)."""
    import torch
    world = dist.get_world_size(group)
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=device)
    if hasattr(dist, "all_gather_into_tensor") and _is_gpu(device):
        dist.all_gather_into_tensor(out, t, group=group)
    else:  # gloo has no all_gather_into_tensor on some versions
        dist.all_gather(list(out.chunk(world)), t, group=group)
    raw = out.cpu().numpy().tobytes()
    k = t.numel()
    return [raw[r * k:(r + 1) * k] for r in range(world)]


def shard_counts(dist, n_local: int, device, group=None) -> list[int]:
    """All-gather of the 8-byte leaf counts; the host needs them (offsets plan the levels)."""
    import time

    import torch
    t0 = time.perf_counter()
    if _is_gpu(device):
        world = dist.get_world_size(group)
        src = torch.full((1,), int(n_local), dtype=torch.int64, device=device)
        out = torch.empty(world, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(out, src, group=group)
        res = [int(x) for x in out.tolist()]
    else:
        raw = _all_gather_bytes(dist, np.array([n_local], dtype=np.uint64).tobytes(), device, group)
        res = [int(np.frombuffer(r, dtype=np.uint64)[0]) for r in raw]
    _coll_add("counts_all_gather", time.perf_counter() - t0, 8)
    return res


def check_ranges(tree, counts: list[int], dist, device, group=None) -> None:
    """Raise ValueError unless the shards hold disjoint contiguous key ranges ordered by rank (every
    non-empty shard's last key < the next non-empty shard's first key; Rust str order = bytes order)."""
    rank = dist.get_rank(group)
    n = counts[rank]
    ends = tree.keys_at([0, n - 1]) if n else [b"", b""]
    lens = _all_gather_bytes(dist, np.array([len(ends[0]), len(ends[1])], dtype=np.uint64).tobytes(), device, group)
    width = max(int(x) for r in lens for x in np.frombuffer(r, dtype=np.uint64)) or 1
    pay = ends[0].ljust(width, b"\0") + ends[1].ljust(width, b"\0")
    got = _all_gather_bytes(dist, pay, device, group)
    prev_last, prev_rank = None, None
    for r, (lr, raw) in enumerate(zip(lens, got)):
        if counts[r] == 0:
            continue
        l0, l1 = (int(x) for x in np.frombuffer(lr, dtype=np.uint64))
        first, last = raw[:l0], raw[width:width + l1]
        if prev_last is not None and not prev_last < first:
            raise ValueError(f"shard key ranges overlap or are out of rank order: rank {prev_rank} ends at "
                             f"{prev_last!r}, rank {r} starts at {first!r} (the seam protocol needs contiguous "
                             f"key ranges ordered by rank)")
        prev_last, prev_rank = last, r


def _native(*trees) -> bool:
    return all(hasattr(t, "sharded_build") for t in trees)


def _comm(dist, device, group):
    from .comm import Comm
    return Comm.from_dist(dist, device, group)


def _absorb(comm) -> None:
    """Move the communicator's collective timings (and host <-> device bytes: coll_traffic) into
    coll_stats."""
    for name, (staged, meta) in comm.traffic().items():
        if staged or meta:
            s = coll_traffic.setdefault(name, [0, 0])
            s[0] += int(staged)
            s[1] += int(meta)
    for name, (secs, calls, nbytes) in comm.stats(reset=True).items():
        if calls:
            s = coll_stats.setdefault(name, [0.0, 0, 0])
            s[0] += secs
            s[1] += calls
            s[2] += int(nbytes)


def sharded_root(tree, keys, values, dist, device="cpu", group=None, on_device: bool = False,
                 validate: bool = True):
    """Build this rank's shard of the global tree and return (global root or None, counts)."""
    if _native(tree):
        comm = _comm(dist, device, group)
        try:
            counts = tree.sharded_build(comm, keys, values, on_device=on_device, range_check=validate)
        except Exception as e:
            _absorb(comm)
            if "key ranges overlap" in str(e):
                raise ValueError(str(e)) from e
            raise
        _absorb(comm)
        return tree.get_root_hash(), counts
    rank = dist.get_rank(group)
    n_local = tree.shard_prepare(keys, values, on_device=on_device)
    counts = shard_counts(dist, n_local, device, group)
    if validate:
        check_ranges(tree, counts, dist, device, group)
    offset, total = sum(counts[:rank]), sum(counts)
    tree.shard_reduce(offset, total)
    return shard_recombine_many([tree], dist, total, device, group)[0], counts


def sequential_root(tree, shard_blobs, global_n: int):
    """Global root of key-range shards built one after another on ONE GPU (configs[3]'s 1B keys on a single
    MI355X: 8 x 125M records never reside together; each shard's records and scratch can be dropped before
    the next one is produced). Per shard g, in key order: mkv_shard_prepare (hash + sort + dedup) ->
    mkv_shard_reduce at offset o_g = the leaves of shards < g inside a tree of global_n leaves ->
    mkv_shard_fringe (<= MKV_FRINGE_BYTES to the host); then one mkv_shard_combine of every fringe —
    rebuild() over the union (/root/reference/src/store/merkle.rs:73-121). shard_blobs yields
    (kb, koff, vb, voff, n) device blobs (tensors or pointers); it may generate each shard lazily.
    global_n is the total leaf count after dedup; a mismatch (duplicate keys inside a shard) raises
    ValueError, because the offsets of later shards would have been wrong. Returns (root, counts)."""
    counts, fringes = [], []
    off = 0
    for blob in shard_blobs:
        n_g = tree.shard_prepare(blob, None, on_device=True)
        if off + n_g > global_n:
            raise ValueError(f"shards hold more than global_n = {global_n} leaves")
        tree.shard_reduce(off, global_n)
        fringes.append(tree.shard_fringe())
        counts.append(n_g)
        off += n_g
    if off != global_n:
        raise ValueError(f"shards hold {off} leaves, not global_n = {global_n}")
    return tree.shard_combine(b"".join(fringes), len(fringes), global_n), counts


def sequential_diff(ta, tb, shard_pairs, global_na: int, global_nb: int):
    """diff_keys of two key-range-sharded replicas (configs[2] x configs[3]: two 1B-key trees) on ONE GPU,
    shard after shard — what 8 ranks do in parallel, each with its own range (sync.rs:67-83 consumes the
    global list). Per shard g in key order: shard_prepare + shard_reduce of both replicas at their global
    offsets (A: o_g inside a tree of global_na leaves, B likewise; offsets are the leaf counts of the
    shards before g), both fringes kept, then the shard-local diff_keys (merkle.rs:171-196): the top-down
    walk from the fringe roots when the two shard plans match, the merge-join otherwise. Ranges are
    ordered, so the per-shard lists concatenate into the global sorted list at the offsets given by their
    counts. shard_pairs yields ((kb, koff, vb, voff, n) of A, same of B) device blobs, possibly generated
    lazily into reused buffers (the trees own copies of their keys).
    Returns (root_a, root_b, [(raw, offs) per shard], [global offset per shard], [diff ms per shard])."""
    import time
    fa, fb, lists, offs, ms = [], [], [], [], []
    oa = ob = at = 0
    for blob_a, blob_b in shard_pairs:
        na = ta.shard_prepare(blob_a, None, on_device=True)
        ta.shard_reduce(oa, global_na)
        fa.append(ta.shard_fringe())
        nb = tb.shard_prepare(blob_b, None, on_device=True)
        tb.shard_reduce(ob, global_nb)
        fb.append(tb.shard_fringe())
        t0 = time.perf_counter()
        raw, o = ta.diff_keys_packed(tb)
        ms.append((time.perf_counter() - t0) * 1e3)
        lists.append((raw, o))
        offs.append(at)
        at += len(o) - 1
        oa += na
        ob += nb
    if oa != global_na or ob != global_nb:
        raise ValueError(f"shards hold {oa} / {ob} leaves, not {global_na} / {global_nb}")
    ra = ta.shard_combine(b"".join(fa), len(fa), global_na)
    rb = tb.shard_combine(b"".join(fb), len(fb), global_nb)
    return ra, rb, lists, offs, ms


def sequential_incremental(shards, global_n: int, replicas: int, warmup: bool = True, device: int = 0):
    """configs[4] at its full size on ONE GPU: a 1B-key tree as key-range shards, base + (replicas - 1)
    variants, each variant applying its own value batch in every shard (1M keys per variant over 8 shards
    of 125K), shard after shard — the 8-rank form runs the shards in parallel. Per shard g: the base shard
    built at its global offset (shard_prepare + shard_reduce), cloned per variant; a STEP = every variant's
    batch through one upsert_device_many (dirty path: merkle.rs:52-56 then the climb) + the base diffed
    against all variants in one shared walk (diff_keys_many, merkle.rs:171-196); the first step is a warm-up
    when `warmup` (the same batches applied again leave the trees and the diffs unchanged); then every
    replica's fringe is kept. After the last shard, each replica's global root is the seam combine of its
    fringes (the recombine the ranks do over RCCL). shards yields ((kb, koff, vb, voff, n) base blob,
    [(kb, koff, vb, voff, m) batch per variant]) device tensors.
    Returns (roots [base, variants...], per-variant [(raw, offs) per shard], [step ms per shard])."""
    import time

    from .merkle import MerkleTree
    fr = [[] for _ in range(replicas)]
    lists = [[] for _ in range(replicas - 1)]
    ms = []
    off = 0
    for blob, batches in shards:
        base = MerkleTree(device)
        n_g = base.shard_prepare(blob, None, on_device=True)
        base.shard_reduce(off, global_n)
        variants = [base.clone() for _ in range(replicas - 1)]
        ptrs = [tuple(x.data_ptr() if hasattr(x, "data_ptr") else x for x in b) for b in batches]

        def step():
            MerkleTree.upsert_device_many(variants, ptrs)
            return base.diff_keys_many_packed(variants)

        if warmup:
            step()
        t0 = time.perf_counter()
        diffs = step()
        ms.append((time.perf_counter() - t0) * 1e3)
        for i, d in enumerate(diffs):
            lists[i].append(d)
        for i, t in enumerate([base] + variants):
            fr[i].append(t.shard_fringe())
        off += n_g
        del base, variants
    if off != global_n:
        raise ValueError(f"shards hold {off} leaves, not global_n = {global_n}")
    holder = MerkleTree(device)
    roots = [holder.shard_combine(b"".join(f), len(f), global_n) for f in fr]
    return roots, lists, ms


def shard_recombine_many(trees, dist, total: int, device="cpu", group=None) -> list:
    """Fringe all-gather + seam combine for k trees (replicas of one key range) in ONE collective:
    after in-place updates (MerkleTree.upsert / upsert_device of keys in the rank's range: the dirty
    path) or after shard_reduce. Returns the k global roots."""
    trees = list(trees)
    k = len(trees)
    if k == 0:
        return []
    if _native(*trees):
        comm = _comm(dist, device, group)
        roots = type(trees[0]).sharded_root_many(trees, comm)
        _absorb(comm)
        return roots
    world = dist.get_world_size(group)
    if _is_gpu(device) and all(hasattr(t, "shard_fringe_device") for t in trees):
        import torch
        src = _buf(device, "fr_in", k * FRINGE_BYTES)
        dst = _buf(device, "fr_out", world * k * FRINGE_BYTES)
        base = src.data_ptr()
        for i, t in enumerate(trees):
            t.shard_fringe_device(base + i * FRINGE_BYTES)  # complete on return
        import time
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(dst[:world * k * FRINGE_BYTES], src[:k * FRINGE_BYTES], group=group)
        torch.cuda.current_stream(device).synchronize()  # the library runs on its own streams
        _coll_add("fringe_all_gather", time.perf_counter() - t0, k * FRINGE_BYTES)
        out = dst.data_ptr()
        return [t.shard_combine_device(out + i * FRINGE_BYTES, world, k * FRINGE_BYTES, total)
                for i, t in enumerate(trees)]
    blocks = _all_gather_bytes(dist, b"".join(t.shard_fringe() for t in trees), device, group)
    return [t.shard_combine(b"".join(b[i * FRINGE_BYTES:(i + 1) * FRINGE_BYTES] for b in blocks), world, total)
            for i, t in enumerate(trees)]


def shard_recombine(tree, dist, total: int, device="cpu", group=None):
    """shard_recombine_many for one tree."""
    return shard_recombine_many([tree], dist, total, device, group)[0]


def sharded_diff(a, b, dist, device="cpu", group=None):
    """diff_keys (merkle.rs:171-196) of two sharded trees with the same key-range partition: each rank
    diffs its own range on the device (top-down when the shard plans match, merge-join when the key sets
    differ), then the divergence counts are all-gathered (8 B/rank) so every rank knows where its keys
    sit in the global sorted list (ranges are ordered by rank, so the concatenation is sorted).
    Returns (this rank's packed keys (bytes array, offsets), global offset, global count)."""
    if _native(a, b):  # the library's own slice + offset (mkv_sharded_diff_local: one 32-B all-gather)
        comm = _comm(dist, device, group)
        kl, off, tot = a.sharded_diff_local(b, comm)
        _absorb(comm)
        return (kl.raw.copy(), kl.offs.copy()), off, tot
    rank = dist.get_rank(group)
    raw, offs = a.diff_keys_packed(b)
    counts = shard_counts(dist, len(offs) - 1, device, group)
    return (raw, offs), sum(counts[:rank]), sum(counts)


def sharded_diff_gather(a, b, dist, device="cpu", group=None):
    """diff_keys (merkle.rs:171-196) of two sharded trees as ONE sorted list on every rank — what
    SyncManager::sync_once consumes whole (sync.rs:67-83). Each rank diffs its own key range on the
    device, then an all-gather-v of the divergent keys: one all-gather of (count, bytes) per rank, one
    all-gather of [u32 key lengths | key bytes] blocks padded to the largest rank's (RCCL over xGMI on a
    GPU group). Ranges are ordered by rank, so the rank-order concatenation is already sorted and unique.
    Returns (key bytes uint8, offsets uint64[n+1])."""
    import time

    import torch
    if _native(a, b):
        comm = _comm(dist, device, group)
        kl = a.sharded_diff(b, comm)
        _absorb(comm)
        return kl.raw.copy(), kl.offs.copy()
    world = dist.get_world_size(group)
    raw, offs = a.diff_keys_packed(b)
    n, nb = len(offs) - 1, int(offs[-1])
    gpu = _is_gpu(device)
    t0 = time.perf_counter()
    meta = _all_gather_tensor(dist, torch.tensor([n, nb], dtype=torch.int64, device=device), group)
    meta = meta.cpu().numpy().reshape(world, 2)
    mn, mb = int(meta[:, 0].max()), int(meta[:, 1].max())
    blk = 4 * mn + mb
    if blk == 0:
        _coll_add("diff_all_gather_v", time.perf_counter() - t0, 16)
        return np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    pay = np.zeros(blk, np.uint8)
    pay[:4 * n].view(np.uint32)[:] = np.diff(offs).astype(np.uint32)
    pay[4 * mn:4 * mn + nb] = raw[:nb]
    src = torch.from_numpy(pay)
    if gpu:
        src = src.to(device, non_blocking=False)
    allp = _all_gather_tensor(dist, src, group).cpu().numpy().reshape(world, blk)
    _coll_add("diff_all_gather_v", time.perf_counter() - t0, 16 + blk)
    lens = np.concatenate([allp[r, :4 * int(meta[r, 0])].view(np.uint32) for r in range(world)])
    out = np.concatenate([allp[r, 4 * mn:4 * mn + int(meta[r, 1])] for r in range(world)])
    o = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, dtype=np.uint64, out=o[1:])
    return out, o


# ---------------------------------------------------------------------------------------------------
# Redistribution of unpartitioned input (SURVEY §8f-3, §8e "sampled splitters")
# ---------------------------------------------------------------------------------------------------
def _backend(dist, group) -> str:
    try:
        return str(dist.get_backend(group)).lower()
    except Exception:  # pragma: no cover - non-default group objects
        return ""


def _all_gather_tensor(dist, t, group=None):
    """All-gather of equal-size tensors into one (world * numel) tensor on t's device."""
    import torch
    world = dist.get_world_size(group)
    if _is_gpu(t.device) and _backend(dist, group) == "nccl":
        out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out
    src = t.cpu()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    return torch.cat(parts).to(t.device)


def _all_to_all(dist, out, inp, out_splits, in_splits, group=None) -> None:
    """all_to_all_single over RCCL for device tensors; staged through host memory for gloo."""
    import time
    outs = [int(x) for x in out_splits]
    ins = [int(x) for x in in_splits]
    t0 = time.perf_counter()
    if _is_gpu(out.device) and _backend(dist, group) == "nccl":
        dist.all_to_all_single(out, inp, outs, ins, group=group)
        import torch
        torch.cuda.current_stream(out.device).synchronize()
    else:
        o = out.cpu() if _is_gpu(out.device) else out
        dist.all_to_all_single(o, inp.cpu(), outs, ins, group=group)
        if o is not out:
            out.copy_(o)
    _coll_add("all_to_all", time.perf_counter() - t0, inp.numel() * inp.element_size())


@dataclass
class Routed:
    """This rank's key range after redistribute: device blobs (kb, koff int64, vb, voff int64) of n
    records ordered by (source rank, source position), and the splitters that cut the ranges."""
    kb: object
    koff: object
    vb: object
    voff: object
    n: int
    splitters: np.ndarray
    sent: np.ndarray      # (world, 3) records / key bytes / value bytes this rank sent to each rank
    received: np.ndarray  # (world, 3) the same, received from each rank

    def blobs(self):
        return (self.kb, self.koff, self.vb, self.voff, self.n)


def redistribute(tree, kb, koff, vb, voff, n: int, dist, device, group=None, samples: int = 4096) -> Routed:
    """Move this rank's n records (device tensors: kb/vb uint8, koff/voff int64 with n + 1 entries, in any
    key order) so that rank r ends with exactly the records of key range r, ranges ordered by rank.

    1. all-gather the record counts; rank r contributes m_r ~ samples * n_r / N evenly spaced key
       prefixes (so the splitters follow the global key distribution), all-gathered;
    2. every rank derives the same world-1 splitters from the gathered samples (mkv_route_splitters);
    3. route_plan: destination of every record + per-destination totals; the (world x world x 3) plan
       matrix is all-gathered so every rank knows its receive sizes;
    4. route_pack into send buffers grouped by destination, then one all-to-all each for key bytes,
       key lengths, value bytes and value lengths (RCCL over xGMI on a GPU group);
    5. route_offsets rebuilds the offsets of the received blobs.
    """
    import torch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = kb.device  # the records' GPU: every buffer the library touches lives there; `device` is the
    # collective device (cpu for gloo), the helpers stage through it as needed
    counts = shard_counts(dist, n, device, group)
    N = sum(counts)
    m = [min(c, -(-samples * c // N)) if N else 0 for c in counts]
    # torch.empty: no fill kernel on torch's stream racing the library's sample writes (the padding
    # beyond m[rank] is never read)
    loc = torch.empty(max(max(m), 1), dtype=torch.int64, device=dev)
    if m[rank]:
        tree.route_sample(kb, koff, n, m[rank], loc)
    gathered = _all_gather_tensor(dist, loc, group).cpu().numpy().view(np.uint64)
    L = loc.numel()
    smp = np.concatenate([gathered[r * L:r * L + m[r]] for r in range(world)]) if N else np.zeros(0, np.uint64)
    from .merkle import route_splitters
    spl = route_splitters(smp, world)
    plan = np.ascontiguousarray(tree.route_plan(kb, koff, vb, voff, n, spl), dtype=np.uint64)
    allp = _all_gather_tensor(dist, torch.from_numpy(plan.view(np.int64).reshape(-1).copy()).to(dev), group)
    allp = allp.cpu().numpy().view(np.uint64).reshape(world, world, 3)  # [source][destination]
    recv = np.ascontiguousarray(allp[:, rank, :])
    kout = torch.empty(max(int(plan[:, 1].sum()), 1), dtype=torch.uint8, device=dev)
    vout = torch.empty(max(int(plan[:, 2].sum()), 1), dtype=torch.uint8, device=dev)
    klen = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    vlen = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    tree.route_pack(kb, koff, vb, voff, n, kout, klen, vout, vlen)
    nr = int(recv[:, 0].sum())
    rk = torch.empty(max(int(recv[:, 1].sum()), 1), dtype=torch.uint8, device=dev)
    rv = torch.empty(max(int(recv[:, 2].sum()), 1), dtype=torch.uint8, device=dev)
    rkl = torch.empty(max(nr, 1), dtype=torch.int32, device=dev)
    rvl = torch.empty(max(nr, 1), dtype=torch.int32, device=dev)
    # all_to_all_single splits along dim 0: give exact-size views (the buffers carry a 1-element floor)
    _all_to_all(dist, rk[:int(recv[:, 1].sum())], kout[:int(plan[:, 1].sum())], recv[:, 1], plan[:, 1], group)
    _all_to_all(dist, rkl[:nr], klen[:n], recv[:, 0], plan[:, 0], group)
    _all_to_all(dist, rv[:int(recv[:, 2].sum())], vout[:int(plan[:, 2].sum())], recv[:, 2], plan[:, 2], group)
    _all_to_all(dist, rvl[:nr], vlen[:n], recv[:, 0], plan[:, 0], group)
    if _is_gpu(dev):
        torch.cuda.current_stream(dev).synchronize()  # the library runs on its own streams
    rko = torch.empty(nr + 1, dtype=torch.int64, device=dev)
    rvo = torch.empty(nr + 1, dtype=torch.int64, device=dev)
    tree.route_offsets(rkl, nr, rko)
    tree.route_offsets(rvl, nr, rvo)
    return Routed(rk, rko, rv, rvo, nr, spl, plan, recv)


def sharded_root_unpartitioned(tree, kb, koff, vb, voff, n: int, dist, device, group=None,
                               samples: int = 4096, validate: bool = True):
    """redistribute + sharded_root: the global root of the union of every rank's records (duplicates
    resolved in rank order), from input in no key order. Returns (root, counts, Routed); keep the Routed
    alive while the tree may still read its blobs (the shard build copies what it keeps)."""
    routed = redistribute(tree, kb, koff, vb, voff, n, dist, device, group, samples)
    root, counts = sharded_root(tree, routed.blobs(), None, dist, device, group, on_device=True,
                                validate=validate)
    return root, counts, routed
