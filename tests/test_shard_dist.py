"""Multi-process (gloo, CPU) tests of the sharded build protocol: merklekv_amd/shard.py orchestration
(all-gather of counts and seam fringes) over a model shard tree; the global root must equal the
unsharded root for uneven, odd-aligned, tiny and empty shards."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from oracle.merkle_oracle import PyMerkleTree
from tests.shard_model import ModelShardTree, plan_levels


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split(keys, cuts):
    ks = sorted(keys)
    out, prev = [], 0
    for c in list(cuts) + [len(ks)]:
        out.append(ks[prev:c])
        prev = c
    return out


def _worker(rank, world, port, shards, values, q):
    import torch.distributed as dist

    from merklekv_amd.shard import sharded_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = shards[rank]
        root, counts = sharded_root(ModelShardTree(), keys, [values[k] for k in keys], dist, device="cpu")
        q.put((rank, root, counts))
    finally:
        dist.destroy_process_group()


def _run(world, shards, values):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shards, values, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world,n,cuts", [
    (2, 1000, [500]),
    (2, 1001, [333]),
    (3, 777, [1, 400]),
    (2, 64, [0]),          # empty first shard
    (3, 5, [2, 2]),        # empty middle shard
])
def test_sharded_root_matches_unsharded_gloo(world, n, cuts):
    keys = [b"key%05d" % i for i in range(n)]
    values = {k: b"val" + k for k in keys}
    ref = PyMerkleTree()
    for k in keys:
        ref.insert(k, values[k])
    shards = _split(keys, cuts)
    res = _run(world, shards, values)
    for rank, root, counts in res:
        assert counts == [len(s) for s in shards]
        assert root == ref.get_root_hash(), rank


def _worker_update(rank, world, port, shards, values, updates, q):
    import torch.distributed as dist

    from merklekv_amd.shard import shard_recombine, sharded_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = shards[rank]
        t = ModelShardTree()
        root0, counts = sharded_root(t, keys, [values[k] for k in keys], dist, device="cpu")
        mine = [(k, v) for k, v in updates if k in set(keys)]
        if mine:
            t.upsert([k for k, _ in mine], [v for _, v in mine])
        root1 = shard_recombine(t, dist, sum(counts), device="cpu")
        q.put((rank, root0, root1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,cuts", [(2, 1001, [333]), (3, 777, [1, 400]), (3, 50, [0, 49])])
def test_sharded_update_recombine_gloo(world, n, cuts):
    """Incremental anti-entropy on shards (configs[4]): each rank applies the value updates of its own
    key range, then shard_recombine (fringe all-gather + seam combine) gives the updated global root."""
    keys = [b"key%05d" % i for i in range(n)]
    values = {k: b"val" + k for k in keys}
    updates = [(keys[i], b"new%d" % i) for i in range(0, n, 7)] + [(keys[-1], b"last"), (keys[0], b"first")]
    ref = PyMerkleTree()
    for k in keys:
        ref.insert(k, values[k])
    root0 = ref.get_root_hash()
    for k, v in updates:
        ref.insert(k, v)
    shards = _split(keys, cuts)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_update, args=(r, world, port, shards, values, updates, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, r0, r1 in res:
        assert r0 == root0 and r1 == ref.get_root_hash(), rank


def test_seam_model_exhaustive_small():
    """Every split point of every size up to 40 into 2 and 3 shards (no processes)."""
    import itertools
    for n in range(1, 41):
        keys = [b"k%03d" % i for i in range(n)]
        ref = PyMerkleTree()
        for k in keys:
            ref.insert(k, k)
        want = ref.get_root_hash()
        for g in (2, 3):
            for cuts in itertools.combinations(range(n + 1), g - 1):
                shards = _split(keys, cuts)
                trees = [ModelShardTree() for _ in shards]
                counts = [t.shard_prepare(s, s) for t, s in zip(trees, shards)]
                fr = b""
                for r, t in enumerate(trees):
                    t.shard_reduce(sum(counts[:r]), n)
                    fr += t.shard_fringe()
                for t in trees:
                    assert t.shard_combine(fr, g, n) == want, (n, cuts)


def test_plan_levels_single_shard_is_whole_tree():
    for n in (1, 2, 3, 7, 1000, 1025):
        p = plan_levels(0, n, n)
        s, sizes = n, []
        while True:
            sizes.append(s)
            if s == 1:
                break
            s = (s + 1) // 2
        assert [c for _, c, _ in p] == sizes and [b for b, _, _ in p] == [0] * len(sizes)


def _worker_generic(rank, world, port, fn, args, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, dist, *args)))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, ("error", type(e).__name__, str(e))))
    finally:
        dist.destroy_process_group()


def _run_fn(world, fn, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_generic, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [v for _, v in sorted(res, key=lambda x: x[0])]


def _fn_overlap(rank, dist, shards, values):
    from merklekv_amd.shard import sharded_root
    keys = shards[rank]
    root, _ = sharded_root(ModelShardTree(), keys, [values[k] for k in keys], dist, device="cpu")
    return root


def test_sharded_root_rejects_overlapping_ranges_gloo():
    """hash-partitioned / overlapping shards would silently give a root that differs from
    merkle.rs; the range check must refuse them on every rank."""
    keys = [b"key%05d" % i for i in range(100)]
    values = {k: k for k in keys}
    bad = [keys[0::2], keys[1::2]]           # interleaved (hash-like) partition
    res = _run_fn(2, _fn_overlap, bad, values)
    assert all(isinstance(r, tuple) and r[0] == "error" and r[1] == "ValueError" for r in res), res
    dup = [keys[:60], keys[50:]]             # overlapping ranges (a key on two ranks)
    res = _run_fn(2, _fn_overlap, dup, values)
    assert all(isinstance(r, tuple) and r[1] == "ValueError" for r in res), res
    ok = [keys[:60], keys[60:]]
    ref = PyMerkleTree()
    for k in keys:
        ref.insert(k, values[k])
    assert _run_fn(2, _fn_overlap, ok, values) == [ref.get_root_hash()] * 2


def _fn_recombine_many(rank, dist, shards, values, updates):
    from merklekv_amd.shard import shard_recombine_many, sharded_root
    keys = shards[rank]
    trees = []
    for r in range(3):  # three replicas of this rank's range
        t = ModelShardTree()
        _, counts = sharded_root(t, keys, [values[k] for k in keys], dist, device="cpu")
        trees.append(t)
    for t, ups in zip(trees, updates):
        mine = [(k, v) for k, v in ups if k in set(keys)]
        if mine:
            t.upsert([k for k, _ in mine], [v for _, v in mine])
    return shard_recombine_many(trees, dist, sum(counts), device="cpu")


def test_sharded_recombine_many_one_collective_gloo():
    """k replicas' fringes share one all-gather (bench configs[4] at N>1); every root must equal the
    unsharded root of that replica's updated records."""
    n = 901
    keys = [b"key%05d" % i for i in range(n)]
    values = {k: b"v" + k for k in keys}
    updates = [[(keys[i], b"u%d" % r) for i in range(r, n, 5 + r)] for r in range(3)]
    want = []
    for ups in updates:
        ref = PyMerkleTree()
        for k in keys:
            ref.insert(k, values[k])
        for k, v in ups:
            ref.insert(k, v)
        want.append(ref.get_root_hash())
    for world, cuts in ((2, [450]), (3, [1, 600])):
        res = _run_fn(world, _fn_recombine_many, _split(keys, cuts), values, updates)
        assert all(r == want for r in res), (world, cuts)


def _fn_sharded_diff(rank, dist, shards_a, shards_b, values_a, values_b):
    from merklekv_amd.shard import sharded_diff, sharded_root
    a, b = ModelShardTree(), ModelShardTree()
    sharded_root(a, shards_a[rank], [values_a[k] for k in shards_a[rank]], dist, device="cpu")
    sharded_root(b, shards_b[rank], [values_b[k] for k in shards_b[rank]], dist, device="cpu")
    (raw, offs), off, tot = sharded_diff(a, b, dist, device="cpu")
    b_ = raw.tobytes()
    return [b_[int(offs[i]):int(offs[i + 1])] for i in range(len(offs) - 1)], off, tot


def test_sharded_mixed_diff_gloo():
    """Global diff of two sharded replicas with value changes, deletions and insertions per shard (the
    shards' leaf counts differ, so each rank merge-joins its range): the rank-ordered concatenation
    equals the unsharded diff (merkle.rs:171-196)."""
    n = 1200
    keys = [b"key%05d" % i for i in range(n)]
    va = {k: b"a" + k for k in keys}
    vb = dict(va)
    for i in range(0, n, 37):
        vb[keys[i]] = b"changed"
    for i in range(5, n, 101):
        vb.pop(keys[i])
    for i in range(0, n, 149):
        vb[keys[i] + b"+new"] = b"inserted"
    splitter = [keys[400], keys[800]]
    def part(ks):
        ks = sorted(ks)
        return [[k for k in ks if k < splitter[0]], [k for k in ks if splitter[0] <= k < splitter[1]],
                [k for k in ks if k >= splitter[1]]]
    ra, rb = PyMerkleTree(), PyMerkleTree()
    for k, v in va.items():
        ra.insert(k, v)
    for k, v in vb.items():
        rb.insert(k, v)
    want = ra.diff_keys(rb)
    res = _run_fn(3, _fn_sharded_diff, part(va), part(vb), va, vb)
    got = []
    for keys_r, off, tot in res:
        assert off == len(got) and tot == len(want)
        got += keys_r
    assert got == want


def _fn_redistribute(rank, dist, inputs, samples):
    import numpy as np
    import torch

    from merklekv_amd.shard import sharded_root_unpartitioned
    from tests.shard_model import ModelShardTree, torch_u8
    keys, vals = inputs[rank]
    kb, vb = torch_u8(b"".join(keys)), torch_u8(b"".join(vals))
    ko = torch.tensor([0] + list(np.cumsum([len(k) for k in keys], dtype=np.int64)), dtype=torch.int64)
    vo = torch.tensor([0] + list(np.cumsum([len(v) for v in vals], dtype=np.int64)), dtype=torch.int64)
    t = ModelShardTree()
    root, counts, routed = sharded_root_unpartitioned(t, kb, ko, vb, vo, len(keys), dist, "cpu", samples=samples)
    return root, counts, list(t.keys), [int(x) for x in routed.splitters], routed.sent.tolist()


def _unpartitioned_inputs(world, seed, n_per_rank, empty_rank=None):
    """Keys in no order on every rank: random suffixes under a few long shared prefixes (ties on the
    8-byte routing prefix), short and empty keys, and duplicates across and within ranks."""
    import random
    rng = random.Random(seed)
    pool = [b"tenant/%04d/object/%06d" % (rng.randrange(3), rng.randrange(10 ** 6)) for _ in range(3 * n_per_rank)]
    pool += [b"", b"a", b"ab", b"tenant/", b"tenant/0", b"zz", b"\x00", b"\xff\xfe"]
    pool += [b"k%05d" % rng.randrange(10 ** 5) for _ in range(2 * n_per_rank)]
    inputs = []
    for r in range(world):
        if r == empty_rank:
            inputs.append(([], []))
            continue
        ks = [rng.choice(pool) for _ in range(n_per_rank)]
        inputs.append((ks, [b"v%d/%d/%d" % (r, i, rng.randrange(99)) for i in range(len(ks))]))
    return inputs


@pytest.mark.parametrize("world,n,empty,samples", [(2, 300, None, 64), (3, 250, 1, 16), (3, 40, None, 4096)])
def test_redistribute_unpartitioned_gloo(world, n, empty, samples):
    """records in no key order on every rank are routed into key-range shards with one
    all-to-all; the sharded root equals the root of all ranks' records inserted in rank order (duplicates:
    last write wins), each rank's range is contiguous, and equal 8-byte prefixes meet on one rank."""
    inputs = _unpartitioned_inputs(world, 1234 + world * n, n, empty)
    ref = PyMerkleTree()
    for ks, vs in inputs:
        for k, v in zip(ks, vs):
            ref.insert(k, v)
    res = _run_fn(world, _fn_redistribute, inputs, samples)
    assert all(not (isinstance(r, tuple) and r and r[0] == "error") for r in res), res
    want_keys = sorted(ref.leaf_map)
    got_keys = []
    for r, (root, counts, keys, spl, sent) in enumerate(res):
        assert root == ref.get_root_hash(), r
        assert counts == [len(x[2]) for x in res]
        assert sum(row[0] for row in sent) == len(inputs[r][0])
        assert spl == res[0][3]
        got_keys += keys
    assert got_keys == want_keys


def test_route_splitters_host():
    """mkv_route_splitters is host code: runs without a GPU (the library loads on CPU)."""
    import numpy as np

    from merklekv_amd.merkle import route_splitters
    s = np.arange(1000, dtype=np.uint64)[::-1].copy()
    assert list(route_splitters(s, 4)) == [250, 500, 750]
    assert list(route_splitters(s, 1)) == []
    assert list(route_splitters(np.zeros(0, np.uint64), 3)) == [2 ** 64 - 1] * 2
    dup = np.array([5] * 10 + [9] * 2, np.uint64)
    assert list(route_splitters(dup, 3)) == [5, 5]


def _fn_diff_gather(rank, dist, shards_a, shards_b, values_a, values_b):
    from merklekv_amd.shard import coll_stats, sharded_diff_gather, sharded_root
    a, b = ModelShardTree(), ModelShardTree()
    sharded_root(a, shards_a[rank], [values_a[k] for k in shards_a[rank]], dist, device="cpu")
    sharded_root(b, shards_b[rank], [values_b[k] for k in shards_b[rank]], dist, device="cpu")
    raw, offs = sharded_diff_gather(a, b, dist, device="cpu")
    b_ = raw.tobytes()
    return [b_[int(offs[i]):int(offs[i + 1])] for i in range(len(offs) - 1)], dict(coll_stats)


@pytest.mark.parametrize("world,empty_b_rank", [(2, None), (3, None), (3, 1)])
def test_sharded_diff_gather_gloo(world, empty_b_rank):
    """the sharded diff assembled into ONE sorted list on every rank (all-gather-v of key
    lengths + bytes) equals diff_keys over the union (merkle.rs:171-196, consumed by sync.rs:67-83),
    including key-set changes at the shard seams (keys inserted right after a splitter, the first key of
    a range deleted) and a rank whose B range is empty."""
    n = 900
    keys = [b"key%05d" % i for i in range(n)]
    va = {k: b"a" + k for k in keys}
    vb = dict(va)
    cuts = [keys[n * (r + 1) // world] for r in range(world - 1)]
    for i in range(0, n, 41):
        vb[keys[i]] = b"changed"
    for c in cuts:
        vb.pop(c)                      # first key of the next range deleted on B
        vb[c + b"\x00"] = b"seam-new"  # new key right after the deleted one, same range
    vb[b"key"] = b"before-everything"  # new smallest key (rank 0)
    vb[b"zzz"] = b"after-everything"   # new largest key (last rank)
    bounds = [b""] + cuts + [None]

    def part(ks):
        ks = sorted(ks)
        return [[k for k in ks if bounds[r] <= k and (bounds[r + 1] is None or k < bounds[r + 1])]
                for r in range(world)]

    pa, pb = part(va), part(vb)
    if empty_b_rank is not None:
        for k in pb[empty_b_rank]:
            vb.pop(k)
        pb[empty_b_rank] = []
    ra, rb = PyMerkleTree(), PyMerkleTree()
    for k, v in va.items():
        ra.insert(k, v)
    for k, v in vb.items():
        rb.insert(k, v)
    want = ra.diff_keys(rb)
    res = _run_fn(world, _fn_diff_gather, pa, pb, va, vb)
    for got, stats in res:
        assert got == want
        assert stats["diff_all_gather_v"][1] == 1


def test_sharded_diff_gather_identical_gloo():
    """Identical replicas: every rank gets the empty list (no key bytes to gather)."""
    keys = [b"k%04d" % i for i in range(300)]
    v = {k: k for k in keys}
    parts = [keys[:100], keys[100:]]
    res = _run_fn(2, _fn_diff_gather, parts, parts, v, v)
    assert [g for g, _ in res] == [[], []]
