"""Sharded build on the device: mkv_shard_prepare/_reduce/_fringe/_combine must give the unsharded
root bit-exactly (seam nodes across unaligned shard boundaries, empty / one-leaf shards, R5 promotion
at the global end only)."""
import itertools
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, gen_records, split_blob  # noqa: E402


def _shards(keys, vals, cuts):
    order = sorted(range(len(keys)), key=lambda i: keys[i])
    ks = [keys[i] for i in order]
    vs = [vals[i] for i in order]
    out, prev = [], 0
    for c in list(cuts) + [len(ks)]:
        out.append((ks[prev:c], vs[prev:c]))
        prev = c
    return out


def _sharded(shards):
    trees = [MerkleTree() for _ in shards]
    counts = [t.shard_prepare(k, v) for t, (k, v) in zip(trees, shards)]
    N = sum(counts)
    fr = b""
    for r, t in enumerate(trees):
        t.shard_reduce(sum(counts[:r]), N)
        fr += t.shard_fringe()
    roots = [t.shard_combine(fr, len(trees), N) for t in trees]
    return roots


def test_sharded_small_exhaustive():
    for n in (1, 2, 3, 5, 8, 13, 33):
        keys = [b"k%04d" % i for i in range(n)]
        t = MerkleTree()
        t.build(keys, keys)
        want = t.get_root_hash()
        for cuts in itertools.combinations(range(n + 1), 2):
            roots = _sharded(_shards(keys, keys, cuts))
            assert all(r == want for r in roots), (n, cuts)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_synthetic_uneven(world):
    n = 200_003
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    want = t.get_root_hash()
    step = n // world
    cuts = [step * i + (i * 7919) % 1000 for i in range(1, world)]
    roots = _sharded(_shards(keys, vals, cuts))
    assert all(r == want for r in roots)


def test_sharded_generator_ranges():
    """The bench's layout: shard g generated on device-side rules with key char 0 in range g."""
    world, n = 4, 50_000
    shards, allk, allv = [], [], []
    for g in range(world):
        kb, ko, vb, vo = gen_records(DEFAULT_SEED, g * n, n, shard=g, nshards=world)
        k, v = split_blob(kb, ko), split_blob(vb, vo)
        shards.append((k, v))
        allk += k
        allv += v
    t = MerkleTree()
    t.build(allk, allv)
    roots = _sharded(shards)
    assert all(r == t.get_root_hash() for r in roots)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import sharded_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kb, ko, vb, vo = gen_records(DEFAULT_SEED, rank * 30_000, 30_000, shard=rank, nshards=world)
        root, counts = sharded_root(MerkleTree(0), (kb, ko), (vb, vo), dist, device="cpu")
        q.put((rank, root))
    finally:
        dist.destroy_process_group()


def test_sharded_two_processes_gloo_same_gpu():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allk, allv = [], []
    for g in range(world):
        kb, ko, vb, vo = gen_records(DEFAULT_SEED, g * 30_000, 30_000, shard=g, nshards=world)
        allk += split_blob(kb, ko)
        allv += split_blob(vb, vo)
    t = MerkleTree()
    t.build(allk, allv)
    assert [r for _, r in res] == [t.get_root_hash()] * world
