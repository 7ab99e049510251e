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


def test_fringe_device_combine_matches_host():
    """mkv_shard_fringe_device / mkv_shard_combine_device (the RCCL path's device-resident buffers):
    the same root as the host fringe path, also when two replicas' fringes share one gathered buffer
    (stride = 2 x MKV_FRINGE_BYTES, what shard_recombine_many hands to the combine)."""
    import torch

    from merklekv_amd._lib import FRINGE_BYTES
    n = 100_003
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    want = t.get_root_hash()
    for world in (1, 3, 8):
        step = n // world
        shards = _shards(keys, vals, [step * i + 17 * i for i in range(1, world)])
        trees = [MerkleTree() for _ in shards]
        counts = [tr.shard_prepare(k, v) for tr, (k, v) in zip(trees, shards)]
        N = sum(counts)
        for r, tr in enumerate(trees):
            tr.shard_reduce(sum(counts[:r]), N)
        buf = torch.zeros(world * 2 * FRINGE_BYTES, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for r, tr in enumerate(trees):  # rank r's block holds [replica 0 | replica 1] (same tree twice)
            tr.shard_fringe_device(buf.data_ptr() + (2 * r) * FRINGE_BYTES)
            tr.shard_fringe_device(buf.data_ptr() + (2 * r + 1) * FRINGE_BYTES)
        host = b"".join(tr.shard_fringe() for tr in trees)
        got = buf.view(world, 2, FRINGE_BYTES)[:, 0].cpu().numpy().tobytes()
        assert got == host, world
        for r, tr in enumerate(trees):
            assert tr.shard_combine_device(buf.data_ptr(), world, 2 * FRINGE_BYTES, N) == want, (world, r)
            assert tr.shard_combine_device(buf.data_ptr() + FRINGE_BYTES, world, 2 * FRINGE_BYTES, N) == want
            assert tr.get_root_hash() == want


def _worker_mixed(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import sharded_diff, sharded_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ka, va, kb_, vb_ = _mixed_shard(rank, world)
        A, B = MerkleTree(0), MerkleTree(0)
        sharded_root(A, ka, va, dist, device="cpu")
        sharded_root(B, kb_, vb_, dist, device="cpu")
        (raw, offs), off, tot = sharded_diff(A, B, dist, device="cpu")
        b = raw.tobytes()
        q.put((rank, [b[int(offs[i]):int(offs[i + 1])] for i in range(len(offs) - 1)], off, tot))
    finally:
        dist.destroy_process_group()


def _mixed_shard(rank, world, n=40_000):
    """Replica A's and B's records of shard `rank` (key char 0 in the rank's range): B has value
    changes, deletions and insertions inside the range, so the shard leaf counts differ."""
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, rank * n, n, shard=rank, nshards=world)
    ka, va = split_blob(kb, ko), split_blob(vb, vo)
    kb_, vb_ = [], []
    for i, (k, v) in enumerate(zip(ka, va)):
        if i % 211 == 5:
            continue                        # deleted on B
        kb_.append(k)
        vb_.append(b"changed" + v[7:] if i % 97 == 3 else v)
    nk, nko, nv, nvo = gen_records(DEFAULT_SEED, 10**9 + rank * 1000, 150, shard=rank, nshards=world)
    kb_ += split_blob(nk, nko)              # inserted on B (same key range)
    vb_ += split_blob(nv, nvo)
    return ka, va, kb_, vb_


def test_sharded_mixed_diff_two_processes_gloo_same_gpu():
    """Sharded diff with key-set changes per shard on the HIP path (each rank merge-joins its range),
    collectives on gloo: the rank-ordered concatenation equals the unsharded device diff and the oracle."""
    import torch.multiprocessing as mp

    from oracle import coracle
    from oracle.merkle_oracle import pack
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_mixed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allA, allB = [[], []], [[], []]
    for r in range(world):
        ka, va, kb_, vb_ = _mixed_shard(r, world)
        allA[0] += ka
        allA[1] += va
        allB[0] += kb_
        allB[1] += vb_
    A, B = MerkleTree(), MerkleTree()
    A.build(*allA)
    B.build(*allB)
    want = A.diff_keys_bytes(B)
    oa = coracle.OracleTree.build(*pack(allA[0]), *pack(allA[1]))
    ob = coracle.OracleTree.build(*pack(allB[0]), *pack(allB[1]))
    assert want == oa.diff(ob)
    got = []
    for _, keys, off, tot in res:
        assert off == len(got) and tot == len(want)
        got += keys
    assert got == want


def _worker_rccl1(q):
    import torch
    import torch.distributed as dist

    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import shard_recombine_many, sharded_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 50_000)
        trees = [MerkleTree(0) for _ in range(3)]
        roots = [sharded_root(t, (kb, ko), (vb, vo), dist, device="cuda")[0] for t in trees]
        again = shard_recombine_many(trees, dist, 50_000, device="cuda")
        q.put((roots, again))
    finally:
        dist.destroy_process_group()


def test_rccl_single_rank_device_fringe_path():
    """The RCCL path of shard.py (device-resident fringe buffers, one all-gather for several trees,
    mkv_shard_combine_device) with the nccl backend at world size 1: same root as the unsharded tree."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl1, args=(q,))
    p.start()
    roots, again = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 50_000)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    assert roots == [t.get_root_hash()] * 3 and again == roots
