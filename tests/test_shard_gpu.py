"""Sharded build on the device: mkv_shard_prepare/_reduce/_fringe/_combine must give the oracle's
root of the union bit-exactly (seam nodes across unaligned shard boundaries, empty / one-leaf shards, R5 promotion
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


def _oracle_root(keys, vals):
    from oracle import coracle
    from oracle.merkle_oracle import pack
    return coracle.OracleTree.build(*pack(keys), *pack(vals)).root()


def test_sharded_small_exhaustive():
    from oracle.merkle_oracle import PyMerkleTree
    for n in (1, 2, 3, 5, 8, 13, 33):
        keys = [b"k%04d" % i for i in range(n)]
        ref = PyMerkleTree()
        for k in keys:
            ref.insert(k, k)
        want = ref.get_root_hash()
        for cuts in itertools.combinations(range(n + 1), 2):
            roots = _sharded(_shards(keys, keys, cuts))
            assert all(r == want for r in roots), (n, cuts)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_synthetic_uneven(world):
    n = 200_003
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    from oracle import coracle
    want = coracle.OracleTree.build(kb, ko, vb, vo).root()
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
    want = _oracle_root(allk, allv)
    roots = _sharded(shards)
    assert all(r == want for r in roots)


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
    assert [r for _, r in res] == [_oracle_root(allk, allv)] * world


def test_fringe_device_combine_matches_host():
    """mkv_shard_fringe_device / mkv_shard_combine_device (the RCCL path's device-resident buffers):
    the same root as the host fringe path, also when two replicas' fringes share one gathered buffer
    (stride = 2 x MKV_FRINGE_BYTES, what shard_recombine_many hands to the combine)."""
    import torch

    from merklekv_amd._lib import FRINGE_BYTES
    from oracle import coracle
    n = 100_003
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    want = coracle.OracleTree.build(kb, ko, vb, vo).root()
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
    import numpy as np
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
        # redistribution over RCCL (all_to_all_single at world size 1) from device tensors
        from merklekv_amd.shard import sharded_root_unpartitioned
        dev = [torch.from_numpy(x.view(np.uint8) if x.dtype == np.uint8 else x.astype(np.int64)).cuda()
               for x in (kb, ko, vb, vo)]
        routed_root, _, routed = sharded_root_unpartitioned(MerkleTree(0), *dev, 50_000, dist, "cuda")
        q.put((roots, again, routed_root, routed.n))
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
    roots, again, routed_root, routed_n = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    from oracle import coracle
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 50_000)
    want = coracle.OracleTree.build(kb, ko, vb, vo).root()
    assert roots == [want] * 3 and again == roots
    assert routed_root == want and routed_n == 50_000


# ---------------------------------------------------------------------------------------------------
# Redistribution of unpartitioned input (csrc/k_route.hip)
# ---------------------------------------------------------------------------------------------------
def _dev_blobs(kb, ko, vb, vo):
    import numpy as np
    import torch
    return [torch.from_numpy(np.array(x, copy=True) if x.dtype == np.uint8 else x.astype(np.int64)).cuda()
            for x in (kb, ko, vb, vo)]


def _mixed_records(seed, n):
    """Ragged records with duplicate keys (same key, different values) and short / shared-prefix keys."""
    import numpy as np

    from oracle.merkle_oracle import pack
    kb, ko, vb, vo = gen_records(seed, 0, n, klen=12, vlen=40, ragged=True)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    rng = np.random.default_rng(seed)
    for i in rng.choice(n, size=n // 20, replace=False):
        keys.append(keys[int(i)])
        vals.append(b"dup-%d" % int(i))
    keys += [b"", b"a", b"prefix--shared-%05d" % 7, b"prefix--shared-%05d" % 3, b"\xff" * 9]
    vals += [b"e", b"", b"x", b"y", b"z"]
    return pack(keys) + pack(vals), keys, vals


def test_route_plan_pack_offsets_vs_model():
    """Single process, no collective: destinations, per-destination totals, destination-grouped send
    buffers (source order kept) and rebuilt offsets equal the host model (tests/shard_model.py)."""
    import numpy as np
    import torch

    from merklekv_amd.merkle import route_splitters
    from tests.shard_model import prefix8
    (kb, ko, vb, vo), keys, vals = _mixed_records(99, 20_000)
    n = len(keys)
    dkb, dko, dvb, dvo = _dev_blobs(kb, ko, vb, vo)
    t = MerkleTree()
    smp = torch.zeros(257, dtype=torch.int64, device="cuda")
    t.route_sample(dkb, dko, n, 257, smp)
    want_smp = [prefix8(keys[((2 * i + 1) * n) // 514]) for i in range(257)]
    assert smp.cpu().numpy().view(np.uint64).tolist() == want_smp
    for world in (1, 2, 5, 256):
        spl = route_splitters(np.array(want_smp, np.uint64), world)
        plan = t.route_plan(dkb, dko, dvb, dvo, n, spl)
        dest = np.searchsorted(spl, np.array([prefix8(k) for k in keys], np.uint64), side="right")
        order = np.argsort(dest, kind="stable")
        for r in range(world):
            sel = dest == r
            assert plan[r].tolist() == [int(sel.sum()), sum(len(keys[i]) for i in np.nonzero(sel)[0]),
                                        sum(len(vals[i]) for i in np.nonzero(sel)[0])], (world, r)
        kout = torch.empty(int(plan[:, 1].sum()) + 1, dtype=torch.uint8, device="cuda")
        vout = torch.empty(int(plan[:, 2].sum()) + 1, dtype=torch.uint8, device="cuda")
        klen = torch.empty(n, dtype=torch.int32, device="cuda")
        vlen = torch.empty(n, dtype=torch.int32, device="cuda")
        t.route_pack(dkb, dko, dvb, dvo, n, kout, klen, vout, vlen)
        assert kout[:-1].cpu().numpy().tobytes() == b"".join(keys[i] for i in order)
        assert vout[:-1].cpu().numpy().tobytes() == b"".join(vals[i] for i in order)
        assert klen.cpu().numpy().tolist() == [len(keys[i]) for i in order]
        assert vlen.cpu().numpy().tolist() == [len(vals[i]) for i in order]
        offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        t.route_offsets(klen, n, offs)
        assert offs.cpu().numpy().tolist() == [0] + np.cumsum([len(keys[i]) for i in order]).tolist()
    with pytest.raises(Exception):  # pack needs the blobs of the last plan
        t.route_pack(dvb, dvo, dkb, dko, n, kout, klen, vout, vlen)


def _worker_route(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from merklekv_amd import MerkleTree
    from merklekv_amd.shard import sharded_root_unpartitioned
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kb, ko, vb, vo = _route_input(rank)
        dev = _dev_blobs(kb, ko, vb, vo)
        t = MerkleTree(0)
        root, counts, routed = sharded_root_unpartitioned(t, *dev, len(ko) - 1, dist, "cuda", samples=2048)
        torch.cuda.synchronize()
        q.put((rank, root, counts, routed.sent.tolist(), routed.received.tolist()))
    finally:
        dist.destroy_process_group()


def _route_input(rank, n=60_000):
    """Unpartitioned records (keys from the whole key space): rank r holds ids [r n/2, r n/2 + n) with
    value field r + 1, so ranks overlap by n/2 keys with different values (the later rank wins)."""
    return gen_records(DEFAULT_SEED, rank * n // 2, n, vfield=rank + 1)


def test_redistribute_two_processes_gloo_same_gpu():
    """Route kernels + all-to-all (gloo, staged) + sharded build: every rank's root equals the oracle
    root of the ranks' inputs inserted in rank order (duplicates across ranks: last write wins)."""
    import torch.multiprocessing as mp

    from oracle import coracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_route, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = [_route_input(r) for r in range(world)]
    keys, vals = [], []
    for kb, ko, vb, vo in parts:
        keys += split_blob(kb, ko)
        vals += split_blob(vb, vo)
    from oracle.merkle_oracle import pack
    want = coracle.OracleTree.build(*pack(keys), *pack(vals))
    for rank, root, counts, sent, received in res:
        assert root == want.root(), rank
        assert sum(counts) == len(want) == 90_000
        assert min(counts) > 0.3 * 90_000  # sampled splitters balance the ranges
    assert res[0][3][1] == res[1][4][0] and res[1][3][0] == res[0][4][1]  # what 0 sends to 1 = what 1 gets


def test_device_entry_points_refuse_host_pointers():
    """A pageable host buffer passed where the ABI wants device memory fails the call (MKV_EINVAL)
    instead of faulting the GPU (tree.cpp need_device_ptr; the r02 rehearsal once passed the gloo
    collective device as the sample buffer)."""
    import numpy as np
    import torch

    from merklekv_amd._lib import MerkleError
    (kb, ko, vb, vo), keys, vals = _mixed_records(5, 1000)
    dkb, dko, dvb, dvo = _dev_blobs(kb, ko, vb, vo)
    n = len(keys)
    t = MerkleTree()
    host_out = torch.zeros(16, dtype=torch.int64)  # CPU tensor
    with pytest.raises(MerkleError, match="not device-accessible"):
        t.route_sample(dkb, dko, n, 16, host_out)
    hko = torch.from_numpy(ko.astype(np.int64))
    with pytest.raises(MerkleError, match="not device-accessible"):
        t.route_plan(dkb, hko, dvb, dvo, n, np.zeros(1, np.uint64))
    with pytest.raises(MerkleError, match="not device-accessible"):
        t.build_device(dkb.data_ptr(), hko.data_ptr(), dvb.data_ptr(), dvo.data_ptr(), n)
    t.build_device(dkb.data_ptr(), dko.data_ptr(), dvb.data_ptr(), dvo.data_ptr(), n)  # still usable
    assert t.get_root_hash() == _oracle_root(keys, vals)
