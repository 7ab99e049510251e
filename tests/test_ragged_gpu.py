"""Ragged records: the lane-refill leaf kernel (k_leaf_ragged, csrc/k_ragged.hip) against the C oracle —
store-like key / value lengths at arbitrary byte offsets, every padding / block / run edge, blob bases at
every byte alignment, records of thousands of blocks beside one-block ones, fixed-shape chunks handed
over by k_leaf_direct, and the key-ownership copy of the records the ragged stage hashed.
Reference inputs are arbitrary &str pairs (/root/reference/src/store/merkle.rs:7-16, :45-49;
/root/reference/src/sync.rs:109-115)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree, leaf_digests  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, pack  # noqa: E402


@pytest.fixture(autouse=True)
def _free_torch_cache():
    yield
    import gc

    import torch
    gc.collect()
    torch.cuda.empty_cache()


def _enc_digest(k: bytes, v: bytes) -> bytes:
    return hashlib.sha256(len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v).digest()


def test_ragged_store_like_1m_vs_oracle():
    """1M records, keys 8-64 B, values 16-256 B, packed (unaligned offsets): root and every leaf digest
    (level 0, in key order) equal the oracle's."""
    n = 1_000_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n, klen=64, vlen=256, ragged=2)
    shani = coracle.set_backend(1)
    try:
        o = coracle.OracleTree.build(kb, ko, vb, vo)
    finally:
        coracle.set_backend(0)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()
    assert shani in (0, 1)


def test_ragged_device_generator_matches_oracle():
    import torch

    from merklekv_amd.merkle import gen_records_ragged_device
    n = 100_003
    want = coracle.gen_records(DEFAULT_SEED, 7, n, klen=64, vlen=256, ragged=2, shard=3, nshards=8)
    kb = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(n * 256, dtype=torch.uint8, device="cuda")
    ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    gen_records_ragged_device(0, DEFAULT_SEED, 7, n, 64, 256, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                              vo.data_ptr(), shard=3, nshards=8)
    gk, gv = ko.cpu().numpy().astype(np.uint64), vo.cpu().numpy().astype(np.uint64)
    assert np.array_equal(gk, want[1]) and np.array_equal(gv, want[3])
    assert np.array_equal(kb[: int(gk[-1])].cpu().numpy(), want[0])
    assert np.array_equal(vb[: int(gv[-1])].cpu().numpy(), want[2])


def _edge_records(rng):
    """Lengths at every field / padding / block edge: total encodings L = 8 + k + v around 55/56 (1 -> 2
    blocks), 119/120, 183/184, 247/248, 375/376, 1975/1976 and beyond, with every key length mod 4 and keys
    that end in the first, second or a later block (the key run / value run splice positions)."""
    keys, vals = [], []
    for Lt in (8, 9, 12, 54, 55, 56, 57, 63, 64, 119, 120, 183, 184, 185, 247, 248, 375, 376, 377, 1975, 1976, 1977,
               2100, 5000):
        for k in (0, 1, 2, 3, 4, 5, 7, 31, 32, 33, 63, 64, 65, 200):
            v = Lt - 8 - k
            if v < 0:
                continue
            keys.append(rng.integers(0, 256, size=k, dtype=np.uint8).tobytes())
            vals.append(rng.integers(0, 256, size=v, dtype=np.uint8).tobytes())
    return keys, vals


def test_ragged_window_and_class_edges_vs_hashlib():
    rng = np.random.default_rng(11)
    keys, vals = _edge_records(rng)
    # shuffled, so that lanes of one wave run records of very different block counts
    order = rng.permutation(len(keys))
    keys = [keys[i] for i in order]
    vals = [vals[i] for i in order]
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        assert g == _enc_digest(k, v), (len(k), len(v))


@pytest.mark.parametrize("kshift,vshift", [(0, 0), (1, 3), (2, 1), (3, 2)])
def test_ragged_device_blobs_at_every_alignment(kshift, vshift):
    """build_device from blobs whose base pointers sit 0-3 bytes past an allocation start (the loads
    clamp to the blob's own byte range): root and leaves equal the oracle's."""
    import torch
    rng = np.random.default_rng(100 + kshift)
    n = 5_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n, klen=64, vlen=256, ragged=2)
    ek, ev = _edge_records(rng)
    keys = [kb[int(ko[i]):int(ko[i + 1])].tobytes() for i in range(n)] + ek
    vals = [vb[int(vo[i]):int(vo[i + 1])].tobytes() for i in range(n)] + ev
    (pk, pko), (pv, pvo) = pack(keys), pack(vals)
    o = coracle.OracleTree.build(pk, pko, pv, pvo)
    dk = torch.zeros(len(pk) + kshift, dtype=torch.uint8, device="cuda")
    dv = torch.zeros(len(pv) + vshift, dtype=torch.uint8, device="cuda")
    dk[kshift:] = torch.from_numpy(pk.copy()).cuda()
    dv[vshift:] = torch.from_numpy(pv.copy()).cuda()
    dko = torch.from_numpy(pko.astype(np.int64)).cuda()
    dvo = torch.from_numpy(pvo.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t = MerkleTree()
    t.build_device(dk.data_ptr() + kshift, dko.data_ptr(), dv.data_ptr() + vshift, dvo.data_ptr(), len(keys))
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 65, 300, 5000])
@pytest.mark.parametrize("shape", ["tiny", "big_ends", "tiny_ends"])
def test_ragged_edge_prefix_and_suffix(n, shape):
    """The records near the blobs' ends (k_leaf_edges: a prefix and a suffix it finds by two searches,
    k_ragged.hip rg_inner): blobs of tiny records only (no interval: every record an edge one), long
    records at both ends around tiny ones, tiny records at both ends around long ones; bases 1 / 3 bytes
    past an allocation start. Root and leaves equal the oracle's."""
    import torch
    rng = np.random.default_rng(1000 + n)
    def lens(i):
        if shape == "tiny":
            return int(rng.integers(0, 4)), int(rng.integers(0, 4))
        end = i < 3 or i >= n - 3
        if shape == "big_ends":
            return (int(rng.integers(60, 300)), int(rng.integers(100, 700))) if end else (int(rng.integers(0, 5)), int(rng.integers(0, 9)))
        return (int(rng.integers(0, 3)), int(rng.integers(0, 3))) if end else (int(rng.integers(8, 64)), int(rng.integers(16, 256)))
    kv = [lens(i) for i in range(n)]
    keys = [rng.integers(0, 256, size=k, dtype=np.uint8).tobytes() for k, _ in kv]
    vals = [rng.integers(0, 256, size=v, dtype=np.uint8).tobytes() for _, v in kv]
    (pk, pko), (pv, pvo) = pack(keys), pack(vals)
    o = coracle.OracleTree.build(pk, pko, pv, pvo)
    dk = torch.zeros(len(pk) + 1, dtype=torch.uint8, device="cuda")
    dv = torch.zeros(len(pv) + 3, dtype=torch.uint8, device="cuda")
    if len(pk):
        dk[1:] = torch.from_numpy(pk.copy()).cuda()
    if len(pv):
        dv[3:] = torch.from_numpy(pv.copy()).cuda()
    dko = torch.from_numpy(pko.astype(np.int64)).cuda()
    dvo = torch.from_numpy(pvo.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t = MerkleTree()
    t.build_device(dk.data_ptr() + 1, dko.data_ptr(), dv.data_ptr() + 3, dvo.data_ptr(), n)
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        assert g == _enc_digest(k, v), (len(k), len(v))


@pytest.mark.parametrize("klen", [3, 32])
def test_ragged_empty_values_every_record_an_edge_one(klen):
    """Empty values everywhere: voff never moves off voff[0], so every record is an edge one (k_leaf_edges,
    one record per lane) — 300K records at key lengths 3 (duplicates: last write wins) and 32, device blobs
    at an unaligned base; root and leaves equal the oracle's."""
    import torch
    rng = np.random.default_rng(4242 + klen)
    n = 300_000
    pk = rng.integers(0, 256, size=n * klen, dtype=np.uint8)
    pko = np.arange(0, n + 1, dtype=np.uint64) * klen
    pv = np.zeros(0, np.uint8)
    pvo = np.zeros(n + 1, np.uint64)
    o = coracle.OracleTree.build(pk, pko, pv, pvo)
    dk = torch.zeros(len(pk) + 1, dtype=torch.uint8, device="cuda")
    dk[1:] = torch.from_numpy(pk.copy()).cuda()
    dv = torch.zeros(16, dtype=torch.uint8, device="cuda")
    dko = torch.from_numpy(pko.astype(np.int64)).cuda()
    dvo = torch.from_numpy(pvo.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t = MerkleTree()
    t.build_device(dk.data_ptr() + 1, dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), n)
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()


def test_ragged_mixed_with_fixed_chunks_and_duplicates():
    """Fixed-shape chunks (32 / 100 B, k_leaf_direct) interleaved with ragged ones, duplicate keys (last
    write wins) and empty keys / values, against the oracle."""
    rng = np.random.default_rng(5)
    fk, fko, fv, fvo = coracle.gen_records(DEFAULT_SEED, 0, 64 * 40)
    rk, rko, rv, rvo = coracle.gen_records(DEFAULT_SEED, 10**6, 64 * 40, klen=64, vlen=256, ragged=2)
    keys, vals = [], []
    for c in range(40):
        src = (fk, fko, fv, fvo) if c % 3 else (rk, rko, rv, rvo)
        for i in range(64 * c, 64 * c + 64):
            keys.append(src[0][int(src[1][i]):int(src[1][i + 1])].tobytes())
            vals.append(src[2][int(src[3][i]):int(src[3][i + 1])].tobytes())
    for i in rng.choice(len(keys), size=200, replace=False):
        keys.append(keys[int(i)])
        vals.append(b"dup" * int(rng.integers(0, 90)))
    keys += [b"", b"e"]
    vals += [b"x" * 77, b""]
    o = coracle.OracleTree.from_pairs(list(zip(keys, vals)))
    t = MerkleTree()
    t.build(keys, vals)
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()


def test_ragged_long_records_beside_short_ones_vs_hashlib():
    """Lane refill: a few records of thousands of blocks (a 256 KiB value, a 12 KiB key) keep their lanes
    busy while the other lanes of the wave take hundreds of one- to four-block records."""
    rng = np.random.default_rng(23)
    keys, vals = [], []
    for i in range(3000):
        if i % 997 == 5:
            keys.append(rng.integers(0, 256, size=int(rng.integers(0, 12_000)), dtype=np.uint8).tobytes())
            vals.append(rng.integers(0, 256, size=int(rng.integers(100_000, 262_144)), dtype=np.uint8).tobytes())
        else:
            keys.append(rng.integers(0, 256, size=int(rng.integers(0, 70)), dtype=np.uint8).tobytes())
            vals.append(rng.integers(0, 256, size=int(rng.integers(0, 200)), dtype=np.uint8).tobytes())
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        assert g == _enc_digest(k, v), (len(k), len(v))


@pytest.mark.parametrize("layout", ["ragged", "fixed_then_ragged", "ragged_then_fixed"])
def test_ragged_build_device_owns_its_keys(layout):
    """build_device from borrowed device blobs: the tree keeps its own copy of the keys (the fixed-shape
    kernel copies the chunks it hashes, k_keycopy_rest the ones it hands to the ragged stage), so after
    the caller overwrites its buffers the sorted keys, a diff and a rebuilt root still equal the oracle's.
    The second build reuses the first one's key buffer (the fused-copy path)."""
    import torch
    n = 64 * 300 + 17
    fk, fko, fv, fvo = coracle.gen_records(DEFAULT_SEED, 0, n)
    rk, rko, rv, rvo = coracle.gen_records(DEFAULT_SEED, 10**6, n, klen=64, vlen=256, ragged=2)
    split = {"ragged": 0, "fixed_then_ragged": 64 * 200 + 5, "ragged_then_fixed": 64 * 100}[layout]
    keys, vals = [], []
    for i in range(n):
        fixed = (i < split) if layout == "fixed_then_ragged" else (layout == "ragged_then_fixed" and i >= split)
        src = (fk, fko, fv, fvo) if fixed else (rk, rko, rv, rvo)
        keys.append(src[0][int(src[1][i]):int(src[1][i + 1])].tobytes())
        vals.append(src[2][int(src[3][i]):int(src[3][i + 1])].tobytes())
    (pk, pko), (pv, pvo) = pack(keys), pack(vals)
    o = coracle.OracleTree.build(pk, pko, pv, pvo)
    dk = torch.from_numpy(pk.copy()).cuda()
    dv = torch.from_numpy(pv.copy()).cuda()
    dko = torch.from_numpy(pko.astype(np.int64)).cuda()
    dvo = torch.from_numpy(pvo.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t = MerkleTree()
    for _ in range(2):
        t.build_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), n)
    dk.fill_(0x5A)
    dko.fill_(0)
    torch.cuda.synchronize()
    assert t.get_root_hash() == o.root()
    assert [k for k, _ in t.leaves()] == [k.decode("utf-8", "surrogateescape") for k, _ in o.leaves()]
    # a replica with a few changed values: the diff names keys from the tree's own copy
    vals2 = list(vals)
    for i in range(0, n, 97):
        vals2[i] = vals2[i] + b"!"
    o2 = coracle.OracleTree.from_pairs(list(zip(keys, vals2)))
    t2 = MerkleTree()
    t2.build(keys, vals2)
    assert t.diff_keys_bytes(t2) == o.diff(o2)
