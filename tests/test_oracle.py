"""CPU tests: pin the oracle (C restatement + hashlib restatement) before trusting it as the checker.

Pins: NIST FIPS 180-4 vectors (the digest sha2 0.10.9 implements), the known-answer roots whose
structure the reference's own tests assert (merkle.rs:239-250, :469-490, :640-668, :581-596,
:616-635, :493-513), and the committed golden fixtures (tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

from oracle.merkle_oracle import DEFAULT_SEED, PyMerkleTree, gen_records, leaf_hash, node_hash, split_blob


@pytest.mark.parametrize("backend", [0, 1])
def test_nist_vectors(oracle_lib, fixtures, backend):
    co = oracle_lib
    got = co.set_backend(backend)
    if backend == 1 and got != 1:
        pytest.skip("no SHA-NI on this host")
    try:
        for msg_hex, dg in fixtures["nist_sha256"]:
            assert co.sha256(bytes.fromhex(msg_hex)).hex() == dg
        assert co.sha256(b"a" * 1_000_000).hex() == fixtures["nist_million_a"]
        # every message length 0..300 against hashlib (padding edge cases around 55/56/64 bytes)
        for L in range(0, 300):
            m = bytes((i * 7 + L) & 0xFF for i in range(L))
            assert co.sha256(m) == hashlib.sha256(m).digest()
    finally:
        co.set_backend(0)


def test_known_answers_c_oracle(oracle_lib, fixtures):
    for name, case in fixtures["known_answers"].items():
        pairs = [(bytes.fromhex(k), bytes.fromhex(v)) for k, v in case["pairs"]]
        t = oracle_lib.OracleTree.from_pairs(pairs)
        assert t.root().hex() == case["root"], name
        for l, lv in enumerate(case["levels"]):
            got = [bytes(row).hex() for row in t.level(l)]
            assert got == lv, (name, l)


def test_manual_roots_relations():
    """The reference's own manual checks (merkle.rs:469-490, :640-668) on the hashlib oracle."""
    h1, h2 = leaf_hash(b"a", b"A"), leaf_hash(b"b", b"B")
    t = PyMerkleTree()
    t.insert(b"a", b"A")
    t.insert(b"b", b"B")
    assert t.get_root_hash() == node_hash(h1, h2)
    hs = [leaf_hash(f"k{i}".encode(), f"v{i}".encode()) for i in range(1, 5)]
    t4 = PyMerkleTree()
    for i in (3, 1, 4, 2):
        t4.insert(f"k{i}".encode(), f"v{i}".encode())
    assert t4.get_root_hash() == node_hash(node_hash(hs[0], hs[1]), node_hash(hs[2], hs[3]))
    t3 = PyMerkleTree()
    for k, v in [(b"a", b"1"), (b"b", b"2"), (b"c", b"3")]:
        t3.insert(k, v)
    la, lb, lc = leaf_hash(b"a", b"1"), leaf_hash(b"b", b"2"), leaf_hash(b"c", b"3")
    assert t3.get_root_hash() == node_hash(node_hash(la, lb), lc)  # R5: c promoted unchanged


def test_sizes_c_oracle(oracle_lib, fixtures):
    for n, root in fixtures["sizes_k_v"].items():
        n = int(n)
        t = oracle_lib.OracleTree.from_pairs([(f"k{i}".encode(), f"v{i}".encode()) for i in range(n)])
        assert t.root().hex() == root, n


def test_synthetic_c_oracle(oracle_lib, fixtures):
    for case in fixtures["synthetic"]:
        kb, ko, vb, vo = oracle_lib.gen_records(case["seed"], 0, case["n"], case["klen"], case["vlen"],
                                                case["ragged"])
        t = oracle_lib.OracleTree.build(kb, ko, vb, vo)
        assert len(t) == case["n_unique"]
        assert t.root().hex() == case["root"]
        for l, want in enumerate(case["level_sha256"]):
            assert hashlib.sha256(t.level(l).tobytes()).hexdigest() == want, l
        lv = t.leaves()
        assert [[k.hex(), h.hex()] for k, h in lv[:16]] == case["first_leaves"]
        assert [[k.hex(), h.hex()] for k, h in lv[-16:]] == case["last_leaves"]


def test_generator_c_matches_numpy(oracle_lib):
    for args in [dict(ragged=False), dict(ragged=True, klen=20, vlen=64), dict(nshards=8, shard=5),
                 dict(nshards=2, shard=1, vfield=2), dict(nshards=3, shard=2), dict(nshards=6, shard=0)]:
        a = gen_records(DEFAULT_SEED, 12345, 300, **args)
        b = oracle_lib.gen_records(DEFAULT_SEED, 12345, 300, **args)
        for x, y in zip(a, b):
            assert np.array_equal(x, y), args


def test_shard_generator_ranges():
    """Key char 0 of shard g lies in the g-th contiguous eighth of the sorted alphabet."""
    alpha = b"-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
    assert list(alpha) == sorted(alpha)
    prev_max = -1
    for g in range(8):
        kb, ko, _, _ = gen_records(7, g * 1000, 1000, nshards=8, shard=g)
        first = kb.reshape(-1, 32)[:, 0]
        assert first.min() > prev_max
        prev_max = first.max()


def test_diff_c_oracle(oracle_lib, fixtures):
    from tests.golden.make_golden import replica_b
    d = fixtures["diff"]
    kb, ko, vb, vo = gen_records(d["seed"], 0, d["n"])
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    bk, bv = replica_b(keys, vals, d["seed"], d["rate_ppm"])
    ta = oracle_lib.OracleTree.from_pairs(list(zip(keys, vals)))
    tb = oracle_lib.OracleTree.from_pairs(list(zip(bk, bv)))
    assert ta.root().hex() == d["root_a"] and tb.root().hex() == d["root_b"]
    assert [k.decode() for k in ta.diff(tb)] == d["diff"]
    assert ta.diff(ta) == []


def test_prefix_roots_c_oracle(oracle_lib, fixtures):
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 1000)
    t = oracle_lib.OracleTree.build(kb, ko, vb, vo)
    for p, want in fixtures["prefix_roots"].items():
        got = t.prefix_root(p.encode())
        assert (got.hex() if got else None) == want, p


def test_upsert_remove_c_oracle(oracle_lib):
    pairs = [(f"k{i}".encode(), f"v{i}".encode()) for i in range(50)]
    t = oracle_lib.OracleTree.from_pairs(pairs)
    py = PyMerkleTree()
    for k, v in pairs:
        py.insert(k, v)
    from oracle.merkle_oracle import pack
    kb, ko = pack([b"k3", b"zz", b"k3"])
    vb, vo = pack([b"x", b"y", b"w"])
    t2 = t.upsert(kb, ko, vb, vo)
    py.insert(b"k3", b"x"); py.insert(b"zz", b"y"); py.insert(b"k3", b"w")
    assert t2.root() == py.get_root_hash()
    kb, ko = pack([b"k1", b"nope", b"zz"])
    t3 = t2.remove(kb, ko)
    for k in (b"k1", b"nope", b"zz"):
        py.remove(k)
    assert t3.root() == py.get_root_hash()
    assert len(t3) == 49


def test_cpu_baselines_match_oracle(oracle_lib):
    """The timed CPU baselines (oracle/cpu_baselines.c) compute the reference's results: cpu_ref's
    bulk build and insert loop (reference data structures, deep-cloned node tree) and cpu_mt's
    parallel build give the oracle root; both diffs give the oracle's divergent-key count."""
    from oracle.merkle_oracle import pack, split_blob
    from tests.golden.make_golden import replica_b
    co = oracle_lib
    for n in (1, 2, 3, 257, 5000):
        kb, ko, vb, vo = co.gen_records(0x4D65726B6C654B56, 0, n)
        want = co.OracleTree.build(kb, ko, vb, vo).root()
        assert co.ref_bulk(kb, ko, vb, vo)[1] == want, n
        assert co.mt_build(kb, ko, vb, vo, 4)[1] == want, n
        assert co.mt_build(kb, ko, vb, vo, 1)[1] == want, n
        if n <= 257:
            assert co.ref_insert_loop(kb, ko, vb, vo)[1] == want, n
    # duplicates: last write wins in every flavour
    keys = [b"k2", b"k1", b"k2", b"k3", b"k1", b"k2"]
    vals = [b"a", b"b", b"c", b"d", b"e", b"f"]
    (kb, ko), (vb, vo) = pack(keys), pack(vals)
    want = co.OracleTree.build(kb, ko, vb, vo).root()
    assert co.ref_bulk(kb, ko, vb, vo)[1] == co.ref_insert_loop(kb, ko, vb, vo)[1] == want
    assert co.mt_build(kb, ko, vb, vo, 3)[1] == want
    # configs[0] shape at 20K: 1 % 80/10/10 replica
    n = 20_000
    kb, ko, vb, vo = co.gen_records(0x4D65726B6C654B56, 0, n)
    bk, bv = replica_b(split_blob(kb, ko), split_blob(vb, vo), 0x4D65726B6C654B56, 10_000)
    (kb2, ko2), (vb2, vo2) = pack(bk), pack(bv)
    ta, tb = co.OracleTree.build(kb, ko, vb, vo), co.OracleTree.build(kb2, ko2, vb2, vo2)
    want = len(ta.diff(tb))
    assert co.ref_diff((kb, ko, vb, vo), (kb2, ko2, vb2, vo2))[1] == want
    for th in (1, 3, 8):
        assert co.mt_diff(ta, tb, th)[1] == want


@pytest.mark.parametrize("G,nper,blog", [(8, 12345, 10), (4, 1000, 3), (8, 1, 1), (2, 3, 1), (8, 4096, 8),
                                         (1, 777, 4), (8, 2048, 11)])
def test_root_stream_matches_tree_build(oracle_lib, G, nper, blog):
    """oracle/root_stream (the streaming restatement that computes the configs[3] golden root,
    tests/golden/roots_sharded.json) equals orc_tree_build over the union of the G key-range shards:
    aligned-block pushes, leaf pushes at unaligned shard seams and the final R5 promotions
    (/root/reference/src/store/merkle.rs:94-118)."""
    import json
    import os
    import subprocess

    from oracle import coracle
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "oracle", "root_stream")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(root, "oracle"), "root_stream"])
    parts = [coracle.gen_records(DEFAULT_SEED, g * nper, nper, shard=g, nshards=G) for g in range(G)]
    kb = np.concatenate([p[0] for p in parts])
    vb = np.concatenate([p[2] for p in parts])
    n = G * nper
    want = coracle.OracleTree.build(kb, np.arange(n + 1, dtype=np.uint64) * 32, vb,
                                    np.arange(n + 1, dtype=np.uint64) * 100).root().hex()
    out = json.loads(subprocess.check_output([exe, str(DEFAULT_SEED), str(G), str(nper), "32", "100", str(blog), "3"]))
    assert out["n"] == n and out["counts"] == [nper] * G
    assert out["root"] == want


def test_roots_sharded_golden_file():
    """The committed configs[3] roots name the generator cases the GPU test rebuilds."""
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "roots_sharded.json")))
    cases = {(c["shards"], c["per_shard"]): c for c in d["cases"]}
    big = cases[(8, 125_000_000)]
    assert big["n"] == 1_000_000_000 and big["seed"] == DEFAULT_SEED and len(big["root"]) == 64
    assert cases[(8, 15_625_000)]["n"] == 125_000_000
