"""Bit-exact parity of the HIP path against the oracle (C restatement + committed golden fixtures).

Integer/byte work, so the bar is exact equality everywhere: leaf digests, every level array, sorted
keys, roots, diff key lists (order included), prefix roots.
"""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree, leaf_digests  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, PyMerkleTree, gen_records, pack, split_blob  # noqa: E402


def levels_of(t: MerkleTree):
    return [t.level_digests(l) for l in range(t.level_count())]


def assert_tree_equal(gpu: MerkleTree, orc, check_levels=True):
    assert len(gpu) == len(orc)
    assert gpu.get_root_hash() == orc.root()
    if check_levels:
        assert gpu.level_count() == orc.nlevels()
        for l in range(orc.nlevels()):
            assert b"".join(gpu.level_digests(l)) == orc.level(l).tobytes(), l
    ol = orc.leaves()
    gl = gpu.leaves()
    assert [k.encode("utf-8", "surrogateescape") for k, _ in gl] == [k for k, _ in ol]
    assert [d for _, d in gl] == [d for _, d in ol]


# ---------------------------------------------------------------- Kernel A alone
def test_leaf_digest_every_length_against_hashlib():
    """Every (|k|, |v|) combination around the 55/56/64-byte padding edges, aligned and unaligned."""
    rng = random.Random(5)
    keys, vals = [], []
    for kl in list(range(0, 20)) + [31, 32, 33, 55, 56, 57, 63, 64, 65, 120, 200]:
        for vl in [0, 1, 3, 4, 5, 44, 45, 46, 47, 48, 52, 56, 60, 64, 100, 119, 120, 121, 300]:
            keys.append(bytes(rng.randrange(256) for _ in range(kl)))
            vals.append(bytes(rng.randrange(256) for _ in range(vl)))
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        enc = len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v
        assert g == hashlib.sha256(enc).digest(), (len(k), len(v))


def test_leaf_digest_uniform_fast_path():
    """Uniform 4-aligned lengths (the fast path) incl. a partial last wave."""
    for kl, vl, n in [(32, 100, 1000), (4, 0, 130), (0, 4, 65), (8, 48, 64), (60, 64, 200)]:
        kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, n, klen=max(kl, 1), vlen=max(vl, 1))
        keys = [k[:kl] for k in split_blob(kb, ko)]
        vals = [v[:vl] for v in split_blob(vb, vo)]
        got = leaf_digests(keys, vals)
        for k, v, g in zip(keys, vals, got):
            assert g == hashlib.sha256(len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v).digest()


def test_leaf_digest_mixed_fixed_and_listed_chunks():
    """k_leaf_direct hashes 64-record chunks of 32-B keys / 100-B values from registers and lists every
    other chunk for k_leaf_list: chunks with one odd record, odd records at chunk edges, a partial last
    chunk, all against hashlib."""
    rng = random.Random(17)
    n = 64 * 90 + 23
    odd = {0, 63, 64, 700, 701, 1279, 2048, 4000, n - 1}
    keys, vals = [], []
    for i in range(n):
        kl = 33 if i in odd and i % 2 == 0 else 32
        vl = 101 if i in odd and i % 2 == 1 else 100
        keys.append(bytes(rng.randrange(256) for _ in range(kl)))
        vals.append(bytes(rng.randrange(256) for _ in range(vl)))
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        assert g == hashlib.sha256(len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v).digest()


def test_leaf_digest_oversized_wave_global_path():
    """A wave whose span does not fit its LDS region hashes straight from HBM."""
    keys = [b"k%d" % i for i in range(70)]
    vals = [bytes([i % 251]) * (300 + 37 * i) for i in range(70)]
    got = leaf_digests(keys, vals)
    for k, v, g in zip(keys, vals, got):
        assert g == hashlib.sha256(len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v).digest()


# ---------------------------------------------------------------- fixtures
def test_known_answers(fixtures):
    for name, case in fixtures["known_answers"].items():
        t = MerkleTree()
        t.build([bytes.fromhex(k) for k, _ in case["pairs"]], [bytes.fromhex(v) for _, v in case["pairs"]])
        assert t.get_root_hash().hex() == case["root"], name
        assert [[h.hex() for h in lv] for lv in levels_of(t)] == case["levels"], name


def test_sizes_k_v(fixtures):
    t = MerkleTree()
    for n, root in fixtures["sizes_k_v"].items():
        n = int(n)
        t.build([f"k{i}" for i in range(n)], [f"v{i}" for i in range(n)])
        assert t.get_root_hash().hex() == root, n


def test_synthetic_fixtures(fixtures):
    for case in fixtures["synthetic"]:
        kb, ko, vb, vo = gen_records(case["seed"], 0, case["n"], klen=case["klen"], vlen=case["vlen"],
                                     ragged=case["ragged"])
        t = MerkleTree()
        t.build((kb, ko), (vb, vo))
        assert len(t) == case["n_unique"]
        assert t.get_root_hash().hex() == case["root"]
        for l, want in enumerate(case["level_sha256"]):
            assert hashlib.sha256(b"".join(t.level_digests(l))).hexdigest() == want, l
        lv = t.leaves()
        assert [[k.encode().hex(), h.hex()] for k, h in lv[:16]] == case["first_leaves"]
        assert [[k.encode().hex(), h.hex()] for k, h in lv[-16:]] == case["last_leaves"]


def test_prefix_roots(fixtures):
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 1000)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    for p, want in fixtures["prefix_roots"].items():
        got = t.prefix_root(p)
        assert (got.hex() if got else None) == want, p


def test_diff_fixture(fixtures):
    from tests.golden.make_golden import replica_b
    d = fixtures["diff"]
    kb, ko, vb, vo = gen_records(d["seed"], 0, d["n"])
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    bk, bv = replica_b(keys, vals, d["seed"], d["rate_ppm"])
    a, b = MerkleTree(), MerkleTree()
    a.build(keys, vals)
    b.build(bk, bv)
    assert a.get_root_hash().hex() == d["root_a"]
    assert b.get_root_hash().hex() == d["root_b"]
    assert a.diff_keys(b) == d["diff"]
    assert b.diff_keys(a) == d["diff"]


# ---------------------------------------------------------------- ordering edge cases vs C oracle
def _check_pairs(oracle_lib, pairs):
    t = MerkleTree()
    t.build([k for k, _ in pairs], [v for _, v in pairs])
    o = oracle_lib.OracleTree.from_pairs(pairs)
    assert_tree_equal(t, o)
    return t, o


def test_long_common_prefixes_refinement(oracle_lib):
    """Keys sharing >8-byte prefixes force the segmented refinement (chunks 1..k and the length pass)."""
    rng = random.Random(11)
    pairs = []
    for i in range(3000):
        p = rng.choice([b"user:000000", b"user:0000001", b"", b"\x00\x00\x00\x00\x00\x00\x00\x00",
                        b"abcdefghabcdefghabcdefgh", b"abcdefgh"])
        suffix = rng.choice([b"", b"\x00", b"\x00\x00", str(rng.randrange(500)).encode(), b"\xff" * rng.randrange(4)])
        pairs.append((p + suffix, b"v%d" % rng.randrange(10 ** 6)))
    _check_pairs(oracle_lib, pairs)


def test_many_tie_runs_heads_list(oracle_lib):
    """Thousands of 8-byte-prefix tie runs (sizes 2..40 around the 16-position short-run limit, first and
    last sorted positions included, duplicates inside runs): the refinement visits runs through the
    head list k_mark_ties appends in arbitrary order."""
    rng = random.Random(23)
    pairs = []
    for g in range(2500):
        size = rng.choice([1, 2, 3, 5, 15, 16, 17, 40])
        head = b"g%07d" % g  # exactly 8 bytes: the whole sorted prefix is shared by the run
        for _ in range(size):
            suffix = rng.choice([b"", b"\x00", b"x", b"%d" % rng.randrange(30), b"\xff\xfe"])
            pairs.append((head + suffix, b"v%d" % rng.randrange(10 ** 6)))
    pairs.append((b"", b"first"))  # a run-free position 0
    pairs.append((b"\xff" * 8 + b"a", b"z1"))  # a run at the last sorted positions
    pairs.append((b"\xff" * 8 + b"b", b"z2"))
    rng.shuffle(pairs)
    _check_pairs(oracle_lib, pairs)


def test_prefix_of_other_key_order(oracle_lib):
    """Rust str Ord: a proper prefix sorts first; zero bytes vs end of string (R3)."""
    ks = [b"ab", b"ab\x00", b"ab\x00\x00", b"ab\x01", b"a", b"", b"abcdefgh", b"abcdefgh\x00", b"abcdefg",
          b"abcdefgh\x00\x00\x00\x00\x00\x00\x00\x00", b"abcdefgh\x00\x00\x00\x00\x00\x00\x00\x00\x00"]
    t, _ = _check_pairs(oracle_lib, [(k, b"v") for k in ks])
    assert [k.encode("utf-8", "surrogateescape") for k in t.inorder_keys()] == sorted(ks)


def test_duplicates_last_write_wins(oracle_lib):
    rng = random.Random(3)
    pairs = [(b"k%d" % rng.randrange(300), b"v%d" % i) for i in range(5000)]
    t, o = _check_pairs(oracle_lib, pairs)
    assert len(t) == len({k for k, _ in pairs})


def test_unicode_nul_ragged(oracle_lib):
    rng = random.Random(7)
    alphabet = ["a", "b", "\0", "é", "中", "🙂", "z", "\x7f"]
    pairs = []
    for _ in range(4000):
        k = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 14))).encode()
        v = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 60))).encode()
        pairs.append((k, v))
    _check_pairs(oracle_lib, pairs)


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 511, 512, 513, 1023, 1024, 1025, 4097, 65537])
def test_synthetic_sizes_vs_oracle(oracle_lib, n):
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + n, 0, n)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    assert_tree_equal(t, oracle_lib.OracleTree.build(kb, ko, vb, vo))


def test_ragged_synthetic_vs_oracle(oracle_lib):
    kb, ko, vb, vo = oracle_lib.gen_records(99, 0, 50000, 24, 300, ragged=True)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    assert_tree_equal(t, oracle_lib.OracleTree.build(kb, ko, vb, vo))


def test_large_1m_vs_oracle(oracle_lib):
    n = 1_000_000
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED, 0, n)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    oracle_lib.set_backend(1)
    try:
        o = oracle_lib.OracleTree.build(kb, ko, vb, vo)
    finally:
        oracle_lib.set_backend(0)
    assert t.get_root_hash() == o.root()
    assert b"".join(t.level_digests(0)) == o.level(0).tobytes()
    assert b"".join(t.level_digests(1)) == o.level(1).tobytes()


# ---------------------------------------------------------------- diff vs oracle
def test_random_diffs_vs_oracle(oracle_lib):
    rng = random.Random(42)
    for trial in range(6):
        base = [(("key%07d" % rng.randrange(10 ** 6)).encode() + (b"\x00" if trial % 2 else b""),
                 b"v%d" % rng.randrange(10 ** 9)) for _ in range(rng.choice([10, 1000, 20000]))]
        other = []
        for k, v in base:
            r = rng.random()
            if r < 0.05:
                continue
            other.append((k, v + b"!" if r < 0.15 else v))
        other += [(b"new%d" % rng.randrange(10 ** 5), b"x") for _ in range(rng.randrange(50))]
        rng.shuffle(other)
        a, b = MerkleTree(), MerkleTree()
        a.build([k for k, _ in base], [v for _, v in base])
        b.build([k for k, _ in other], [v for _, v in other])
        oa = oracle_lib.OracleTree.from_pairs(base)
        ob = oracle_lib.OracleTree.from_pairs(other)
        assert a.diff_keys_bytes(b) == oa.diff(ob)
        assert b.diff_keys_bytes(a) == ob.diff(oa)


def test_diff_shared_long_prefixes_vs_oracle(oracle_lib):
    keys = [b"tenant/0001/object/%08d" % i for i in range(5000)]
    a_pairs = [(k, b"A") for k in keys]
    b_pairs = [(k, b"A" if i % 97 else b"B") for i, k in enumerate(keys) if i % 211] + [(b"tenant/0001/object/", b"z")]
    a, b = MerkleTree(), MerkleTree()
    a.build([k for k, _ in a_pairs], [v for _, v in a_pairs])
    b.build([k for k, _ in b_pairs], [v for _, v in b_pairs])
    oa = oracle_lib.OracleTree.from_pairs(a_pairs)
    ob = oracle_lib.OracleTree.from_pairs(b_pairs)
    assert a.diff_keys_bytes(b) == oa.diff(ob)


@pytest.mark.parametrize("extra", [True, False])
def test_diff_distinct_keys_equal_prefix_equal_value_vs_oracle(oracle_lib, extra):
    """R7 (merkle.rs:181-190) compares KEYS; the merge-join pairs leaves by 8-byte prefix + digest and
    falls back to the full keys when the digests differ. Distinct keys with one 8-byte prefix (also the
    zero-padding twins "pfx_0001" / "pfx_0001\\0") carrying IDENTICAL values sit on opposite sides: their
    digests differ (the key is hashed), so the fallback must report both keys. extra=True adds a key on
    one side (unequal leaf counts: merge-join), False keeps the counts equal (top-down walk)."""
    common = [(b"cmn/%06d" % i, b"same") for i in range(3000)]
    a_only = [(b"pfx_0000-alpha", b"v"), (b"pfx_0001", b"v"), (b"pfx_0002\x00\x00", b"w"), (b"zz-edge-a", b"q")]
    b_only = [(b"pfx_0000-beta", b"v"), (b"pfx_0001\x00", b"v"), (b"pfx_0002\x00", b"w"), (b"zz-edge-b", b"q")]
    a_pairs = common + a_only
    b_pairs = common + b_only + ([(b"zzz-extra", b"x")] if extra else [])
    a, b = MerkleTree(), MerkleTree()
    a.build([k for k, _ in a_pairs], [v for _, v in a_pairs])
    b.build([k for k, _ in b_pairs], [v for _, v in b_pairs])
    want = oracle_lib.OracleTree.from_pairs(a_pairs).diff(oracle_lib.OracleTree.from_pairs(b_pairs))
    assert want == sorted(k for k, _ in a_only + b_only + ([(b"zzz-extra", b"")] if extra else []))
    assert a.diff_keys_bytes(b) == want
    assert b.diff_keys_bytes(a) == want


@pytest.mark.parametrize("na,nb", [
    (16384, 16384 - 1),       # 32767 merged outputs: 64 tiles, one partition group, last tile short
    (16383, 16385),           # exactly 64 tiles: the group's end split is the array end
    (16385, 16384),           # 65 tiles: a second group holding one tile
    (64 * 512 * 3, 700),      # three groups, B much shorter (splits clamp at B's end)
    (5, 40000),               # A much shorter
    (0, 3000),                # empty A
    (3000, 0),                # empty B
])
def test_merge_join_partition_group_edges_vs_oracle(oracle_lib, na, nb):
    """The merge-join's one-launch partition (a wave per 64 tiles: cooperative boundary searches, then
    per-tile searches between them) at tile-count edges; unequal leaf counts force the merge-join."""
    keys = sorted({b"%09d" % (i * 7919 % 1000003) for i in range(max(na, nb) + 2000)})
    a_pairs = [(k, b"a") for k in keys[:na]]
    # B: A's keys shifted by one position (key sets differ), every 13th value changed
    b_keys = keys[1:nb + 1] if nb <= len(keys) - 1 else keys[:nb]
    b_pairs = [(k, b"a" if i % 13 else b"b") for i, k in enumerate(b_keys)]
    a, b = MerkleTree(), MerkleTree()
    if a_pairs:
        a.build([k for k, _ in a_pairs], [v for _, v in a_pairs])
    if b_pairs:
        b.build([k for k, _ in b_pairs], [v for _, v in b_pairs])
    oa = oracle_lib.OracleTree.from_pairs(a_pairs)
    ob = oracle_lib.OracleTree.from_pairs(b_pairs)
    assert a.diff_keys_bytes(b) == oa.diff(ob)
    assert b.diff_keys_bytes(a) == ob.diff(oa)


def _near_identical(rng, n, shared_prefix, events):
    """Base replica + variant with 0.2 % value changes and the given structural events."""
    pre = b"tenant/0001/obj/" if shared_prefix else b""
    keys = sorted({pre + b"%016x" % rng.getrandbits(64) for _ in range(n)})
    base = [(k, b"v" + k[-6:]) for k in keys]
    var = [(k, v + b"!" if rng.random() < 0.002 else v) for k, v in base]
    for ev in events:
        if ev == "insert_first":  # odd shift at the start: every later tile pairs in phase 1
            var.append((pre + b"0", b"new"))
        elif ev == "insert_last":
            var.append((pre + b"\xff", b"new"))
        elif ev == "random":  # sparse inserts + deletes
            drop = set(rng.sample(range(len(var)), n // 1000))
            var = [p for i, p in enumerate(var) if i not in drop]
            var += [(pre + b"%016x" % rng.getrandbits(64) + b"+", b"ins") for _ in range(n // 1000)]
    return base, var


@pytest.mark.parametrize("n,shared_prefix,events", [
    (300_000, False, ("insert_last",)),
    (300_000, False, ("insert_first",)),
    (300_017, False, ("random",)),
    (257, False, ("insert_first",)),
    (100_000, True, ("insert_first",)),
    (100_003, True, ("random",)),
])
def test_merge_join_near_identical_vs_oracle(oracle_lib, n, shared_prefix, events):
    """Merge-join (unequal leaf counts) on near-identical replicas: the aligned wave-tile fast path in
    both pairing phases, partial last tiles, and shared 8-byte prefixes (aligned check passes on the
    prefixes, the full key compare rejects misaligned pairs and the general merge takes over)."""
    rng = random.Random(hash((n, shared_prefix, events)) & 0xFFFF)
    base, var = _near_identical(rng, n, shared_prefix, events)
    a, b = MerkleTree(), MerkleTree()
    a.build([k for k, _ in base], [v for _, v in base])
    b.build([k for k, _ in var], [v for _, v in var])
    oa = oracle_lib.OracleTree.from_pairs(base)
    ob = oracle_lib.OracleTree.from_pairs(var)
    expect = oa.diff(ob)
    assert expect  # the variant always differs
    assert a.diff_keys_bytes(b) == expect
    assert b.diff_keys_bytes(a) == ob.diff(oa)


def test_diff_empty_trees():
    a, b = MerkleTree(), MerkleTree()
    assert a.diff_keys(b) == []
    b.insert("x", "1")
    assert a.diff_keys(b) == ["x"] and b.diff_keys(a) == ["x"]


# ---------------------------------------------------------------- batches (upsert/remove/apply)
def test_insert_remove_sequences_vs_python_oracle():
    rng = random.Random(17)
    t, py = MerkleTree(), PyMerkleTree()
    for step in range(40):
        for _ in range(rng.randrange(1, 60)):
            k = b"k%d" % rng.randrange(200)
            if rng.random() < 0.3:
                t.remove(k)
                py.remove(k)
            else:
                v = b"v%d" % rng.randrange(1000)
                t.insert(k, v)
                py.insert(k, v)
        assert t.get_root_hash() == py.get_root_hash(), step
        assert len(t) == len(py.leaf_map)
        assert [k.encode() for k in t.inorder_keys()] == py.inorder_keys()


def test_upsert_remove_batches_vs_oracle(oracle_lib):
    kb, ko, vb, vo = oracle_lib.gen_records(5, 0, 20000, 16, 40, ragged=True)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = oracle_lib.OracleTree.build(kb, ko, vb, vo)
    kb2, ko2, vb2, vo2 = oracle_lib.gen_records(5, 15000, 10000, 16, 40, ragged=True, vfield=3)
    t.upsert((kb2, ko2), (vb2, vo2))
    o = o.upsert(kb2, ko2, vb2, vo2)
    assert_tree_equal(t, o)
    keys = split_blob(kb, ko)[::3]
    rb, ro = pack(keys)
    t.remove_many((rb, ro))
    o = o.remove(rb, ro)
    assert_tree_equal(t, o)


def test_clone_is_deep():
    a = MerkleTree()
    a.build([f"k{i}" for i in range(100)], [f"v{i}" for i in range(100)])
    b = a.clone()
    b.insert("k5", "changed")
    assert a.get_root_hash() != b.get_root_hash()
    assert a.diff_keys(b) == ["k5"]


def test_level_structure_and_views():
    n = 1000
    t = MerkleTree()
    t.build([f"k{i}" for i in range(n)], [f"v{i}" for i in range(n)])
    sizes = [len(t.level_digests(l)) for l in range(t.level_count())]
    s, want = n, []
    while True:
        want.append(s)
        if s == 1:
            break
        s = (s + 1) // 2
    assert sizes == want
    assert t.node_count() == 2 * n - 1
    assert len(t.preorder_hashes()) == 2 * n - 1
    py = PyMerkleTree()
    for i in range(n):
        py.insert(f"k{i}".encode(), f"v{i}".encode())
    assert [t.level_digests(l) for l in range(len(sizes))] == py.levels()


# ---------------------------------------------------------------- top-down diff (equal leaf counts)
@pytest.mark.parametrize("n,stride", [(1, 1), (2, 1), (3, 2), (1000, 7), (65_537, 1000), (200_000, 97)])
def test_topdown_value_only_vs_oracle(oracle_lib, n, stride):
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + 5, 0, n)
    vb2 = vb.copy().reshape(n, 100)
    vb2[::stride, 3] ^= 1  # value-only divergence: same key set, same leaf count
    vb2 = vb2.reshape(-1)
    a, b = MerkleTree(), MerkleTree()
    a.build((kb, ko), (vb, vo))
    b.build((kb, ko), (vb2, vo))
    oa = oracle_lib.OracleTree.build(kb, ko, vb, vo)
    ob = oracle_lib.OracleTree.build(kb, ko, vb2, vo)
    want = oa.diff(ob)
    assert len(want) == len(range(0, n, stride))
    assert a.diff_keys_bytes(b) == want
    assert b.diff_keys_bytes(a) == want


@pytest.mark.parametrize("n,klen,stride", [(400_000, 32, 48), (100_000, 200, 48)])
def test_topdown_onewait_capacity_overflow_and_regrowth(oracle_lib, n, klen, stride):
    """The one-wait top-down diff stages its key list in a capacity sized from earlier calls. First call on
    a fresh handle: the list outgrows it (more keys than the capacity, or more key bytes: 200-B keys) and
    the refs path copies it; the capacity grows, so the second call fits (a large result: the staging
    block is handed over); a one-key diff then gets a right-sized copy. Every result equals the oracle's
    (/root/reference/src/store/merkle.rs:171-196)."""
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + 9, 0, n, klen=klen, vlen=100)
    vb2 = vb.copy().reshape(n, 100)
    vb2[::stride, 7] ^= 1
    vb2 = vb2.reshape(-1)
    vb3 = vb.copy().reshape(n, 100)
    vb3[n // 2, 0] ^= 1
    vb3 = vb3.reshape(-1)
    a, b, c = MerkleTree(), MerkleTree(), MerkleTree()
    a.build((kb, ko), (vb, vo))
    b.build((kb, ko), (vb2, vo))
    c.build((kb, ko), (vb3, vo))
    oa = oracle_lib.OracleTree.build(kb, ko, vb, vo)
    want_b = oa.diff(oracle_lib.OracleTree.build(kb, ko, vb2, vo))
    want_c = oa.diff(oracle_lib.OracleTree.build(kb, ko, vb3, vo))
    assert len(want_b) == len(range(0, n, stride)) and len(want_c) == 1
    first = a.diff_keys_bytes(b)   # overflow: copied from the refs
    second = a.diff_keys_bytes(b)  # fits the grown capacity
    small = a.diff_keys_bytes(c)   # right-sized copy of a one-key list
    again = a.diff_keys_bytes(b)
    assert first == want_b and second == want_b and again == want_b
    assert small == want_c


def test_topdown_positions_across_bitmap_blocks(oracle_lib):
    """Divergent leaves at chosen sorted positions: word / uint4 / 32768-leaf block edges, a dense run
    and the last leaf (the sorted-position compaction of the walk); repeated diffs on one handle, then a
    larger tree diffed by the same handle (the position bitmap must come back zero every time)."""
    a = MerkleTree()
    for n, seed in ((70_001, 21), (70_001, 22), (140_003, 23)):
        kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + seed, 0, n)
        order = np.lexsort(kb.reshape(n, 32).T[::-1])  # input index of each sorted position
        pos = {0, 1, 31, 32, 127, 128, 129, 32767, 32768, 32769, 65535, n - 2, n - 1} | set(range(40_000, 40_200))
        vb2 = vb.copy().reshape(n, 100)
        vb2[order[sorted(pos)], 7] ^= 1
        vb2 = vb2.reshape(-1)
        b = MerkleTree()
        a.build((kb, ko), (vb, vo))
        b.build((kb, ko), (vb2, vo))
        oa = oracle_lib.OracleTree.build(kb, ko, vb, vo)
        ob = oracle_lib.OracleTree.build(kb, ko, vb2, vo)
        want = oa.diff(ob)
        assert len(want) == len(pos)
        for _ in range(2):
            assert a.diff_keys_bytes(b) == want
        assert b.diff_keys_bytes(a) == want


def test_topdown_equal_count_key_swap_falls_back(oracle_lib):
    """Same leaf count but different key sets: divergent positions hold different keys -> merge-join."""
    n = 10_000
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + 6, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    keys2 = list(keys)
    keys2[17] = b"!" + keys2[17][1:]        # one key replaced (sorts first), count unchanged
    keys2[4242] = keys2[4242][:-1] + b"~"
    vals2 = list(vals)
    vals2[99] = b"changed"
    a, b = MerkleTree(), MerkleTree()
    a.build(keys, vals)
    b.build(keys2, vals2)
    oa = oracle_lib.OracleTree.from_pairs(list(zip(keys, vals)))
    ob = oracle_lib.OracleTree.from_pairs(list(zip(keys2, vals2)))
    assert a.diff_keys_bytes(b) == oa.diff(ob)
    assert b.diff_keys_bytes(a) == ob.diff(oa)


@pytest.mark.parametrize("n", [100, 5_000, 300_000])
def test_topdown_screen_every_position_shifted(oracle_lib, n):
    """Equal counts, the largest key replaced by one that sorts first: every sorted position shifts, so the
    key-set screen (sampled prefixes, beside the walk's top) stops the walk at its gated jump — or, for
    trees too small for one, the leaf-key check does — and the merge-join answers. Twice per handle (the
    screen's slots are rewritten, never zeroed), then a value-only diff on the same handle."""
    kb, ko, vb, vo = oracle_lib.gen_records(DEFAULT_SEED + 31, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    keys2 = list(keys)
    last = max(range(n), key=lambda i: keys[i])
    keys2[last] = b"\x00" + keys2[last][1:]
    a, b = MerkleTree(), MerkleTree()
    a.build(keys, vals)
    b.build(keys2, vals)
    oa = oracle_lib.OracleTree.from_pairs(list(zip(keys, vals)))
    ob = oracle_lib.OracleTree.from_pairs(list(zip(keys2, vals)))
    for _ in range(2):
        assert a.diff_keys_bytes(b) == oa.diff(ob)
    vals3 = list(vals)
    vals3[n // 3] = b"changed"
    c = MerkleTree()
    c.build(keys, vals3)
    assert a.diff_keys_bytes(c) == [keys[n // 3]]


@pytest.mark.parametrize("klen", [12, 37, 60, 64, 90])
def test_topdown_key_tail_change_falls_back(klen):
    """Equal counts and 8-byte prefixes; one key differs only in its last byte (aligned and unaligned
    key storage, keys up to and beyond the 64-byte batched compare): the leaf check must see it."""
    rng = random.Random(klen)
    n = 3000
    keys = [bytes(rng.choice(b"abcdefgh") for _ in range(klen)) for _ in range(n)]
    keys = sorted(set(keys))
    vals = [b"v%d" % i for i in range(len(keys))]
    keys2 = list(keys)
    j = len(keys) // 2
    keys2[j] = keys2[j][:-1] + (b"z" if keys2[j][-1:] != b"z" else b"y")
    assert keys2[j] not in set(keys)
    vals2 = list(vals)
    vals2[7] = b"changed"
    a, b = MerkleTree(), MerkleTree()
    a.build(keys, vals)
    b.build(keys2, vals2)
    want = sorted({keys[7], keys[j], keys2[j]})
    assert a.diff_keys_bytes(b) == want
    assert b.diff_keys_bytes(a) == want


def test_topdown_identical_trees_empty():
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 5000)
    a, b = MerkleTree(), MerkleTree()
    a.build((kb, ko), (vb, vo))
    b.build((kb, ko), (vb, vo))
    assert a.diff_keys(b) == [] and a.diff_first_key(b) is None


# ---------------------------------------------------------------- sort window past shared key bytes
def _shared_prefix_pairs(rng, shape, n):
    alpha = b"-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
    def rnd(m):
        return bytes(rng.choice(alpha) for _ in range(m))
    if shape == "tenant19":      # 19 shared bytes, 13 random: window at byte 19 after 3 hist passes
        ks = [b"tenant/0001/object/" + rnd(13) for _ in range(n)]
    elif shape == "user5":       # 5 shared bytes then digits: window at byte 5
        ks = [b"user:%d" % rng.randrange(10 ** 9) for _ in range(n)]
    elif shape == "long41":      # 41 shared bytes, short suffixes, some keys equal to the prefix
        base = b"x" * 33 + b"/shared/"
        ks = [base + (rnd(rng.randrange(0, 4)) if i % 50 else b"") for i in range(n)]
    elif shape == "dups":        # shared 12 bytes + few distinct suffixes: duplicates, last write wins
        ks = [b"bucket-0042/" + rnd(2) for _ in range(n)]
    elif shape == "nul_pad":     # shared bytes that are NULs, keys of the prefix length and longer
        ks = [b"\x00" * 9 + (rnd(rng.randrange(0, 6)) if i % 7 else b"") for i in range(n)]
    else:                        # "mixed": one key breaks the sharing at byte 0 -> window stays at 0
        ks = [b"tenant/0001/object/" + rnd(13) for _ in range(n - 1)] + [b"a"]
    return [(k, b"v%d" % rng.randrange(10 ** 6)) for k in ks]


@pytest.mark.parametrize("shape", ["tenant19", "user5", "long41", "dups", "nul_pad", "mixed"])
def test_shared_prefix_sort_window_vs_oracle(oracle_lib, shape):
    """Keys that share leading bytes (the realistic "tenant/..." / "user:" shapes): the prefix sort moves
    its window past the shared bytes (tree.cpp sort_unique), the tree keeps offset-0 key prefixes for
    diff / locate / merge. Build, diff against a mutated replica, and a key-set batch merge vs the oracle."""
    rng = random.Random(hash(shape) & 0xFFFF)
    pairs = _shared_prefix_pairs(rng, shape, 40_000)
    t, o = _check_pairs(oracle_lib, pairs)
    # replica with value changes, deletions and insertions of the same shape
    cur = dict(pairs)
    ks = sorted(cur)
    other = dict(cur)
    for k in ks[::97]:
        other[k] = b"changed"
    for k in ks[5::211]:
        other.pop(k, None)
    for k, v in _shared_prefix_pairs(rng, shape, 300):
        other[k + b"~new"] = v
    t2 = MerkleTree()
    t2.build(list(other), list(other.values()))
    o2 = oracle_lib.OracleTree.from_pairs(list(other.items()))
    assert t2.get_root_hash() == o2.root()
    assert t.diff_keys_bytes(t2) == o.diff(o2)
    # key-set batch merged into the existing tree (sorted batch, offset-0 prefixes on both sides)
    batch = [(k + b"~b", b"b") for k, _ in _shared_prefix_pairs(rng, shape, 500)] + [(ks[3], b"upd")]
    t.upsert([k for k, _ in batch], [v for _, v in batch])
    o3 = oracle_lib.OracleTree.from_pairs(pairs + batch)
    assert t.get_root_hash() == o3.root()
    assert t.diff_keys_bytes(t2) == o3.diff(o2)


# ---------------------------------------------------------------- key byte-entropy shapes (round 2)
def _entropy_pairs(rng, shape, n):
    b64 = b"-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
    if shape == "bits1":        # 1 bit per byte: every window byte sorted, long tie runs refined
        ks = [bytes(rng.choice(b"ab") for _ in range(12)) for _ in range(n)]
    elif shape == "bytes8":     # 8 bits per byte, ragged lengths
        ks = [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 12))) for _ in range(n)]
    elif shape == "b64":   # 6 bits per byte
        ks = [bytes(rng.choice(b64) for _ in range(10)) for _ in range(n)]
    elif shape == "skew":       # a few values at some positions, a constant position, skewed frequencies
        ks = [bytes([rng.choice(b"abc"), 0x2F, rng.choice(b"xy" * 30 + b"z")]) +
              bytes(rng.choice(b64[:20]) for _ in range(rng.randrange(0, 7))) for _ in range(n)]
    elif shape == "short_nul":  # lengths 0..3 incl. NUL bytes: zero padding vs real NULs
        ks = [bytes(rng.choice(b"\x00\x01A") for _ in range(rng.randrange(0, 4))) for _ in range(n)]
    else:                       # "dec": decimal digits, 10 values per position (4 bits, 3.3 bits entropy)
        ks = [b"%012d" % rng.randrange(10 ** 12) for _ in range(n)]
    return [(k, b"v%d" % i) for i, k in enumerate(ks)]


@pytest.mark.parametrize("shape,n", [("bits1", 50_000), ("bytes8", 120_000), ("b64", 200_000),
                                     ("skew", 60_000), ("short_nul", 5_000), ("dec", 150_000)])
def test_key_entropy_shapes_vs_oracle(oracle_lib, shape, n):
    """Key sets whose bytes carry 1, 3.3, 6 or 8 bits each (the adaptive digit choice of the prefix sort
    stops at different bytes, mid-byte entropy), constant and skewed positions, NULs vs zero padding,
    duplicates (last write wins): build + diff against the oracle."""
    rng = random.Random(sum(shape.encode()))
    pairs = _entropy_pairs(rng, shape, n)
    t, o = _check_pairs(oracle_lib, pairs)
    other = dict(pairs)
    ks = sorted(other)
    for k in ks[::53]:
        other[k] = b"changed"
    for k in ks[7::101]:
        other.pop(k)
    t2 = MerkleTree()
    t2.build(list(other), list(other.values()))
    o2 = oracle_lib.OracleTree.from_pairs(list(other.items()))
    assert t2.get_root_hash() == o2.root()
    assert t.diff_keys_bytes(t2) == o.diff(o2)



def test_sort_window_hint_across_builds(oracle_lib):
    """One handle rebuilt over key sets with different shared prefixes: the first histogram pass starts
    at the previous build's shared length (tree.cpp sort_unique) and must fall back to a second pass
    whenever that hint is wrong (longer, shorter, none, single key)."""
    rng = random.Random(23)
    t = MerkleTree()
    shapes = ["tenant19", "tenant19", "user5", "mixed", "tenant19", "one", "long41", "tenant19", "b64"]
    for shape in shapes:
        if shape == "one":
            pairs = [(b"tenant/0001/object/zz", b"v")]
        elif shape == "b64":
            pairs = _entropy_pairs(rng, "b64", 20_000)
        else:
            pairs = _shared_prefix_pairs(rng, shape, 20_000)
        t.build([k for k, _ in pairs], [v for _, v in pairs])
        assert_tree_equal(t, oracle_lib.OracleTree.from_pairs(pairs), check_levels=False)


@pytest.mark.parametrize("layout", ["disjoint", "overlap_half", "interleaved", "reversed_disjoint"])
def test_merge_join_partition_far_from_interpolation_vs_oracle(oracle_lib, layout):
    """Equal leaf counts with different key sets (fingerprints differ: straight to the merge-join) whose
    merge-path splits lie far from the |A| / (|A| + |B|) interpolation the partition's first, exponential
    round probes around (k_diff.hip k_diff_partition): up to n/2 = 100K positions away, beyond its
    +-65,535 reach, so the 33-ary rounds finish the search."""
    n = 200_000
    keys = sorted({b"%010d" % (i * 104729 % 1000000007) for i in range(2 * n + 10)})[: 2 * n]
    if layout == "disjoint":
        ka, kb = keys[:n], keys[n:]
    elif layout == "reversed_disjoint":
        ka, kb = keys[n:], keys[:n]
    elif layout == "overlap_half":
        ka, kb = keys[:n], keys[n // 2: n // 2 + n]
    else:
        ka, kb = keys[0::2], keys[1::2]
    a_pairs = [(k, b"x") for k in ka]
    b_pairs = [(k, b"x" if i % 11 else b"y") for i, k in enumerate(kb)]
    a, b = MerkleTree(), MerkleTree()
    a.build([k for k, _ in a_pairs], [v for _, v in a_pairs])
    b.build([k for k, _ in b_pairs], [v for _, v in b_pairs])
    oa = oracle_lib.OracleTree.from_pairs(a_pairs)
    ob = oracle_lib.OracleTree.from_pairs(b_pairs)
    assert a.diff_keys_bytes(b) == oa.diff(ob)
    assert b.diff_keys_bytes(a) == ob.diff(oa)
