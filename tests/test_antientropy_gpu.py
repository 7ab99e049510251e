"""Anti-entropy end to end on the device (sync.rs:56-87, README.md:315-341):
  * mkv_tree_build_digests: a tree from shipped (key, leaf digest) pairs equals the tree of the records;
  * exchange_diff's key-set fallback runs on the device (shadow tree + merge-join), no host set diff;
  * sync_once: diff -> fetch remote values -> set/delete locally (sync.rs:74-83) -> update the local
    tree (dirty path for value-only divergence, batch merge for key-set changes); both replicas' roots
    converge, and the local store equals the remote store;
  * HASH [pattern] with the server's '*' convention (server.rs:651-656) against the golden fixture.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.antientropy import Peer, exchange_diff, sync_once  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, PyMerkleTree, leaf_hash, split_blob  # noqa: E402


def _tree(store: dict) -> MerkleTree:
    t = MerkleTree()
    ks = sorted(store)
    t.build(ks, [store[k] for k in ks])
    return t


@pytest.mark.parametrize("n", [0, 1, 2, 3, 1000, 65_537])
def test_build_digests_equals_build(n):
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n) if n else (np.zeros(0, np.uint8), np.zeros(1, np.uint64),
                                                                        np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    a = MerkleTree()
    a.build((kb, ko), (vb, vo))
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    dig = b"".join(leaf_hash(k, v) for k, v in zip(keys, vals))
    b = MerkleTree.from_digests((kb, ko), np.frombuffer(dig, np.uint8) if dig else np.zeros(0, np.uint8))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    assert b.get_root_hash() == a.get_root_hash() == o.root()  # both against the oracle, not each other
    assert len(b) == len(a) == len(o)
    if n:
        raw, offs, d = a.leaves_packed()
        raw2, offs2, d2 = b.leaves_packed()
        assert np.array_equal(raw, raw2) and np.array_equal(offs, offs2) and np.array_equal(d, d2)
        assert np.array_equal(d, o.level(0))
        assert a.diff_keys_bytes(b) == []


def test_build_digests_duplicates_last_wins():
    keys = [b"k2", b"k1", b"k2", b"k3", b"k1"]
    vals = [b"a", b"b", b"c", b"d", b"e"]
    ref = PyMerkleTree()
    for k, v in zip(keys, vals):
        ref.insert(k, v)
    t = MerkleTree.from_digests(keys, [leaf_hash(k, v) for k, v in zip(keys, vals)])
    assert t.get_root_hash() == ref.get_root_hash()


def _replicas(n, seed, mixed):
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    local = dict(zip(keys, vals))
    remote = dict(local)
    rng = np.random.default_rng(seed)
    for i in rng.choice(n, size=max(1, n // 100), replace=False):
        remote[keys[i]] = b"changed-" + vals[i][:20]
    if mixed:
        for i in rng.choice(n, size=max(1, n // 1000), replace=False):
            remote.pop(keys[i], None)
        for j in range(max(1, n // 1000)):
            remote[b"new/%08d" % j] = b"fresh-%d" % j
        for i in rng.choice(n, size=max(1, n // 2000), replace=False):  # local-only keys get deleted
            local[b"local-only/%06d" % i] = b"x"
    return local, remote


@pytest.mark.parametrize("n,mixed", [(20_000, False), (20_000, True), (300_000, True)])
def test_sync_once_converges(n, mixed):
    local, remote = _replicas(n, 7 + n, mixed)
    lt, rt = _tree(local), _tree(remote)
    want_diff = lt.diff_keys_bytes(rt)
    oracle_l, oracle_r = PyMerkleTree(), PyMerkleTree()
    for k, v in local.items():
        oracle_l.insert(k, v)
    for k, v in remote.items():
        oracle_r.insert(k, v)
    assert want_diff == oracle_l.diff_keys(oracle_r)
    rep = sync_once(lt, local, Peer(rt, remote))
    assert rep.diffs == want_diff
    assert rep.path == ("batch merge" if mixed else "dirty-path upsert")
    assert rep.stats.fallback == mixed
    assert local == remote  # the store is now the peer's (sync.rs:74-83)
    assert lt.get_root_hash() == rt.get_root_hash() == oracle_r.get_root_hash()
    assert lt.diff_keys_bytes(rt) == []
    again = sync_once(lt, local, Peer(rt, remote))
    assert again.path == "identical" and again.diffs == []


def test_sync_once_edge_cases():
    # empty local: everything is inserted
    local, remote = {}, {b"a": b"1", b"b": b"2", b"c": b"3"}
    lt, rt = MerkleTree(), _tree(remote)
    rep = sync_once(lt, local, Peer(rt, remote))
    assert rep.set_keys == 3 and local == remote and lt.get_root_hash() == rt.get_root_hash()
    # empty remote: everything local is deleted; both roots None (R6)
    local, remote = {b"a": b"1", b"b": b"2"}, {}
    lt, rt = _tree(local), MerkleTree()
    rep = sync_once(lt, local, Peer(rt, remote))
    assert rep.deleted_keys == 2 and local == {} and lt.get_root_hash() is None and rt.get_root_hash() is None
    # same key count, different keys (positions line up by count only): the key check falls back
    local, remote = {b"a": b"1", b"b": b"2"}, {b"a": b"1", b"c": b"2"}
    lt, rt = _tree(local), _tree(remote)
    got, st = exchange_diff(lt, Peer(rt, remote))
    assert got == [b"b", b"c"] and st.fallback
    sync_once(lt, local, Peer(rt, remote))
    assert local == remote and lt.get_root_hash() == rt.get_root_hash()


def test_hash_pattern_fixture(fixtures):
    fx = fixtures["hash_patterns"]
    t = MerkleTree()
    t.build([k.encode() for k in fx["keys"]], [v.encode() for v in fx["values"]])
    for p, want in fx["roots"].items():
        got = t.hash_pattern(p)
        assert (got.hex() if got else None) == want, p
    assert t.hash_pattern(None) == t.hash_pattern("*") == t.get_root_hash()
    # the raw range reduction treats '*' as a byte: keys "*", "*a", "*b", "**"
    ref = PyMerkleTree()
    for k, v in zip(fx["keys"], fx["values"]):
        ref.insert(k.encode(), v.encode())
    assert t.prefix_root("*") == ref.prefix_root(b"*") != t.get_root_hash()
    assert t.hash_command("c") == "HASH c " + "0" * 64 + "\r\n"
    assert t.hash_command() == "HASH " + t.get_root_hash().hex() + "\r\n"
