"""Incremental anti-entropy update (BASELINE configs[4]): value-only upsert batches take the dirty path
(k_update.hip) and must equal the reference's insert-then-rebuild (merkle.rs:52-56) bit-exactly: root,
every level array, and diffs against the pre-update tree. Sharded trees: in-place shard updates +
fringe/combine give the unsharded root; top-down diff from the shard's fringe roots equals the
unsharded diff restricted to the shard. Checked against the C oracle (oracle/merkle_oracle.c)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED, pack, split_blob  # noqa: E402


def _levels(t: MerkleTree):
    return [b"".join(t.level_digests(l)) for l in range(t.level_count())]


def _oracle_levels(o):
    return [o.level(l).tobytes() for l in range(o.nlevels())]


def _batch(keys, idx, tag):
    """Update records for keys[idx] (in the given order, duplicates allowed) with fresh values."""
    ks = [keys[int(i)] for i in idx]
    vs = [b"upd-%s-%d-%d" % (tag.encode(), j, int(i)) for j, i in enumerate(idx)]
    return ks, vs


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 64, 1000, 4097, 65537])
def test_dirty_path_matches_rebuild(n):
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    rng = np.random.default_rng(n)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    base = t.clone()
    m = max(1, n // 7)
    idx = list(rng.integers(0, n, size=m))
    idx += [n - 1, 0] + idx[: max(1, m // 3)]  # last leaf (R5 promotion path), first, duplicates
    ks, vs = _batch(keys, idx, "a")
    t.upsert(ks, vs)
    kb2, ko2 = pack(ks)
    vb2, vo2 = pack(vs)
    o2 = o.upsert(kb2, ko2, vb2, vo2)
    assert t.get_root_hash() == o2.root()
    assert _levels(t) == _oracle_levels(o2)
    assert base.diff_keys_bytes(t) == o.diff(o2)
    # a second batch on the updated tree (bitmap must be clean again)
    idx2 = list(rng.integers(0, n, size=max(1, n // 3)))
    ks3, vs3 = _batch(keys, idx2, "b")
    t.upsert(ks3, vs3)
    kb3, ko3 = pack(ks3)
    vb3, vo3 = pack(vs3)
    o3 = o2.upsert(kb3, ko3, vb3, vo3)
    assert t.get_root_hash() == o3.root()
    assert _levels(t) == _oracle_levels(o3)


def test_dirty_path_same_value_is_noop():
    n = 1000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    want = t.get_root_hash()
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    t.upsert(keys[10:20], vals[10:20])
    assert t.get_root_hash() == want


def test_batch_with_new_key_falls_back_exactly():
    n = 3000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    ks = [keys[5], b"zz-new-key", keys[5], keys[2999]]
    vs = [b"1", b"2", b"3", b"4"]
    t.upsert(ks, vs)
    o2 = o.upsert(*pack(ks), *pack(vs))
    assert len(t) == n + 1
    assert t.get_root_hash() == o2.root()
    assert _levels(t) == _oracle_levels(o2)


def test_upsert_device_dirty_and_fallback():
    import torch
    n = 20000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    for tag, ks in (("dirty", [keys[i] for i in range(0, n, 97)] + [keys[3]]),
                    ("fallback", [keys[1], b"brand-new"])):
        vs = [b"v-%s-%d" % (tag.encode(), i) for i in range(len(ks))]
        bk, bo = pack(ks)
        bv, bvo = pack(vs)
        dk = torch.from_numpy(bk.copy()).cuda()
        dko = torch.from_numpy(bo.astype(np.int64)).cuda()
        dv = torch.from_numpy(bv.copy()).cuda()
        dvo = torch.from_numpy(bvo.astype(np.int64)).cuda()
        torch.cuda.synchronize()
        t.upsert_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), len(ks))
        o = o.upsert(bk, bo, bv, bvo)
        assert t.get_root_hash() == o.root(), tag
    assert _levels(t) == _oracle_levels(o)


@pytest.mark.parametrize("base_off", [1000, 4, 3])
def test_fixed_length_keys_at_offset_base(base_off):
    """Trees whose keys all have one length address them arithmetically (kb + koff[0] + s x len,
    DiffSide::klen). Device inputs whose offsets start at base_off (a slice of a larger buffer; 3 leaves
    the key bytes unaligned) over 2^20 + 100 keys (so the update locates through the hash index): root,
    value-only update (locate + dirty climb), merge of a new key, diffs — all vs the oracle
    (merkle.rs:52-56, :73-121, :171-204)."""
    import torch
    n = (1 << 20) + 100
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    dk = torch.zeros(base_off + len(kb) + 16, dtype=torch.uint8)
    dk[base_off:base_off + len(kb)] = torch.from_numpy(kb)
    dk = dk.cuda()
    dko = torch.from_numpy(ko.astype(np.int64) + base_off).cuda()
    dv = torch.from_numpy(vb.copy()).cuda()
    dvo = torch.from_numpy(vo.astype(np.int64)).cuda()
    torch.cuda.synchronize()
    t = MerkleTree()
    t.build_device(dk.data_ptr(), dko.data_ptr(), dv.data_ptr(), dvo.data_ptr(), n)
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    assert t.get_root_hash() == o.root()
    base, ob = t.clone(), o
    rng = np.random.default_rng(base_off)
    idx = sorted(int(i) for i in rng.choice(n, 5000, replace=False))
    uk, uv = [keys[i] for i in idx], [b"u-%d" % i for i in idx]
    t.upsert(uk, uv)  # value-only: hash-index locate + dirty climb
    o = o.upsert(*pack(uk), *pack(uv))
    assert t.get_root_hash() == o.root()
    assert base.diff_keys_bytes(t) == ob.diff(o) == sorted(uk)
    assert t.diff_keys_bytes(base) == o.diff(ob)
    nk = keys[7][:-1] + b"#"  # one new key of the same length: merge path, the tree stays fixed-length
    t.upsert([nk], [b"new"])
    o = o.upsert(*pack([nk]), *pack([b"new"]))
    assert t.get_root_hash() == o.root()
    assert base.diff_keys_bytes(t) == ob.diff(o)


@pytest.mark.parametrize("n,m", [(20000, 300), (70001, 9000)])
def test_upsert_device_many_matches_separate_calls(n, m):
    """Batched dirty climb of several replicas (shared level plan) + a replica of another size (own
    group) + one batch with a new key (general path) == separate upserts == oracle."""
    import torch
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    rng = np.random.default_rng(m)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    small_n = n // 3
    kbs, kos, vbs, vos = coracle.gen_records(DEFAULT_SEED, 0, small_n)
    small = MerkleTree()
    small.build((kbs, kos), (vbs, vos))
    osmall = coracle.OracleTree.build(kbs, kos, vbs, vos)
    trees = [base.clone() for _ in range(4)] + [small]
    refs = [base.clone() for _ in range(4)] + [small.clone()]
    batches, keep, expect = [], [], []
    for r in range(5):
        pool = keys if r < 4 else split_blob(kbs, kos)
        idx = list(rng.integers(0, len(pool), size=m)) + [len(pool) - 1, 0]
        ks = [pool[int(i)] for i in idx]
        if r == 3:
            ks.append(b"zz-new-key-%d" % r)  # key-set change: this tree leaves the group
        vs = [b"many-%d-%d-%d" % (r, j, int(i)) for j, i in enumerate(idx)] + [b"nv"] * (len(ks) - len(idx))
        bk, bo = pack(ks)
        bv, bvo = pack(vs)
        d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
             torch.from_numpy(bv.copy()).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
        keep.append(d)
        batches.append((d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(ks)))
        expect.append((o if r < 4 else osmall).upsert(bk, bo, bv, bvo))
    torch.cuda.synchronize()
    MerkleTree.upsert_device_many(trees, batches)
    for t, b in zip(refs, batches):
        t.upsert_device(*b)
    for r in range(5):
        assert trees[r].get_root_hash() == expect[r].root() == refs[r].get_root_hash(), r
        assert _levels(trees[r]) == _oracle_levels(expect[r]), r
    # a second batched round on the same handles (bitmaps must be clean again)
    MerkleTree.upsert_device_many(trees[:3], batches[:3])
    for r in range(3):
        refs[r].upsert_device(*batches[r])
        assert trees[r].get_root_hash() == refs[r].get_root_hash(), r


def _shard_trees(kb, ko, vb, vo, cuts):
    """Sorted records split at cuts -> prepared+reduced+combined shard trees."""
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    order = sorted(range(len(keys)), key=lambda i: keys[i])
    ks = [keys[i] for i in order]
    vs = [vals[i] for i in order]
    bounds = [0] + list(cuts) + [len(ks)]
    trees = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        t = MerkleTree()
        t.shard_prepare(ks[a:b], vs[a:b])
        trees.append(t)
    N = len(ks)
    fr = b""
    for r, t in enumerate(trees):
        t.shard_reduce(bounds[r], N)
        fr += t.shard_fringe()
    roots = [t.shard_combine(fr, len(trees), N) for t in trees]
    return trees, ks, bounds, roots


def _recombine(trees, N):
    fr = b"".join(t.shard_fringe() for t in trees)
    return [t.shard_combine(fr, len(trees), N) for t in trees]


@pytest.mark.parametrize("n,cuts", [(1001, (333, 700)), (40000, (1, 16384, 16385, 39999)), (7, (3,)),
                                    (200003, (1, 2, 77777, 131072, 131073, 199999, 200002))])
def test_sharded_dirty_update_and_topdown_diff(n, cuts):
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    trees, ks, bounds, roots = _shard_trees(kb, ko, vb, vo, cuts)
    full = MerkleTree()
    full.build((kb, ko), (vb, vo))
    assert all(r == full.get_root_hash() for r in roots)
    base = [t.clone() for t in trees]
    base_full = full.clone()
    rng = np.random.default_rng(n)
    idx = sorted(set(int(i) for i in rng.integers(0, n, size=max(2, n // 50)))) + [n - 1]
    upd_k = [ks[i] for i in idx]
    upd_v = [b"new-%d" % i for i in idx]
    full.upsert(upd_k, upd_v)
    for r, t in enumerate(trees):
        a, b = bounds[r], bounds[r + 1]
        sel = [j for j, i in enumerate(idx) if a <= i < b]
        if sel:
            t.upsert([upd_k[j] for j in sel], [upd_v[j] for j in sel])
    roots2 = _recombine(trees, n)
    assert all(r == full.get_root_hash() for r in roots2)
    want = base_full.diff_keys_bytes(full)
    assert want == sorted(set(upd_k))
    got = []
    for b0, t in zip(base, trees):
        got += b0.diff_keys_bytes(t)
    assert got == want


def test_sharded_upsert_new_key_rejected():
    n = 100
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    trees, ks, bounds, roots = _shard_trees(kb, ko, vb, vo, (50,))
    from merklekv_amd import MerkleError
    with pytest.raises(MerkleError):
        trees[0].upsert([b"not-a-leaf"], [b"x"])


def test_merge_batches_key_set_changes_vs_oracle():
    """Key-set-changing batches take the sorted-batch merge: new keys, value updates,
    removes (present and absent), duplicates within a batch in both orders, and enough rounds that the
    key storage is repacked. Every round: root + all levels + leaves equal the oracle's."""
    rng = np.random.default_rng(77)
    n = 3000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    state = dict(zip(split_blob(kb, ko), split_blob(vb, vo)))
    for rnd in range(6):
        keys, vals, rm = [], [], []
        pool = sorted(state)
        for _ in range(2500):
            r = rng.random()
            if r < 0.35 and pool:
                k = pool[int(rng.integers(0, len(pool)))]          # update an existing key
                keys.append(k); vals.append(b"u%d-%d" % (rnd, len(keys))); rm.append(0)
            elif r < 0.6 and pool:
                k = pool[int(rng.integers(0, len(pool)))]          # remove an existing key
                keys.append(k); vals.append(b""); rm.append(1)
            elif r < 0.65:
                keys.append(b"absent-%d" % int(rng.integers(0, 10**9))); vals.append(b""); rm.append(1)
            else:
                k = b"new-%d-%d" % (rnd, int(rng.integers(0, 10**3)))  # repeats: in-batch duplicates
                keys.append(k); vals.append(b"n%d" % len(keys)); rm.append(0)
        # explicit duplicate orders: insert-then-remove and remove-then-insert of the same key
        keys += [b"dup-a-%d" % rnd, b"dup-a-%d" % rnd, b"dup-b-%d" % rnd, b"dup-b-%d" % rnd]
        vals += [b"x", b"", b"", b"y"]
        rm += [0, 1, 1, 0]
        t.apply(keys, vals, rm)
        for k, v, r in zip(keys, vals, rm):  # sequential semantics (merkle.rs:52-62)
            if r:
                state.pop(k, None)
            else:
                state[k] = v
        items = sorted(state.items())
        o = coracle.OracleTree.build(*pack([k for k, _ in items]), *pack([v for _, v in items]))
        assert len(t) == len(o), rnd
        assert t.get_root_hash() == o.root(), rnd
        assert _levels(t) == _oracle_levels(o), rnd
        assert [k.encode("utf-8", "surrogateescape") for k, _ in t.leaves()] == [k for k, _ in items], rnd


def test_diff_many_matches_pairwise_and_oracle():
    """mkv_tree_diff_many (configs[4]'s 1-vs-7 replica diff): one shared top-down walk for same-key-set
    replicas, pairwise fallback for the rest; every result equals its own diff_keys and the oracle."""
    n = 20011
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    obase = coracle.OracleTree.build(kb, ko, vb, vo)
    rng = np.random.default_rng(5)
    variants, oracles = [], []
    for v in range(7):
        t = base.clone()
        m = [0, 1, 50, 300, 2000, 5, 100][v]
        idx = [int(i) for i in rng.integers(0, n, size=m)] + ([n - 1] if v == 4 else [])
        ks = [keys[i] for i in idx]
        vs = [b"v%d-%d" % (v, j) for j in range(len(idx))]
        o = obase
        if ks:
            t.upsert(ks, vs)
            o = obase.upsert(*pack(ks), *pack(vs))
        if v == 5:  # key-set change: one removal + one insert keeps n but shifts positions
            t.remove_many([keys[7]])
            t.upsert([b"zzz-new"], [b"x"])
            o = o.remove(*pack([keys[7]])).upsert(*pack([b"zzz-new"]), *pack([b"x"]))
        variants.append(t)
        oracles.append(o)
    small = MerkleTree()  # different size: pairwise merge-join
    small.build((kb[: 32 * 100], ko[:101]), (vb[: 100 * 100], vo[:101]))
    variants.append(small)
    oracles.append(coracle.OracleTree.build(kb[: 32 * 100], ko[:101], vb[: 100 * 100], vo[:101]))
    got = base.diff_keys_many_packed(variants)
    for i, (t, o) in enumerate(zip(variants, oracles)):
        raw, offs = got[i]
        b, oo = raw.tobytes(), offs.tolist()
        lst = [b[oo[j]:oo[j + 1]] for j in range(len(oo) - 1)]
        assert lst == base.diff_keys_bytes(t), i
        assert lst == obase.diff(o), i


def test_keyset_identity_follows_clones_and_key_changes():
    """Diffs between trees sharing a key-set id (a clone plus value-only updates) skip the leaf-key
    check; any build or key insert/remove on either side must bring the check back."""
    n = 6007
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED + 3, 0, n)
    keys = split_blob(kb, ko)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    obase = coracle.OracleTree.build(kb, ko, vb, vo)
    c = base.clone()
    c.upsert([keys[11], keys[3000]], [b"c1", b"c2"])           # value-only: key set kept
    oc = obase.upsert(*pack([keys[11], keys[3000]]), *pack([b"c1", b"c2"]))
    assert base.diff_keys_bytes(c) == obase.diff(oc)
    # the base swaps one key for another (same count, same level plan): positions shift
    base.remove_many([keys[5]])
    base.upsert([b"~~late-key"], [b"x"])
    obase = obase.remove(*pack([keys[5]])).upsert(*pack([b"~~late-key"]), *pack([b"x"]))
    assert len(base) == len(c)
    assert base.diff_keys_bytes(c) == obase.diff(oc)
    assert c.diff_keys_bytes(base) == oc.diff(obase)
    got = base.diff_keys_many_packed([c, c.clone()])
    for raw, offs in got:
        b, oo = raw.tobytes(), offs.tolist()
        assert [b[oo[j]:oo[j + 1]] for j in range(len(oo) - 1)] == obase.diff(oc)
    # a clone rebuilt from different keys of the same count
    d = c.clone()
    keys2 = list(keys)
    keys2[100] = b"!" + keys2[100][1:]
    vals = split_blob(vb, vo)
    d.build(keys2, vals)
    od = coracle.OracleTree.from_pairs(list(zip(keys2, vals)))
    assert c.diff_keys_bytes(d) == oc.diff(od)


def test_antientropy_exchange_matches_diff_and_moves_little():
    """Top-down exchange (README.md:310-347): same result as diff_keys; for a sparse value-only
    divergence only a small fraction of the tree's digests cross the wire; key-set changes fall back."""
    from merklekv_amd.antientropy import Peer, exchange_diff
    n = 50_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    a = MerkleTree()
    a.build((kb, ko), (vb, vo))
    b = a.clone()
    idx = [3, 777, 4096, 20000, 49999]
    b.upsert([keys[i] for i in idx], [b"changed"] * len(idx))
    got, st = exchange_diff(a, Peer(b))
    assert got == a.diff_keys_bytes(b) == sorted(keys[i] for i in idx)
    assert not st.fallback and st.digests_sent < n // 20
    same, st2 = exchange_diff(a, Peer(a.clone()))
    assert same == [] and st2.digests_sent == 1
    c = a.clone()
    c.remove_many([keys[10]])
    c.upsert([b"zz-extra"], [b"v"])
    got3, st3 = exchange_diff(a, Peer(c))
    assert got3 == a.diff_keys_bytes(c) and st3.fallback
    d = MerkleTree()
    d.build((kb[: 32 * 1000], ko[:1001]), (vb[: 100 * 1000], vo[:1001]))
    got4, st4 = exchange_diff(a, Peer(d))
    assert got4 == a.diff_keys_bytes(d) and st4.fallback


def test_keylist_views_zero_copy_and_shared_blocks():
    """KeyList views over the pinned result blocks: equal to the copied lists; per-variant views of one
    mkv_tree_diff_many share a block, and freeing one leaves the others valid."""
    import gc
    n = 5000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    vs = []
    for v in range(3):
        t = base.clone()
        t.upsert([keys[i] for i in range(v, n, 97)], [b"x%d" % v] * len(range(v, n, 97)))
        vs.append(t)
    want = [base.diff_keys_bytes(t) for t in vs]
    views = base.diff_keys_many_view(vs)
    del views[0]
    gc.collect()
    for w, kl in zip(want[1:], views):
        b, o = kl.raw.tobytes(), kl.offs.tolist()
        assert [b[o[i]:o[i + 1]] for i in range(len(kl))] == w
    one = base.diff_keys_view(vs[2])
    b, o = one.raw.tobytes(), one.offs.tolist()
    assert [b[o[i]:o[i + 1]] for i in range(len(one))] == want[2]


def test_clone_keyset_change_then_batched_update_and_diff_vs_oracle():
    """the key-set id is a correctness input of the batched dirty path (a replica's batch is
    located in the first tree of its group) and of the batched walk (leaf-key check skipped). A clone
    that swaps keys through apply() (same count, same level plan) must leave the group: a batched
    upsert over [orig, clone] and diff_many against the original must still equal the oracle."""
    import torch
    n = 9001
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED + 17, 0, n)
    keys = split_blob(kb, ko)
    orig = MerkleTree()
    orig.build((kb, ko), (vb, vo))
    o_orig = coracle.OracleTree.build(kb, ko, vb, vo)
    clone = orig.clone()
    # apply(): remove two keys, insert two new ones (count and level plan unchanged, positions shift)
    new_keys = [b"!!first-new", b"~~last-new"]
    clone.apply([keys[10], keys[4000]] + new_keys, [b"", b""] + [b"n1", b"n2"], [1, 1, 0, 0])
    o_clone = o_orig.remove(*pack([keys[10], keys[4000]])).upsert(*pack(new_keys), *pack([b"n1", b"n2"]))
    assert len(clone) == len(orig) == n
    assert clone.get_root_hash() == o_clone.root()
    rng = np.random.default_rng(3)
    live = [k for k in keys if k not in (keys[10], keys[4000])]
    batches, keep, oracles = [], [], []
    for r, (t, o, pool) in enumerate(((orig, o_orig, keys), (clone, o_clone, live + new_keys))):
        idx = [int(i) for i in rng.integers(0, len(pool), size=257)]
        ks = [pool[i] for i in idx] + ([new_keys[1]] if r else [keys[10]])  # keys only this tree holds
        vs = [b"b%d-%d" % (r, j) for j in range(len(ks))]
        bk, bo = pack(ks)
        bv, bvo = pack(vs)
        d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
             torch.from_numpy(bv.copy()).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
        keep.append(d)
        batches.append((d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(ks)))
        oracles.append(o.upsert(bk, bo, bv, bvo))
    torch.cuda.synchronize()
    base = orig.clone()  # the pre-update original, for the batched diff
    MerkleTree.upsert_device_many([orig, clone], batches)
    assert orig.get_root_hash() == oracles[0].root()
    assert clone.get_root_hash() == oracles[1].root()
    assert _levels(clone) == _oracle_levels(oracles[1])
    got = base.diff_keys_many_packed([orig, clone])
    for (raw, offs), o in zip(got, oracles):
        b, oo = raw.tobytes(), offs.tolist()
        assert [b[oo[j]:oo[j + 1]] for j in range(len(oo) - 1)] == o_orig.diff(o)


@pytest.mark.parametrize("n,m,k", [(300_000, 140_000, 2), (40_000, 5_000, 3)])
def test_batched_update_fixed_shape_hash_vs_oracle(n, m, k):
    """The batched update hash (k_leaf_multi) on 32/100-B records takes the compile-time register path
    (and, for k x m >= 2^18 records, the plain round form); one batch mixes in a 99-B value so a wave falls
    back to the generic path mid-batch. Roots and every level equal the oracle's insert-then-rebuild."""
    import torch
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    rng = np.random.default_rng(n + m)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    kv = kb.reshape(n, 32)
    trees, keep, expect = [base.clone() for _ in range(k)], [], []
    for r in range(k):
        idx = rng.integers(0, n, size=m)
        bk = np.ascontiguousarray(kv[idx]).reshape(-1)
        vals = rng.integers(0, 256, size=(m, 100), dtype=np.uint8)
        vlens = np.full(m, 100, np.uint64)
        if r == 1:
            vlens[m // 2] = 99  # one ragged record: its wave takes the generic path
        bv = np.concatenate([vals[i, : int(vlens[i])] for i in range(m)]) if r == 1 else vals.reshape(-1)
        bo = np.arange(m + 1, dtype=np.uint64) * 32
        bvo = np.zeros(m + 1, np.uint64)
        bvo[1:] = np.cumsum(vlens)
        d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
             torch.from_numpy(np.ascontiguousarray(bv)).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
        keep.append(d)
        expect.append(o.upsert(bk, bo, np.ascontiguousarray(bv), bvo))
    torch.cuda.synchronize()
    MerkleTree.upsert_device_many(trees, [(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), m)
                                          for d in keep])
    for r in range(k):
        assert trees[r].get_root_hash() == expect[r].root(), r
        assert _levels(trees[r]) == _oracle_levels(expect[r]), r


@pytest.mark.parametrize("n", [262_144, 262_100, 300_000])
def test_locate_top_sample_edges_take_dirty_path(n):
    """Value batches hitting the smallest and largest keys: the locate's LDS top sample (LOC_TOP entries at
    a stride of the 1/64 samples) must bracket keys past its last entry (n = 262,144: 4,096 samples at
    stride 2, the last sample beyond the top sample) — a miss there is exact (merge fallback) but leaves
    the dirty path, so the test also checks that the dirty path ran (update_counts()[0] > 0)."""
    import torch
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    srt = sorted(keys)
    rng = np.random.default_rng(n)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    ks = srt[-300:] + srt[:300] + [srt[int(i)] for i in rng.integers(0, n, size=400)]
    vs = [b"edge-%d-%d" % (n, j) for j in range(len(ks))]
    bk, bo = pack(ks)
    bv, bvo = pack(vs)
    d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
         torch.from_numpy(bv.copy()).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
    torch.cuda.synchronize()
    exp = o.upsert(bk, bo, bv, bvo)
    single = base.clone()
    single.upsert_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(ks))
    many = [base.clone() for _ in range(2)]
    MerkleTree.upsert_device_many(many, [(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(),
                                          len(ks))] * 2)
    for t in [single] + many:
        assert t.get_root_hash() == exp.root()
        assert t.update_counts()[0] == len(set(ks))  # every batch key located: the dirty path ran


def test_value_only_diffs_take_the_topdown_walk():
    """Equal key sets with changed values: the pair diff and the batched 1-vs-k diff must come from the
    top-down walk (its divergent leaf count equals the result), not from the exact merge-join fallback."""
    n = 200_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    rng = np.random.default_rng(7)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    variants, expect = [], []
    for r in range(3):
        idx = sorted(set(int(i) for i in rng.integers(0, n, size=200)))
        vs2 = list(vals)
        for i in idx:
            vs2[i] = b"changed-%d-%d" % (r, i)
        bv, bvo = pack(vs2)
        t = MerkleTree()
        t.build((kb, ko), (bv, bvo))
        variants.append(t)
        expect.append(o.diff(coracle.OracleTree.build(kb, ko, bv, bvo)))
    assert base.diff_keys_bytes(variants[0]) == expect[0]
    ws = base.walk_stats()
    assert ws["launches"] > 0 and ws["divergent_positions"] == len(expect[0])
    got = base.diff_keys_many_packed(variants)
    for (raw, offs), e in zip(got, expect):
        assert split_blob(raw, offs) == e
    ws = base.walk_stats()
    assert ws["launches"] > 0 and ws["divergent_positions"] == sum(len(e) for e in expect)


@pytest.mark.parametrize("n,dens", [(300007, "sparse"), (300007, "medium"), (300007, "dense"), (4099, "dense"),
                                    (131072, "runs")])
def test_dirty_climb_passes_and_rendezvous_vs_oracle(n, dens):
    """The dirty climb (k_update.hip k_dirty_climb) in every regime its passes take: sparse batches (one
    dirty leaf per ~1000: every wave's lanes climb apart, merge at the pass boundaries and across waves),
    medium and dense ones (most merges inside a wave; a batch 3x the tree with duplicates), and long runs
    of one key (130 writes of a key straddle the 64-entry batches of the first pass; the last write wins,
    merkle.rs:54). Five replicas in one batched call (upsert_device_many), then every level array of every
    replica against the oracle's insert-then-rebuild (merkle.rs:52-56, :73-121)."""
    import torch
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    rng = np.random.default_rng(n + len(dens))
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    trees = [base.clone() for _ in range(5)]
    keep, batches, expect = [], [], []
    for r in range(5):
        m = {"sparse": max(1, n // 1000), "medium": n // 50, "dense": 3 * n, "runs": 200}[dens] + 17 * r
        idx = list(rng.integers(0, n, size=m))
        if dens == "runs":
            hot = int(rng.integers(0, n))
            idx = idx[:40] + [hot] * 130 + idx[40:] + [n - 1]
        ks = [keys[int(i)] for i in idx]
        vs = [b"climb-%d-%d-%d" % (r, j, int(i)) for j, i in enumerate(idx)]
        bk, bo = pack(ks)
        bv, bvo = pack(vs)
        d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
             torch.from_numpy(bv.copy()).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
        keep.append(d)
        batches.append((d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(ks)))
        expect.append(o.upsert(bk, bo, bv, bvo))
    torch.cuda.synchronize()
    MerkleTree.upsert_device_many(trees, batches)
    for r in range(5):
        assert trees[r].get_root_hash() == expect[r].root(), r
        assert _levels(trees[r]) == _oracle_levels(expect[r]), r
        assert sum(trees[r].update_counts()) > 0  # the dirty path ran (no fallback to the batch merge)


def test_hash_index_locate_shared_prefixes_and_missing_keys():
    """Trees of >= 2^20 keys locate batch keys through the hash index (k_update.hip locate_hix): keys that
    share a 19-byte prefix (the sample search's worst case, the index's hash covers the whole key), batch
    keys at both ends and repeated, then a batch with a key that is not a leaf (empty slot: counted
    missing, the exact merge path runs). Roots vs the oracle's insert-then-rebuild (merkle.rs:52-56)."""
    n = (1 << 20) + 4097
    keys = [b"tenant/0001/object/%010d" % (7 * i) for i in range(n)]
    vals = [b"v%d" % i for i in range(n)]
    kb, ko = pack(keys)
    vb, vo = pack(vals)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    rng = np.random.default_rng(20)
    idx = list(rng.integers(0, n, size=5000)) + [0, n - 1, n - 1, 1, n - 2]
    ks, vs = _batch(keys, idx, "hix")
    t.upsert(ks, vs)
    o2 = o.upsert(*pack(ks), *pack(vs))
    assert t.get_root_hash() == o2.root()
    assert t.update_counts()[0] == len(set(int(i) for i in idx))  # every key located: the dirty path ran
    ks3 = [keys[3], b"tenant/0001/object/0000000001", keys[n - 1]]  # 1 is no multiple of 7: not a leaf
    vs3 = [b"a", b"b", b"c"]
    t.upsert(ks3, vs3)
    o3 = o2.upsert(*pack(ks3), *pack(vs3))
    assert t.get_root_hash() == o3.root()
    assert len(t) == n + 1  # the new key was inserted by the merge path


def test_fixed_length_key_lists_follow_key_length_changes():
    """Key lists of trees whose keys all have one length skip the length gather (offsets k x len,
    tree.cpp pair_klen); a merged batch with a key of another length must turn that off, and trees of
    two different fixed lengths must not use it. Every list vs the oracle's R7 diff (merkle.rs:171-204)."""
    n = 20000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    assert len(set(len(k) for k in keys)) == 1
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    ob = coracle.OracleTree.build(kb, ko, vb, vo)
    t = base.clone()
    t.upsert([keys[5], b"short", keys[n - 1]], [b"x", b"y", b"z"])  # a 5-byte key: merge path
    o = ob.upsert(*pack([keys[5], b"short", keys[n - 1]]), *pack([b"x", b"y", b"z"]))
    assert t.get_root_hash() == o.root()
    assert base.diff_keys_bytes(t) == ob.diff(o)
    assert t.diff_keys_bytes(base) == o.diff(ob)
    # value-only update of the merged tree (dirty path keeps its key set), then diff again
    t.upsert([b"short", keys[7]], [b"y2", b"w"])
    o = o.upsert(*pack([b"short", keys[7]]), *pack([b"y2", b"w"]))
    assert base.diff_keys_bytes(t) == ob.diff(o)
    # two trees of different fixed lengths (every key of one tree is 2 bytes longer)
    k2 = [k + b"zz" for k in keys[:n // 2]] + keys[n // 2:]
    kb2, ko2 = pack(k2)
    t2 = MerkleTree()
    t2.build((kb2, ko2), (vb, vo))
    o2 = coracle.OracleTree.build(kb2, ko2, vb, vo)
    assert base.diff_keys_bytes(t2) == ob.diff(o2)
    k3 = [k + b"zz" for k in keys]
    kb3, ko3 = pack(k3)
    t3 = MerkleTree()
    t3.build((kb3, ko3), (vb, vo))
    o3 = coracle.OracleTree.build(kb3, ko3, vb, vo)
    assert base.diff_keys_bytes(t3) == ob.diff(o3)


def test_fixed_length_offsets_written_by_host_across_pool_cycles():
    """The one-wait diff of fixed-length keys has the host write the list's offsets k x len into the
    pinned staging block and keeps them while the block cycles through the pinned pool
    (tree.cpp PinnedBlock::fill_offsets; only the key bytes cross PCIe). Results of growing and shrinking
    size and of a second key length, some kept alive across calls so the blocks change hands, must all
    carry exact offsets and keys (R7, merkle.rs:171-204: the changed keys, sorted); the same for the
    batched 1-vs-k list (keylist_from_refs_async) and its per-variant views."""
    n = 60000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    k2 = [k + b"zz" for k in keys]
    kb2, ko2 = pack(k2)
    b1, b2 = MerkleTree(), MerkleTree()
    b1.build((kb, ko), (vb, vo))
    b2.build((kb2, ko2), (vb, vo))
    rng = np.random.default_rng(11)
    held = []
    for rnd, m in enumerate([10, 3000, 50, 20000, 5, 8000, 1, 12000]):
        for bt, ks in ((b1, keys), (b2, k2)):
            t = bt.clone()
            idx = sorted(int(i) for i in rng.choice(n, m, replace=False))
            t.upsert([ks[i] for i in idx], [b"new-%d" % rnd] * m)
            d = bt.diff_keys_view(t)
            L = len(ks[0])
            assert len(d) == m
            assert np.array_equal(d.offs, np.arange(m + 1, dtype=np.uint64) * np.uint64(L))
            raw = d.raw.tobytes()
            assert [raw[i * L:(i + 1) * L] for i in range(m)] == sorted(ks[i] for i in idx)
            held.append(d)
        held = held[-3:]
        # the batched 1-vs-k walk's shared list (host-written offsets too), split per variant
        for bt, ks in ((b1, keys), (b2, k2)):
            vs, want = [], []
            for v in range(3):
                t = bt.clone()
                idx = sorted(int(i) for i in rng.choice(n, m // (v + 1) + 1, replace=False))
                t.upsert([ks[i] for i in idx], [b"b-%d-%d" % (rnd, v)] * len(idx))
                vs.append(t)
                want.append(sorted(ks[i] for i in idx))
            L = len(ks[0])
            for d, w in zip(bt.diff_keys_many_view(vs), want):
                assert len(d) == len(w)
                assert np.array_equal(d.offs, np.arange(len(w) + 1, dtype=np.uint64) * np.uint64(L))
                raw = d.raw.tobytes()
                assert [raw[i * L:(i + 1) * L] for i in range(len(w))] == w
                held.append(d)
            held = held[-4:]


def test_batched_diff_per_variant_split_each_call():
    """The batched 1-vs-k diff splits one shared key list into per-variant lists from counters the walk
    writes into pinned memory; with fixed-length keys the key list needs no length readback, so the call
    must still wait for those counters. Rounds of shrinking, uneven per-variant batches on fresh clones
    (the pinned staging is reused, nothing else synchronises), every list vs the oracle's R7 diff."""
    n = 200000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    base = MerkleTree()
    base.build((kb, ko), (vb, vo))
    ob = coracle.OracleTree.build(kb, ko, vb, vo)
    rng = np.random.default_rng(77)
    for rnd, scale in enumerate((3000, 1500, 700, 300)):
        variants = [base.clone() for _ in range(4)]
        expect = []
        for i, v in enumerate(variants):
            m = scale * (i + 1) // 2 + 7 * rnd
            idx = rng.choice(n, size=m, replace=False)
            ks, vs = _batch(keys, idx, "r%d-%d" % (rnd, i))
            v.upsert(ks, vs)
            expect.append(ob.diff(ob.upsert(*pack(ks), *pack(vs))))
        got = base.diff_keys_many_packed(variants)
        for i, (raw, offs) in enumerate(got):
            b, o = raw.tobytes(), offs.tolist()
            assert [b[o[j]:o[j + 1]] for j in range(len(o) - 1)] == expect[i], (rnd, i)


@pytest.mark.parametrize("run", [1, 2, 63, 64, 65, 1000, 100_000])
def test_dirty_climb_hot_key_long_runs_vs_oracle(run):
    """One key written `run` times in a batch (plus scattered writes before and after it): the lane holding
    the run's LAST write finds the run's start by galloping back + a binary search over the sorted entries
    (a serial walk back was O(run) dependent loads on one lane). The last write wins (merkle.rs:54);
    root and every level array vs the oracle's insert-then-rebuild (merkle.rs:52-56, :73-121)."""
    import torch
    n = 200_003
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys = split_blob(kb, ko)
    rng = np.random.default_rng(run)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    hot = int(rng.integers(1, n - 1))
    idx = list(rng.integers(0, n, size=300)) + [hot] * run + list(rng.integers(0, n, size=300)) + [hot - 1, hot + 1]
    ks, vs = _batch(keys, idx, "hot")
    bk, bo = pack(ks)
    bv, bvo = pack(vs)
    d = [torch.from_numpy(bk.copy()).cuda(), torch.from_numpy(bo.astype(np.int64)).cuda(),
         torch.from_numpy(bv.copy()).cuda(), torch.from_numpy(bvo.astype(np.int64)).cuda()]
    torch.cuda.synchronize()
    t.upsert_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), len(ks))
    o2 = o.upsert(bk, bo, bv, bvo)
    assert t.get_root_hash() == o2.root()
    assert _levels(t) == _oracle_levels(o2)
    assert sum(t.update_counts()) > 0  # the dirty path ran
