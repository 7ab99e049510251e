"""configs[3] on one GPU: 1B keys sharded by key range over 8 GPUs, rehearsed as 8
in-process shards on one device with the exact per-rank protocol (shard_prepare -> counts -> shard_reduce
-> fringe -> combine; diffs per shard, rank order = global order).

  * 10M keys in 8 generator key ranges (shard=g, nshards=8): the global root of the sharded build and the
    concatenated per-shard value-only (top-down) and mixed (merge-join) diffs equal the C oracle on the
    union (/root/reference/src/store/merkle.rs:73-121, :171-196);
  * 125M keys (one configs[3] GPU's worth, split 8 ways) through the device fringe path
    (shard_fringe_device / shard_combine_device, stride = k x MKV_FRINGE_BYTES, two replicas per gathered
    block): root == the unsharded device build of the same records, and the sharded diffs equal the
    constructed divergent set with global offsets from the counts.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED  # noqa: E402

K, V = 32, 100
W = 8


@pytest.fixture(autouse=True)
def _free_torch_cache():
    yield
    import gc

    import torch
    gc.collect()
    torch.cuda.empty_cache()


def _concat(parts):
    """Union blob of fixed-shape shard blobs (kb, ko, vb, vo) in rank order."""
    kb = np.concatenate([p[0] for p in parts])
    vb = np.concatenate([p[2] for p in parts])
    n = sum(len(p[1]) - 1 for p in parts)
    return kb, np.arange(n + 1, dtype=np.uint64) * K, vb, np.arange(n + 1, dtype=np.uint64) * V


def _fixed(kb, vb):
    n = len(kb) // K
    return kb, np.arange(n + 1, dtype=np.uint64) * K, vb, np.arange(n + 1, dtype=np.uint64) * V


def _sharded_host(parts):
    """The per-rank protocol with host fringes; returns (trees, roots, counts)."""
    trees = [MerkleTree() for _ in parts]
    counts = [t.shard_prepare((kb, ko), (vb, vo)) for t, (kb, ko, vb, vo) in zip(trees, parts)]
    N = sum(counts)
    for r, t in enumerate(trees):
        t.shard_reduce(sum(counts[:r]), N)
    fr = b"".join(t.shard_fringe() for t in trees)
    return trees, [t.shard_combine(fr, len(trees), N) for t in trees], counts


def _replica_b(g, kb, vb, mixed):
    """Shard g's B records: every 1000th value changed; mixed also deletes every 1201st record and
    inserts 1/1000 new keys of the same key range."""
    k2, v2 = kb.reshape(-1, K), vb.reshape(-1, V).copy()
    n = len(k2)
    v2[np.arange(3 + g, n, 1000), 5] ^= 0x10
    if not mixed:
        return k2.reshape(-1), v2.reshape(-1)
    keep = np.ones(n, bool)
    keep[np.arange(11 + g, n, 1201)] = False
    m = n // 1000
    nk, _, nv, _ = coracle.gen_records(DEFAULT_SEED, 10**12 + g * m, m, shard=g, nshards=W)
    return (np.concatenate([k2[keep].reshape(-1), nk]), np.concatenate([v2[keep].reshape(-1), nv]))


def test_sharded_8way_10m_vs_oracle():
    ng = 1_250_000
    parts = [coracle.gen_records(DEFAULT_SEED, g * ng, ng, shard=g, nshards=W) for g in range(W)]
    shani = coracle.set_backend(1)  # SHA-NI oracle backend (cross-checked vs portable in test_oracle)
    try:
        oa = coracle.OracleTree.build(*_concat(parts))
        trees_a, roots_a, counts_a = _sharded_host(parts)
        assert counts_a == [ng] * W
        assert roots_a == [oa.root()] * W
        for mixed in (False, True):
            bparts = [_fixed(*_replica_b(g, p[0], p[2], mixed)) for g, p in enumerate(parts)]
            ob = coracle.OracleTree.build(*_concat(bparts))
            trees_b, roots_b, counts_b = _sharded_host(bparts)
            assert roots_b == [ob.root()] * W, mixed
            want = oa.diff(ob)
            got, offs = [], []
            for ta, tb in zip(trees_a, trees_b):
                offs.append(len(got))
                got += ta.diff_keys_bytes(tb)
            assert got == want, mixed
            assert len(want) >= W * ng // 1000
            del trees_b
    finally:
        coracle.set_backend(0)
    assert shani in (0, 1)


def _dev_shard(torch, g, ng, kall, vall):
    """Generate shard g's records into its slice of the union buffers; returns device offsets."""
    from merklekv_amd.merkle import gen_records_device
    ko = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    kv = kall[g * ng * K:(g + 1) * ng * K]
    vv = vall[g * ng * V:(g + 1) * ng * V]
    gen_records_device(0, DEFAULT_SEED, g * ng, ng, K, V, kv.data_ptr(), ko.data_ptr(), vv.data_ptr(),
                       vo.data_ptr(), shard=g, nshards=W)
    return kv, ko, vv, vo


def _sharded_device(torch, blobs):
    """The RCCL path's device-resident fringe buffers: every shard writes its fringe into a (world x 2 x
    FRINGE_BYTES) buffer (two replica slots per rank, like shard_recombine_many), combined from there."""
    from merklekv_amd._lib import FRINGE_BYTES
    trees = [MerkleTree() for _ in blobs]
    counts = [t.shard_prepare(b, None, on_device=True) for t, b in zip(trees, blobs)]
    N = sum(counts)
    for r, t in enumerate(trees):
        t.shard_reduce(sum(counts[:r]), N)
    buf = torch.zeros(len(trees) * 2 * FRINGE_BYTES, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for r, t in enumerate(trees):
        t.shard_fringe_device(buf.data_ptr() + (2 * r + 1) * FRINGE_BYTES)  # slot 1 of rank r
    roots = [t.shard_combine_device(buf.data_ptr() + FRINGE_BYTES, len(trees), 2 * FRINGE_BYTES, N)
             for t in trees]
    return trees, roots, counts


def test_sharded_8way_125m_device_fringe():
    import torch
    ng = 125_000_000 // W
    n = ng * W
    kall = torch.empty(n * K + 64, dtype=torch.uint8, device="cuda")
    vall = torch.empty(n * V + 64, dtype=torch.uint8, device="cuda")
    shards = [_dev_shard(torch, g, ng, kall, vall) for g in range(W)]
    torch.cuda.synchronize()
    blobs = [(kv, ko, vv, vo, ng) for kv, ko, vv, vo in shards]
    trees_a, roots_a, counts = _sharded_device(torch, blobs)
    assert counts == [ng] * W
    # the unsharded device build of the same records (the 10M sharded test pins both to the oracle)
    uko = torch.arange(0, n + 1, device="cuda", dtype=torch.int64) * K
    uvo = torch.arange(0, n + 1, device="cuda", dtype=torch.int64) * V
    torch.cuda.synchronize()
    whole = MerkleTree()
    whole.build_device(kall.data_ptr(), uko.data_ptr(), vall.data_ptr(), uvo.data_ptr(), n)
    want_root = whole.get_root_hash()
    del whole, uko, uvo
    torch.cuda.empty_cache()
    assert roots_a == [want_root] * W
    assert want_root == _golden_root(W, ng)  # pinned by the CPU oracle (tests/golden/roots_sharded.json)
    # replicas: value-only (top-down per shard) and mixed (merge-join per shard), 0.1 % per shard
    g_ = torch.Generator(device="cuda")
    g_.manual_seed(31)
    for mode in ("value_only", "mixed"):
        bl, exp = [], []
        for g, (kv, ko, vv, vo) in enumerate(shards):
            k2, v2 = kv.view(ng, K), vv.view(ng, V).clone()
            perm = torch.randperm(ng, device="cuda", generator=g_)
            nd = ng // 1000
            if mode == "value_only":
                chg, rm, new = perm[:nd], perm[:0], 0
            else:
                c, r = nd * 8 // 10, nd // 10
                chg, rm, new = perm[:c], perm[c:c + r], nd - c - r
            v2[chg, 9] ^= 4
            keep = torch.ones(ng, dtype=torch.bool, device="cuda")
            keep[rm] = False
            kB, vB = k2[keep], v2[keep]
            e = [k2[chg], k2[rm]]
            if new:
                from merklekv_amd.merkle import gen_records_device
                nkb = torch.empty(new * K + 64, dtype=torch.uint8, device="cuda")
                nvb = torch.empty(new * V + 64, dtype=torch.uint8, device="cuda")
                nko = torch.empty(new + 1, dtype=torch.int64, device="cuda")
                nvo = torch.empty(new + 1, dtype=torch.int64, device="cuda")
                gen_records_device(0, DEFAULT_SEED, 10**12 + g * new, new, K, V, nkb.data_ptr(), nko.data_ptr(),
                                   nvb.data_ptr(), nvo.data_ptr(), shard=g, nshards=W)
                torch.cuda.synchronize()
                kB = torch.cat([kB, nkb[: new * K].view(new, K)])
                vB = torch.cat([vB, nvb[: new * V].view(new, V)])
                e.append(nkb[: new * K].view(new, K))
            nb = kB.shape[0]
            kBf, vBf = kB.contiguous().view(-1), vB.contiguous().view(-1)
            bl.append((kBf, torch.arange(0, nb + 1, device="cuda", dtype=torch.int64) * K, vBf,
                       torch.arange(0, nb + 1, device="cuda", dtype=torch.int64) * V, nb))
            ex = torch.cat(e).cpu().numpy()
            exp.append(ex[np.lexsort(ex.T[::-1])])
            del v2, kB, vB
        torch.cuda.synchronize()
        trees_b, roots_b, counts_b = _sharded_device(torch, bl)
        assert len(set(roots_b)) == 1 and roots_b[0] != want_root
        want = np.concatenate(exp)  # ranges are ordered by rank: the concatenation is the global order
        got, offs = [], []
        for ta, tb in zip(trees_a, trees_b):
            raw, o = ta.diff_keys_packed(tb)
            offs.append(sum(len(x) for x in got))
            got.append(raw.reshape(-1, K))
        cnt = [len(x) for x in got]
        assert offs == [sum(cnt[:r]) for r in range(W)]  # global offsets from the counts
        g_all = np.concatenate(got)
        assert np.array_equal(g_all, want), mode
        assert (np.lexsort(g_all.T[::-1]) == np.arange(len(g_all))).all()  # globally sorted
        del trees_b, bl
        torch.cuda.empty_cache()


def _golden_root(shards, per_shard):
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "roots_sharded.json")))
    for c in d["cases"]:
        if c["shards"] == shards and c["per_shard"] == per_shard and c["seed"] == DEFAULT_SEED:
            return bytes.fromhex(c["root"])
    raise KeyError((shards, per_shard))


def test_configs3_1b_root_sequential_shards_vs_golden():
    """configs[3] at its full size: 1B keys = 8 key ranges x 125M records (generator shard g of 8, records
    [g * 125M, (g + 1) * 125M)), built on ONE GPU shard after shard (shard.sequential_root: prepare ->
    reduce at the shard's global offset -> fringe; each shard's records regenerated into the same buffers),
    then the seam combine of the 8 fringes. The root equals the golden root the CPU oracle computed over
    the same 1B records (tests/golden/roots_sharded.json, oracle/root_stream.c, merkle.rs:73-121)."""
    import torch

    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import sequential_root
    ng, nsh = 125_000_000, 8
    kb = torch.empty(ng * K + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(ng * V + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(ng + 1, dtype=torch.int64, device="cuda")

    def shards():
        for g in range(nsh):
            gen_records_device(0, DEFAULT_SEED, g * ng, ng, K, V, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                               vo.data_ptr(), shard=g, nshards=nsh)
            torch.cuda.synchronize()
            yield (kb, ko, vb, vo, ng)

    t = MerkleTree()
    root, counts = sequential_root(t, shards(), ng * nsh)
    assert counts == [ng] * nsh
    assert root == _golden_root(nsh, ng)
    del t, kb, vb, ko, vo


def _sorted_rows(a):
    return a[np.lexsort(a.T[::-1])] if len(a) else a


def _b_shard(torch, g, ng, kv, ko, vv, vo, mode):
    """Replica B of shard g (0.1 % of the records): value_only flips a byte of every 1000th value (rows
    3 + g mod 1000); mixed removes every tenth of those rows and inserts as many new keys of the same key
    range, so both replicas keep n_g leaves per shard (equal global offsets, different key sets -> the
    merge-join). Returns (B blob, expected divergent keys of the shard, sorted)."""
    from merklekv_amd.merkle import gen_records_device
    rows = torch.arange(3 + g, ng, 1000, device="cuda")
    k2, v2 = kv[: ng * K].view(ng, K), vv[: ng * V].view(ng, V).clone()
    if mode == "value_only":
        v2[rows, 9] ^= 4
        torch.cuda.synchronize()
        return (kv, ko, v2.view(-1), vo, ng), _sorted_rows(k2[rows].cpu().numpy())
    rm = rows[(rows // 1000) % 10 == 0]
    chg = rows[(rows // 1000) % 10 != 0]
    v2[chg, 9] ^= 4
    keep = torch.ones(ng, dtype=torch.bool, device="cuda")
    keep[rm] = False
    new = rm.numel()
    nkb = torch.empty(new * K + 64, dtype=torch.uint8, device="cuda")
    nvb = torch.empty(new * V + 64, dtype=torch.uint8, device="cuda")
    nko = torch.empty(new + 1, dtype=torch.int64, device="cuda")
    nvo = torch.empty(new + 1, dtype=torch.int64, device="cuda")
    gen_records_device(0, DEFAULT_SEED, 10**12 + g * new, new, K, V, nkb.data_ptr(), nko.data_ptr(), nvb.data_ptr(),
                       nvo.data_ptr(), shard=g, nshards=W)
    torch.cuda.synchronize()
    kB = torch.cat([k2[keep], nkb[: new * K].view(new, K)]).contiguous().view(-1)
    vB = torch.cat([v2[keep], nvb[: new * V].view(new, V)]).contiguous().view(-1)
    del v2
    exp = torch.cat([k2[chg], k2[rm], nkb[: new * K].view(new, K)]).cpu().numpy()
    offk = torch.arange(0, ng + 1, device="cuda", dtype=torch.int64) * K
    offv = torch.arange(0, ng + 1, device="cuda", dtype=torch.int64) * V
    torch.cuda.synchronize()
    return (kB, offk, vB, offv, ng), _sorted_rows(exp)


@pytest.mark.parametrize("mode", ["value_only", "mixed"])
def test_configs3_1b_diff_sequential_vs_construction(mode):
    """configs[2] x configs[3] at full size: the diff of two 1B-key replicas (8 key ranges x 125M, 0.1 %
    divergence) on ONE GPU, shard after shard (shard.sequential_diff: both replicas' shards prepared and
    reduced at their global offsets, the shard-local diff — top-down from the fringe roots for value-only
    changes, merge-join for key-set changes — each list at its global offset from the counts). The
    concatenated 1B diff equals the constructed divergent set and is globally sorted
    (/root/reference/src/store/merkle.rs:171-196, consumed whole by sync.rs:67-83); replica A's global
    root is the CPU oracle's golden 1B root (tests/golden/roots_sharded.json)."""
    import torch

    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import sequential_diff
    ng, nsh = 125_000_000, W
    kb = torch.empty(ng * K + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(ng * V + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    exp = []

    def pairs():
        for g in range(nsh):
            gen_records_device(0, DEFAULT_SEED, g * ng, ng, K, V, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                               vo.data_ptr(), shard=g, nshards=nsh)
            torch.cuda.synchronize()
            blob_b, e = _b_shard(torch, g, ng, kb, ko, vb, vo, mode)
            exp.append(e)
            yield (kb, ko, vb, vo, ng), blob_b
            del blob_b

    ta, tb = MerkleTree(), MerkleTree()
    ra, rb, lists, offs, ms = sequential_diff(ta, tb, pairs(), ng * nsh, ng * nsh)
    assert ra == _golden_root(nsh, ng)
    assert rb is not None and rb != ra
    got = np.concatenate([raw.reshape(-1, K) for raw, _ in lists])
    want = np.concatenate(exp)  # ranges ordered by shard: the concatenation is the global order
    assert offs == [sum(len(o) - 1 for _, o in lists[:g]) for g in range(nsh)]
    assert len(got) == len(want) >= nsh * (ng // 1000)
    assert np.array_equal(got, want), mode
    assert (np.lexsort(got.T[::-1]) == np.arange(len(got))).all()  # globally sorted
    del ta, tb, kb, vb, ko, vo


def _c4_batches(torch, g, ng, kv, R, m):
    """configs[4]'s batches of shard g: variant r writes m random values at m random positions
    (duplicates: the last write wins), seeded by (r, g) so a second pass reproduces them."""
    out = []
    uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * K
    uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * V
    for r in range(R - 1):
        gen = torch.Generator(device="cuda")
        gen.manual_seed(1000 * r + g)
        sel = torch.randint(0, ng, (m,), device="cuda", generator=gen)
        uvb = torch.randint(45, 122, (m, V), device="cuda", generator=gen, dtype=torch.uint8)
        out.append((kv[: ng * K].view(ng, K)[sel].contiguous().view(-1), uko, uvb.contiguous().view(-1), uvo, m, sel))
    return out


def test_configs4_1b_incremental_sequential_vs_construction():
    """configs[4] at full size on ONE GPU: a 1B-key tree as 8 key-range shards of 125M, base + 7 variants,
    each variant applying 125K value updates per shard (1M per variant), shard after shard
    (shard.sequential_incremental: dirty path for all 7 variants in one call, then the base diffed against
    all 7 in one shared walk, every replica's fringe kept; per replica the global root from the seam
    combine of its 8 fringes). Base root = the golden 1B root; each variant's concatenated diff = its
    updated keys, globally sorted; variant 0's global root = a fresh sequential build of its updated
    records (merkle.rs:52-56 and :73-121)."""
    import torch

    from merklekv_amd.merkle import gen_records_device
    from merklekv_amd.shard import sequential_incremental, sequential_root
    ng, nsh, R, m = 125_000_000, W, 8, 125_000
    N = ng * nsh
    kb = torch.empty(ng * K + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(ng * V + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(ng + 1, dtype=torch.int64, device="cuda")
    exp = [[] for _ in range(R - 1)]

    def gen(g):
        gen_records_device(0, DEFAULT_SEED, g * ng, ng, K, V, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(),
                           vo.data_ptr(), shard=g, nshards=nsh)
        torch.cuda.synchronize()

    def shards():
        for g in range(nsh):
            gen(g)
            bs = _c4_batches(torch, g, ng, kb, R, m)
            for r, b in enumerate(bs):
                exp[r].append(_sorted_rows(kb[: ng * K].view(ng, K)[torch.unique(b[5])].cpu().numpy()))
            yield (kb, ko, vb, vo, ng), [b[:5] for b in bs]
            del bs

    roots, lists, ms = sequential_incremental(shards(), N, R)
    assert roots[0] == _golden_root(nsh, ng)
    assert len(set(roots)) == R
    for r in range(R - 1):
        got = np.concatenate([raw.reshape(-1, K) for raw, _ in lists[r]])
        want = np.concatenate(exp[r])
        assert np.array_equal(got, want), r
        assert (np.lexsort(got.T[::-1]) == np.arange(len(got))).all()
    exp.clear()

    def variant0():
        for g in range(nsh):
            gen(g)
            ukb, uko, uvb, uvo, mm, sel = _c4_batches(torch, g, ng, kb, R, m)[0]
            last = {}
            for j, i in enumerate(sel.cpu().tolist()):
                last[i] = j
            idx = torch.tensor(list(last.keys()), device="cuda")
            src = torch.tensor(list(last.values()), device="cuda")
            vb[: ng * V].view(ng, V)[idx] = uvb.view(m, V)[src]
            torch.cuda.synchronize()
            yield (kb, ko, vb, vo, ng)

    t = MerkleTree()
    fresh, counts = sequential_root(t, variant0(), N)
    assert counts == [ng] * nsh
    assert fresh == roots[1]
    del t, kb, vb, ko, vo
