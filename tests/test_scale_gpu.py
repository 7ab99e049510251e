"""BASELINE configs at full size, checked by the oracle where it finishes in seconds and by
size-independent properties elsewhere:
  configs[0]  100K keys + a 1 % 80/10/10 replica: both roots and the diff bit-exact vs the C oracle;
  configs[1]  10M keys: root bit-exact vs the C oracle (host-blob and device-resident inputs);
  configs[2]  two 100M-key replicas (and 20M), 0.1 % divergence, value-only (top-down) and mixed
              80/10/10 (merge-join): the divergent set equals the constructed one byte for byte;
  configs[4]  a 125M-key tree (one GPU's shard of the 1B-key tree), 8 replicas = base + 7 clones, each
              clone applies its own 125K-key value batch in one mkv_tree_upsert_device_many call: two
              variants' roots equal a fresh build of their updated records, and diff_keys_many returns
              exactly each batch's unique keys; plus repeated dirty updates on 20M == fresh builds.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from merklekv_amd import MerkleTree  # noqa: E402
from merklekv_amd.merkle import gen_records_device  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED  # noqa: E402

K, V = 32, 100


def _dev_records(torch, n, idx0=0, vfield=1):
    kb = torch.empty(n * K + 64, dtype=torch.uint8, device="cuda")
    vb = torch.empty(n * V + 64, dtype=torch.uint8, device="cuda")
    ko = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    vo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    gen_records_device(0, DEFAULT_SEED, idx0, n, K, V, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(),
                       vfield=vfield)
    torch.cuda.synchronize()
    return kb, ko, vb, vo


def _build_dev(torch, kflat, vflat, n):
    ko = torch.arange(0, n + 1, device="cuda", dtype=torch.int64) * K
    vo = torch.arange(0, n + 1, device="cuda", dtype=torch.int64) * V
    torch.cuda.synchronize()  # torch's stream vs the library's: inputs must be complete before the call
    t = MerkleTree()
    t.build_device(kflat.data_ptr(), ko.data_ptr(), vflat.data_ptr(), vo.data_ptr(), n)
    return t


def test_10m_root_bit_exact_vs_oracle():
    import torch
    n = 10_000_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    want = coracle.OracleTree.build(kb, ko, vb, vo).root()
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    assert t.get_root_hash() == want
    del t
    dkb, dko, dvb, dvo = _dev_records(torch, n)
    t2 = MerkleTree()
    t2.build_device(dkb.data_ptr(), dko.data_ptr(), dvb.data_ptr(), dvo.data_ptr(), n)
    assert t2.get_root_hash() == want


def _sorted_rows(a: np.ndarray) -> np.ndarray:
    return a[np.lexsort(a.T[::-1])] if len(a) else a


@pytest.fixture(autouse=True)
def _free_torch_cache():
    yield
    import gc

    import torch
    gc.collect()
    torch.cuda.empty_cache()  # the library allocates with hipMalloc directly: hand cached blocks back


def test_configs0_100k_build_and_1pct_mixed_diff_vs_oracle():
    """BASELINE configs[0] exactly: 100K synthetic 32 B / 100 B records; replica B with 1 % events
    (80 % value changes, 10 % deletions, 10 % insertions: tests/golden/make_golden.py replica_b)."""
    from tests.golden.make_golden import replica_b
    from oracle.merkle_oracle import pack, split_blob
    n = 100_000
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    bk, bv = replica_b(keys, vals, DEFAULT_SEED, 10_000)
    (bkb, bko), (bvb, bvo) = pack(bk), pack(bv)
    oa = coracle.OracleTree.build(kb, ko, vb, vo)
    ob = coracle.OracleTree.build(bkb, bko, bvb, bvo)
    a, b = MerkleTree(), MerkleTree()
    a.build((kb, ko), (vb, vo))
    b.build((bkb, bko), (bvb, bvo))
    assert a.get_root_hash() == oa.root() and b.get_root_hash() == ob.root()
    want = oa.diff(ob)
    assert 900 <= len(want) <= 1100  # ~1 % of 100K
    assert a.diff_keys_bytes(b) == want
    assert b.diff_keys_bytes(a) == want
    assert a.diff_first_key(b) == (want[0].decode() if want else None)


@pytest.mark.parametrize("n", [20_000_000, 100_000_000], ids=["20m", "100m"])
@pytest.mark.parametrize("mode", ["value_only", "mixed"])
def test_replica_diff_exact(mode, n):
    """configs[2] at full size (100M) and 20M: A.diff_keys(B) == the constructed divergent set."""
    import torch
    kb, ko, vb, vo = _dev_records(torch, n)
    kv, vv = kb[: n * K].view(n, K), vb[: n * V].view(n, V)
    A = _build_dev(torch, kb, vb, n)
    ndiv = n // 1000
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    perm = torch.randperm(n, device="cuda", generator=g)
    if mode == "value_only":
        chg, rm, new = perm[:ndiv], perm[:0], 0
    else:
        c, r = ndiv * 8 // 10, ndiv // 10
        chg, rm, new = perm[:c], perm[c:c + r], ndiv - c - r
    v2 = vv.clone()
    v2[chg, 7] ^= 2
    keep = torch.ones(n, dtype=torch.bool, device="cuda")
    keep[rm] = False
    kB, vB = kv[keep], v2[keep]
    if new:
        nk, _, nv, _ = _dev_records(torch, new, idx0=10**12)
        kB = torch.cat([kB, nk[: new * K].view(new, K)])
        vB = torch.cat([vB, nv[: new * V].view(new, V)])
    B = _build_dev(torch, kB.contiguous().view(-1), vB.contiguous().view(-1), kB.shape[0])
    exp = torch.cat([kv[chg], kv[rm]] + ([kB[-new:]] if new else [])).cpu().numpy()
    raw, offs = A.diff_keys_packed(B)
    assert len(offs) - 1 == ndiv
    assert np.array_equal(raw.reshape(-1, K), _sorted_rows(exp))
    # symmetric: B vs A gives the same set
    raw2, _ = B.diff_keys_packed(A)
    assert np.array_equal(raw2, raw)
    del A, B, kb, vb, kB, vB, v2


def test_125m_eight_replica_incremental():
    """configs[4] per GPU: 125M-key tree, base + 7 clones, 125K-key value batch per clone."""
    import torch
    n, m, R = 125_000_000, 125_000, 8
    kb, ko, vb, vo = _dev_records(torch, n)
    kv, vv = kb[: n * K].view(n, K), vb[: n * V].view(n, V)
    base = MerkleTree()
    base.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    root0 = base.get_root_hash()
    variants = [base.clone() for _ in range(R - 1)]
    assert all(t.get_root_hash() == root0 for t in variants)
    g = torch.Generator(device="cuda")
    g.manual_seed(125)
    batches, keep = [], []
    uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * K
    uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * V
    for r in range(R - 1):
        sel = torch.randint(0, n, (m,), device="cuda", generator=g)  # duplicates: last write wins
        ukb = kv[sel].contiguous().view(-1)
        uvb = torch.randint(45, 122, (m, V), device="cuda", generator=g, dtype=torch.uint8).contiguous()
        batches.append((ukb, uvb, sel))
        keep.append((ukb, uko, uvb, uvo))
    torch.cuda.synchronize()
    MerkleTree.upsert_device_many(variants, [(a.data_ptr(), b.data_ptr(), c.data_ptr(), d.data_ptr(), m)
                                             for a, b, c, d in keep])
    roots = [t.get_root_hash() for t in variants]
    assert len(set(roots)) == R - 1 and root0 not in roots
    diffs = base.diff_keys_many_packed(variants)
    for r, ((raw, offs), (_, _, sel)) in enumerate(zip(diffs, batches)):
        uniq = torch.unique(sel)
        exp = _sorted_rows(kv[uniq].cpu().numpy())
        assert len(offs) - 1 == uniq.numel(), r
        assert np.array_equal(raw.reshape(-1, K), exp), r
    del diffs, variants
    import gc
    gc.collect()
    for r in (0, R - 2):  # two variants: root == fresh build of the updated records
        ukb, uvb, sel = batches[r]
        vv2 = vv.clone()
        last = {}
        for j, i in enumerate(sel.cpu().tolist()):
            last[i] = j
        idx = torch.tensor(list(last.keys()), device="cuda")
        src = torch.tensor(list(last.values()), device="cuda")
        vv2[idx] = uvb.view(m, V)[src]
        torch.cuda.synchronize()
        fresh = MerkleTree()
        fresh.build_device(kb.data_ptr(), ko.data_ptr(), vv2.data_ptr(), vo.data_ptr(), n)
        assert fresh.get_root_hash() == roots[r], r
        del fresh, vv2
        torch.cuda.empty_cache()


def test_20m_dirty_updates_equal_fresh_build():
    import torch
    n = 20_000_000
    kb, ko, vb, vo = _dev_records(torch, n)
    t = MerkleTree()
    t.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
    vv = vb[: n * V].view(n, V)
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    for rnd in range(3):
        m = 20_000 * (rnd + 1)
        sel = torch.randint(0, n, (m,), device="cuda", generator=g)  # duplicates: last write wins
        newv = torch.randint(45, 122, (m, V), device="cuda", generator=g, dtype=torch.uint8)
        ukb = kb[: n * K].view(n, K)[sel].contiguous().view(-1)
        uko = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * K
        uvo = torch.arange(0, m + 1, device="cuda", dtype=torch.int64) * V
        newv = newv.contiguous()
        torch.cuda.synchronize()
        t.upsert_device(ukb.data_ptr(), uko.data_ptr(), newv.view(-1).data_ptr(), uvo.data_ptr(), m)
        # apply the same batch to the records (sequential semantics: later duplicates overwrite)
        vv[sel] = newv  # index_put with duplicates is not ordered: resolve explicitly below
        last = {}
        for j, i in enumerate(sel.cpu().tolist()):
            last[i] = j
        idx = torch.tensor(list(last.keys()), device="cuda")
        src = torch.tensor(list(last.values()), device="cuda")
        vv[idx] = newv[src]
        torch.cuda.synchronize()
        fresh = MerkleTree()
        fresh.build_device(kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), n)
        assert t.get_root_hash() == fresh.get_root_hash(), rnd
        del fresh
