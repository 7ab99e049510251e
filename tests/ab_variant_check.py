"""Child process of tests/test_ab_variants_gpu.py: runs one small build + diff workload under the A/B
knobs in its environment (MKV_LEAF_RAGGED, MKV_DIFF_PART, MKV_DIFF_FUSED, MKV_TOP_SHA, ... are read once
per process by the library) and checks every result against the C oracle (test infrastructure:
oracle/ is the checker, never the thing measured). Prints "ok" and exits 0 on success.
Reference semantics: /root/reference/src/store/merkle.rs:73-121 (rebuild), :171-196 (diff_keys)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from merklekv_amd import MerkleTree  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.merkle_oracle import DEFAULT_SEED  # noqa: E402


def check(cond, what):
    if not cond:
        print("FAIL", what, flush=True)
        sys.exit(1)


def main():
    # ragged store-like records (listing + bucketing + the selected ragged hash kernel)
    n = 200_003
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 3, n, klen=64, vlen=256, ragged=2)
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    t = MerkleTree()
    t.build((kb, ko), (vb, vo))
    check(t.get_root_hash() == o.root(), "ragged root")
    check(b"".join(t.level_digests(0)) == o.level(0).tobytes(), "ragged leaves")
    # fixed shape (k_leaf_direct) + reduction (fused launches + top)
    kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, 300_001)
    o = coracle.OracleTree.build(kb, ko, vb, vo)
    a = MerkleTree()
    a.build((kb, ko), (vb, vo))
    check(a.get_root_hash() == o.root(), "fixed root")
    # mixed divergence (merge-join): changed values, deletes, inserts
    rng = random.Random(7)
    base = [(("k%09d" % rng.randrange(10 ** 9)).encode(), b"v%d" % i) for i in range(60_000)]
    other = []
    for k, v in base:
        r = rng.random()
        if r < 0.01:
            continue
        other.append((k, v + b"!" if r < 0.03 else v))
    other += [(("n%08d" % rng.randrange(10 ** 8)).encode(), b"x") for _ in range(700)]
    rng.shuffle(other)
    ta, tb = MerkleTree(), MerkleTree()
    ta.build([k for k, _ in base], [v for _, v in base])
    tb.build([k for k, _ in other], [v for _, v in other])
    oa, ob = coracle.OracleTree.from_pairs(base), coracle.OracleTree.from_pairs(other)
    check(ta.diff_keys_bytes(tb) == oa.diff(ob), "mixed diff a-b")
    check(tb.diff_keys_bytes(ta) == ob.diff(oa), "mixed diff b-a")
    check(ta.get_root_hash() == oa.root() and tb.get_root_hash() == ob.root(), "mixed roots")
    # value-only divergence on equal key sets (top-down walk, or merge-join under MKV_DIFF_TOPDOWN=0)
    vals = [(k, v + b"?" if i % 97 == 0 else v) for i, (k, v) in enumerate(base)]
    tc = MerkleTree()
    tc.build([k for k, _ in vals], [v for _, v in vals])
    oc = coracle.OracleTree.from_pairs(vals)
    check(ta.diff_keys_bytes(tc) == oa.diff(oc), "value-only diff")
    print("ok", flush=True)


if __name__ == "__main__":
    main()
