"""Generate tests/golden/fixtures.json with the hashlib restatement in oracle/merkle_oracle.py.

Run from the repo root:  python tests/golden/make_golden.py
The Rust reference cannot be built in this image (no cargo/rustc, crates not vendored), so these
vectors come from an independent restatement of merkle.rs (R1-R7) whose SHA-256 is OpenSSL's (via
hashlib); each case is tied to the reference test that pins its structure. NIST FIPS 180-4 vectors pin
the digest itself. Fixtures are data only (inputs and expected outputs).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.merkle_oracle import (DEFAULT_SEED, PyMerkleTree, gen_records, leaf_hash, mutate_plan,  # noqa: E402
                                  split_blob)


def tree_of(pairs):
    t = PyMerkleTree()
    for k, v in pairs:
        t.insert(k, v)
    return t


def hx(b):
    return None if b is None else b.hex()


def level_checksums(t):
    return [hashlib.sha256(b"".join(lv)).hexdigest() for lv in t.levels()]


def synth_case(n, seed=DEFAULT_SEED, ragged=False, klen=32, vlen=100):
    kb, ko, vb, vo = gen_records(seed, 0, n, klen=klen, vlen=vlen, ragged=ragged)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    t = tree_of(zip(keys, vals))
    leaves = t.leaves()
    return {
        "n": n, "seed": seed, "ragged": ragged, "klen": klen, "vlen": vlen,
        "n_unique": len(leaves),
        "root": hx(t.get_root_hash()),
        "first_leaves": [[k.hex(), h.hex()] for k, h in leaves[:16]],
        "last_leaves": [[k.hex(), h.hex()] for k, h in leaves[-16:]],
        "level_sha256": level_checksums(t),
        "input_digest_sha256": hashlib.sha256(b"".join(leaf_hash(k, v) for k, v in zip(keys, vals))).hexdigest(),
    }, t, keys, vals


def replica_b(keys, vals, seed, rate_ppm):
    n = len(keys)
    changed, deleted, n_ins = mutate_plan(seed, n, rate_ppm)
    kb2, ko2, vb2, vo2 = gen_records(seed, 0, n, vfield=2)
    v2 = split_blob(vb2, vo2)
    bk, bv = [], []
    for i in range(n):
        if deleted[i]:
            continue
        bk.append(keys[i])
        bv.append(v2[i] if changed[i] else vals[i])
    kb3, ko3, vb3, vo3 = gen_records(seed, n, n_ins)
    bk += split_blob(kb3, ko3)
    bv += split_blob(vb3, vo3)
    return bk, bv


def main():
    fx = {}
    fx["nist_sha256"] = [
        ["", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"],
        ["abc".encode().hex(), "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"],
        [b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(),
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"],
        [b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu".hex(),
         "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"],
    ]
    fx["nist_million_a"] = "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"

    ka = {
        "single_k_v": ([("k", "v")], "merkle.rs:239-250"),
        "two_a_b": ([("a", "A"), ("b", "B")], "merkle.rs:469-490, :984-1003"),
        "four_k1_k4": ([(f"k{i}", f"v{i}") for i in range(1, 5)], "merkle.rs:640-668, :1006-1023"),
        "odd_a_b_c": ([("a", "1"), ("b", "2"), ("c", "3")], "merkle.rs:581-596"),
        "stress_k0_k199": ([(f"k{i}", f"v{i}") for i in range(200)], "merkle.rs:616-635"),
        "empty_strings": ([("", ""), ("x", "")], "merkle.rs:493-513"),
        "nul_unicode": ([("", ""), ("", "nonempty"), ("nonempty", ""), ("has\0nul", "v"), ("k", "va\0lue"),
                         ("a\0b", "\0\0\0"), ("α", "1"), ("中文", "值"), ("emoji🙂", "ok")], "merkle.rs:493-513, :755-774"),
        "colon_a_colon_b": ([("x", "y"), ("a:", "b")], "merkle.rs:425-444"),
        "colon_a_b": ([("x", "y"), ("a", ":b")], "merkle.rs:425-444"),
    }
    fx["known_answers"] = {}
    for name, (pairs, cite) in ka.items():
        t = tree_of((k.encode(), v.encode()) for k, v in pairs)
        fx["known_answers"][name] = {
            "pairs": [[k.encode().hex(), v.encode().hex()] for k, v in pairs],
            "root": hx(t.get_root_hash()),
            "levels": [[h.hex() for h in lv] for lv in t.levels()],
            "cite": cite,
        }

    # odd/even sizes: keys k{i}, values v{i} (reference stress-test naming)
    sizes = list(range(1, 130)) + [255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2047, 2049]
    fx["sizes_k_v"] = {}
    for n in sizes:
        t = tree_of((f"k{i}".encode(), f"v{i}".encode()) for i in range(n))
        fx["sizes_k_v"][str(n)] = hx(t.get_root_hash())

    fx["synthetic"] = []
    for n, ragged in [(1000, False), (10000, False), (3000, True)]:
        case, t, keys, vals = synth_case(n, ragged=ragged, klen=32 if not ragged else 12,
                                         vlen=100 if not ragged else 150)
        fx["synthetic"].append(case)

    # diff fixture: config-1 shape at 5k with 1% divergence
    n, seed, rate = 5000, DEFAULT_SEED, 10000
    kb, ko, vb, vo = gen_records(seed, 0, n)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    bk, bv = replica_b(keys, vals, seed, rate)
    ta, tb = tree_of(zip(keys, vals)), tree_of(zip(bk, bv))
    fx["diff"] = {
        "n": n, "seed": seed, "rate_ppm": rate, "n_b": len(bk),
        "root_a": hx(ta.get_root_hash()), "root_b": hx(tb.get_root_hash()),
        "diff": [k.decode() for k in ta.diff_keys(tb)],
    }
    # prefix roots on the 1000-key synthetic set
    kb, ko, vb, vo = gen_records(DEFAULT_SEED, 0, 1000)
    t = tree_of(zip(split_blob(kb, ko), split_blob(vb, vo)))
    fx["prefix_roots"] = {p: hx(t.prefix_root(p.encode())) for p in ["", "A", "Zz", "a", "-", "_", "zzzz", "q9"]}

    # HASH [pattern] (server.rs:651-656): None / "" / "*" select every key, anything else is a prefix;
    # a key that starts with '*' is reachable only through a real prefix such as "*a"
    hk = [b"*", b"*a", b"*b", b"a*", b"ab", b"b", b"", b"**"]
    hv = [b"v%d" % i for i in range(len(hk))]
    th = tree_of(zip(hk, hv))
    def hash_cmd(pat):
        return th.prefix_root(b"" if pat in ("", "*") else pat.encode())
    fx["hash_patterns"] = {"keys": [k.decode() for k in hk], "values": [v.decode() for v in hv],
                           "roots": {p: hx(hash_cmd(p)) for p in ["", "*", "*a", "**", "a", "b", "c"]}}

    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures.json")
    with open(out, "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
