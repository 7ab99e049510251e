"""Pure-Python restatement of MerkleKV's Merkle tree — TEST INFRASTRUCTURE ONLY.

Independent second oracle (SHA-256 from hashlib/OpenSSL, not from merkle_oracle.c) used to generate
the committed golden fixtures under tests/golden/ and to cross-check the C oracle at small sizes.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import anything under
oracle/; the product path (merklekv_amd/) never does.

Rules restated (all cites are /root/reference/src/store/merkle.rs):
  R1 encode_leaf        :7-16    u32_be(len k) || k || u32_be(len v) || v
  R2 compute_leaf_hash  :45-49   SHA-256(R1)
  R3 leaf order         :80-81   bytes lexicographic, shorter prefix first (Rust String Ord)
  R4 internal node      :99-103  SHA-256(left || right)
  R5 odd promotion      :111-114 last node of an odd level promoted unchanged
  R6 empty              :74-77   root None
  R7 diff_keys          :171-196 sorted keys missing on one side or with differing leaf digests
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np


def encode_leaf(key: bytes, value: bytes) -> bytes:
    """R1, merkle.rs:7-16."""
    return struct.pack(">I", len(key)) + key + struct.pack(">I", len(value)) + value


def leaf_hash(key: bytes, value: bytes) -> bytes:
    """R2, merkle.rs:45-49."""
    return hashlib.sha256(encode_leaf(key, value)).digest()


def node_hash(left: bytes, right: bytes) -> bytes:
    """R4, merkle.rs:99-103."""
    return hashlib.sha256(left + right).digest()


def reduce_levels(leaf_digests: list[bytes]) -> list[list[bytes]]:
    """rebuild() loop, merkle.rs:94-118 (R4/R5). Returns all levels, level 0 = leaves."""
    if not leaf_digests:
        return []
    levels = [list(leaf_digests)]
    cur = levels[0]
    while len(cur) > 1:
        nxt = []
        for j in range(0, len(cur), 2):
            if j + 1 < len(cur):
                nxt.append(node_hash(cur[j], cur[j + 1]))
            else:
                nxt.append(cur[j])  # R5 promotion
        levels.append(nxt)
        cur = nxt
    return levels


class PyMerkleTree:
    """Mirror of MerkleTree (merkle.rs:27-205) with the same method names."""

    def __init__(self):
        self.leaf_map: dict[bytes, bytes] = {}

    def insert(self, key: bytes, value: bytes) -> None:  # :52-56
        self.leaf_map[key] = leaf_hash(key, value)

    def remove(self, key: bytes) -> None:  # :59-62
        self.leaf_map.pop(key, None)

    def leaves(self) -> list[tuple[bytes, bytes]]:  # :133-138
        return sorted(self.leaf_map.items(), key=lambda kv: kv[0])

    def inorder_keys(self) -> list[bytes]:  # :126-130
        return sorted(self.leaf_map)

    def levels(self) -> list[list[bytes]]:
        return reduce_levels([h for _, h in self.leaves()])

    def get_root_hash(self) -> bytes | None:  # :65-67
        lv = self.levels()
        return lv[-1][0] if lv else None

    def node_count(self) -> int:  # :156-163 — every pairing adds one node; promotion adds none
        n = len(self.leaf_map)
        return 2 * n - 1 if n else 0

    def diff_keys(self, other: "PyMerkleTree") -> list[bytes]:  # :171-196
        out = []
        for k in sorted(set(self.leaf_map) | set(other.leaf_map)):
            a, b = self.leaf_map.get(k), other.leaf_map.get(k)
            if a is None or b is None or a != b:
                out.append(k)
        return out

    def diff_first_key(self, other: "PyMerkleTree") -> bytes | None:  # :199-204
        d = self.diff_keys(other)
        return d[0] if d else None

    def prefix_root(self, prefix: bytes) -> bytes | None:
        """HASH <prefix> (server.rs:647-685): fresh tree over keys with the prefix."""
        lv = reduce_levels([h for k, h in self.leaves() if k.startswith(prefix)])
        return lv[-1][0] if lv else None


# ---------------------------------------------------------------------------------------------
# Synthetic generator (same definition as orc_gen_records in merkle_oracle.c and the device one)
# ---------------------------------------------------------------------------------------------
SORTED_ALPHA = b"-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz"
DEFAULT_SEED = 0x4D65726B6C654B56  # "MerkleKV"
_M = (1 << 64) - 1
_GOLD = 0x9E3779B97F4A7C15


def mix64_np(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gen_word_np(seed: int, idx: np.ndarray, field: int, j: int) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = ((idx << np.uint64(12)) | np.uint64((field << 6) | j)) + np.uint64(1)
        return mix64_np(np.uint64(seed) + np.uint64(_GOLD) * x)


def gen_records(seed: int, idx0: int, n: int, klen: int = 32, vlen: int = 100, ragged: bool = False,
                shard: int = 0, nshards: int = 1, vfield: int = 1):
    """Vectorised twin of orc_gen_records: returns (kb, koff, vb, voff) numpy arrays."""
    alpha = np.frombuffer(SORTED_ALPHA, dtype=np.uint8)
    idx = np.arange(idx0, idx0 + n, dtype=np.uint64)
    if ragged == 2:  # store-like ragged: keys [klen/8, klen], values [vlen/16, vlen] (orc_gen_records mode 2)
        kmin, vmin = max(1, klen // 8), vlen // 16
        kl = (kmin + gen_word_np(seed, idx, 62, 0) % np.uint64(klen - kmin + 1)).astype(np.int64)
        vl = (vmin + gen_word_np(seed, idx, 62, 1) % np.uint64(vlen - vmin + 1)).astype(np.int64)
    elif ragged:
        kl = (1 + gen_word_np(seed, idx, 62, 0) % np.uint64(klen)).astype(np.int64)
        vl = (gen_word_np(seed, idx, 62, 1) % np.uint64(vlen + 1)).astype(np.int64)
    else:
        kl = np.full(n, klen, dtype=np.int64)
        vl = np.full(n, vlen, dtype=np.int64)

    def chars(field, lens, maxlen, restrict):
        out = np.zeros((n, max(maxlen, 1)), dtype=np.uint8)
        for c in range(maxlen):
            if c % 10 == 0:
                w = gen_word_np(seed, idx, field, c // 10)
            x = ((w >> np.uint64(6 * (c % 10))) & np.uint64(63)).astype(np.int64)
            if c == 0 and restrict and nshards > 1:
                lo, hi = shard * 64 // nshards, (shard + 1) * 64 // nshards
                x = lo + x % (hi - lo)
            out[:, c] = alpha[x]
        mask = np.arange(max(maxlen, 1))[None, :] < lens[:, None]
        return out[mask]

    kb = chars(0, kl, klen, True)
    vb = chars(vfield, vl, vlen, False)
    koff = np.zeros(n + 1, dtype=np.uint64)
    voff = np.zeros(n + 1, dtype=np.uint64)
    koff[1:] = np.cumsum(kl)
    voff[1:] = np.cumsum(vl)
    return kb, koff, vb, voff


def mutate_plan(seed: int, n: int, rate_ppm: int, idx0: int = 0):
    """Replica-B plan: per record class = word(seed, idx, 63, 0) % 1e6;
    class < 0.8*rate -> value changed (value field 2), < 0.9*rate -> deleted; plus n*rate/1e7 inserted
    records with fresh indices. Returns (changed_mask, deleted_mask, n_inserted)."""
    idx = np.arange(idx0, idx0 + n, dtype=np.uint64)
    cls = (gen_word_np(seed, idx, 63, 0) % np.uint64(1_000_000)).astype(np.int64)
    changed = cls < (rate_ppm * 8) // 10
    deleted = (~changed) & (cls < (rate_ppm * 9) // 10)
    n_ins = (n * rate_ppm) // 10_000_000
    return changed, deleted, n_ins


def split_blob(b: np.ndarray, off: np.ndarray) -> list[bytes]:
    raw = b.tobytes()
    o = off.tolist()
    return [raw[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def pack(items: list[bytes]):
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items])
    blob = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, dtype=np.uint8)
    return blob, off
