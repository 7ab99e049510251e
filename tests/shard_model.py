"""Pure-Python model of a shard tree (TEST INFRASTRUCTURE): same protocol and fringe byte format as
mkv_shard_prepare / _reduce / _fringe / _combine, computed with the hashlib oracle. Lets the
torch.distributed orchestration in merklekv_amd/shard.py and the seam math be tested on CPU with gloo.
"""
from __future__ import annotations

import struct

import numpy as np

from oracle.merkle_oracle import PyMerkleTree, node_hash, pack


def torch_u8(b: bytes):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.zeros(0, dtype=torch.uint8)

ENTRY = struct.Struct("<IIQ32s")  # level, valid, idx, digest  (MKV_FRINGE_ENTRY_BYTES = 48)
MAX_ENTRIES = 130


def plan_levels(o: int, n: int, N: int):
    """(base, count, size) per level: the owned global node range of a shard (tree.cpp plan_levels)."""
    out = []
    if N == 0:
        return out
    a, e, S = o, o + n, N
    while True:
        out.append((a, max(0, e - a), S))
        if S == 1:
            break
        a, e, S = (a + 1) // 2, ((e + 1) // 2 if e == S else e // 2), (S + 1) // 2
    return out


def _split_np(b, o, n):
    raw = b.numpy().tobytes()
    offs = o.numpy()
    return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]


def prefix8(k: bytes) -> int:
    """Zero-padded 8-byte big-endian prefix (k_route.hip be_prefix8)."""
    return int.from_bytes(k[:8].ljust(8, b"\0"), "big")


class ModelShardTree:
    # ---- redistribution model (k_route.hip) over CPU tensors ----
    def route_sample(self, kb, koff, n, m, out):
        keys = _split_np(kb, koff, n)
        for i in range(m):
            out[i] = np.uint64(prefix8(keys[((2 * i + 1) * n) // (2 * m)])).view(np.int64)

    def route_plan(self, kb, koff, vb, voff, n, splitters):
        keys, vals = _split_np(kb, koff, n), _split_np(vb, voff, n)
        spl = [int(x) for x in np.asarray(splitters, np.uint64)]
        world = len(spl) + 1
        dest = [sum(1 for s in spl if s <= prefix8(k)) for k in keys]
        self._route = sorted(range(n), key=lambda i: dest[i])  # stable: source order within a destination
        out = np.zeros((world, 3), np.uint64)
        for i in range(n):
            out[dest[i]] += np.array([1, len(keys[i]), len(vals[i])], np.uint64)
        self._route_recs = (keys, vals)
        return out

    def route_pack(self, kb, koff, vb, voff, n, kout, klen, vout, vlen):
        keys, vals = self._route_recs
        ks = b"".join(keys[i] for i in self._route)
        vs = b"".join(vals[i] for i in self._route)
        kout[:len(ks)] = torch_u8(ks)
        vout[:len(vs)] = torch_u8(vs)
        for j, i in enumerate(self._route):
            klen[j] = len(keys[i])
            vlen[j] = len(vals[i])

    def route_offsets(self, lens, n, out):
        out[0] = 0
        if n:
            out[1:n + 1] = lens[:n].to(out.dtype).cumsum(0)

    def shard_prepare(self, keys, values, on_device=False):
        if on_device:  # (kb, koff, vb, voff, n) CPU tensors, as redistribute returns them
            kb, ko, vb, vo, n = keys
            keys, values = _split_np(kb, ko, n), _split_np(vb, vo, n)
        t = PyMerkleTree()
        for k, v in zip(keys, values):
            t.insert(k, v)
        self.leaves = [h for _, h in t.leaves()]
        self.keys = [k for k, _ in t.leaves()]
        return len(self.leaves)

    def keys_at(self, pos):
        return [self.keys[int(p)] for p in pos]

    def diff_keys_packed(self, other):
        """merkle.rs:171-196 over this shard's leaves (the device path runs per rank the same way)."""
        a, b = PyMerkleTree(), PyMerkleTree()
        a.leaf_map.update(zip(self.keys, self.leaves))
        b.leaf_map.update(zip(other.keys, other.leaves))
        return pack(a.diff_keys(b))

    def upsert(self, keys, values):
        """Value-only batch on keys already in this shard (the dirty path's contract): leaves change in
        place, the owned levels are recomputed with the same plan."""
        t = PyMerkleTree()
        for k, h in zip(self.keys, self.leaves):
            t.leaf_map[k] = h
        for k, v in zip(keys, values):
            assert k in t.leaf_map, "dirty path: key must already be a leaf"
            t.insert(k, v)
        self.leaves = [h for _, h in t.leaves()]
        self.shard_reduce(self.plan[0][0], self.plan[0][2])

    def shard_reduce(self, offset, total):
        self.plan = plan_levels(offset, len(self.leaves), total)
        self.levels = [list(self.leaves)]
        for l in range(1, len(self.plan)):
            a, c, _ = self.plan[l]
            pa, _, pS = self.plan[l - 1]
            prev = self.levels[-1]
            cur = []
            for j in range(a, a + c):
                c0 = 2 * j - pa
                cur.append(node_hash(prev[c0], prev[c0 + 1]) if 2 * j + 1 < pS else prev[c0])
            self.levels.append(cur)

    def shard_fringe(self) -> bytes:
        ents = []
        L = len(self.plan)
        for l, (a, c, _) in enumerate(self.plan):
            if not c:
                continue
            for x in sorted({a, a + c - 1}):
                owned_parent = False
                if l + 1 < L:
                    a2, c2, _ = self.plan[l + 1]
                    owned_parent = a2 <= x // 2 < a2 + c2
                if not owned_parent:
                    ents.append(ENTRY.pack(l, 1, x, self.levels[l][x - a]))
        assert len(ents) <= MAX_ENTRIES
        return b"".join(ents) + b"\0" * (ENTRY.size * (MAX_ENTRIES - len(ents)))

    def shard_combine(self, fringes: bytes, world: int, total: int):
        if total == 0:
            return None
        ents = []
        for r in range(world):
            blk = fringes[r * ENTRY.size * MAX_ENTRIES:(r + 1) * ENTRY.size * MAX_ENTRIES]
            for i in range(MAX_ENTRIES):
                lv, valid, idx, h = ENTRY.unpack_from(blk, i * ENTRY.size)
                if not valid:
                    break
                ents.append((lv, idx, h))
        ents.sort()
        S = []
        s = total
        while True:
            S.append(s)
            if s == 1:
                break
            s = (s + 1) // 2
        cur: list[tuple[int, bytes]] = []
        for l in range(len(S)):
            computed = []
            if l > 0:
                for i, (x, h) in enumerate(cur):
                    if x % 2:
                        continue
                    if x + 1 < S[l - 1]:
                        assert i + 1 < len(cur) and cur[i + 1][0] == x + 1, "seam sibling missing"
                        computed.append((x // 2, node_hash(h, cur[i + 1][1])))
                    else:
                        computed.append((x // 2, h))
            cur = sorted(computed + [(idx, h) for lv, idx, h in ents if lv == l])
        assert len(cur) == 1
        return cur[0][1]
