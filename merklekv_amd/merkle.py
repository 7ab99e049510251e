"""MerkleTree — the reference's `crate::store::merkle::MerkleTree` API on the MI355X.

Mirrors /root/reference/src/store/merkle.rs method for method (same names, argument meaning and
empty/None behaviour) over the C ABI of include/mkv_merkle.h. All hashing, ordering, reduction and
diffing runs in the HIP kernels of merklekv_amd/csrc; this module only packs arguments.

Per-call semantics are identical to the reference even though `insert`/`remove` are batched: the
reference rebuilds the whole tree after every insert (merkle.rs:52-56) and that rebuild depends only on
the final leaf map, so queued operations are applied as one ordered batch (last write wins, removes
honoured in order) right before anything observes the tree.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence

import numpy as np

from ._lib import FRINGE_BYTES, Blob, MerkleError, check, lib

__all__ = ["MerkleTree", "NodeView", "KeyList", "pack_blob", "MerkleError"]


def _b(x) -> bytes:
    if isinstance(x, str):
        return x.encode("utf-8", "surrogateescape")
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    raise TypeError(f"key/value must be str or bytes, got {type(x).__name__}")


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


class _Packed:
    """Keeps the numpy buffers of a host mkv_blob alive for the duration of a call."""

    def __init__(self, blob_bytes: np.ndarray, offsets: np.ndarray):
        self.bytes = np.ascontiguousarray(blob_bytes, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.n = len(self.offsets) - 1

    def blob(self) -> Blob:
        return Blob(self.bytes.ctypes.data if self.bytes.size else None,
                    self.offsets.ctypes.data, self.n)


def pack_blob(items: Sequence[bytes] | tuple) -> _Packed:
    """Pack byte strings (or pass through a (bytes_array, offsets_array) pair)."""
    if isinstance(items, tuple) and len(items) == 2 and isinstance(items[1], np.ndarray):
        return _Packed(items[0], items[1])
    items = [_b(x) for x in items]
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum(np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items)))
    raw = b"".join(items)
    return _Packed(np.frombuffer(raw, dtype=np.uint8) if raw else np.zeros(0, np.uint8), off)


def _keylist_packed(handle) -> tuple[np.ndarray, np.ndarray]:
    """(bytes, offsets[n+1]) copies of a library-owned key list (one memcpy each)."""
    n = C.c_uint64()
    bp = C.c_void_p()
    op = C.c_void_p()
    check(lib().mkv_keylist_get(handle, C.byref(n), C.byref(bp), C.byref(op)))
    cnt = n.value
    if cnt == 0:
        return np.zeros(0, np.uint8), np.zeros(1, np.uint64)
    offs = np.ctypeslib.as_array(C.cast(op, C.POINTER(C.c_uint64)), shape=(cnt + 1,)).copy()
    o0, o1 = int(offs[0]), int(offs[-1])  # offsets[0] may be nonzero (a view into a shared block)
    raw = (np.ctypeslib.as_array(C.cast(bp, C.POINTER(C.c_uint8)), shape=(o1,))[o0:].copy() if o1 > o0
           else np.zeros(0, np.uint8))
    offs -= np.uint64(o0)
    return raw, offs


class KeyList:
    """Zero-copy view of a library-owned key list (pinned host memory written by the device): .raw is
    the key bytes, .offs the offsets rebased to 0 (n+1). The list is freed with this object. len() is
    available at once; .raw / .offs wait for the list's copy into host memory if it is still in flight
    (mkv_tree_diff_many returns before that copy ends)."""

    def __init__(self, handle):
        self._h = handle
        n = C.c_uint64()
        check(lib().mkv_keylist_get(handle, C.byref(n), None, None))
        self.n = n.value
        self._raw = None
        self._offs = None
        if self.n == 0:
            self._raw, self._offs = np.zeros(0, np.uint8), np.zeros(1, np.uint64)

    def _views(self):
        n = C.c_uint64()
        bp = C.c_void_p()
        op = C.c_void_p()
        check(lib().mkv_keylist_get(self._h, C.byref(n), C.byref(bp), C.byref(op)))
        offs = np.ctypeslib.as_array(C.cast(op, C.POINTER(C.c_uint64)), shape=(self.n + 1,))
        o0, o1 = int(offs[0]), int(offs[-1])
        self._raw = np.ctypeslib.as_array(C.cast(bp, C.POINTER(C.c_uint8)), shape=(o1,))[o0:]
        self._offs = offs if o0 == 0 else offs - np.uint64(o0)

    @property
    def raw(self) -> np.ndarray:
        if self._raw is None:
            self._views()
        return self._raw

    @property
    def offs(self) -> np.ndarray:
        """Offsets rebased to 0 (a list sharing one block with other lists is rebased on first use)."""
        if self._offs is None:
            self._views()
        return self._offs

    def __len__(self):
        return self.n

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().mkv_keylist_free(h)
            except Exception:
                pass
            self._h = None


def _keylist(handle) -> list[bytes]:
    raw, offs = _keylist_packed(handle)
    if len(offs) == 1:
        return []
    b = raw.tobytes()
    o = offs.tolist()
    return [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]


class NodeView:
    """Read-only view of a node of the implicit tree, shaped like the reference's MerkleNode
    (merkle.rs:18-25): .hash, .left, .right (None at leaves), .key (leaves only). A promoted node
    (R5, merkle.rs:111-114) is the same node as its only child, exactly as in the reference."""

    def __init__(self, tree: "MerkleTree", level: int, idx: int):
        sizes = tree._level_sizes()
        # resolve promotion chains down to the node that actually owns this hash
        while level > 0 and 2 * idx + 1 >= sizes[level - 1]:
            level, idx = level - 1, 2 * idx
        self._t, self.level, self.idx = tree, level, idx

    @property
    def hash(self) -> bytes:
        return self._t.level_digests(self.level)[self.idx]

    @property
    def left(self):
        return None if self.level == 0 else NodeView(self._t, self.level - 1, 2 * self.idx)

    @property
    def right(self):
        return None if self.level == 0 else NodeView(self._t, self.level - 1, 2 * self.idx + 1)

    @property
    def key(self):
        return _s(self._t._leaf_keys()[self.idx]) if self.level == 0 else None


class MerkleTree:
    """MerkleTree::new() (merkle.rs:36-41). `device` = HIP device index."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().mkv_tree_create(device, C.byref(h)))
        self._h = h
        self.device = device
        self._pending: list[tuple[bool, bytes, bytes]] = []
        self._cache: dict = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().mkv_tree_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ mutation
    def insert(self, key, value) -> None:
        """insert(&mut self, key, value) — merkle.rs:52-56."""
        self._pending.append((False, _b(key), _b(value)))
        self._cache.clear()

    def remove(self, key) -> None:
        """remove(&mut self, key) — merkle.rs:59-62."""
        self._pending.append((True, _b(key), b""))
        self._cache.clear()

    def build(self, keys, values) -> None:
        """new() + n x insert(k_i, v_i) as one device build (sync.rs:104-143, server.rs:661-669).
        keys/values: sequences of str/bytes, or (bytes_array, offsets_array) pairs."""
        self._pending.clear()
        self._cache.clear()
        pk, pv = pack_blob(keys), pack_blob(values)
        if pk.n != pv.n:
            raise ValueError("keys and values differ in length")
        check(lib().mkv_tree_build(self._h, pk.blob(), pv.blob()))

    def build_digests(self, keys, digests) -> None:
        """Tree from shipped (key, leaf digest) pairs (mkv_tree_build_digests): same as build() over the
        original records, without their values (a peer's leaves(), merkle.rs:133-138). digests: bytes
        or uint8 array of 32 x len(keys), or a sequence of 32-byte digests."""
        self._pending.clear()
        self._cache.clear()
        pk = pack_blob(keys)
        if not isinstance(digests, (bytes, bytearray, memoryview, np.ndarray)):
            digests = b"".join(digests)
        d = np.ascontiguousarray(np.frombuffer(bytes(digests), np.uint8) if not isinstance(digests, np.ndarray)
                                 else digests.reshape(-1).astype(np.uint8, copy=False))
        if d.size != 32 * pk.n:
            raise ValueError("need 32 digest bytes per key")
        check(lib().mkv_tree_build_digests(self._h, pk.blob(), d.ctypes.data if d.size else None))

    @classmethod
    def from_digests(cls, keys, digests, device: int = 0) -> "MerkleTree":
        t = cls(device)
        t.build_digests(keys, digests)
        return t

    def build_wire(self, scan_response: bytes, get_responses: bytes) -> None:
        """build_remote_merkle_snapshot (sync.rs:122-143) from the raw SCAN response and the concatenated
        GET responses; parsed on the device (mkv_tree_build_wire)."""
        self._pending.clear()
        self._cache.clear()
        sb = np.frombuffer(scan_response, np.uint8) if scan_response else np.zeros(1, np.uint8)
        gb = np.frombuffer(get_responses, np.uint8) if get_responses else np.zeros(1, np.uint8)
        check(lib().mkv_tree_build_wire(self._h, sb.ctypes.data, len(scan_response), gb.ctypes.data,
                                        len(get_responses)))

    def upsert(self, keys, values) -> None:
        """Batch of insert() calls on the current contents (one device rebuild)."""
        self._flush()
        self._cache.clear()
        pk, pv = pack_blob(keys), pack_blob(values)
        check(lib().mkv_tree_upsert(self._h, pk.blob(), pv.blob()))

    def upsert_device(self, kb_ptr: int, koff_ptr: int, vb_ptr: int, voff_ptr: int, n: int) -> None:
        """upsert() of a batch already resident in HBM (device pointers). A batch of existing keys takes
        the dirty path (only changed leaves and their ancestors are rehashed)."""
        self._flush()
        self._cache.clear()
        check(lib().mkv_tree_upsert_device(self._h, Blob(kb_ptr, koff_ptr, n), Blob(vb_ptr, voff_ptr, n)))

    @staticmethod
    def upsert_device_many(trees, batches) -> None:
        """upsert_device() on k distinct trees at once: batches[i] = (kb_ptr, koff_ptr, vb_ptr, voff_ptr, n)
        for trees[i]. Replicas sharing a key set share the dirty climb (mkv_tree_upsert_device_many)."""
        trees = list(trees)
        batches = list(batches)
        if len(trees) != len(batches):
            raise ValueError("one batch per tree")
        k = len(trees)
        if k == 0:
            return
        for t in trees:
            t._flush()
            t._cache.clear()
        hs = (C.c_void_p * k)(*[t._h.value for t in trees])
        kbs = (Blob * k)(*[Blob(b[0], b[1], b[4]) for b in batches])
        vbs = (Blob * k)(*[Blob(b[2], b[3], b[4]) for b in batches])
        check(lib().mkv_tree_upsert_device_many(hs, kbs, vbs, k))

    def apply(self, keys, values, is_remove) -> None:
        """Mixed ordered batch: record i is remove(k_i) if is_remove[i] else insert(k_i, v_i)."""
        self._flush()
        self._cache.clear()
        pk, pv = pack_blob(keys), pack_blob(values)
        rm = np.ascontiguousarray(np.asarray(is_remove, dtype=np.uint8))
        if pk.n != pv.n or rm.size != pk.n:
            raise ValueError("keys, values and is_remove differ in length")
        if pk.n:
            check(lib().mkv_tree_apply(self._h, pk.blob(), pv.blob(), rm.ctypes.data))

    def remove_many(self, keys) -> None:
        self._flush()
        self._cache.clear()
        check(lib().mkv_tree_remove(self._h, pack_blob(keys).blob()))

    def _flush(self) -> None:
        if not self._pending:
            return
        ops, self._pending = self._pending, []
        self._cache.clear()
        keys = [k for _, k, _ in ops]
        vals = [v for _, _, v in ops]
        pk, pv = pack_blob(keys), pack_blob(vals)
        any_rm = any(r for r, _, _ in ops)
        all_rm = all(r for r, _, _ in ops)
        if all_rm:
            check(lib().mkv_tree_remove(self._h, pk.blob()))
        elif not any_rm:
            if len(self) == 0:
                check(lib().mkv_tree_build(self._h, pk.blob(), pv.blob()))
            else:
                check(lib().mkv_tree_upsert(self._h, pk.blob(), pv.blob()))
        else:
            rm = np.array([1 if r else 0 for r, _, _ in ops], dtype=np.uint8)
            check(lib().mkv_tree_apply(self._h, pk.blob(), pv.blob(), rm.ctypes.data))

    # ------------------------------------------------------------------ queries
    def __len__(self) -> int:
        self._flush()
        n = C.c_uint64()
        check(lib().mkv_tree_len(self._h, C.byref(n)))
        return n.value

    def get_root_hash(self) -> bytes | None:
        """get_root_hash() — merkle.rs:65-67 (None for the empty tree, R6)."""
        self._flush()
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        check(lib().mkv_tree_root(self._h, out, C.byref(has)))
        return bytes(out) if has.value else None

    @property
    def root(self) -> NodeView | None:
        """The public `root` field (merkle.rs:29) as a node view."""
        self._flush()
        sizes = self._level_sizes()
        return NodeView(self, len(sizes) - 1, 0) if sizes else None

    def _level_sizes(self) -> list[int]:
        if "sizes" not in self._cache:
            L = C.c_uint32()
            check(lib().mkv_tree_level_count(self._h, C.byref(L)))
            sizes = []
            for l in range(L.value):
                c = C.c_uint64()
                check(lib().mkv_tree_level(self._h, l, C.byref(c), None))
                sizes.append(c.value)
            self._cache["sizes"] = sizes
        return self._cache["sizes"]

    def level_count(self) -> int:
        self._flush()
        return len(self._level_sizes())

    def level_digests(self, level: int) -> list[bytes]:
        """Level `level` of the implicit tree (0 = leaves in key order)."""
        self._flush()
        key = ("level", level)
        if key not in self._cache:
            c = C.c_uint64()
            check(lib().mkv_tree_level(self._h, level, C.byref(c), None))
            buf = np.zeros(max(c.value, 1) * 32, np.uint8)
            check(lib().mkv_tree_level(self._h, level, C.byref(c), buf.ctypes.data))
            raw = buf.tobytes()
            self._cache[key] = [raw[32 * i:32 * i + 32] for i in range(c.value)]
        return self._cache[key]

    def _leaf_keys(self) -> list[bytes]:
        if "keys" not in self._cache:
            kl = C.c_void_p()
            check(lib().mkv_tree_leaves(self._h, C.byref(kl), None))
            try:
                self._cache["keys"] = _keylist(kl)
            finally:
                lib().mkv_keylist_free(kl)
        return self._cache["keys"]

    def leaves_packed(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """leaves() as arrays: (key bytes, offsets[n+1], digests n x 32) — what a peer ships when key
        sets differ (mkv_tree_leaves)."""
        self._flush()
        n = len(self)
        dig = np.zeros((max(n, 1), 32), np.uint8)
        kl = C.c_void_p()
        check(lib().mkv_tree_leaves(self._h, C.byref(kl), dig.ctypes.data))
        try:
            raw, offs = _keylist_packed(kl)
        finally:
            lib().mkv_keylist_free(kl)
        return raw, offs, dig[:n]

    def inorder_keys(self) -> list[str]:
        """inorder_keys() — merkle.rs:126-130."""
        self._flush()
        return [_s(k) for k in self._leaf_keys()]

    def leaves(self) -> list[tuple[str, bytes]]:
        """leaves() — merkle.rs:133-138: (key, leaf digest) in key order."""
        self._flush()
        keys = self._leaf_keys()
        dig = self.level_digests(0) if keys else []
        return [(_s(k), d) for k, d in zip(keys, dig)]

    def preorder_hashes(self) -> list[bytes]:
        """preorder_hashes() — merkle.rs:142-153 (a promoted node is visited once, as in the reference)."""
        self._flush()
        sizes = self._level_sizes()
        if not sizes:
            return []
        lv = [self.level_digests(l) for l in range(len(sizes))]
        out: list[bytes] = []
        stack = [(len(sizes) - 1, 0, True)]
        while stack:
            l, j, emit = stack.pop()
            if emit:
                out.append(lv[l][j])
            if l == 0:
                continue
            if 2 * j + 1 < sizes[l - 1]:
                stack.append((l - 1, 2 * j + 1, True))
                stack.append((l - 1, 2 * j, True))
            else:
                stack.append((l - 1, 2 * j, False))  # promoted: same node, do not emit twice
        return out

    def node_count(self) -> int:
        """node_count() — merkle.rs:156-163."""
        self._flush()
        c = C.c_uint64()
        check(lib().mkv_tree_node_count(self._h, C.byref(c)))
        return c.value

    def diff_keys(self, other: "MerkleTree") -> list[str]:
        """diff_keys(&other) — merkle.rs:171-196: sorted keys missing on one side or differing."""
        return [_s(k) for k in self.diff_keys_bytes(other)]

    def diff_keys_bytes(self, other: "MerkleTree") -> list[bytes]:
        self._flush()
        other._flush()
        kl = C.c_void_p()
        check(lib().mkv_tree_diff(self._h, other._h, C.byref(kl)))
        try:
            return _keylist(kl)
        finally:
            lib().mkv_keylist_free(kl)

    def diff_keys_packed(self, other: "MerkleTree") -> tuple[np.ndarray, np.ndarray]:
        """diff_keys as the C ABI returns it: packed key bytes + offsets[n+1] (numpy copies)."""
        self._flush()
        other._flush()
        kl = C.c_void_p()
        check(lib().mkv_tree_diff(self._h, other._h, C.byref(kl)))
        try:
            return _keylist_packed(kl)
        finally:
            lib().mkv_keylist_free(kl)

    def diff_keys_view(self, other: "MerkleTree") -> KeyList:
        """diff_keys as a zero-copy KeyList over the library's pinned result (no host-side copy)."""
        self._flush()
        other._flush()
        kl = C.c_void_p()
        check(lib().mkv_tree_diff(self._h, other._h, C.byref(kl)))
        return KeyList(kl)

    def diff_keys_many_view(self, others) -> list[KeyList]:
        self._flush()
        for o in others:
            o._flush()
        k = len(others)
        hs = (C.c_void_p * max(k, 1))(*[o._h.value for o in others])
        outs = (C.c_void_p * max(k, 1))()
        check(lib().mkv_tree_diff_many(self._h, hs, k, outs))
        return [KeyList(C.c_void_p(outs[i])) for i in range(k)]

    def diff_keys_many_packed(self, others) -> list[tuple[np.ndarray, np.ndarray]]:
        """[diff_keys_packed(o) for o in others] — one shared top-down walk for replicas with this
        tree's key set (mkv_tree_diff_many)."""
        self._flush()
        for o in others:
            o._flush()
        k = len(others)
        hs = (C.c_void_p * max(k, 1))(*[o._h.value for o in others])
        outs = (C.c_void_p * max(k, 1))()
        check(lib().mkv_tree_diff_many(self._h, hs, k, outs))
        res = []
        try:
            for i in range(k):
                res.append(_keylist_packed(C.c_void_p(outs[i])))
        finally:
            for i in range(k):
                if outs[i]:
                    lib().mkv_keylist_free(C.c_void_p(outs[i]))
        return res

    def diff_keys_many(self, others) -> list[list[str]]:
        out = []
        for raw, offs in self.diff_keys_many_packed(others):
            b, o = raw.tobytes(), offs.tolist()
            out.append([_s(b[o[i]:o[i + 1]]) for i in range(len(o) - 1)])
        return out

    # ------------------------------------------------------------------ anti-entropy exchange
    def node_digests(self, level: int, idx) -> bytes:
        """Digests of nodes (level, idx[k]) — what a peer serves (README.md:310-347)."""
        self._flush()
        ia = np.ascontiguousarray(np.asarray(idx, dtype=np.uint64))
        out = np.zeros(max(ia.size, 1) * 32, np.uint8)
        check(lib().mkv_tree_node_digests(self._h, level, ia.ctypes.data, ia.size, out.ctypes.data))
        return out[: 32 * ia.size].tobytes()

    def compare_nodes(self, level: int, idx, peer: bytes) -> np.ndarray:
        """The idx[k] whose local digest differs from the peer's digest peer[32k:32k+32]."""
        self._flush()
        ia = np.ascontiguousarray(np.asarray(idx, dtype=np.uint64))
        pb = np.frombuffer(peer, dtype=np.uint8) if peer else np.zeros(1, np.uint8)
        out = np.zeros(max(ia.size, 1), np.uint64)
        n = C.c_uint64()
        check(lib().mkv_tree_compare_nodes(self._h, level, ia.ctypes.data, pb.ctypes.data, ia.size, out.ctypes.data,
                                           C.byref(n)))
        return out[: n.value]

    def keys_at(self, pos) -> list[bytes]:
        """Keys at sorted leaf positions (inorder_keys()[p], merkle.rs:126-130)."""
        self._flush()
        pa = np.ascontiguousarray(np.asarray(pos, dtype=np.uint64))
        kl = C.c_void_p()
        check(lib().mkv_tree_keys_at(self._h, pa.ctypes.data if pa.size else None, pa.size, C.byref(kl)))
        try:
            return _keylist(kl)
        finally:
            lib().mkv_keylist_free(kl)

    def diff_first_key(self, other: "MerkleTree") -> str | None:
        """diff_first_key(&other) — merkle.rs:199-204."""
        d = self.diff_keys(other)
        return d[0] if d else None

    def prefix_root(self, prefix) -> bytes | None:
        """Root of a fresh tree over the keys starting with the byte prefix (mkv_tree_prefix_root). This is
        the raw range reduction: "*" is a literal byte here; hash_pattern() has the HASH command's
        wildcard convention."""
        self._flush()
        p = _b(prefix)
        buf = (C.c_uint8 * max(len(p), 1)).from_buffer_copy(p or b"\0")
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        check(lib().mkv_tree_prefix_root(self._h, buf, len(p), out, C.byref(has)))
        return bytes(out) if has.value else None

    def hash_pattern(self, pattern=None) -> bytes | None:
        """HASH [pattern] (server.rs:647-685): None, "" and "*" mean every key (server.rs:651-656),
        anything else is a prefix; None result = the empty set (the server prints 64 zeros)."""
        self._flush()
        p = b"" if pattern is None else _b(pattern)
        buf = (C.c_uint8 * max(len(p), 1)).from_buffer_copy(p or b"\0")
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        check(lib().mkv_tree_hash_pattern(self._h, buf, len(p), out, C.byref(has)))
        return bytes(out) if has.value else None

    def hash_command(self, pattern=None) -> str:
        """The server's HASH response line (server.rs:672-682), root or 64 zeros."""
        r = self.hash_pattern(pattern)
        hx = r.hex() if r is not None else "0" * 64
        pat = "" if pattern is None else (pattern if isinstance(pattern, str) else _s(pattern))
        return f"HASH {hx}\r\n" if not pat else f"HASH {pat} {hx}\r\n"

    def clone(self) -> "MerkleTree":
        """#[derive(Clone)] — merkle.rs:27."""
        self._flush()
        t = MerkleTree(self.device)
        check(lib().mkv_tree_clone(self._h, t._h))
        return t

    __copy__ = clone

    # ------------------------------------------------------------------ profiling
    def prof_enable(self, on: bool = True) -> None:
        check(lib().mkv_prof_enable(self._h, 1 if on else 0))

    def prof_reset(self) -> None:
        check(lib().mkv_prof_reset(self._h))

    def prof_read(self, group: str) -> tuple[float, int]:
        ms = C.c_double()
        cnt = C.c_uint64()
        check(lib().mkv_prof_read(self._h, group.encode(), C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    def update_counts(self) -> list[int]:
        """Per-level dirty entry counts of this tree's last dirty-path update (mkv_tree_update_counts)."""
        out = (C.c_uint64 * 64)()
        nl = C.c_uint32()
        check(lib().mkv_tree_update_counts(self._h, out, 64, C.byref(nl)))
        return [out[i] for i in range(min(nl.value, 64))]

    def walk_stats(self) -> dict:
        """The last top-down walk with this tree as the base (mkv_tree_walk_stats): a batched walk of
        diff_keys_many or an unsharded pair walk."""
        out = (C.c_uint64 * 4)()
        check(lib().mkv_tree_walk_stats(self._h, out))
        return {"entries": out[0], "bytes": out[1], "divergent_positions": out[2], "launches": out[3]}

    # ------------------------------------------------------------------ sharded build
    def shard_prepare(self, keys, values, on_device: bool = False) -> int:
        n = C.c_uint64()
        if on_device:
            kb, ko, vb, vo, cnt = (x.data_ptr() if hasattr(x, "data_ptr") else x for x in keys)
            check(lib().mkv_shard_prepare(self._h, Blob(kb, ko, cnt), Blob(vb, vo, cnt), 1, C.byref(n)))
        else:
            pk, pv = pack_blob(keys), pack_blob(values)
            check(lib().mkv_shard_prepare(self._h, pk.blob(), pv.blob(), 0, C.byref(n)))
        self._cache.clear()
        return n.value

    def shard_reduce(self, global_offset: int, global_n: int) -> None:
        check(lib().mkv_shard_reduce(self._h, global_offset, global_n))
        self._cache.clear()

    def shard_fringe(self) -> bytes:
        buf = (C.c_uint8 * FRINGE_BYTES)()
        check(lib().mkv_shard_fringe(self._h, buf))
        return bytes(buf)

    def shard_combine(self, fringes: bytes, world: int, global_n: int) -> bytes | None:
        src = (C.c_uint8 * len(fringes)).from_buffer_copy(fringes)
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        check(lib().mkv_shard_combine(self._h, src, world, global_n, out, C.byref(has)))
        return bytes(out) if has.value else None

    def shard_fringe_device(self, dptr: int) -> None:
        """Write this shard's fringe (MKV_FRINGE_BYTES) into device memory at dptr (complete on return)."""
        check(lib().mkv_shard_fringe_device(self._h, dptr))

    def shard_combine_device(self, dptr: int, world: int, stride: int, global_n: int) -> bytes | None:
        """Global root from `world` all-gathered fringe blocks in device memory (block r at dptr + r * stride)."""
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        check(lib().mkv_shard_combine_device(self._h, dptr, world, stride, global_n, out, C.byref(has)))
        return bytes(out) if has.value else None

    # ------------------------------------------------------------------ sharded entry points (comm.cpp)
    # `comm` is a merklekv_amd.comm.Comm; the library runs the collectives itself (RCCL or the host form).
    def sharded_build(self, comm, keys, values, on_device: bool = False, range_check: bool = True) -> list[int]:
        """mkv_sharded_build: this rank's key range -> afterwards get_root_hash() is the GLOBAL root on
        every rank (bit-exact with one tree over all ranks' records). Returns every rank's leaf count."""
        counts = (C.c_uint64 * comm.world)()
        if on_device:
            kb, ko, vb, vo, cnt = (x.data_ptr() if hasattr(x, "data_ptr") else x for x in keys)
            kblob, vblob = Blob(kb, ko, cnt), Blob(vb, vo, cnt)
        else:
            pk, pv = pack_blob(keys), pack_blob(values)
            kblob, vblob = pk.blob(), pv.blob()
        self._pending.clear()
        self._cache.clear()
        comm.check(lib().mkv_sharded_build(self._h, comm.handle, kblob, vblob, int(bool(on_device)),
                                           int(bool(range_check)), counts))
        return list(counts)

    def sharded_root(self, comm) -> bytes | None:
        """mkv_sharded_root: the global root again after in-range updates of this shard."""
        self._flush()
        self._cache.clear()
        out = (C.c_uint8 * 32)()
        has = C.c_int()
        comm.check(lib().mkv_sharded_root(self._h, comm.handle, out, C.byref(has)))
        return bytes(out) if has.value else None

    @staticmethod
    def sharded_root_many(trees, comm) -> list:
        """mkv_sharded_root_many: global roots of k replicas of one key range, ONE all-gather."""
        trees = list(trees)
        k = len(trees)
        for t in trees:
            t._flush()
            t._cache.clear()
        hs = (C.c_void_p * max(k, 1))(*[t._h.value for t in trees])
        roots = (C.c_uint8 * (32 * max(k, 1)))()
        has = (C.c_int * max(k, 1))()
        comm.check(lib().mkv_sharded_root_many(hs, k, comm.handle, roots, has))
        raw = bytes(roots)
        return [raw[32 * i:32 * i + 32] if has[i] else None for i in range(k)]

    def sharded_diff(self, other: "MerkleTree", comm) -> KeyList:
        """mkv_sharded_diff: diff_keys of two sharded trees with one key-range partition, as ONE sorted
        list on every rank (what sync_once consumes, sync.rs:67-83)."""
        self._flush()
        other._flush()
        kl = C.c_void_p()
        comm.check(lib().mkv_sharded_diff(self._h, other._h, comm.handle, C.byref(kl)))
        return KeyList(kl)

    def sharded_diff_local(self, other: "MerkleTree", comm):
        """mkv_sharded_diff_local: this rank's slice of the global divergent-key list, its global offset
        and the global length — one 32-B all-gather. Returns (KeyList, offset, total)."""
        self._flush()
        other._flush()
        kl, off, tot = C.c_void_p(), C.c_uint64(), C.c_uint64()
        comm.check(lib().mkv_sharded_diff_local(self._h, other._h, comm.handle, C.byref(kl), C.byref(off),
                                                C.byref(tot)))
        return KeyList(kl), off.value, tot.value

    # ------------------------------------------------------------------ redistribution (f-3)
    # Tensor arguments are device tensors on this tree's GPU: key / value bytes (uint8), offsets (int64,
    # n + 1 entries), lengths (int32 holding u32). See shard.redistribute for the collective flow.
    def route_sample(self, kb, koff, n: int, m: int, out) -> None:
        """m evenly spaced 8-byte big-endian key prefixes of the n records into out (int64, m entries)."""
        check(lib().mkv_route_sample(self._h, Blob(kb.data_ptr(), koff.data_ptr(), n), m, out.data_ptr()))

    def route_plan(self, kb, koff, vb, voff, n: int, splitters) -> np.ndarray:
        """Destinations of the n records under world-1 splitters: (world, 3) uint64 = records, key bytes,
        value bytes per destination rank."""
        spl = np.ascontiguousarray(splitters, dtype=np.uint64)
        world = len(spl) + 1
        out = np.zeros((world, 3), np.uint64)
        check(lib().mkv_route_plan(self._h, Blob(kb.data_ptr(), koff.data_ptr(), n),
                                   Blob(vb.data_ptr(), voff.data_ptr(), n), world,
                                   spl.ctypes.data if len(spl) else None, out.ctypes.data))
        return out

    def route_pack(self, kb, koff, vb, voff, n: int, kout, klen, vout, vlen) -> None:
        """Send buffers grouped by destination (source order kept) after route_plan on the same records."""
        check(lib().mkv_route_pack(self._h, Blob(kb.data_ptr(), koff.data_ptr(), n),
                                   Blob(vb.data_ptr(), voff.data_ptr(), n), kout.data_ptr(), klen.data_ptr(),
                                   vout.data_ptr(), vlen.data_ptr()))

    def route_offsets(self, lens, n: int, out) -> None:
        """out[0..n] (int64) = exclusive scan of n u32 lengths."""
        check(lib().mkv_route_offsets(self._h, lens.data_ptr(), n, out.data_ptr()))

    def build_device(self, kb_ptr: int, koff_ptr: int, vb_ptr: int, voff_ptr: int, n: int) -> None:
        """Build from records already resident in HBM (device pointers)."""
        self._pending.clear()
        self._cache.clear()
        check(lib().mkv_tree_build_device(self._h, Blob(kb_ptr, koff_ptr, n), Blob(vb_ptr, voff_ptr, n)))


def leaf_digests(keys, values, device: int = 0) -> list[bytes]:
    """Kernel A alone: R2 digests of (key, value) records in input order."""
    pk, pv = pack_blob(keys), pack_blob(values)
    out = np.zeros(max(pk.n, 1) * 32, np.uint8)
    check(lib().mkv_leaf_digests(device, pk.blob(), pv.blob(), out.ctypes.data))
    raw = out.tobytes()
    return [raw[32 * i:32 * i + 32] for i in range(pk.n)]


def gen_records_device(device: int, seed: int, idx0: int, n: int, klen: int, vlen: int, kb: int, koff: int,
                       vb: int, voff: int, shard: int = 0, nshards: int = 1, vfield: int = 1) -> None:
    check(lib().mkv_gen_records_device(device, seed, idx0, n, klen, vlen, shard, nshards, vfield, kb, koff, vb,
                                       voff))


def gen_records_ragged_device(device: int, seed: int, idx0: int, n: int, klen: int, vlen: int, kb: int, koff: int,
                              vb: int, voff: int, shard: int = 0, nshards: int = 1, vfield: int = 1) -> None:
    """Store-like ragged records (keys [klen/8, klen] B, values [vlen/16, vlen] B, packed): the oracle's
    gen_records(..., ragged=2). kb >= n*klen, vb >= n*vlen bytes; koff/voff n + 1 entries."""
    check(lib().mkv_gen_records_ragged_device(device, seed, idx0, n, klen, vlen, shard, nshards, vfield, kb, koff, vb,
                                              voff))


def route_splitters(samples, world: int) -> np.ndarray:
    """world-1 splitters (uint64) from every rank's prefix samples (mkv_route_splitters, host only)."""
    smp = np.ascontiguousarray(samples, dtype=np.uint64)
    out = np.zeros(max(world - 1, 1), np.uint64)
    check(lib().mkv_route_splitters(smp.ctypes.data if len(smp) else None, len(smp), world, out.ctypes.data))
    return out[:world - 1]


def pool_stats() -> dict:
    """Pinned key-list pool counters (mkv_pool_stats)."""
    a = (C.c_uint64 * 6)()
    check(lib().mkv_pool_stats(a))
    return {"host_mallocs": a[0], "host_frees": a[1], "bytes_pinned": a[2], "pin_ms": a[3] / 1e6,
            "pooled_blocks": a[4], "pooled_bytes": a[5]}


def debug_trace() -> str:
    """Host phase trace of this thread's last diff call (mkv_debug_trace)."""
    n = C.c_uint64()
    buf = C.create_string_buffer(4096)
    check(lib().mkv_debug_trace(buf, 4096, C.byref(n)))
    return buf.value.decode()


def pool_trim() -> None:
    check(lib().mkv_pool_trim())


def version() -> str:
    return lib().mkv_version().decode()
