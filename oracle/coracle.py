"""ctypes binding of oracle/liboracle.so (the C restatement) — TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by merklekv_amd/.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        L.orc_set_sha_backend.argtypes = [C.c_int]
        L.orc_set_sha_backend.restype = C.c_int
        L.orc_cpu_has_shani.restype = C.c_int
        L.orc_sha256.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.orc_leaf_digest.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.orc_node_digest.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_tree_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_tree_build.restype = C.c_void_p
        L.orc_tree_build_digests.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_tree_build_digests.restype = C.c_void_p
        L.orc_tree_upsert.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_uint64]
        L.orc_tree_upsert.restype = C.c_void_p
        L.orc_tree_remove.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_tree_remove.restype = C.c_void_p
        L.orc_tree_free.argtypes = [C.c_void_p]
        L.orc_tree_len.argtypes = [C.c_void_p]
        L.orc_tree_len.restype = C.c_uint64
        L.orc_tree_root.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_tree_root.restype = C.c_int
        L.orc_tree_nlevels.argtypes = [C.c_void_p]
        L.orc_tree_nlevels.restype = C.c_uint32
        L.orc_tree_level.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.orc_tree_level.restype = C.c_uint64
        L.orc_tree_leaf.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(u8p), C.POINTER(C.c_uint64), C.c_void_p]
        L.orc_tree_diff.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(u8p), C.POINTER(u64p)]
        L.orc_tree_diff.restype = C.c_uint64
        L.orc_tree_prefix_root.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.orc_tree_prefix_root.restype = C.c_int
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_gen_word.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]
        L.orc_gen_word.restype = C.c_uint64
        L.orc_gen_records.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_uint32, C.c_uint32, C.c_uint32] + [C.c_void_p] * 4
        L.orc_bench_build.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_void_p]
        L.orc_bench_build.restype = C.c_double
        L.orc_bench_leaf_hash.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_void_p]
        L.orc_bench_leaf_hash.restype = C.c_double
        for name in ("orc_ref_bulk", "orc_ref_insert_loop"):
            getattr(L, name).argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_void_p]
            getattr(L, name).restype = C.c_double
        L.orc_ref_diff.argtypes = [C.c_void_p] * 4 + [C.c_uint64] + [C.c_void_p] * 4 + [C.c_uint64, u64p]
        L.orc_ref_diff.restype = C.c_double
        L.orc_mt_build.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_int, C.c_void_p]
        L.orc_mt_build.restype = C.c_double
        L.orc_mt_diff.argtypes = [C.c_void_p, C.c_void_p, C.c_int, u64p]
        L.orc_mt_diff.restype = C.c_double
        _LIB = L
    return _LIB


def ref_bulk(kb, ko, vb, vo):
    """cpu_ref one bulk build (reference data structures, one rebuild): (seconds, root)."""
    out = (C.c_uint8 * 32)()
    s = lib().orc_ref_bulk(_p(kb), _p(ko), _p(vb), _p(vo), len(ko) - 1, out)
    return s, bytes(out) if len(ko) > 1 else None


def ref_insert_loop(kb, ko, vb, vo):
    """cpu_ref new() + n x insert() (a rebuild per insert): (seconds, root)."""
    out = (C.c_uint8 * 32)()
    s = lib().orc_ref_insert_loop(_p(kb), _p(ko), _p(vb), _p(vo), len(ko) - 1, out)
    return s, bytes(out) if len(ko) > 1 else None


def ref_diff(a, b):
    """cpu_ref diff_keys between two record sets a, b = (kb, ko, vb, vo): (seconds, count)."""
    c = C.c_uint64()
    s = lib().orc_ref_diff(*(_p(x) for x in a), len(a[1]) - 1, *(_p(x) for x in b), len(b[1]) - 1, C.byref(c))
    return s, c.value


def mt_build(kb, ko, vb, vo, threads):
    out = (C.c_uint8 * 32)()
    s = lib().orc_mt_build(_p(kb), _p(ko), _p(vb), _p(vo), len(ko) - 1, threads, out)
    return s, bytes(out) if len(ko) > 1 else None


def mt_diff(ta: "OracleTree", tb: "OracleTree", threads):
    c = C.c_uint64()
    s = lib().orc_mt_diff(ta.h, tb.h, threads, C.byref(c))
    return s, c.value


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a.size else None


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    return np.ascontiguousarray(x, dtype=np.uint8)


def sha256(msg: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    m = _u8(msg)
    lib().orc_sha256(_p(m) if m.size else None, len(m), _p(out))
    return out.tobytes()


def set_backend(b: int) -> int:
    return lib().orc_set_sha_backend(b)


def gen_records(seed, idx0, n, klen=32, vlen=100, ragged=False, shard=0, nshards=1, vfield=1):
    kb = np.zeros(max(n * klen, 1), np.uint8)
    vb = np.zeros(max(n * vlen, 1), np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    lib().orc_gen_records(seed, idx0, n, klen, vlen, int(ragged), shard, nshards, vfield, _p(kb), _p(koff),
                          _p(vb), _p(voff))
    return kb[: int(koff[-1])], koff, vb[: int(voff[-1])], voff


class OracleTree:
    """Owned handle to an orc_tree."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def build(cls, kb, koff, vb, voff):
        kb, vb = _u8(kb), _u8(vb)
        koff = np.ascontiguousarray(koff, np.uint64)
        voff = np.ascontiguousarray(voff, np.uint64)
        n = len(koff) - 1
        return cls(lib().orc_tree_build(_p(kb), _p(koff), _p(vb), _p(voff), n))

    @classmethod
    def from_pairs(cls, pairs):
        from oracle.merkle_oracle import pack
        kb, koff = pack([k for k, _ in pairs])
        vb, voff = pack([v for _, v in pairs])
        return cls.build(kb, koff, vb, voff)

    def upsert(self, kb, koff, vb, voff) -> "OracleTree":
        kb, vb = _u8(kb), _u8(vb)
        koff = np.ascontiguousarray(koff, np.uint64)
        voff = np.ascontiguousarray(voff, np.uint64)
        return OracleTree(lib().orc_tree_upsert(self.h, _p(kb), _p(koff), _p(vb), _p(voff), len(koff) - 1))

    def remove(self, kb, koff) -> "OracleTree":
        kb = _u8(kb)
        koff = np.ascontiguousarray(koff, np.uint64)
        return OracleTree(lib().orc_tree_remove(self.h, _p(kb), _p(koff), len(koff) - 1))

    def __del__(self):
        if getattr(self, "h", None) and _LIB is not None:
            _LIB.orc_tree_free(self.h)
            self.h = None

    def __len__(self):
        return lib().orc_tree_len(self.h)

    def root(self) -> bytes | None:
        out = np.zeros(32, np.uint8)
        return out.tobytes() if lib().orc_tree_root(self.h, _p(out)) else None

    def nlevels(self) -> int:
        return lib().orc_tree_nlevels(self.h)

    def level(self, l: int) -> np.ndarray:
        cnt = lib().orc_tree_level(self.h, l, None)
        out = np.zeros((max(cnt, 1), 32), np.uint8)
        lib().orc_tree_level(self.h, l, _p(out))
        return out[:cnt]

    def leaves(self) -> list[tuple[bytes, bytes]]:
        out = []
        kp = u8p()
        kl = C.c_uint64()
        dg = np.zeros(32, np.uint8)
        for i in range(len(self)):
            lib().orc_tree_leaf(self.h, i, C.byref(kp), C.byref(kl), _p(dg))
            out.append((C.string_at(kp, kl.value) if kl.value else b"", dg.tobytes()))
        return out

    def diff(self, other: "OracleTree") -> list[bytes]:
        kb = u8p()
        ko = u64p()
        n = lib().orc_tree_diff(self.h, other.h, C.byref(kb), C.byref(ko))
        offs = [ko[i] for i in range(n + 1)]
        raw = C.string_at(kb, offs[-1]) if offs[-1] else b""
        lib().orc_free(C.cast(kb, C.c_void_p))
        lib().orc_free(C.cast(ko, C.c_void_p))
        return [raw[offs[i]:offs[i + 1]] for i in range(n)]

    def prefix_root(self, prefix: bytes) -> bytes | None:
        out = np.zeros(32, np.uint8)
        p = _u8(prefix)
        ok = lib().orc_tree_prefix_root(self.h, _p(p) if p.size else None, len(p), _p(out))
        return out.tobytes() if ok else None
