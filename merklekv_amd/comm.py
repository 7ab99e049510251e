"""Communicator of the library's sharded entry points (mkv_comm, include/mkv_merkle.h).

The collectives of a sharded build / root / diff run INSIDE the C library (csrc/comm.cpp), so a host in
any language drives multi-GPU key-range shards through the same C ABI (the reference's SyncManager is
Rust, sync.rs:56-87; it has no sharding of its own, merkle.rs:27-32). Two forms:

  * RCCL (`Comm.rccl`): rank 0 makes the 128-byte unique id (mkv_comm_unique_id), it is shared out of
    band (here: a broadcast over the caller's torch.distributed group), every rank calls
    mkv_comm_init_rank on its GPU. Payloads stay in device memory (all-gathers over xGMI); the host reads
    only the 32-B status / count words of each operation (`traffic()`).
  * host (`Comm.host`): the caller's all-gather of equal-size host byte payloads, as a C callback
    (here: torch.distributed over gloo — the CPU tests and several ranks sharing one GPU).

`Comm.from_dist` picks the form from the group's backend and the collective device, and caches one
communicator per (group, device, form).
"""
from __future__ import annotations

import ctypes as C
import warnings

from ._lib import ALLGATHER_FN, COLL_KINDS, COMM_ID_BYTES, MerkleError, check, lib

__all__ = ["Comm"]

_cache: dict = {}


class Comm:
    """Owns one mkv_comm handle (destroyed with the object)."""

    def __init__(self, handle, rank: int, world: int, form: str, keep=None):
        self._h = handle
        self.rank, self.world, self.form = rank, world, form
        self._keep = keep  # the host form's ctypes callback (must outlive the handle)
        self.error: BaseException | None = None  # last exception raised inside the host callback

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        check(lib().mkv_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rccl(cls, uid: bytes, rank: int, world: int, device: int) -> "Comm":
        """RCCL communicator of `world` ranks, this one on HIP device `device` (collective call)."""
        h = C.c_void_p()
        src = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        check(lib().mkv_comm_init_rank(src, rank, world, device, C.byref(h)))
        return cls(h, rank, world, "rccl")

    @classmethod
    def host(cls, rank: int, world: int, all_gather) -> "Comm":
        """Host communicator over `all_gather(payload: bytes) -> list[bytes]` (world equal-size parts in
        rank order)."""
        box: dict = {}

        def _cb(ctx, send, recv, nbytes):
            try:
                parts = all_gather(C.string_at(send, nbytes))
                joined = b"".join(parts)
                if len(parts) != world or len(joined) != world * nbytes:
                    raise ValueError(f"all_gather returned {len(parts)} parts / {len(joined)} bytes for "
                                     f"world {world} x {nbytes}")
                C.memmove(recv, joined, len(joined))
                return 0
            except BaseException as e:  # never unwind through the C frames
                box["comm"].error = e
                return 1

        fn = ALLGATHER_FN(_cb)
        h = C.c_void_p()
        check(lib().mkv_comm_create_host(rank, world, fn, None, C.byref(h)))
        c = cls(h, rank, world, "host", keep=fn)
        box["comm"] = c
        return c

    @classmethod
    def from_dist(cls, dist, device="cpu", group=None) -> "Comm":
        """The cached communicator of a torch.distributed group: RCCL when the collective device is a GPU
        and the group's backend is "nccl" (RCCL on ROCm), else the host form over the group (gloo)."""
        import torch
        dev = torch.device(device)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        try:
            backend = str(dist.get_backend(group)).lower()
        except Exception:  # pragma: no cover - non-default group objects
            backend = ""
        form = "rccl" if dev.type == "cuda" and backend == "nccl" else "host"
        key = (id(group), rank, world, str(dev), form)
        c = _cache.get(key)
        if c is not None:
            return c
        from .shard import _all_gather_bytes
        c = None
        if form == "rccl":
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            t = torch.zeros(COMM_ID_BYTES + 1, dtype=torch.uint8, device=dev)
            if rank == 0:
                try:
                    t[:COMM_ID_BYTES].copy_(torch.frombuffer(bytearray(cls.unique_id()), dtype=torch.uint8))
                    t[COMM_ID_BYTES] = 1
                except MerkleError as e:  # no RCCL in this process: every rank takes the host form
                    warnings.warn(f"merklekv_amd: RCCL communicator unavailable ({e}); host all-gather instead")
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            if int(t[COMM_ID_BYTES].item()):
                c = cls.rccl(t[:COMM_ID_BYTES].cpu().numpy().tobytes(), rank, world, idx)
        if c is None:  # host form over the group (gloo, or the group's own device collectives)
            coll_dev = "cpu" if form == "host" else dev
            c = cls.host(rank, world, lambda p: _all_gather_bytes(dist, p, coll_dev, group))
        _cache[key] = c
        return c

    def check(self, status: int) -> None:
        """check() that re-raises the host callback's own exception when it caused the failure."""
        if status != 0 and self.error is not None:
            e, self.error = self.error, None
            raise MerkleError(status, f"host all-gather failed: {e!r}") from e
        check(status)

    def all_gather(self, payload: bytes) -> list[bytes]:
        """mkv_comm_all_gather: every rank's equal-size payload, rank order (collective)."""
        n = len(payload)
        src = (C.c_uint8 * max(n, 1)).from_buffer_copy(payload.ljust(max(n, 1), b"\0"))
        dst = (C.c_uint8 * max(n * self.world, 1))()
        self.check(lib().mkv_comm_all_gather(self._h, src, dst, n))
        raw = bytes(dst)
        return [raw[r * n:(r + 1) * n] for r in range(self.world)]

    def stats(self, reset: bool = False) -> dict:
        """{kind: (seconds, calls, payload bytes per rank)} of the collectives this communicator ran."""
        n = len(COLL_KINDS)
        s, k, b = (C.c_double * n)(), (C.c_uint64 * n)(), (C.c_uint64 * n)()
        check(lib().mkv_comm_stats(self._h, s, k, b, int(reset)))
        return {COLL_KINDS[i]: (s[i], k[i], b[i]) for i in range(n)}

    def traffic(self) -> dict:
        """{kind: (host-staged payload bytes, meta bytes)} since creation / the last stats reset
        (mkv_comm_traffic: the RCCL form stages no payload bytes for the sharded operations)."""
        n = len(COLL_KINDS)
        s, m = (C.c_uint64 * n)(), (C.c_uint64 * n)()
        check(lib().mkv_comm_traffic(self._h, s, m))
        return {COLL_KINDS[i]: (s[i], m[i]) for i in range(n)}

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            lib().mkv_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def clear_cache() -> None:
    """Destroy the cached communicators (before the torch.distributed group goes away)."""
    for c in _cache.values():
        c.close()
    _cache.clear()
