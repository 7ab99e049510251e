"""ctypes binding of the C ABI in include/mkv_merkle.h (libmerklekv_hip.so, built in-tree for gfx950).

The product path has no fallback: if the shared library is missing or no HIP device is present, calls
raise MerkleError. Nothing here imports or calls oracle/.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MKV_LIB_PATH: an alternative build of the same library (A/B runs of two kernel versions in one call)
LIB_PATH = os.environ.get("MKV_LIB_PATH") or os.path.join(_HERE, "lib", "libmerklekv_hip.so")

MKV_OK, MKV_EINVAL, MKV_EHIP, MKV_ENOMEM, MKV_ESTATE = 0, 1, 2, 3, 4
FRINGE_ENTRY_BYTES = 48
FRINGE_MAX_ENTRIES = 130
FRINGE_BYTES = FRINGE_ENTRY_BYTES * FRINGE_MAX_ENTRIES
ROUTE_MAX_WORLD = 256

# Every symbol include/mkv_merkle.h declares (tests check the .so exports all of them).
EXPORTS = [
    "mkv_tree_create", "mkv_tree_destroy", "mkv_tree_clone", "mkv_tree_build", "mkv_tree_build_device",
    "mkv_tree_build_wire",
    "mkv_tree_upsert", "mkv_tree_upsert_device", "mkv_tree_upsert_device_many", "mkv_tree_remove", "mkv_tree_apply", "mkv_tree_root", "mkv_tree_len",
    "mkv_tree_node_count", "mkv_tree_level_count", "mkv_tree_level", "mkv_tree_leaves", "mkv_tree_diff",
    "mkv_tree_diff_many", "mkv_tree_node_digests", "mkv_tree_compare_nodes", "mkv_tree_keys_at",
    "mkv_tree_prefix_root", "mkv_keylist_get", "mkv_keylist_free", "mkv_last_error", "mkv_shard_prepare",
    "mkv_shard_reduce", "mkv_shard_fringe", "mkv_shard_combine", "mkv_prof_enable", "mkv_prof_reset",
    "mkv_prof_read", "mkv_gen_records_device", "mkv_gen_records_ragged_device", "mkv_tree_update_counts",
    "mkv_tree_walk_stats", "mkv_leaf_digests", "mkv_version",
    "mkv_tree_build_digests", "mkv_tree_hash_pattern", "mkv_shard_fringe_device", "mkv_shard_combine_device",
    "mkv_pool_trim", "mkv_pool_stats", "mkv_debug_trace",
    "mkv_route_sample", "mkv_route_splitters", "mkv_route_plan", "mkv_route_pack", "mkv_route_offsets",
    "mkv_comm_unique_id", "mkv_comm_init_rank", "mkv_comm_create_host", "mkv_comm_rank", "mkv_comm_destroy",
    "mkv_comm_stats", "mkv_comm_all_gather", "mkv_sharded_build", "mkv_sharded_root", "mkv_sharded_root_many", "mkv_sharded_diff",
    "mkv_sharded_diff_local", "mkv_comm_traffic", "mkv_comm_inject_fault",
]

COMM_ID_BYTES = 128
COLL_KINDS = ["counts_all_gather", "range_all_gather", "fringe_all_gather", "diff_all_gather_v",
              "user_all_gather"]  # MKV_COLL_*
# int (*mkv_allgather_fn)(void *ctx, const void *send, void *recv, uint64_t bytes)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)


class MerkleError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"mkv status {status}: {msg}")
        self.status = status


class Blob(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("offsets", C.c_void_p), ("n", C.c_uint64)]


_lib = None


def lib():
    """Load the HIP library (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MerkleError(MKV_EHIP, f"native library missing: {LIB_PATH} (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    P = C.POINTER
    sig = {
        "mkv_tree_create": ([i32, P(vp)], i32),
        "mkv_tree_destroy": ([vp], None),
        "mkv_tree_clone": ([vp, vp], i32),
        "mkv_tree_build": ([vp, Blob, Blob], i32),
        "mkv_tree_build_device": ([vp, Blob, Blob], i32),
        "mkv_tree_build_wire": ([vp, vp, u64, vp, u64], i32),
        "mkv_tree_upsert": ([vp, Blob, Blob], i32),
        "mkv_tree_upsert_device": ([vp, Blob, Blob], i32),
        "mkv_tree_upsert_device_many": ([P(vp), P(Blob), P(Blob), u32], i32),
        "mkv_tree_remove": ([vp, Blob], i32),
        "mkv_tree_apply": ([vp, Blob, Blob, vp], i32),
        "mkv_tree_root": ([vp, vp, P(i32)], i32),
        "mkv_tree_len": ([vp, P(u64)], i32),
        "mkv_tree_node_count": ([vp, P(u64)], i32),
        "mkv_tree_level_count": ([vp, P(u32)], i32),
        "mkv_tree_level": ([vp, u32, P(u64), vp], i32),
        "mkv_tree_leaves": ([vp, P(vp), vp], i32),
        "mkv_tree_diff": ([vp, vp, P(vp)], i32),
        "mkv_tree_diff_many": ([vp, P(vp), u32, P(vp)], i32),
        "mkv_tree_node_digests": ([vp, u32, vp, u64, vp], i32),
        "mkv_tree_compare_nodes": ([vp, u32, vp, vp, u64, vp, P(u64)], i32),
        "mkv_tree_keys_at": ([vp, vp, u64, P(vp)], i32),
        "mkv_tree_prefix_root": ([vp, vp, u64, vp, P(i32)], i32),
        "mkv_keylist_get": ([vp, P(u64), P(vp), P(vp)], i32),
        "mkv_keylist_free": ([vp], None),
        "mkv_last_error": ([], C.c_char_p),
        "mkv_shard_prepare": ([vp, Blob, Blob, i32, P(u64)], i32),
        "mkv_shard_reduce": ([vp, u64, u64], i32),
        "mkv_shard_fringe": ([vp, vp], i32),
        "mkv_shard_combine": ([vp, vp, u32, u64, vp, P(i32)], i32),
        "mkv_prof_enable": ([vp, i32], i32),
        "mkv_prof_reset": ([vp], i32),
        "mkv_prof_read": ([vp, C.c_char_p, P(C.c_double), P(u64)], i32),
        "mkv_gen_records_device": ([i32, u64, u64, u64, u32, u32, u32, u32, u32, vp, vp, vp, vp], i32),
        "mkv_gen_records_ragged_device": ([i32, u64, u64, u64, u32, u32, u32, u32, u32, vp, vp, vp, vp], i32),
        "mkv_tree_update_counts": ([vp, vp, u32, vp], i32),
        "mkv_tree_walk_stats": ([vp, vp], i32),
        "mkv_leaf_digests": ([i32, Blob, Blob, vp], i32),
        "mkv_version": ([], C.c_char_p),
        "mkv_tree_build_digests": ([vp, Blob, vp], i32),
        "mkv_tree_hash_pattern": ([vp, vp, u64, vp, P(i32)], i32),
        "mkv_shard_fringe_device": ([vp, vp], i32),
        "mkv_shard_combine_device": ([vp, vp, u32, u64, u64, vp, P(i32)], i32),
        "mkv_pool_trim": ([], i32),
        "mkv_pool_stats": ([vp], i32),
        "mkv_debug_trace": ([vp, u64, P(u64)], i32),
        "mkv_route_sample": ([vp, Blob, u32, vp], i32),
        "mkv_route_splitters": ([vp, u64, u32, vp], i32),
        "mkv_route_plan": ([vp, Blob, Blob, u32, vp, vp], i32),
        "mkv_route_pack": ([vp, Blob, Blob, vp, vp, vp, vp], i32),
        "mkv_route_offsets": ([vp, vp, u64, vp], i32),
        "mkv_comm_unique_id": ([vp], i32),
        "mkv_comm_init_rank": ([vp, i32, i32, i32, P(vp)], i32),
        "mkv_comm_create_host": ([i32, i32, ALLGATHER_FN, vp, P(vp)], i32),
        "mkv_comm_rank": ([vp, P(i32), P(i32)], i32),
        "mkv_comm_destroy": ([vp], None),
        "mkv_comm_stats": ([vp, vp, vp, vp, i32], i32),
        "mkv_comm_all_gather": ([vp, vp, vp, u64], i32),
        "mkv_sharded_build": ([vp, vp, Blob, Blob, i32, i32, vp], i32),
        "mkv_sharded_root": ([vp, vp, vp, P(i32)], i32),
        "mkv_sharded_root_many": ([P(vp), u32, vp, vp, vp], i32),
        "mkv_sharded_diff": ([vp, vp, vp, P(vp)], i32),
        "mkv_sharded_diff_local": ([vp, vp, vp, P(vp), P(u64), P(u64)], i32),
        "mkv_comm_traffic": ([vp, vp, vp], i32),
        "mkv_comm_inject_fault": ([vp, i32], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(status: int) -> None:
    if status != MKV_OK:
        raise MerkleError(status, lib().mkv_last_error().decode(errors="replace"))
