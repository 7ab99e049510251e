"""merklekv_amd — MI355X-native Merkle anti-entropy hot path of MerkleKV.

Public API mirrors /root/reference/src/store/merkle.rs (MerkleTree) and its callers
(src/sync.rs SyncManager, src/server.rs HASH). Compute runs in HIP kernels (merklekv_amd/csrc) behind
the C ABI in include/mkv_merkle.h.
"""
from ._lib import LIB_PATH, MerkleError
from .merkle import MerkleTree, NodeView, leaf_digests, pack_blob, version

__all__ = ["MerkleTree", "NodeView", "MerkleError", "leaf_digests", "pack_blob", "version", "LIB_PATH"]
