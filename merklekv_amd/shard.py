"""Sharded (multi-GPU) tree build: one process per GPU, contiguous key ranges ordered by rank.

SURVEY.md §8e. Per rank: hash + sort + dedup the local range (mkv_shard_prepare), all-gather the leaf
counts (8 B/rank) -> global leaf offset o_g and total N, reduce every node whose leaf span lies inside
[o_g, o_g + n_g) (mkv_shard_reduce), export the seam fringe (<= 2 nodes per level, MKV_FRINGE_BYTES),
all-gather fringes, and hash the seam nodes on the device (mkv_shard_combine). Every rank ends with the
same global root, bit-exact with the single-tree root. Collectives go through torch.distributed: on
ROCm the "nccl" backend is RCCL over xGMI; "gloo" is used by the CPU tests.

`tree` is anything with the shard_* methods of merklekv_amd.MerkleTree.
"""
from __future__ import annotations

import numpy as np


def _all_gather_bytes(dist, payload: bytes, device, group=None) -> list[bytes]:
    """All-gather of equal-size byte payloads: one collective into one buffer, one copy back."""
    import torch
    world = dist.get_world_size(group)
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=device)
    if hasattr(dist, "all_gather_into_tensor") and (device is None or torch.device(device).type != "cpu"):
        dist.all_gather_into_tensor(out, t, group=group)
    else:  # gloo has no all_gather_into_tensor on some versions
        dist.all_gather(list(out.chunk(world)), t, group=group)
    raw = out.cpu().numpy().tobytes()
    k = t.numel()
    return [raw[r * k:(r + 1) * k] for r in range(world)]


def shard_counts(dist, n_local: int, device, group=None) -> list[int]:
    raw = _all_gather_bytes(dist, np.array([n_local], dtype=np.uint64).tobytes(), device, group)
    return [int(np.frombuffer(r, dtype=np.uint64)[0]) for r in raw]


def sharded_root(tree, keys, values, dist, device="cpu", group=None, on_device: bool = False):
    """Build this rank's shard of the global tree and return (global root or None, counts)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    n_local = tree.shard_prepare(keys, values, on_device=on_device)
    counts = shard_counts(dist, n_local, device, group)
    offset, total = sum(counts[:rank]), sum(counts)
    tree.shard_reduce(offset, total)
    fringes = _all_gather_bytes(dist, tree.shard_fringe(), device, group)
    root = tree.shard_combine(b"".join(fringes), world, total)
    return root, counts


def shard_recombine(tree, dist, total: int, device="cpu", group=None):
    """After an in-place update of this rank's shard (MerkleTree.upsert / upsert_device of keys in its
    range: the dirty path), all-gather the new fringes and recompute the seam nodes and global root."""
    world = dist.get_world_size(group)
    fringes = _all_gather_bytes(dist, tree.shard_fringe(), device, group)
    return tree.shard_combine(b"".join(fringes), world, total)
