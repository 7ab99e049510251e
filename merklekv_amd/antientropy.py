"""Anti-entropy between two peers: the top-down exchange (README.md:310-347) and the
apply step of SyncManager::sync_once (src/sync.rs:56-87).

The reference describes (but does not implement: src/sync.rs ships the whole key set) a protocol in
which node A asks node B for the root hash, then for the children of every divergent node, descending
only into divergent branches until the inconsistent keys are found. Here each round is two device
calls: the serving peer gathers the requested node digests (`mkv_tree_node_digests`), the requester
compares them with its own nodes (`mkv_tree_compare_nodes`). Rounds descend `jump` levels at a time
(all 2^jump descendants of each divergent node are requested), trading a few more digests per round for
fewer network round trips. At the leaves both peers name the keys at the divergent positions
(`mkv_tree_keys_at`).

When those keys differ, or the leaf counts differ, the key sets differ and positions no longer line up.
The peer then ships its (key, leaf digest) pairs — the information SyncManager pulls with SCAN + GET
(src/sync.rs:122-143), without the values — and the requester builds a shadow tree from them on the
device (`mkv_tree_build_digests`, no Kernel A) and diffs it with `mkv_tree_diff` (merge-join). No host
set arithmetic: every comparison runs in the HIP kernels.

`sync_once` then does what sync.rs:74-83 does with the divergent keys — fetch each one's remote value
(GET; NOT_FOUND means "delete locally"), set/delete it in the local store — and also brings the local
tree along: a value-only divergence goes through the dirty path (`mkv_tree_upsert`: only the changed
leaves and their ancestors are rehashed), a key-set divergence through the batch merge
(`mkv_tree_apply`). Afterwards the local root equals the peer's.

`Peer` is the serving side's request handler: everything it returns is bytes that would cross the wire,
which is what `ExchangeStats` counts.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class ExchangeStats:
    rounds: int = 0
    digests_sent: int = 0          # node digests the serving peer shipped
    index_bytes_sent: int = 0      # node indices the requester shipped
    key_bytes_sent: int = 0        # key bytes both sides shipped at the end (or the fallback's leaves)
    value_bytes_sent: int = 0      # values of divergent keys fetched by sync_once
    fallback: bool = False
    per_level: list = field(default_factory=list)

    @property
    def bytes_on_wire(self) -> int:
        return 32 * self.digests_sent + self.index_bytes_sent + self.key_bytes_sent + self.value_bytes_sent


class Peer:
    """Request handler of the serving replica: its MerkleTree and (optionally) its key-value store
    (any mapping key -> value; the reference's KVEngineStoreTrait::get, served by GET)."""

    def __init__(self, tree, store=None):
        self.tree = tree
        self.store = store

    def shape(self) -> tuple[int, int]:
        return len(self.tree), self.tree.level_count()

    def digests(self, level: int, idx: np.ndarray) -> bytes:
        return self.tree.node_digests(level, idx)

    def keys_at(self, pos: np.ndarray) -> list[bytes]:
        return self.tree.keys_at(pos)

    def leaf_pairs(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """leaves() (merkle.rs:133-138) packed: key bytes, offsets, n x 32 digests."""
        return self.tree.leaves_packed()

    def get_values(self, keys: list[bytes]) -> list:
        """GET per key (server.rs:548-553 / sync.rs:192-214): the value, or None for NOT_FOUND."""
        if self.store is None:
            raise RuntimeError("this peer serves no values (Peer(tree, store=None))")
        return [self.store.get(k) for k in keys]


def _descendants(idx: np.ndarray, k: int) -> np.ndarray:
    if idx.size == 0:
        return idx
    base = (idx.astype(np.uint64) << np.uint64(k))[:, None]
    return (base + np.arange(1 << k, dtype=np.uint64)[None, :]).reshape(-1)


def exchange_diff(local, remote: Peer, jump: int = 4) -> tuple[list[bytes], ExchangeStats]:
    """Keys that differ between `local` (a MerkleTree) and the peer — the same sorted set as
    local.diff_keys(remote_tree) (merkle.rs:171-196) — plus what crossed the wire."""
    st = ExchangeStats()
    n_local = len(local)
    n_remote, _ = remote.shape()
    if n_local == 0 and n_remote == 0:
        return [], st
    if n_local == n_remote and n_local > 0:
        L = local.level_count()
        sizes = local._level_sizes()
        level, front = L - 1, np.zeros(1, np.uint64)
        while True:
            front = front[front < np.uint64(sizes[level])]
            peer = remote.digests(level, front)
            st.rounds += 1
            st.digests_sent += front.size
            st.index_bytes_sent += 8 * front.size
            front = local.compare_nodes(level, front, peer)
            st.per_level.append((level, int(front.size)))
            if level == 0 or front.size == 0:
                break
            k = min(jump, level)
            front = _descendants(front, k)
            level -= k
        if front.size == 0:
            return [], st
        mine = local.keys_at(front)
        theirs = remote.keys_at(front)
        st.key_bytes_sent += sum(len(k) for k in mine) + sum(len(k) for k in theirs)
        if mine == theirs:  # same keys at every divergent position: value differences only
            return mine, st
    # Key sets differ: the peer ships its (key, leaf digest) pairs; a shadow tree is built from them on
    # the device (mkv_tree_build_digests, no re-hash) and diffed with the device merge-join.
    st.fallback = True
    kraw, koffs, dig = remote.leaf_pairs()
    st.key_bytes_sent += int(kraw.size) + 8 * int(koffs.size) + int(dig.size)
    shadow = type(local).from_digests((kraw, koffs), dig, device=local.device)
    return local.diff_keys_bytes(shadow), st


@dataclass
class SyncReport:
    diffs: list
    set_keys: int
    deleted_keys: int
    path: str                      # "identical" | "dirty-path upsert" | "batch merge"
    stats: ExchangeStats


def sync_once(local, local_store, remote: Peer, jump: int = 4) -> SyncReport:
    """SyncManager::sync_once (sync.rs:56-87): make the local replica equal to the remote one.
    local: MerkleTree of the local data; local_store: the local key-value mapping (set / delete, as
    sync.rs:74-83 does on the store). The local tree is updated with the same changes, so afterwards
    local.get_root_hash() == the peer's root."""
    diffs, st = exchange_diff(local, remote, jump)
    if not diffs:  # sync.rs:68-71 "already identical"
        return SyncReport([], 0, 0, "identical", st)
    vals = remote.get_values(diffs)
    st.value_bytes_sent += sum(len(v) for v in vals if v is not None)
    st.key_bytes_sent += sum(len(k) for k in diffs)  # the GET requests
    is_rm = np.array([v is None for v in vals], dtype=np.uint8)
    for k, v in zip(diffs, vals):  # sync.rs:74-83: set when the remote has the key, else delete
        if v is None:
            local_store.pop(k, None)
        else:
            local_store[k] = v
    vv = [b"" if v is None else v for v in vals]
    if not st.fallback and not is_rm.any():
        local.upsert(diffs, vv)  # every divergent key is a local leaf: dirty-path rehash
        path = "dirty-path upsert"
    else:
        local.apply(diffs, vv, is_rm)  # inserts / deletes shift positions: batch sort + merge
        path = "batch merge"
    return SyncReport(diffs, int(len(diffs) - is_rm.sum()), int(is_rm.sum()), path, st)
