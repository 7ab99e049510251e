"""Top-down anti-entropy exchange between two peers (README.md:310-347).

The reference describes (but does not implement: src/sync.rs ships the whole key set) a protocol in
which node A asks node B for the root hash, then for the children of every divergent node, descending
only into divergent branches until the inconsistent keys are found. Here each round is two device
calls: the serving peer gathers the requested node digests (`mkv_tree_node_digests`), the requester
compares them with its own nodes (`mkv_tree_compare_nodes`). Rounds descend `jump` levels at a time
(all 2^jump descendants of each divergent node are requested), trading a few more digests per round for
fewer network round trips. At the leaves both peers name the keys at the divergent positions
(`mkv_tree_keys_at`); when those keys differ, or the leaf counts differ, the key sets differ and the
exchange falls back to shipping every (key, leaf digest) pair — what SyncManager does today
(src/sync.rs:104-143) — and diffing locally.

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
    key_bytes_sent: int = 0        # key bytes both sides shipped at the end
    fallback: bool = False
    per_level: list = field(default_factory=list)

    @property
    def bytes_on_wire(self) -> int:
        return 32 * self.digests_sent + self.index_bytes_sent + self.key_bytes_sent


class Peer:
    """Request handler of the serving replica (wraps its MerkleTree)."""

    def __init__(self, tree):
        self.tree = tree

    def shape(self) -> tuple[int, int]:
        return len(self.tree), self.tree.level_count()

    def digests(self, level: int, idx: np.ndarray) -> bytes:
        return self.tree.node_digests(level, idx)

    def keys_at(self, pos: np.ndarray) -> list[bytes]:
        return self.tree.keys_at(pos)

    def all_leaves(self) -> list[tuple[bytes, bytes]]:
        keys = self.tree._leaf_keys()
        return list(zip(keys, self.tree.level_digests(0)))


def _descendants(idx: np.ndarray, k: int) -> np.ndarray:
    if idx.size == 0:
        return idx
    base = (idx.astype(np.uint64) << np.uint64(k))[:, None]
    return (base + np.arange(1 << k, dtype=np.uint64)[None, :]).reshape(-1)


def exchange_diff(local, remote: Peer, jump: int = 4) -> tuple[list[bytes], ExchangeStats]:
    """Keys that differ between `local` (a MerkleTree) and the peer — the same sorted set as
    local.diff_keys(remote_tree) (merkle.rs:171-196) — plus what crossed the wire."""
    st = ExchangeStats()
    n_local, L_local = len(local), local.level_count()
    n_remote, L_remote = remote.shape()
    if n_local == 0 and n_remote == 0:
        return [], st
    if n_local == n_remote and n_local > 0:
        L = L_local
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
    # key sets differ: ship every (key, digest) and diff locally (src/sync.rs:104-143 behaviour)
    st.fallback = True
    theirs = dict(remote.all_leaves())
    st.key_bytes_sent += sum(len(k) + 32 for k in theirs)
    mine = dict(zip(local._leaf_keys(), local.level_digests(0)))
    out = sorted(k for k in set(mine) | set(theirs) if mine.get(k) != theirs.get(k))
    return out, st
