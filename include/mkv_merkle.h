/*
 * mkv_merkle.h — C ABI of the MI355X (gfx950) Merkle anti-entropy hot path.
 *
 * Drop-in boundary for MerkleKV's `crate::store::merkle::MerkleTree` (/root/reference/src/store/merkle.rs).
 * The reference exposes a concrete Rust struct, no trait or plugin registry; its callers are
 * SyncManager (src/sync.rs:104-143, :67) and the HASH command (src/server.rs:647-685). Each entry point
 * below names the reference method it replaces. All functions are `extern "C"`, take plain pointers
 * and sizes, and return mkv_status (0 = OK); on failure mkv_last_error() holds a thread-local message.
 * There is no CPU fallback: without a HIP device every compute call fails with MKV_EHIP.
 *
 * Threading: a handle is not thread-safe (the reference mutates through &mut self, serialised by the
 * callers' tokio Mutex, server.rs:386-390). Calls block until results are host-visible.
 * Ownership: input blobs are borrowed for the duration of the call; outputs go to caller buffers or to
 * library-owned mkv_keylist objects freed with mkv_keylist_free.
 */
#ifndef MKV_MERKLE_H
#define MKV_MERKLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t mkv_status;
#define MKV_OK 0
#define MKV_EINVAL 1 /* bad argument */
#define MKV_EHIP 2   /* HIP runtime / device error (includes "no GPU") */
#define MKV_ENOMEM 3 /* device allocation failed */
#define MKV_ESTATE 4 /* call not valid in the handle's current state */

typedef struct mkv_tree mkv_tree;       /* opaque: device-resident sorted keys, leaf digests, all levels */
typedef struct mkv_keylist mkv_keylist; /* opaque: packed key list returned by diff / leaves */

/* Packed byte strings: item i is bytes[offsets[i] .. offsets[i+1]), offsets has n+1 entries.
 * Host memory unless a function says "device". Keys/values are hashed as the bytes given (the
 * reference takes &str, i.e. UTF-8; R1 length prefixes are u32, so each item must be < 4 GiB). */
typedef struct {
    const uint8_t *bytes;
    const uint64_t *offsets;
    uint64_t n;
} mkv_blob;

/* ---------------- MerkleTree API (merkle.rs) ---------------- */

/* MerkleTree::new() — merkle.rs:36-41. Binds the handle to HIP device `hip_device`. */
mkv_status mkv_tree_create(int hip_device, mkv_tree **out);
void mkv_tree_destroy(mkv_tree *t);

/* #[derive(Clone)] (merkle.rs:27): dst (an existing handle on the same device) becomes a deep copy of src. */
mkv_status mkv_tree_clone(const mkv_tree *src, mkv_tree *dst);

/* new() + n x insert(k_i, v_i) in order — merkle.rs:52-56 called by sync.rs:110-115, :130-134 and
 * server.rs:664-667. Replaces the tree's contents. Duplicate keys: last write wins (merkle.rs:54). */
mkv_status mkv_tree_build(mkv_tree *t, mkv_blob keys, mkv_blob values);
/* Same with device pointers (bytes/offsets already resident in HBM on the tree's device). The caller
 * must have completed the work that produced them (the library runs on its own non-blocking streams
 * and does not order itself after other streams or runtimes, e.g. torch's); offsets must be monotone
 * with offsets[n] inside the allocation — they are trusted, not validated. */
mkv_status mkv_tree_build_device(mkv_tree *t, mkv_blob keys, mkv_blob values);

/* A tree from shipped (key, leaf digest) pairs: digests = n x 32 bytes, digest i = SHA-256(R1 encoding
 * of key i and its value) as the peer computed it (merkle.rs:45-49). Same result as mkv_tree_build over
 * the original records (duplicates: last wins), without the values and without Kernel A. This is the
 * anti-entropy fallback when key sets differ: SyncManager ships a peer's snapshot (sync.rs:122-143); a
 * peer that serves its leaves() (merkle.rs:133-138) lets the requester diff on the device. */
mkv_status mkv_tree_build_digests(mkv_tree *t, mkv_blob keys, const uint8_t *digests);

/* SyncManager::build_remote_merkle_snapshot (sync.rs:122-143) straight from the wire bytes: scan = the
 * SCAN response ("KEYS <n>\r\n" + n key lines, server.rs:580-587), gets = the n GET responses in key order
 * concatenated ("VALUE <v>\r\n" or "NOT_FOUND\r\n", server.rs:551-552). Parsed on the device with the
 * client's read_line + trim_end semantics (sync.rs:150-214); NOT_FOUND keys are skipped; malformed
 * responses -> MKV_EINVAL with the reference's error text. Replaces the tree's contents. */
mkv_status mkv_tree_build_wire(mkv_tree *t, const uint8_t *scan, uint64_t scan_len, const uint8_t *gets,
                               uint64_t gets_len);

/* n x insert(k_i, v_i) on the existing contents — merkle.rs:52-56 (sequential semantics, one rebuild).
 * When every key is already a leaf (value-only anti-entropy batch, BASELINE configs[4]) only the changed
 * leaves and their ancestors are rehashed (dirty path); otherwise the batch is merged and the tree
 * rebuilt. On a sharded tree only the dirty path is allowed (new keys -> MKV_ESTATE) and the global
 * root is stale until mkv_shard_fringe + all-gather + mkv_shard_combine. */
mkv_status mkv_tree_upsert(mkv_tree *t, mkv_blob keys, mkv_blob values);
/* Same with device pointers (batch already resident in HBM; same contract as mkv_tree_build_device). */
mkv_status mkv_tree_upsert_device(mkv_tree *t, mkv_blob keys, mkv_blob values);
/* k x mkv_tree_upsert_device(trees[i], keys[i], values[i]) — the anti-entropy round that applies one
 * value batch to each of k replicas (sync.rs:62-90 calls insert per repaired key on each node; configs[4]
 * applies a 125K-key batch to each of 7 replicas). Results are identical to k separate calls. Replicas
 * with one level plan (same key set) share the dirty climb: one launch per tree level for all of them.
 * Trees must be distinct. */
mkv_status mkv_tree_upsert_device_many(mkv_tree *const *trees, const mkv_blob *keys, const mkv_blob *values,
                                       uint32_t k);
/* n x remove(k_i) — merkle.rs:59-62. Missing keys are ignored. */
mkv_status mkv_tree_remove(mkv_tree *t, mkv_blob keys);
/* Mixed batch: record i is remove(k_i) if is_remove[i] else insert(k_i, v_i), applied in order. values
 * must have the same n as keys (the value of a remove record is ignored). */
mkv_status mkv_tree_apply(mkv_tree *t, mkv_blob keys, mkv_blob values, const uint8_t *is_remove);

/* get_root_hash() — merkle.rs:65-67. *has_root = 0 for the empty tree (R6: root None). */
mkv_status mkv_tree_root(const mkv_tree *t, uint8_t out32[32], int *has_root);
/* Number of leaves (leaf_map.len()). */
mkv_status mkv_tree_len(const mkv_tree *t, uint64_t *n);
/* node_count() — merkle.rs:156-163 (= 2n-1 for n>0: each pairing adds one node, promotion adds none). */
mkv_status mkv_tree_node_count(const mkv_tree *t, uint64_t *count);
/* Implicit level arrays (the reference's MerkleNode tree, merkle.rs:18-25, laid out per level):
 * level 0 = leaf digests in key order, level nlevels-1 = root. out may be NULL to query *count. */
mkv_status mkv_tree_level_count(const mkv_tree *t, uint32_t *nlevels);
mkv_status mkv_tree_level(const mkv_tree *t, uint32_t level, uint64_t *count, uint8_t *out);
/* leaves() / inorder_keys() — merkle.rs:126-138: sorted keys (library-owned list) and, if digests_out
 * != NULL, the n*32 leaf digests in the same order. */
mkv_status mkv_tree_leaves(const mkv_tree *t, mkv_keylist **keys, uint8_t *digests_out);
/* diff_keys(&other) — merkle.rs:171-196: sorted unique keys missing on one side or with different leaf
 * digests. diff_first_key (merkle.rs:199-204) is element 0. Both trees must be on the same device. */
mkv_status mkv_tree_diff(const mkv_tree *a, const mkv_tree *b, mkv_keylist **out);
/* k x diff_keys(a, others[i]) (merkle.rs:171-196), outs[i] as from mkv_tree_diff. Variants with a's level
 * plan and key set share one top-down walk (configs[4]: a base replica against 7 updated replicas);
 * the others are diffed pairwise. Results are identical to k separate calls. */
mkv_status mkv_tree_diff_many(const mkv_tree *a, const mkv_tree *const *others, uint32_t k, mkv_keylist **outs);
/* ---- anti-entropy exchange between peers (the top-down protocol of README.md:310-347) ----
 * A peer serves digests of nodes by (level, index); the requester compares them with its own nodes and
 * descends only into divergent ones, so only divergent branches cross the network. Both trees must hold
 * the same key set (equal leaf counts) for the positions to line up; keys at the divergent leaf
 * positions are then exchanged with mkv_tree_keys_at (merklekv_amd/antientropy.py drives the rounds). */
/* out[k*32..] = digest of node (level, idx[k]); a node past the level's end reads as 32 zero bytes. */
mkv_status mkv_tree_node_digests(const mkv_tree *t, uint32_t level, const uint64_t *idx, uint64_t m, uint8_t *out);
/* out_idx[0..*n_out) = the idx[k] whose local digest differs from peer[k*32..] (order kept). */
mkv_status mkv_tree_compare_nodes(const mkv_tree *t, uint32_t level, const uint64_t *idx, const uint8_t *peer,
                                  uint64_t m, uint64_t *out_idx, uint64_t *n_out);
/* Keys at sorted leaf positions pos[0..m) (inorder_keys()[pos[k]], merkle.rs:126-130). */
mkv_status mkv_tree_keys_at(const mkv_tree *t, const uint64_t *pos, uint64_t m, mkv_keylist **out);

/* HASH <prefix> — server.rs:647-685: root of a fresh tree over the keys starting with prefix
 * (*has_root = 0 when none: the server prints 64 zeros). plen = 0 gives the whole-tree root. */
mkv_status mkv_tree_prefix_root(const mkv_tree *t, const uint8_t *prefix, uint64_t plen, uint8_t out32[32],
                                int *has_root);

/* HASH [pattern] with the server's pattern convention (server.rs:651-656): pattern NULL / empty / "*"
 * selects every key (scan("")), anything else is a byte prefix (scan(p)). A key that itself starts with
 * '*' is therefore only reachable through mkv_tree_prefix_root, exactly as in the reference. */
mkv_status mkv_tree_hash_pattern(const mkv_tree *t, const uint8_t *pattern, uint64_t plen, uint8_t out32[32],
                                 int *has_root);

/* Key i of a list is bytes[offsets[i] .. offsets[i+1]) (offsets has n+1 entries; offsets[0] may be
 * nonzero). The memory stays valid until mkv_keylist_free. The lists of mkv_tree_diff_many may still be
 * on their way into host memory when the call returns (the copy overlaps the caller's next work): n is
 * available at once; asking for bytes or offsets waits for the copy. */
mkv_status mkv_keylist_get(const mkv_keylist *l, uint64_t *n, const uint8_t **bytes, const uint64_t **offsets);
void mkv_keylist_free(mkv_keylist *l);

const char *mkv_last_error(void);

/* ---------------- sharded build (one process per GPU, key-range shards) ----------------
 * Shard g holds a contiguous key range; ranges are ordered by rank. Flow per rank:
 *   mkv_shard_prepare(keys, values)          -> local leaf count n_g (hash + sort + dedup)
 *   [host all-gathers n_g, computes o_g = sum_{h<g} n_h, N = sum n_h]
 *   mkv_shard_reduce(o_g, N)                 -> every node whose leaf span lies inside [o_g, o_g+n_g)
 *   mkv_shard_fringe(buf)                    -> the <= 2 owned nodes per level whose parent is not owned
 *   [host all-gathers the fringe buffers over RCCL]
 *   mkv_shard_combine(all, world, N)         -> global root, identical on every rank (seam nodes hashed
 *                                               on the device). Bit-exact with the unsharded tree.
 * Incremental: mkv_tree_upsert[_device] of existing keys in the shard's range, then fringe + all-gather +
 * combine again. mkv_tree_diff of two shards with the same (o_g, n_g, N) walks top-down from the
 * shard's fringe roots. */
#define MKV_FRINGE_ENTRY_BYTES 48
#define MKV_FRINGE_MAX_ENTRIES 130
#define MKV_FRINGE_BYTES (MKV_FRINGE_ENTRY_BYTES * MKV_FRINGE_MAX_ENTRIES)
mkv_status mkv_shard_prepare(mkv_tree *t, mkv_blob keys, mkv_blob values, int on_device, uint64_t *n_local);
mkv_status mkv_shard_reduce(mkv_tree *t, uint64_t global_offset, uint64_t global_n);
mkv_status mkv_shard_fringe(const mkv_tree *t, uint8_t *out /* MKV_FRINGE_BYTES */);
mkv_status mkv_shard_combine(mkv_tree *t, const uint8_t *fringes /* world x MKV_FRINGE_BYTES */, uint32_t world,
                             uint64_t global_n, uint8_t out32[32], int *has_root);
/* Device-resident forms for an RCCL all-gather (no host staging of the fringes): fringe_device writes
 * MKV_FRINGE_BYTES into device memory on the tree's device and returns when it is complete;
 * combine_device reads `world` gathered blocks at dfringes + r * stride_bytes (stride >= MKV_FRINGE_BYTES,
 * multiple of 16; several trees' fringes can share one all-gather), orders them on the device and
 * returns the global root. The caller must have completed the collective before the call. */
mkv_status mkv_shard_fringe_device(const mkv_tree *t, uint8_t *dout);
mkv_status mkv_shard_combine_device(mkv_tree *t, const uint8_t *dfringes, uint32_t world, uint64_t stride_bytes,
                                    uint64_t global_n, uint8_t out32[32], int *has_root);

/* ---------------- multi-GPU over a communicator: the collectives inside the library --------
 * One process per GPU; rank r holds the records of key range r, ranges ordered by rank. The sharded entry
 * points run the all-gathers themselves, so a host in any language (the reference's SyncManager is Rust,
 * sync.rs:56-87) needs no collective layer of its own. Two communicator forms:
 *   RCCL (xGMI): mkv_comm_unique_id on one rank, the 128 bytes shared out of band (TCP, a file, MPI),
 *     then mkv_comm_init_rank on every rank (ncclCommInitRank). Payloads (boundary keys, fringes, key
 *     lists) stay in device memory: packed, all-gathered, checked and compacted on the device; the host
 *     reads only each operation's 32-B status / count words per rank (mkv_comm_traffic: `meta`) and a
 *     diff's final result.
 * Failure: every operation's first collective carries each rank's status word, and so does every later
 * collective of it, so when one rank's local step fails (bad blob, out of memory) EVERY rank returns an
 * error from the same call (the failing rank its own, the others that rank's code) — no rank is left
 * waiting in a collective. Staging buffers that must grow are allocated before a 32-B status round on
 * buffers reserved at creation, so an allocation failure after the meta all-gather reaches every rank too.
 * Every wait on a collective is bounded (MKV_WAIT_TIMEOUT_S, default 120 s): a rank whose peers never join
 * (a rank that never calls the operation, a dead link) aborts the RCCL communicator (ncclCommAbort) and
 * returns MKV_EHIP; later calls on that communicator return MKV_ESTATE.
 *   host: mkv_comm_create_host with the caller's all-gather (gloo, MPI, a test harness): fn gathers
 *     `bytes` from every rank into recv in rank order (host memory) and returns 0.
 * Replaces: the host-side count / fringe / key-list exchanges a caller had to write around
 * mkv_shard_* (above); the reference itself has no sharding (one MerkleTree per node, merkle.rs:27-32). */
typedef struct mkv_comm mkv_comm;
#define MKV_COMM_ID_BYTES 128
typedef int (*mkv_allgather_fn)(void *ctx, const void *send, void *recv, uint64_t bytes);
mkv_status mkv_comm_unique_id(uint8_t id[MKV_COMM_ID_BYTES]);
mkv_status mkv_comm_init_rank(const uint8_t id[MKV_COMM_ID_BYTES], int rank, int world, int hip_device, mkv_comm **out);
mkv_status mkv_comm_create_host(int rank, int world, mkv_allgather_fn fn, void *ctx, mkv_comm **out);
mkv_status mkv_comm_rank(const mkv_comm *c, int *rank, int *world);
/* Test hook (no reference counterpart): the next local step of this rank between an operation's meta
 * all-gather and its block all-gather fails with MKV_ENOMEM, as a failed staging allocation would; every
 * rank must then return an error from that call. where = 0 clears it. */
#define MKV_FAULT_AFTER_META 1
mkv_status mkv_comm_inject_fault(mkv_comm *c, int where);
/* All-gather of `bytes` host bytes per rank through the communicator (recv: world x bytes, rank order);
 * what the sharded entry points use for their metadata. Collective; needs no GPU in the host form. */
mkv_status mkv_comm_all_gather(mkv_comm *c, const void *send, void *recv, uint64_t bytes);
/* Per-kind collective timings since creation / the last reset: host wall seconds around each all-gather
 * and the wait for its result, calls, payload bytes per rank. Kinds: */
#define MKV_COLL_COUNTS 0 /* leaf counts (8 B) */
#define MKV_COLL_RANGE 1  /* range check: first / last key per shard */
#define MKV_COLL_FRINGE 2 /* seam fringes (k x MKV_FRINGE_BYTES) */
#define MKV_COLL_DIFF 3   /* divergent keys: (count, bytes) meta + per-rank blocks, or the local slice's counts */
#define MKV_COLL_USER 4   /* mkv_comm_all_gather: the caller's own bytes */
#define MKV_COLL_KINDS 5
mkv_status mkv_comm_stats(mkv_comm *c, double secs[MKV_COLL_KINDS], uint64_t calls[MKV_COLL_KINDS],
                          uint64_t bytes[MKV_COLL_KINDS], int reset);
/* Host <-> device bytes moved around the collectives since creation / the last stats reset, per kind:
 * staged = payload bytes copied between host and device to feed or read a collective (0 for the RCCL
 * form's sharded operations; the host form's payloads are host memory by definition and not counted),
 * meta = the status / count words the host reads back for control flow (32 B per rank per operation, plus
 * 24-B verdicts of the device block checks). */
mkv_status mkv_comm_traffic(const mkv_comm *c, uint64_t staged[MKV_COLL_KINDS], uint64_t meta[MKV_COLL_KINDS]);
void mkv_comm_destroy(mkv_comm *c);
/* Collective sharded build of this rank's records (device blobs when on_device != 0, else host blobs):
 * hash + sort + dedup, all-gather of the leaf counts, range check when range_check != 0 (every shard's
 * keys below the next non-empty shard's, else MKV_EINVAL; three more small all-gathers), in-shard
 * reduction, fringe all-gather, device seam combine. Afterwards mkv_tree_root is the GLOBAL root on every
 * rank, bit-exact with one tree over all records (merkle.rs:73-121). counts_out (optional, world
 * entries): every rank's leaf count. */
mkv_status mkv_sharded_build(mkv_tree *t, mkv_comm *c, mkv_blob keys, mkv_blob values, int on_device,
                             int range_check, uint64_t *counts_out);
/* Global root again after in-place updates of the shard (mkv_tree_upsert[_device] of keys in its range):
 * fringe all-gather + seam combine (merkle.rs:52-56 then :65-67). _many: k replicas of one key range, ONE
 * all-gather for all of them; roots = k x 32 bytes. */
mkv_status mkv_sharded_root(mkv_tree *t, mkv_comm *c, uint8_t out32[32], int *has_root);
mkv_status mkv_sharded_root_many(mkv_tree *const *ts, uint32_t k, mkv_comm *c, uint8_t *roots, int *has_root);
/* diff_keys (merkle.rs:171-196) of two sharded trees over the same partition, as ONE sorted list on every
 * rank — what SyncManager::sync_once consumes (sync.rs:67): local device diff, all-gather of (count,
 * bytes), then the lists themselves: RCCL form an all-gather-v (grouped send / receive) of device blocks
 * sized by each rank's own list, host form one all-gather of blocks padded to the largest rank's. Rank
 * order is key order. */
mkv_status mkv_sharded_diff(const mkv_tree *a, const mkv_tree *b, mkv_comm *c, mkv_keylist **out);
/* This rank's slice of that global list: the sorted divergent keys of its own key range (one device ->
 * host copy) and their position in the global list — the sum of the lower ranks' counts, from ONE 32-B
 * all-gather ("each rank writes its compacted keys at its global offset"). A sharded apply
 * (sync.rs:74-83 sets / deletes per key) needs only its own slice, so the host traffic of a global diff does
 * not grow with the number of ranks. global_total (optional): the global list's length. */
mkv_status mkv_sharded_diff_local(const mkv_tree *a, const mkv_tree *b, mkv_comm *c, mkv_keylist **out,
                                  uint64_t *global_offset, uint64_t *global_total);

/* ---------------- redistribution of unpartitioned input ----------------
 * The sharded build needs rank r to hold every key of range r. Records that sit on the ranks in no key
 * order (a store snapshot per GPU, as sync.rs:104-143 collects one) are moved there with one all-to-all:
 *   mkv_route_sample(keys, m, s)        -> m evenly spaced 8-byte big-endian key prefixes (device)
 *   [host all-gathers every rank's samples; m_r proportional to the rank's record count]
 *   mkv_route_splitters(all, world, s)  -> world-1 splitters (host only, same result on every rank)
 *   mkv_route_plan(keys, values, s)     -> per destination: records, key bytes, value bytes (host)
 *   [host all-gathers the plans: what every rank receives from every rank]
 *   mkv_route_pack(...)                 -> send buffers grouped by destination, source order kept
 *   [all-to-all of key bytes, key lengths, value bytes, value lengths over RCCL]
 *   mkv_route_offsets(lens, n, offs)    -> offsets of the received blobs, then mkv_shard_prepare(on_device)
 * Range r = keys whose zero-padded 8-byte prefix p has s[r-1] <= p < s[r]: prefix order agrees with the
 * reference's String order (R3), so ranges are ordered by rank, and equal prefixes (hence duplicate keys)
 * always meet on one rank. Received records are ordered by (source rank, source position): a key present
 * on several ranks resolves as if the ranks' inputs were concatenated in rank order (last write wins).
 * All record arrays are device pointers; lengths travel as u32 (a key or value of 4 GiB or more is refused). */
#define MKV_ROUTE_MAX_WORLD 256
mkv_status mkv_route_sample(mkv_tree *t, mkv_blob keys, uint32_t m, uint64_t *samples_dev);
mkv_status mkv_route_splitters(const uint64_t *samples, uint64_t ns, uint32_t world, uint64_t *splitters);
mkv_status mkv_route_plan(mkv_tree *t, mkv_blob keys, mkv_blob values, uint32_t world, const uint64_t *splitters,
                          uint64_t *counts /* world x 3: records, key bytes, value bytes */);
/* After mkv_route_plan on the same tree and blobs: kout / vout = key / value bytes grouped by destination
 * (sizes: the plan's byte totals), klen / vlen = u32 lengths (keys.n entries each). Complete on return. */
mkv_status mkv_route_pack(mkv_tree *t, mkv_blob keys, mkv_blob values, uint8_t *kout, uint32_t *klen, uint8_t *vout,
                          uint32_t *vlen);
/* offs[0..n] = exclusive scan of n u32 lengths (offs[n] = total). Complete on return. */
mkv_status mkv_route_offsets(mkv_tree *t, const uint32_t *lens, uint64_t n, uint64_t *offs);

/* ---------------- measurement / test utilities (not part of the reference API) ---------------- */
/* Per-kernel-group device time accumulated with HIP events on the tree's stream when enabled.
 * Groups: "leaf_hash", "sort", "gather", "reduce", "diff", "update", "total_build". */
mkv_status mkv_prof_enable(mkv_tree *t, int on);
mkv_status mkv_prof_reset(mkv_tree *t);
mkv_status mkv_prof_read(const mkv_tree *t, const char *group, double *total_ms, uint64_t *count);
/* Synthetic records (same generator as oracle/merkle_oracle.c) written to device buffers:
 * kb >= n*klen, vb >= n*vlen, koff/voff n+1 entries. Synchronous. */
/* Introspection (benches / tests): per-level dirty entry counts of the tree's last dirty-path update
 * (level 0 = changed leaves, level l > 0 = rehashed nodes), and the last top-down walk this tree ran as
 * the base (a batched walk of mkv_tree_diff_many or a pair walk of mkv_tree_diff, sharded or not):
 * out[0] = frontier entries expanded, out[1] = digest bytes the walk compared, out[2] = divergent leaf
 * positions, out[3] = launches. Both synchronise the tree's stream. */
mkv_status mkv_tree_update_counts(const mkv_tree *t, uint64_t *out, uint32_t cap, uint32_t *nlevels);
mkv_status mkv_tree_walk_stats(const mkv_tree *t, uint64_t out[4]);
mkv_status mkv_gen_records_device(int hip_device, uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen,
                                  uint32_t vlen, uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb,
                                  uint64_t *koff, uint8_t *vb, uint64_t *voff);
/* Ragged ("store-like") synthetic records for benches / tests: keys of [max(1, klen/8), klen] bytes and
 * values of [vlen/16, vlen] bytes, packed back to back (records start at arbitrary byte offsets); the same
 * definition as the oracle's orc_gen_records(ragged = 2). kb >= n*klen, vb >= n*vlen bytes. */
mkv_status mkv_gen_records_ragged_device(int hip_device, uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen,
                                         uint32_t vlen, uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb,
                                         uint64_t *koff, uint8_t *vb, uint64_t *voff);
/* Leaf digests only (Kernel A) over host records; out = n*32 bytes. */
mkv_status mkv_leaf_digests(int hip_device, mkv_blob keys, mkv_blob values, uint8_t *out);
/* Pinned key-list pool (results of diff / leaves / keys_at live in pinned host blocks recycled through
 * a bounded pool; MKV_POOL_MAX_MB caps it, default 1024). trim frees every pooled block now (it is also
 * emptied when the last tree is destroyed). stats: out6 = {hipHostMalloc calls, hipHostFree calls,
 * bytes pinned in total, host ns spent in both, blocks pooled now, bytes pooled now}. */
mkv_status mkv_pool_trim(void);
mkv_status mkv_pool_stats(uint64_t out6[6]);
/* Host phase trace of the last diff call on this thread: "label=µs;label=µs;..." (µs since the call
 * started; labels at the blocking points: device waits, readbacks, copies). *len = full length. */
mkv_status mkv_debug_trace(char *buf, uint64_t cap, uint64_t *len);
/* Library version string. */
const char *mkv_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MKV_MERKLE_H */
