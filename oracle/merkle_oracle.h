/*
 * merkle_oracle.h — CPU restatement of MerkleKV's Merkle tree (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the HIP path in merklekv_amd/. It is NOT part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as
 * the checker / the timed CPU baseline. The product library never links or calls it.
 *
 * Every function restates /root/reference/src/store/merkle.rs (snapshot 2025-09-26):
 *   R1 encode_leaf          merkle.rs:7-16   u32_be(|k|) || k || u32_be(|v|) || v
 *   R2 compute_leaf_hash    merkle.rs:45-49  SHA-256(R1)  (sha2 0.10.9, Cargo.lock:1227-1230)
 *   R3 leaf order           merkle.rs:80-81  Rust String Ord = memcmp, shorter prefix first
 *   R4 internal node        merkle.rs:99-103 SHA-256(left32 || right32), no domain prefix
 *   R5 odd promotion        merkle.rs:111-114 last node of an odd level promoted unchanged
 *   R6 empty tree           merkle.rs:74-77, :65-67  root None
 *   R7 diff_keys            merkle.rs:171-196 sorted unique keys missing on one side or differing
 *   insert/remove           merkle.rs:52-62  upsert/delete (last write wins) then full rebuild
 *
 * The Rust reference cannot be compiled in this image (no cargo/rustc, crates not vendored), so
 * oracle/_ref does not exist; parity is pinned by NIST FIPS 180-4 vectors, the relational tests
 * of merkle.rs:207-1184 and hashlib-generated fixtures (tests/golden/).
 */
#ifndef MERKLE_ORACLE_H
#define MERKLE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SHA-256 backend: 0 = portable FIPS 180-4 C (default, the checker), 1 = x86 SHA-NI (timed baseline;
 * the reference's sha2 crate selects SHA-NI at run time too). Returns the backend actually set. */
int orc_set_sha_backend(int backend);
int orc_cpu_has_shani(void);

void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);
/* R1+R2, merkle.rs:7-16 + :45-49 */
void orc_leaf_digest(const uint8_t *k, uint64_t klen, const uint8_t *v, uint64_t vlen, uint8_t out[32]);
/* R4, merkle.rs:99-103 */
void orc_node_digest(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]);

typedef struct orc_tree orc_tree;

/* new() + n x insert(k_i, v_i) in order (merkle.rs:36-41, :52-56): records are packed blobs
 * with offsets[n+1]. */
orc_tree *orc_tree_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                         uint64_t n);
/* Same, from precomputed leaf digests (digests[i] is record i's R2 digest). */
orc_tree *orc_tree_build_digests(const uint8_t *kb, const uint64_t *koff, const uint8_t *digests, uint64_t n);
/* insert() batch on an existing tree (sequential semantics, last write wins); returns a new tree. */
orc_tree *orc_tree_upsert(const orc_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                          const uint64_t *voff, uint64_t n);
/* remove() batch (merkle.rs:59-62); returns a new tree. */
orc_tree *orc_tree_remove(const orc_tree *t, const uint8_t *kb, const uint64_t *koff, uint64_t n);
void orc_tree_free(orc_tree *t);

uint64_t orc_tree_len(const orc_tree *t);
/* returns 1 and writes the root if non-empty, 0 for the empty tree (R6) */
int orc_tree_root(const orc_tree *t, uint8_t out[32]);
uint32_t orc_tree_nlevels(const orc_tree *t);
/* level l node count; copies the level's digests into out (may be NULL) */
uint64_t orc_tree_level(const orc_tree *t, uint32_t l, uint8_t *out);
/* sorted leaf i: key pointer/length (owned by the tree) and digest (merkle.rs:133-138) */
void orc_tree_leaf(const orc_tree *t, uint64_t i, const uint8_t **key, uint64_t *klen, uint8_t digest[32]);

/* R7 diff (merkle.rs:171-196). Returns count; *out_kb / *out_koff are malloc'd (free with orc_free). */
uint64_t orc_tree_diff(const orc_tree *a, const orc_tree *b, uint8_t **out_kb, uint64_t **out_koff);
/* Root of the leaves whose key starts with prefix (HASH <prefix>, server.rs:647-685); 0 if none. */
int orc_tree_prefix_root(const orc_tree *t, const uint8_t *prefix, uint64_t plen, uint8_t out[32]);
void orc_free(void *p);

/* ---- synthetic workload generator (shared definition with tests/golden and the device generator) ----
 * mix64 = splitmix64 finaliser; word(seed, idx, field, j) = mix64(seed + GOLD * (((idx<<12)|(field<<6)|j) + 1))
 * keys: klen chars, values: vlen chars from the sorted URL-safe base64 alphabet; key char 0 is restricted
 * to shard g of G (G | 64) so shards are contiguous key ranges. */
uint64_t orc_gen_word(uint64_t seed, uint64_t idx, uint32_t field, uint32_t j);
/* Generate records idx in [idx0, idx0+n) (fields: key 0, value `vfield`). Fixed lengths klen/vlen;
 * ragged == 1: klen = 1 + w%klen, vlen = w'%(vlen+1) per record; ragged == 2 ("store-like"): klen in
 * [max(1, klen/8), klen], vlen in [vlen/16, vlen]. Buffers: kb >= n*klen, vb >= n*vlen. */
void orc_gen_records(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, int ragged,
                     uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb,
                     uint64_t *voff);

/* ---- timed CPU baseline ---- build over packed records, single thread; returns seconds. */
double orc_bench_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t root_out[32]);
double orc_bench_leaf_hash(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                           uint64_t n, uint8_t *digests_out);

/* ---- timed CPU baselines (cpu_baselines.c; bench.py cpu_baseline leg) ----
 * cpu_ref: the reference's data structures (SipHash HashMap of heap Strings / Vecs, deep-cloned node
 * tree per level, merkle.rs:52-121, :171-196), single thread. cpu_mt: optimised, `threads` host threads.
 * Each returns seconds of the timed part. */
double orc_ref_bulk(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    uint8_t root_out[32]);
double orc_ref_insert_loop(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                           uint64_t n, uint8_t root_out[32]);
double orc_ref_diff(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    const uint8_t *kb2, const uint64_t *koff2, const uint8_t *vb2, const uint64_t *voff2, uint64_t n2,
                    uint64_t *count);
double orc_mt_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    int threads, uint8_t root_out[32]);
double orc_mt_diff(const orc_tree *a, const orc_tree *b, int threads, uint64_t *count);

#ifdef __cplusplus
}
#endif
#endif
