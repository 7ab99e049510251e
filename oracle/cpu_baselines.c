/*
 * cpu_baselines.c — timed CPU baselines for bench.py (TEST INFRASTRUCTURE ONLY, linked into
 * liboracle.so; never part of the product library).
 *
 * Two flavours of MerkleKV's Merkle tree on the host:
 *
 *  cpu_ref — reference-faithful, single thread: the data structures and allocation pattern of
 *            /root/reference/src/store/merkle.rs, restated in C:
 *              leaf_map    HashMap<String, Vec<u8>> (merkle.rs:31) — open addressing, SipHash-1-3 keys
 *                          (Rust's default hasher), every key a heap String, every digest a heap Vec;
 *              insert      compute_leaf_hash (encode_leaf into a fresh Vec, SHA-256, .to_vec()) + map
 *                          insert (new String; an overwrite drops the old digest) + rebuild (:52-56);
 *              rebuild     collect (&key, &digest) refs, sort_by key (:79-81), leaf nodes with cloned
 *                          hash Vec and key String (:83-91), then per level: parent = SHA-256(l || r)
 *                          with BOTH CHILDREN DEEP-CLONED into new boxes (:107-108), odd last node
 *                          cloned (:111-114), old level dropped (recursive frees) (:117), old root
 *                          dropped when the new one is assigned (:120);
 *              diff_keys   BTreeSet of the union of keys (:175-177) — here the union of key refs is
 *                          sorted and deduplicated (the same O(u log u) key compares), then two
 *                          HashMap lookups per key and a String clone per divergent key (:181-193).
 *            SHA-256 uses SHA-NI when the CPU has it (sha2 0.10.9 selects it at run time).
 *  cpu_mt  — optimised, all host cores (pthreads): parallel leaf hashing, parallel chunk sort + merge,
 *            parallel level reduction, range-partitioned parallel merge diff. Same results.
 *
 * Both produce the reference's root and diff (checked against the oracle by tests/test_oracle.py).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "merkle_oracle.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* ============================================================================================
 * cpu_ref
 * ============================================================================================ */

/* SipHash-1-3 (Rust std's DefaultHasher), fixed keys. */
static inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }
#define SIPROUND                                                                          \
    do {                                                                                  \
        v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);                         \
        v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;                                            \
        v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;                                            \
        v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);                         \
    } while (0)
static uint64_t siphash13(const uint8_t *p, size_t n) {
    const uint64_t k0 = 0x0706050403020100ULL, k1 = 0x0f0e0d0c0b0a0908ULL;
    uint64_t v0 = k0 ^ 0x736f6d6570736575ULL, v1 = k1 ^ 0x646f72616e646f6dULL;
    uint64_t v2 = k0 ^ 0x6c7967656e657261ULL, v3 = k1 ^ 0x7465646279746573ULL;
    const size_t end = n & ~(size_t)7;
    for (size_t i = 0; i < end; i += 8) {
        uint64_t m;
        memcpy(&m, p + i, 8);
        v3 ^= m;
        SIPROUND;
        v0 ^= m;
    }
    uint64_t b = (uint64_t)n << 56;
    for (size_t i = end; i < n; ++i) b |= (uint64_t)p[i] << (8 * (i - end));
    v3 ^= b;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    SIPROUND; SIPROUND; SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

typedef struct {
    uint8_t *key;   /* String */
    uint32_t klen;
    uint8_t *hash;  /* Vec<u8>(32) */
} ref_slot;

typedef struct ref_node {
    uint8_t *hash;            /* Vec<u8> */
    struct ref_node *left;    /* Option<Box<MerkleNode>> */
    struct ref_node *right;
    uint8_t *key;             /* Option<String> */
    uint32_t klen;
} ref_node;

typedef struct {
    ref_slot *slots;
    uint64_t cap, len;
    ref_node root;
    int has_root;
} ref_tree;

static int rkey_cmp(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    uint32_t m = la < lb ? la : lb;
    int c = m ? memcmp(a, b, m) : 0;
    return c ? c : (la > lb) - (la < lb);
}

static uint8_t *dup(const uint8_t *p, size_t n) {
    uint8_t *q = (uint8_t *)malloc(n ? n : 1);
    if (n) memcpy(q, p, n);
    return q;
}

static void node_clone_into(const ref_node *s, ref_node *d) {
    d->hash = dup(s->hash, 32);
    d->key = s->key ? dup(s->key, s->klen) : NULL;
    d->klen = s->klen;
    d->left = d->right = NULL;
    if (s->left) {
        d->left = (ref_node *)malloc(sizeof(ref_node));
        node_clone_into(s->left, d->left);
    }
    if (s->right) {
        d->right = (ref_node *)malloc(sizeof(ref_node));
        node_clone_into(s->right, d->right);
    }
}

static void node_drop(ref_node *n) {
    free(n->hash);
    free(n->key);
    if (n->left) {
        node_drop(n->left);
        free(n->left);
    }
    if (n->right) {
        node_drop(n->right);
        free(n->right);
    }
}

static void map_grow(ref_tree *t) {
    uint64_t nc = t->cap ? 2 * t->cap : 16;
    ref_slot *ns = (ref_slot *)calloc(nc, sizeof(ref_slot));
    for (uint64_t i = 0; i < t->cap; ++i) {
        if (!t->slots[i].key) continue;
        uint64_t h = siphash13(t->slots[i].key, t->slots[i].klen) & (nc - 1);
        while (ns[h].key) h = (h + 1) & (nc - 1);
        ns[h] = t->slots[i];
    }
    free(t->slots);
    t->slots = ns;
    t->cap = nc;
}

static int cmp_slot_ptr(const void *a, const void *b) {
    const ref_slot *x = *(ref_slot *const *)a, *y = *(ref_slot *const *)b;
    return rkey_cmp(x->key, x->klen, y->key, y->klen);
}

/* rebuild(), merkle.rs:73-121 */
static void ref_rebuild(ref_tree *t) {
    if (t->len == 0) {
        if (t->has_root) node_drop(&t->root);
        t->has_root = 0;
        return;
    }
    ref_slot **leaves = (ref_slot **)malloc(t->len * sizeof(ref_slot *));
    uint64_t n = 0;
    for (uint64_t i = 0; i < t->cap; ++i)
        if (t->slots[i].key) leaves[n++] = &t->slots[i];
    qsort(leaves, n, sizeof(ref_slot *), cmp_slot_ptr);
    ref_node *nodes = (ref_node *)malloc(n * sizeof(ref_node));
    for (uint64_t i = 0; i < n; ++i) {
        nodes[i].hash = dup(leaves[i]->hash, 32);
        nodes[i].key = dup(leaves[i]->key, leaves[i]->klen);
        nodes[i].klen = leaves[i]->klen;
        nodes[i].left = nodes[i].right = NULL;
    }
    free(leaves);
    while (n > 1) {
        const uint64_t p = (n + 1) / 2;
        ref_node *lvl = (ref_node *)malloc(p * sizeof(ref_node));
        for (uint64_t j = 0; j < p; ++j) {
            if (2 * j + 1 < n) {
                uint8_t m[64];
                memcpy(m, nodes[2 * j].hash, 32);
                memcpy(m + 32, nodes[2 * j + 1].hash, 32);
                lvl[j].hash = (uint8_t *)malloc(32);
                orc_sha256(m, 64, lvl[j].hash);
                lvl[j].left = (ref_node *)malloc(sizeof(ref_node));
                node_clone_into(&nodes[2 * j], lvl[j].left);
                lvl[j].right = (ref_node *)malloc(sizeof(ref_node));
                node_clone_into(&nodes[2 * j + 1], lvl[j].right);
                lvl[j].key = NULL;
                lvl[j].klen = 0;
            } else {
                node_clone_into(&nodes[2 * j], &lvl[j]);
            }
        }
        for (uint64_t i = 0; i < n; ++i) node_drop(&nodes[i]);  /* nodes = new_level drops the old Vec */
        free(nodes);
        nodes = lvl;
        n = p;
    }
    if (t->has_root) node_drop(&t->root);
    t->root = nodes[0];
    t->has_root = 1;
    free(nodes);
}

/* compute_leaf_hash (merkle.rs:45-49): encode_leaf into a fresh Vec (:7-16), hash, finalize().to_vec() */
static uint8_t *ref_leaf_hash(const uint8_t *k, uint32_t kl, const uint8_t *v, uint32_t vl) {
    uint8_t *enc = (uint8_t *)malloc(8 + (size_t)kl + vl);
    enc[0] = (uint8_t)(kl >> 24); enc[1] = (uint8_t)(kl >> 16); enc[2] = (uint8_t)(kl >> 8); enc[3] = (uint8_t)kl;
    memcpy(enc + 4, k, kl);
    uint8_t *q = enc + 4 + kl;
    q[0] = (uint8_t)(vl >> 24); q[1] = (uint8_t)(vl >> 16); q[2] = (uint8_t)(vl >> 8); q[3] = (uint8_t)vl;
    memcpy(q + 4, v, vl);
    uint8_t *h = (uint8_t *)malloc(32);
    orc_sha256(enc, 8 + (size_t)kl + vl, h);
    free(enc);
    return h;
}

/* leaf_map.insert(key.to_string(), hash) (merkle.rs:54) */
static void ref_map_insert(ref_tree *t, const uint8_t *k, uint32_t kl, uint8_t *hash) {
    uint8_t *ks = dup(k, kl);  /* key.to_string() */
    if ((t->len + 1) * 8 > t->cap * 7) map_grow(t);
    uint64_t h = siphash13(ks, kl) & (t->cap - 1);
    while (t->slots[h].key) {
        if (rkey_cmp(t->slots[h].key, t->slots[h].klen, ks, kl) == 0) {
            free(t->slots[h].hash);  /* old value dropped */
            t->slots[h].hash = hash;
            free(ks);                /* the new key String is dropped (HashMap keeps the old one) */
            return;
        }
        h = (h + 1) & (t->cap - 1);
    }
    t->slots[h].key = ks;
    t->slots[h].klen = kl;
    t->slots[h].hash = hash;
    ++t->len;
}

static const uint8_t *ref_map_get(const ref_tree *t, const uint8_t *k, uint32_t kl) {
    if (!t->cap) return NULL;
    uint64_t h = siphash13(k, kl) & (t->cap - 1);
    while (t->slots[h].key) {
        if (rkey_cmp(t->slots[h].key, t->slots[h].klen, k, kl) == 0) return t->slots[h].hash;
        h = (h + 1) & (t->cap - 1);
    }
    return NULL;
}

static void ref_free(ref_tree *t) {
    for (uint64_t i = 0; i < t->cap; ++i) {
        free(t->slots[i].key);
        free(t->slots[i].hash);
    }
    free(t->slots);
    if (t->has_root) node_drop(&t->root);
    memset(t, 0, sizeof(*t));
}

static void ref_fill(ref_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                     uint64_t n, int rebuild_each) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t kl = (uint32_t)(koff[i + 1] - koff[i]), vl = (uint32_t)(voff[i + 1] - voff[i]);
        ref_map_insert(t, kb + koff[i], kl, ref_leaf_hash(kb + koff[i], kl, vb + voff[i], vl));
        if (rebuild_each) ref_rebuild(t);
    }
}

/* The reference's data structures and rebuild, timed: n x (compute_leaf_hash + map insert) then ONE
 * rebuild (what a bulk load would cost if insert did not rebuild). Returns seconds. */
double orc_ref_bulk(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    uint8_t root_out[32]) {
    ref_tree t;
    memset(&t, 0, sizeof(t));
    const double t0 = now_s();
    ref_fill(&t, kb, koff, vb, voff, n, 0);
    ref_rebuild(&t);
    const double t1 = now_s();
    if (t.has_root) memcpy(root_out, t.root.hash, 32);
    else memset(root_out, 0, 32);
    ref_free(&t);
    return t1 - t0;
}

/* The reference's public API as its callers use it (sync.rs:110-115, server.rs:664-667):
 * new() + n x insert(), each insert rebuilding the whole tree (O(n^2 log n)). Returns seconds. */
double orc_ref_insert_loop(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                           uint64_t n, uint8_t root_out[32]) {
    ref_tree t;
    memset(&t, 0, sizeof(t));
    const double t0 = now_s();
    ref_fill(&t, kb, koff, vb, voff, n, 1);
    const double t1 = now_s();
    if (t.has_root) memcpy(root_out, t.root.hash, 32);
    else memset(root_out, 0, 32);
    ref_free(&t);
    return t1 - t0;
}

typedef struct {
    const uint8_t *k;
    uint32_t l;
} kref;

static int cmp_kref(const void *a, const void *b) {
    const kref *x = (const kref *)a, *y = (const kref *)b;
    return rkey_cmp(x->k, x->l, y->k, y->l);
}

/* diff_keys (merkle.rs:171-196) between two reference-structured trees built from the two record sets;
 * only the diff is timed. Returns seconds; *count = divergent keys. */
double orc_ref_diff(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    const uint8_t *kb2, const uint64_t *koff2, const uint8_t *vb2, const uint64_t *voff2, uint64_t n2,
                    uint64_t *count) {
    ref_tree a, b;
    memset(&a, 0, sizeof(a));
    memset(&b, 0, sizeof(b));
    ref_fill(&a, kb, koff, vb, voff, n, 0);
    ref_fill(&b, kb2, koff2, vb2, voff2, n2, 0);
    const double t0 = now_s();
    kref *u = (kref *)malloc((a.len + b.len + 1) * sizeof(kref));
    uint64_t m = 0;
    for (uint64_t i = 0; i < a.cap; ++i)
        if (a.slots[i].key) u[m++] = (kref){a.slots[i].key, a.slots[i].klen};
    for (uint64_t i = 0; i < b.cap; ++i)
        if (b.slots[i].key) u[m++] = (kref){b.slots[i].key, b.slots[i].klen};
    qsort(u, m, sizeof(kref), cmp_kref);  /* BTreeSet<&String>: ordered union */
    uint64_t cap = 64, cnt = 0;
    uint8_t **out = (uint8_t **)malloc(cap * sizeof(uint8_t *));
    for (uint64_t i = 0; i < m; ++i) {
        if (i && cmp_kref(&u[i - 1], &u[i]) == 0) continue;
        const uint8_t *h1 = ref_map_get(&a, u[i].k, u[i].l), *h2 = ref_map_get(&b, u[i].k, u[i].l);
        if (!h1 || !h2 || memcmp(h1, h2, 32) != 0) {
            if (cnt == cap) {
                cap *= 2;
                out = (uint8_t **)realloc(out, cap * sizeof(uint8_t *));
            }
            out[cnt++] = dup(u[i].k, u[i].l);  /* k.clone() */
        }
    }
    const double t1 = now_s();
    for (uint64_t i = 0; i < cnt; ++i) free(out[i]);
    free(out);
    free(u);
    ref_free(&a);
    ref_free(&b);
    *count = cnt;
    return t1 - t0;
}

/* ============================================================================================
 * cpu_mt
 * ============================================================================================ */
typedef struct {
    const uint8_t *kb, *vb;
    const uint64_t *koff, *voff;
    uint64_t *idx;
    uint8_t *dig;
    uint64_t lo, hi;
} mt_job;

static void *mt_hash(void *p) {
    mt_job *j = (mt_job *)p;
    for (uint64_t i = j->lo; i < j->hi; ++i)
        orc_leaf_digest(j->kb + j->koff[i], j->koff[i + 1] - j->koff[i], j->vb + j->voff[i],
                        j->voff[i + 1] - j->voff[i], j->dig + 32 * i);
    return NULL;
}

typedef struct {
    const uint8_t *kb;
    const uint64_t *koff;
} mt_sc;

static int mt_idx_cmp(const void *pa, const void *pb, void *arg) {
    const mt_sc *s = (const mt_sc *)arg;
    uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
    int c = rkey_cmp(s->kb + s->koff[a], (uint32_t)(s->koff[a + 1] - s->koff[a]), s->kb + s->koff[b],
                     (uint32_t)(s->koff[b + 1] - s->koff[b]));
    return c ? c : (a > b) - (a < b);
}

static void *mt_sort(void *p) {
    mt_job *j = (mt_job *)p;
    mt_sc sc = {j->kb, j->koff};
    for (uint64_t i = j->lo; i < j->hi; ++i) j->idx[i] = i;
    qsort_r(j->idx + j->lo, j->hi - j->lo, sizeof(uint64_t), mt_idx_cmp, &sc);
    return NULL;
}

typedef struct {
    const uint8_t *kb;
    const uint64_t *koff;
    const uint64_t *src;
    uint64_t *dst;
    uint64_t a0, a1, b0, b1, o;
} mt_merge_job;

static void *mt_merge(void *p) {
    mt_merge_job *m = (mt_merge_job *)p;
    mt_sc sc = {m->kb, m->koff};
    uint64_t i = m->a0, j = m->b0, o = m->o;
    while (i < m->a1 && j < m->b1)
        m->dst[o++] = mt_idx_cmp(&m->src[j], &m->src[i], &sc) < 0 ? m->src[j++] : m->src[i++];
    while (i < m->a1) m->dst[o++] = m->src[i++];
    while (j < m->b1) m->dst[o++] = m->src[j++];
    return NULL;
}

typedef struct {
    const uint8_t *c;
    uint8_t *p;
    uint64_t cn, lo, hi;
} mt_lvl_job;

static void *mt_level(void *p) {
    mt_lvl_job *j = (mt_lvl_job *)p;
    for (uint64_t x = j->lo; x < j->hi; ++x) {
        if (2 * x + 1 < j->cn) orc_node_digest(j->c + 64 * x, j->c + 64 * x + 32, j->p + 32 * x);
        else memcpy(j->p + 32 * x, j->c + 64 * x, 32);
    }
    return NULL;
}

/* Optimised build on `threads` host threads: returns seconds, writes the root. */
double orc_mt_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                    int threads, uint8_t root_out[32]) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    mt_job jobs[256];
    uint8_t *dig = (uint8_t *)malloc(n ? 32 * n : 32);
    uint64_t *idx = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
    uint64_t *tmp = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
    const double t0 = now_s();
    /* 1) leaf digests + per-chunk sorts */
    uint64_t bounds[257];
    for (int i = 0; i <= threads; ++i) bounds[i] = n * (uint64_t)i / (uint64_t)threads;
    for (int i = 0; i < threads; ++i) {
        jobs[i] = (mt_job){kb, vb, koff, voff, idx, dig, bounds[i], bounds[i + 1]};
        pthread_create(&th[i], NULL, mt_hash, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, mt_sort, &jobs[i]);
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    /* 2) pairwise merges of sorted runs, in parallel per round */
    int runs = threads;
    uint64_t *src = idx, *dst = tmp;
    while (runs > 1) {
        mt_merge_job mj[128];
        int k = 0;
        for (int r = 0; r < runs; r += 2) {
            const uint64_t a0 = bounds[r], a1 = bounds[r + 1], b1 = r + 1 < runs ? bounds[r + 2] : a1;
            mj[k] = (mt_merge_job){kb, koff, src, dst, a0, a1, a1, b1, a0};
            pthread_create(&th[k], NULL, mt_merge, &mj[k]);
            ++k;
        }
        for (int i = 0; i < k; ++i) pthread_join(th[i], NULL);
        int nr = 0;
        for (int r = 0; r < runs; r += 2) bounds[nr++] = bounds[r];
        bounds[nr] = n;
        runs = nr;
        uint64_t *s = src;
        src = dst;
        dst = s;
    }
    /* 3) dedup (keep the last write) + leaf level in key order */
    uint64_t m = 0;
    uint8_t *lvl0 = (uint8_t *)malloc(n ? 32 * n : 32);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t a = src[i];
        if (i + 1 < n) {
            const uint64_t b = src[i + 1];
            if (rkey_cmp(kb + koff[a], (uint32_t)(koff[a + 1] - koff[a]), kb + koff[b], (uint32_t)(koff[b + 1] - koff[b])) == 0)
                continue;
        }
        memcpy(lvl0 + 32 * m++, dig + 32 * a, 32);
    }
    /* 4) levels, each split across the threads when large */
    uint8_t *cur = lvl0, *nxt = (uint8_t *)malloc(m ? 32 * ((m + 1) / 2) + 32 : 32);
    uint64_t s = m;
    while (s > 1) {
        const uint64_t p = (s + 1) / 2;
        const int T = p >= 65536 ? threads : 1;
        mt_lvl_job lj[256];
        for (int i = 0; i < T; ++i) {
            lj[i] = (mt_lvl_job){cur, nxt, s, p * (uint64_t)i / (uint64_t)T, p * (uint64_t)(i + 1) / (uint64_t)T};
            if (T > 1) pthread_create(&th[i], NULL, mt_level, &lj[i]);
            else mt_level(&lj[i]);
        }
        if (T > 1)
            for (int i = 0; i < T; ++i) pthread_join(th[i], NULL);
        uint8_t *t = cur;
        cur = nxt;
        nxt = t;
        s = p;
    }
    const double t1 = now_s();
    if (m) memcpy(root_out, cur, 32);
    else memset(root_out, 0, 32);
    free(dig);
    free(idx);
    free(tmp);
    free(cur);
    free(nxt);
    return t1 - t0;
}

typedef struct {
    const orc_tree *a, *b;
    uint64_t a0, a1, b0, b1, cnt;
} mt_diff_job;

static inline void leaf_key(const orc_tree *t, uint64_t i, const uint8_t **k, uint32_t *l) {
    uint64_t kl;
    orc_tree_leaf(t, i, k, &kl, NULL);
    *l = (uint32_t)kl;
}

static void *mt_diff(void *p) {
    mt_diff_job *j = (mt_diff_job *)p;
    uint64_t i = j->a0, k = j->b0, c = 0;
    uint8_t da[32], db[32];
    while (i < j->a1 || k < j->b1) {
        if (k >= j->b1) { ++c; ++i; continue; }
        if (i >= j->a1) { ++c; ++k; continue; }
        const uint8_t *ka, *kb_;
        uint32_t la, lb;
        leaf_key(j->a, i, &ka, &la);
        leaf_key(j->b, k, &kb_, &lb);
        const int cmp = rkey_cmp(ka, la, kb_, lb);
        if (cmp < 0) { ++c; ++i; }
        else if (cmp > 0) { ++c; ++k; }
        else {
            const uint8_t *x;
            uint64_t xl;
            orc_tree_leaf(j->a, i, &x, &xl, da);
            orc_tree_leaf(j->b, k, &x, &xl, db);
            c += memcmp(da, db, 32) != 0;
            ++i; ++k;
        }
    }
    j->cnt = c;
    return NULL;
}

/* lower bound of key (k, l) in tree t's sorted leaves */
static uint64_t lower_bound_key(const orc_tree *t, const uint8_t *k, uint32_t l) {
    uint64_t lo = 0, hi = orc_tree_len(t);
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        const uint8_t *x;
        uint64_t xl;
        orc_tree_leaf(t, mid, &x, &xl, NULL);
        if (rkey_cmp(x, (uint32_t)xl, k, l) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* Parallel diff_keys count over key ranges split at A's leaves (sorted merge per range). */
double orc_mt_diff(const orc_tree *a, const orc_tree *b, int threads, uint64_t *count) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    mt_diff_job jobs[256];
    const uint64_t na = orc_tree_len(a), nb = orc_tree_len(b);
    const double t0 = now_s();
    uint64_t prev_a = 0, prev_b = 0;
    for (int i = 0; i < threads; ++i) {
        uint64_t ea = i + 1 == threads ? na : na * (uint64_t)(i + 1) / (uint64_t)threads;
        uint64_t eb = nb;
        if (i + 1 < threads && ea < na) {
            const uint8_t *k;
            uint64_t kl;
            orc_tree_leaf(a, ea, &k, &kl, NULL);
            eb = lower_bound_key(b, k, (uint32_t)kl);
        }
        jobs[i] = (mt_diff_job){a, b, prev_a, ea, prev_b, eb, 0};
        prev_a = ea;
        prev_b = eb;
        pthread_create(&th[i], NULL, mt_diff, &jobs[i]);
    }
    uint64_t c = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        c += jobs[i].cnt;
    }
    const double t1 = now_s();
    *count = c;
    return t1 - t0;
}
