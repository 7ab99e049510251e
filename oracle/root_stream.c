/*
 * root_stream.c — global Merkle root over G generator key-range shards, streamed shard by shard
 * (TEST INFRASTRUCTURE ONLY: it computes the configs[3] golden root committed under tests/golden/; the
 * product never links or runs it).
 *
 * configs[3] is "1B keys sharded by key range across 8 GPUs". One orc_tree over 1B records would need
 * ~170 GB of host memory, so this program restates the same rules without materialising the tree:
 *   R1 + R2  leaf digest = SHA-256(u32_be|k| || k || u32_be|v| || v)   merkle.rs:7-16, :45-49
 *   R3       leaves in byte order of the key                              merkle.rs:80-81
 *   R4 + R5  pairwise parents, the odd last node of a level promoted     merkle.rs:94-118
 * Shard g holds records idx in [g*nper, (g+1)*nper) drawn with key char 0 restricted to the g-th slice of
 * the sorted alphabet (orc_gen_records(shard = g, nshards = G)), so shard g's sorted keys are the global
 * leaves [g*nper, (g+1)*nper) and the global leaf order is the concatenation of the shards' sorted keys.
 * Each shard is generated, hashed, sorted (radix on the first two key bytes, then a comparison sort per
 * bucket) and its digests pushed in order into a streaming reducer: pend[l] holds the left node of an open
 * pair at level l; pushing a node at level l pairs it with pend[l] (parent at l+1) or leaves it pending.
 * Full 2^B-leaf blocks whose global start is a multiple of 2^B are reduced in parallel and pushed as
 * level-B nodes (a complete aligned block contains no promotion). At the end each still-pending node below
 * the top is the odd last node of its level and is promoted unchanged one level up (R5), which yields
 * exactly the level arrays of rebuild(). The result is checked against orc_tree_build on small unions by
 * tests/test_oracle.py::test_root_stream_matches_tree_build.
 *
 * usage: root_stream SEED G NPER [KLEN VLEN BLOCK_LOG2 THREADS]   (fixed KLEN <= 32, VLEN)
 * prints one JSON object: root hex, leaf count, per-shard counts, sha backend, seconds.
 */
#define _GNU_SOURCE
#include "merkle_oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    uint8_t k[32];
    uint8_t d[32];
} rec_t;

static uint64_t g_seed, g_nper;
static uint32_t g_G, g_klen, g_vlen, g_blog, g_threads;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* ---- streaming reducer (R4/R5) ---- */
#define MAXL 80
static uint8_t pend[MAXL][32];
static int has_pend[MAXL];

static void push_node(uint32_t l, const uint8_t h[32]) {
    uint8_t cur[32];
    memcpy(cur, h, 32);
    while (has_pend[l]) {
        orc_node_digest(pend[l], cur, cur);
        has_pend[l] = 0;
        ++l;
    }
    memcpy(pend[l], cur, 32);
    has_pend[l] = 1;
}

/* End of the leaf stream: every pending node that is not the top is its level's odd last node (level
 * count odd <=> a pending node there), promoted unchanged (merkle.rs:111-114). */
static int finish(uint8_t root[32]) {
    for (uint32_t l = 0; l + 1 < MAXL; ++l) {
        if (!has_pend[l]) continue;
        int above = 0;
        for (uint32_t m = l + 1; m < MAXL; ++m) above |= has_pend[m];
        if (!above) {
            memcpy(root, pend[l], 32);
            return 1;
        }
        uint8_t x[32];
        memcpy(x, pend[l], 32);
        has_pend[l] = 0;
        push_node(l + 1, x);
    }
    return 0;
}

/* ---- per-shard work, parallel ---- */
static rec_t *A, *Bv;  /* generated records (A), bucketed (Bv) */
static uint64_t *hist; /* threads x 65536 */
static uint64_t cur_idx0;
static uint32_t cur_shard;

typedef struct {
    uint32_t tid;
} targ;

static void range_of(uint32_t tid, uint64_t n, uint64_t *lo, uint64_t *hi) {
    *lo = n * tid / g_threads;
    *hi = n * (tid + 1) / g_threads;
}

static void *gen_hash(void *p) {
    const uint32_t tid = ((targ *)p)->tid;
    uint64_t lo, hi;
    range_of(tid, g_nper, &lo, &hi);
    const uint64_t CH = 65536;
    uint8_t *kb = malloc(CH * g_klen + 64), *vb = malloc(CH * g_vlen + 64);
    uint64_t *ko = malloc((CH + 1) * 8), *vo = malloc((CH + 1) * 8);
    uint64_t *h = hist + (uint64_t)tid * 65536;
    memset(h, 0, 65536 * 8);
    for (uint64_t s = lo; s < hi; s += CH) {
        const uint64_t c = hi - s < CH ? hi - s : CH;
        orc_gen_records(g_seed, cur_idx0 + s, c, g_klen, g_vlen, 0, cur_shard, g_G, 1, kb, ko, vb, vo);
        for (uint64_t i = 0; i < c; ++i) {
            rec_t *r = &A[s + i];
            memset(r->k, 0, 32);
            memcpy(r->k, kb + ko[i], g_klen);
            orc_leaf_digest(kb + ko[i], g_klen, vb + vo[i], g_vlen, r->d);
            h[((uint32_t)r->k[0] << 8) | r->k[1]]++;
        }
    }
    free(kb);
    free(vb);
    free(ko);
    free(vo);
    return NULL;
}

static void *scatter(void *p) {
    const uint32_t tid = ((targ *)p)->tid;
    uint64_t lo, hi;
    range_of(tid, g_nper, &lo, &hi);
    uint64_t *h = hist + (uint64_t)tid * 65536; /* holds this thread's start offsets per bucket */
    for (uint64_t i = lo; i < hi; ++i) Bv[h[((uint32_t)A[i].k[0] << 8) | A[i].k[1]]++] = A[i];
    return NULL;
}

static uint64_t bstart[65537];
static atomic_uint_fast64_t next_bucket;
static atomic_uint_fast64_t dup_count;

static int rec_cmp(const void *a, const void *b) { return memcmp(((const rec_t *)a)->k, ((const rec_t *)b)->k, 32); }

static void *sort_buckets(void *p) {
    (void)p;
    for (;;) {
        uint64_t b = atomic_fetch_add(&next_bucket, 1);
        if (b >= 65536) break;
        uint64_t s = bstart[b], e = bstart[b + 1];
        if (e - s > 1) qsort(Bv + s, e - s, sizeof(rec_t), rec_cmp);
        for (uint64_t i = s + 1; i < e; ++i)
            if (!memcmp(Bv[i - 1].k, Bv[i].k, 32)) atomic_fetch_add(&dup_count, 1);
    }
    return NULL;
}

/* full aligned blocks [blk0, blk0 + nblk) of this shard (global block index), roots into broots */
static uint64_t blk_first_leaf, blk_count;
static uint8_t (*broots)[32];
static atomic_uint_fast64_t next_block;

static void *reduce_blocks(void *p) {
    (void)p;
    const uint64_t bs = 1ull << g_blog;
    uint8_t(*buf)[32] = malloc(bs * 32);
    for (;;) {
        uint64_t b = atomic_fetch_add(&next_block, 1);
        if (b >= blk_count) break;
        const rec_t *src = Bv + blk_first_leaf + b * bs;
        for (uint64_t i = 0; i < bs; ++i) memcpy(buf[i], src[i].d, 32);
        for (uint64_t m = bs; m > 1; m >>= 1)
            for (uint64_t j = 0; j < m / 2; ++j) orc_node_digest(buf[2 * j], buf[2 * j + 1], buf[j]);
        memcpy(broots[b], buf[0], 32);
    }
    free(buf);
    return NULL;
}

static void run_threads(void *(*fn)(void *)) {
    pthread_t th[256];
    targ a[256];
    for (uint32_t t = 0; t < g_threads; ++t) {
        a[t].tid = t;
        pthread_create(&th[t], NULL, fn, &a[t]);
    }
    for (uint32_t t = 0; t < g_threads; ++t) pthread_join(th[t], NULL);
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s SEED G NPER [KLEN VLEN BLOCK_LOG2 THREADS]\n", argv[0]);
        return 2;
    }
    g_seed = strtoull(argv[1], NULL, 0);
    g_G = (uint32_t)strtoul(argv[2], NULL, 0);
    g_nper = strtoull(argv[3], NULL, 0);
    g_klen = argc > 4 ? (uint32_t)strtoul(argv[4], NULL, 0) : 32;
    g_vlen = argc > 5 ? (uint32_t)strtoul(argv[5], NULL, 0) : 100;
    g_blog = argc > 6 ? (uint32_t)strtoul(argv[6], NULL, 0) : 20;
    g_threads = argc > 7 ? (uint32_t)strtoul(argv[7], NULL, 0) : 8;
    if (g_klen == 0 || g_klen > 32 || g_G == 0 || g_G > 64 || 64 % g_G || g_threads == 0 || g_threads > 256 ||
        g_blog == 0 || g_blog > 30) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    const int shani = orc_set_sha_backend(1); /* cross-checked against the portable backend in tests */
    const double t0 = now_s();
    A = malloc(g_nper * sizeof(rec_t));
    Bv = malloc(g_nper * sizeof(rec_t));
    hist = malloc((uint64_t)g_threads * 65536 * 8);
    if (!A || !Bv || !hist) {
        fprintf(stderr, "out of memory\n");
        return 1;
    }
    const uint64_t bs = 1ull << g_blog;
    broots = malloc((g_nper / bs + 2) * 32);
    uint64_t total = 0;
    printf("{\"seed\": %llu, \"shards\": %u, \"per_shard\": %llu, \"klen\": %u, \"vlen\": %u, \"counts\": [",
           (unsigned long long)g_seed, g_G, (unsigned long long)g_nper, g_klen, g_vlen);
    for (uint32_t g = 0; g < g_G; ++g) {
        cur_shard = g;
        cur_idx0 = (uint64_t)g * g_nper;
        run_threads(gen_hash);
        /* bucket offsets: bucket-major, thread-minor (stable by input index) */
        uint64_t off = 0;
        for (uint32_t b = 0; b < 65536; ++b) {
            bstart[b] = off;
            for (uint32_t t = 0; t < g_threads; ++t) {
                uint64_t c = hist[(uint64_t)t * 65536 + b];
                hist[(uint64_t)t * 65536 + b] = off;
                off += c;
            }
        }
        bstart[65536] = off;
        run_threads(scatter);
        atomic_store(&next_bucket, 0);
        atomic_store(&dup_count, 0);
        run_threads(sort_buckets);
        if (atomic_load(&dup_count)) {
            fprintf(stderr, "shard %u: %llu duplicate keys (generator uniqueness violated)\n", g,
                    (unsigned long long)atomic_load(&dup_count));
            return 1;
        }
        /* stream the shard's leaves [total, total + nper) */
        uint64_t i = 0;
        while (i < g_nper && ((total + i) & (bs - 1))) push_node(0, Bv[i++].d);
        blk_first_leaf = i;
        blk_count = (g_nper - i) / bs;
        atomic_store(&next_block, 0);
        run_threads(reduce_blocks);
        for (uint64_t b = 0; b < blk_count; ++b) push_node(g_blog, broots[b]);
        for (i = blk_first_leaf + blk_count * bs; i < g_nper; ++i) push_node(0, Bv[i].d);
        total += g_nper;
        printf("%s%llu", g ? ", " : "", (unsigned long long)g_nper);
        fflush(stdout);
    }
    uint8_t root[32];
    const int ok = total ? finish(root) : 0;
    printf("], \"n\": %llu, \"root\": \"", (unsigned long long)total);
    if (ok)
        for (int j = 0; j < 32; ++j) printf("%02x", root[j]);
    printf("\", \"sha_backend\": \"%s\", \"threads\": %u, \"seconds\": %.1f}\n", shani ? "sha-ni" : "portable",
           g_threads, now_s() - t0);
    free(A);
    free(Bv);
    free(hist);
    free(broots);
    return 0;
}
