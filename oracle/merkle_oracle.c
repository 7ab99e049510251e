/*
 * merkle_oracle.c — CPU restatement of /root/reference/src/store/merkle.rs (TEST INFRASTRUCTURE ONLY).
 * See merkle_oracle.h for the rule list (R1-R7) and citations. Plain C11; SHA-NI path is x86-only and
 * used only for the timed baseline.
 */
#define _GNU_SOURCE
#include "merkle_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------------------------------------
 * SHA-256, FIPS 180-4 (the algorithm sha2 0.10.9 implements; Cargo.toml:21, Cargo.lock:1227-1230)
 * ------------------------------------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void compress_portable(uint32_t s[8], const uint8_t *blk) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) | ((uint32_t)blk[4 * t + 2] << 8) |
               (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

#if defined(__x86_64__)
__attribute__((target("sha,sse4.1,ssse3"))) static void compress_shani(uint32_t s[8], const uint8_t *blk) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i *)&s[0]);
    __m128i st1 = _mm_loadu_si128((const __m128i *)&s[4]);
    tmp = _mm_shuffle_epi32(tmp, 0xB1);
    st1 = _mm_shuffle_epi32(st1, 0x1B);
    __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);
    st1 = _mm_blend_epi16(st1, tmp, 0xF0);
    __m128i abef = st0, cdgh = st1;
    __m128i m[4];
    for (int i = 0; i < 16; ++i) {
        __m128i x;
        if (i < 4) {
            x = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk + 16 * i)), MASK);
        } else {
            __m128i t = _mm_sha256msg1_epu32(m[i & 3], m[(i + 1) & 3]);
            t = _mm_add_epi32(t, _mm_alignr_epi8(m[(i + 3) & 3], m[(i + 2) & 3], 4));
            x = _mm_sha256msg2_epu32(t, m[(i + 3) & 3]);
        }
        m[i & 3] = x;
        __m128i msg = _mm_add_epi32(x, _mm_loadu_si128((const __m128i *)&K256[4 * i]));
        st1 = _mm_sha256rnds2_epu32(st1, st0, msg);
        msg = _mm_shuffle_epi32(msg, 0x0E);
        st0 = _mm_sha256rnds2_epu32(st0, st1, msg);
    }
    st0 = _mm_add_epi32(st0, abef);
    st1 = _mm_add_epi32(st1, cdgh);
    tmp = _mm_shuffle_epi32(st0, 0x1B);
    st1 = _mm_shuffle_epi32(st1, 0xB1);
    st0 = _mm_blend_epi16(tmp, st1, 0xF0);
    st1 = _mm_alignr_epi8(st1, tmp, 8);
    _mm_storeu_si128((__m128i *)&s[0], st0);
    _mm_storeu_si128((__m128i *)&s[4], st1);
}
#endif

typedef void (*compress_fn)(uint32_t s[8], const uint8_t *blk);
static compress_fn g_compress = compress_portable;

int orc_cpu_has_shani(void) {
#if defined(__x86_64__)
    __builtin_cpu_init();
    return __builtin_cpu_supports("sha") ? 1 : 0;
#else
    return 0;
#endif
}

int orc_set_sha_backend(int backend) {
#if defined(__x86_64__)
    if (backend == 1 && orc_cpu_has_shani()) {
        g_compress = compress_shani;
        return 1;
    }
#endif
    g_compress = compress_portable;
    return 0;
}

/* Streaming hasher over a sequence of byte pieces. */
typedef struct {
    uint32_t s[8];
    uint8_t buf[64];
    size_t fill;
    uint64_t total;
} sha_ctx;

static void sha_init(sha_ctx *c) {
    memcpy(c->s, H0, sizeof H0);
    c->fill = 0;
    c->total = 0;
}
static void sha_update(sha_ctx *c, const uint8_t *p, size_t n) {
    c->total += n;
    while (n) {
        if (c->fill == 0 && n >= 64) {
            g_compress(c->s, p);
            p += 64;
            n -= 64;
            continue;
        }
        size_t take = 64 - c->fill;
        if (take > n) take = n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += take;
        p += take;
        n -= take;
        if (c->fill == 64) {
            g_compress(c->s, c->buf);
            c->fill = 0;
        }
    }
}
static void sha_final(sha_ctx *c, uint8_t out[32]) {
    uint64_t bits = c->total * 8;
    c->buf[c->fill++] = 0x80;
    if (c->fill > 56) {
        memset(c->buf + c->fill, 0, 64 - c->fill);
        g_compress(c->s, c->buf);
        c->fill = 0;
    }
    memset(c->buf + c->fill, 0, 56 - c->fill);
    for (int i = 0; i < 8; ++i) c->buf[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
    g_compress(c->s, c->buf);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(c->s[i] >> 24);
        out[4 * i + 1] = (uint8_t)(c->s[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->s[i] >> 8);
        out[4 * i + 3] = (uint8_t)(c->s[i]);
    }
}

void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
    sha_ctx c;
    sha_init(&c);
    sha_update(&c, msg, len);
    sha_final(&c, out);
}

/* R1 + R2: merkle.rs:7-16 (encode_leaf) and :45-49 (compute_leaf_hash). The encoding is streamed into
 * the hasher piecewise; the byte sequence hashed is exactly u32be(klen)||k||u32be(vlen)||v. */
void orc_leaf_digest(const uint8_t *k, uint64_t klen, const uint8_t *v, uint64_t vlen, uint8_t out[32]) {
    uint8_t kl[4] = {(uint8_t)(klen >> 24), (uint8_t)(klen >> 16), (uint8_t)(klen >> 8), (uint8_t)klen};
    uint8_t vl[4] = {(uint8_t)(vlen >> 24), (uint8_t)(vlen >> 16), (uint8_t)(vlen >> 8), (uint8_t)vlen};
    sha_ctx c;
    sha_init(&c);
    sha_update(&c, kl, 4);
    sha_update(&c, k, klen);
    sha_update(&c, vl, 4);
    sha_update(&c, v, vlen);
    sha_final(&c, out);
}

/* R4: merkle.rs:99-103 — parent = SHA-256(left.hash || right.hash). */
void orc_node_digest(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
    uint8_t m[64];
    memcpy(m, l, 32);
    memcpy(m + 32, r, 32);
    orc_sha256(m, 64, out);
}

/* ------------------------------------------------------------------------------------------------
 * Tree: sorted unique keys (owned), leaf digests, and the level arrays the reference's pointer tree
 * is isomorphic to (level l has ceil(n/2^l) nodes; R5 promotion copies the last node unchanged).
 * ------------------------------------------------------------------------------------------------ */
struct orc_tree {
    uint64_t n;
    uint8_t *kb;      /* sorted keys, packed */
    uint64_t *koff;   /* n+1 */
    uint32_t nlev;    /* number of levels (0 for empty, 1 for a single leaf) */
    uint64_t *lcnt;   /* per level node count */
    uint64_t *loff;   /* per level node offset into nodes */
    uint8_t *nodes;   /* all levels, 32 B per node; level 0 = leaf digests in key order */
};

/* R3: Rust `str` Ord (merkle.rs:80-81) = lexicographic bytes, shorter prefix first. */
static int key_cmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    uint64_t m = la < lb ? la : lb;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c;
    return (la > lb) - (la < lb);
}

typedef struct {
    const uint8_t *kb;
    const uint64_t *koff;
} sort_ctx;

static int idx_cmp(const void *pa, const void *pb, void *arg) {
    const sort_ctx *s = (const sort_ctx *)arg;
    uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
    int c = key_cmp(s->kb + s->koff[a], s->koff[a + 1] - s->koff[a], s->kb + s->koff[b], s->koff[b + 1] - s->koff[b]);
    if (c) return c;
    return (a > b) - (a < b); /* equal keys: insertion order, so the last write is last */
}

/* rebuild(), merkle.rs:73-121: levels bottom-up, pairs hashed left-to-right, odd last node promoted. */
static void build_levels(orc_tree *t) {
    uint64_t n = t->n;
    t->nlev = 0;
    if (n == 0) return;
    uint32_t L = 1;
    for (uint64_t s = n; s > 1; s = (s + 1) / 2) ++L;
    t->nlev = L;
    t->lcnt = (uint64_t *)malloc(L * sizeof(uint64_t));
    t->loff = (uint64_t *)malloc(L * sizeof(uint64_t));
    uint64_t tot = 0, s = n;
    for (uint32_t l = 0; l < L; ++l) {
        t->lcnt[l] = s;
        t->loff[l] = tot;
        tot += s;
        s = (s + 1) / 2;
    }
    uint8_t *nodes = (uint8_t *)realloc(t->nodes, tot * 32);
    t->nodes = nodes;
    for (uint32_t l = 1; l < L; ++l) {
        const uint8_t *c = nodes + 32 * t->loff[l - 1];
        uint8_t *p = nodes + 32 * t->loff[l];
        uint64_t cn = t->lcnt[l - 1];
        for (uint64_t j = 0; j < t->lcnt[l]; ++j) {
            if (2 * j + 1 < cn)
                orc_node_digest(c + 64 * j, c + 64 * j + 32, p + 32 * j);
            else
                memcpy(p + 32 * j, c + 64 * j, 32); /* R5: promote unchanged */
        }
    }
}

/* Sequential insert semantics over (key, digest) records: sort by key then insertion order, keep the
 * last occurrence of each key (HashMap::insert overwrite, merkle.rs:54), then rebuild. */
orc_tree *orc_tree_build_digests(const uint8_t *kb, const uint64_t *koff, const uint8_t *digests, uint64_t n) {
    orc_tree *t = (orc_tree *)calloc(1, sizeof(orc_tree));
    uint64_t *idx = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; ++i) idx[i] = i;
    sort_ctx sc = {kb, koff};
    if (n > 1) qsort_r(idx, n, sizeof(uint64_t), idx_cmp, &sc);
    /* dedup: keep last of each equal run */
    uint64_t m = 0, kbytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t a = idx[i];
        if (i + 1 < n) {
            uint64_t b = idx[i + 1];
            if (key_cmp(kb + koff[a], koff[a + 1] - koff[a], kb + koff[b], koff[b + 1] - koff[b]) == 0) continue;
        }
        idx[m++] = a;
        kbytes += koff[a + 1] - koff[a];
    }
    t->n = m;
    t->kb = (uint8_t *)malloc(kbytes ? kbytes : 1);
    t->koff = (uint64_t *)malloc((m + 1) * sizeof(uint64_t));
    t->nodes = (uint8_t *)malloc(m ? m * 32 : 1);
    uint64_t o = 0;
    for (uint64_t i = 0; i < m; ++i) {
        uint64_t a = idx[i], l = koff[a + 1] - koff[a];
        t->koff[i] = o;
        if (l) memcpy(t->kb + o, kb + koff[a], l);
        o += l;
        memcpy(t->nodes + 32 * i, digests + 32 * a, 32);
    }
    t->koff[m] = o;
    free(idx);
    build_levels(t);
    return t;
}

orc_tree *orc_tree_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                         uint64_t n) {
    uint8_t *dg = (uint8_t *)malloc(n ? n * 32 : 1);
    for (uint64_t i = 0; i < n; ++i)
        orc_leaf_digest(kb + koff[i], koff[i + 1] - koff[i], vb + voff[i], voff[i + 1] - voff[i], dg + 32 * i);
    orc_tree *t = orc_tree_build_digests(kb, koff, dg, n);
    free(dg);
    return t;
}

orc_tree *orc_tree_upsert(const orc_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                          const uint64_t *voff, uint64_t n) {
    uint64_t m = t->n, tot = m + n;
    uint64_t kbytes = t->koff[m] + (n ? koff[n] - koff[0] : 0);
    uint8_t *ckb = (uint8_t *)malloc(kbytes ? kbytes : 1);
    uint64_t *ckoff = (uint64_t *)malloc((tot + 1) * sizeof(uint64_t));
    uint8_t *dg = (uint8_t *)malloc(tot ? tot * 32 : 1);
    memcpy(ckb, t->kb, t->koff[m]);
    for (uint64_t i = 0; i <= m; ++i) ckoff[i] = t->koff[i];
    if (m) memcpy(dg, t->nodes, 32 * m);
    uint64_t o = t->koff[m];
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t l = koff[i + 1] - koff[i];
        memcpy(ckb + o, kb + koff[i], l);
        o += l;
        ckoff[m + i + 1] = o;
        orc_leaf_digest(kb + koff[i], l, vb + voff[i], voff[i + 1] - voff[i], dg + 32 * (m + i));
    }
    orc_tree *r = orc_tree_build_digests(ckb, ckoff, dg, tot);
    free(ckb);
    free(ckoff);
    free(dg);
    return r;
}

orc_tree *orc_tree_remove(const orc_tree *t, const uint8_t *kb, const uint64_t *koff, uint64_t n) {
    uint64_t m = t->n;
    uint8_t *keep = (uint8_t *)malloc(m ? m : 1);
    memset(keep, 1, m);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *k = kb + koff[i];
        uint64_t l = koff[i + 1] - koff[i];
        uint64_t lo = 0, hi = m;
        while (lo < hi) {
            uint64_t mid = (lo + hi) / 2;
            int c = key_cmp(t->kb + t->koff[mid], t->koff[mid + 1] - t->koff[mid], k, l);
            if (c < 0) lo = mid + 1; else hi = mid;
        }
        if (lo < m && key_cmp(t->kb + t->koff[lo], t->koff[lo + 1] - t->koff[lo], k, l) == 0) keep[lo] = 0;
    }
    uint64_t c = 0;
    for (uint64_t i = 0; i < m; ++i) c += keep[i];
    uint64_t *sel = (uint64_t *)malloc((c + 1) * sizeof(uint64_t));
    uint64_t j = 0;
    for (uint64_t i = 0; i < m; ++i)
        if (keep[i]) sel[j++] = i;
    uint64_t kbytes = 0;
    for (uint64_t i = 0; i < c; ++i) kbytes += t->koff[sel[i] + 1] - t->koff[sel[i]];
    uint8_t *ckb = (uint8_t *)malloc(kbytes ? kbytes : 1);
    uint64_t *ckoff = (uint64_t *)malloc((c + 1) * sizeof(uint64_t));
    uint8_t *dg = (uint8_t *)malloc(c ? c * 32 : 1);
    uint64_t o = 0;
    for (uint64_t i = 0; i < c; ++i) {
        uint64_t a = sel[i], l = t->koff[a + 1] - t->koff[a];
        ckoff[i] = o;
        memcpy(ckb + o, t->kb + t->koff[a], l);
        o += l;
        memcpy(dg + 32 * i, t->nodes + 32 * a, 32);
    }
    ckoff[c] = o;
    orc_tree *r = orc_tree_build_digests(ckb, ckoff, dg, c);
    free(keep);
    free(sel);
    free(ckb);
    free(ckoff);
    free(dg);
    return r;
}

void orc_tree_free(orc_tree *t) {
    if (!t) return;
    free(t->kb);
    free(t->koff);
    free(t->lcnt);
    free(t->loff);
    free(t->nodes);
    free(t);
}

uint64_t orc_tree_len(const orc_tree *t) { return t->n; }

int orc_tree_root(const orc_tree *t, uint8_t out[32]) {
    if (t->n == 0) return 0;
    memcpy(out, t->nodes + 32 * t->loff[t->nlev - 1], 32);
    return 1;
}

uint32_t orc_tree_nlevels(const orc_tree *t) { return t->nlev; }

uint64_t orc_tree_level(const orc_tree *t, uint32_t l, uint8_t *out) {
    if (l >= t->nlev) return 0;
    if (out) memcpy(out, t->nodes + 32 * t->loff[l], 32 * t->lcnt[l]);
    return t->lcnt[l];
}

void orc_tree_leaf(const orc_tree *t, uint64_t i, const uint8_t **key, uint64_t *klen, uint8_t digest[32]) {
    *key = t->kb + t->koff[i];
    *klen = t->koff[i + 1] - t->koff[i];
    if (digest) memcpy(digest, t->nodes + 32 * i, 32);
}

/* R7, merkle.rs:171-196: iterate the sorted union; push k if missing on one side or digests differ. */
uint64_t orc_tree_diff(const orc_tree *a, const orc_tree *b, uint8_t **out_kb, uint64_t **out_koff) {
    uint64_t i = 0, j = 0, cnt = 0, bytes = 0, cap = 16, bcap = 256;
    uint64_t *off = (uint64_t *)malloc((cap + 1) * sizeof(uint64_t));
    uint8_t *kb = (uint8_t *)malloc(bcap);
    off[0] = 0;
    while (i < a->n || j < b->n) {
        const uint8_t *k;
        uint64_t l;
        int push;
        if (j >= b->n) {
            k = a->kb + a->koff[i]; l = a->koff[i + 1] - a->koff[i]; push = 1; ++i;
        } else if (i >= a->n) {
            k = b->kb + b->koff[j]; l = b->koff[j + 1] - b->koff[j]; push = 1; ++j;
        } else {
            const uint8_t *ka = a->kb + a->koff[i], *kb2 = b->kb + b->koff[j];
            uint64_t la = a->koff[i + 1] - a->koff[i], lb = b->koff[j + 1] - b->koff[j];
            int c = key_cmp(ka, la, kb2, lb);
            if (c < 0) { k = ka; l = la; push = 1; ++i; }
            else if (c > 0) { k = kb2; l = lb; push = 1; ++j; }
            else {
                k = ka; l = la;
                push = memcmp(a->nodes + 32 * i, b->nodes + 32 * j, 32) != 0;
                ++i; ++j;
            }
        }
        if (!push) continue;
        if (cnt == cap) { cap *= 2; off = (uint64_t *)realloc(off, (cap + 1) * sizeof(uint64_t)); }
        while (bytes + l > bcap) { bcap *= 2; kb = (uint8_t *)realloc(kb, bcap); }
        memcpy(kb + bytes, k, l);
        bytes += l;
        off[++cnt] = bytes;
    }
    *out_kb = kb;
    *out_koff = off;
    return cnt;
}

/* HASH <prefix> (server.rs:647-685): a fresh tree over the leaves whose key starts with prefix.
 * The prefix set is contiguous in sorted order; its leaf digests are reused. */
int orc_tree_prefix_root(const orc_tree *t, const uint8_t *prefix, uint64_t plen, uint8_t out[32]) {
    uint64_t lo = t->n, hi = 0;
    for (uint64_t i = 0; i < t->n; ++i) {
        uint64_t l = t->koff[i + 1] - t->koff[i];
        if (l >= plen && (plen == 0 || memcmp(t->kb + t->koff[i], prefix, plen) == 0)) {
            if (i < lo) lo = i;
            hi = i + 1;
        }
    }
    if (lo >= hi) return 0;
    uint64_t s = hi - lo;
    uint8_t *cur = (uint8_t *)malloc(32 * s);
    memcpy(cur, t->nodes + 32 * lo, 32 * s);
    while (s > 1) {
        uint64_t p = (s + 1) / 2;
        for (uint64_t j = 0; j < p; ++j) {
            if (2 * j + 1 < s) orc_node_digest(cur + 64 * j, cur + 64 * j + 32, cur + 32 * j);
            else memmove(cur + 32 * j, cur + 64 * j, 32);
        }
        s = p;
    }
    memcpy(out, cur, 32);
    free(cur);
    return 1;
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------------------------------------
 * Synthetic generator: deterministic splitmix64 stream keyed by (seed, idx, field, j).
 * ------------------------------------------------------------------------------------------------ */
static const char SORTED_ALPHA[65] = "-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz";

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t orc_gen_word(uint64_t seed, uint64_t idx, uint32_t field, uint32_t j) {
    return mix64(seed + 0x9E3779B97F4A7C15ULL * (((idx << 12) | ((uint64_t)field << 6) | j) + 1));
}

static void gen_chars(uint64_t seed, uint64_t idx, uint32_t field, uint32_t len, uint32_t shard, uint32_t nshards,
                      uint8_t *out) {
    uint64_t w = 0;
    for (uint32_t c = 0; c < len; ++c) {
        if (c % 10 == 0) w = orc_gen_word(seed, idx, field, c / 10);
        uint32_t x = (uint32_t)(w >> (6 * (c % 10))) & 63;
        if (c == 0 && field == 0 && nshards > 1) {
            const uint32_t lo = shard * 64 / nshards, hi = (shard + 1) * 64 / nshards;
            x = lo + x % (hi - lo);
        }
        out[c] = (uint8_t)SORTED_ALPHA[x];
    }
}

void orc_gen_records(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, int ragged,
                     uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb,
                     uint64_t *voff) {
    uint64_t ko = 0, vo = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t idx = idx0 + i;
        uint32_t kl = klen, vl = vlen;
        if (ragged == 1) {
            kl = 1 + (uint32_t)(orc_gen_word(seed, idx, 62, 0) % klen);
            vl = (uint32_t)(orc_gen_word(seed, idx, 62, 1) % (vlen + 1));
        } else if (ragged == 2) {  /* "store-like" ragged: keys [klen/8, klen], values [vlen/16, vlen] */
            const uint32_t kmin = klen / 8 ? klen / 8 : 1, vmin = vlen / 16;
            kl = kmin + (uint32_t)(orc_gen_word(seed, idx, 62, 0) % (klen - kmin + 1));
            vl = vmin + (uint32_t)(orc_gen_word(seed, idx, 62, 1) % (vlen - vmin + 1));
        }
        koff[i] = ko;
        voff[i] = vo;
        gen_chars(seed, idx, 0, kl, shard, nshards, kb + ko);
        gen_chars(seed, idx, vfield, vl, 0, 1, vb + vo);
        ko += kl;
        vo += vl;
    }
    koff[n] = ko;
    voff[n] = vo;
}

/* ------------------------------------------------------------------------------------------------
 * Timed CPU baseline (bench.py cpu_baseline): one bulk build = one rebuild() over n records.
 * ------------------------------------------------------------------------------------------------ */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double orc_bench_build(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t root_out[32]) {
    double t0 = now_s();
    orc_tree *t = orc_tree_build(kb, koff, vb, voff, n);
    double t1 = now_s();
    if (!orc_tree_root(t, root_out)) memset(root_out, 0, 32);
    orc_tree_free(t);
    return t1 - t0;
}

double orc_bench_leaf_hash(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                           uint64_t n, uint8_t *digests_out) {
    double t0 = now_s();
    for (uint64_t i = 0; i < n; ++i)
        orc_leaf_digest(kb + koff[i], koff[i + 1] - koff[i], vb + voff[i], voff[i + 1] - voff[i],
                        digests_out + 32 * i);
    return now_s() - t0;
}
