// k_update.hip — incremental anti-entropy update: dirty-path rehash of a value-only batch
// (BASELINE configs[4]).
//
// The reference re-sorts and re-hashes the whole tree after every insert (merkle.rs:52-56 -> :73-121).
// When every key of an upsert batch is already a leaf, the key order and the level shapes are unchanged
// (R3/R5 depend only on the key set), so only the leaves whose digests change and their ancestors need
// hashing: per level at most min(m, S_l) nodes instead of S_l.
//
//   k_locate        batch key -> sorted leaf position (binary search on the u64 prefixes, full-key
//                   compare inside equal-prefix runs); counts keys that are not leaves (caller falls
//                   back to the batch merge for those batches).
//   (radix sort of (tree << pbits | position, batch index); stable, so the last write of a key is the
//   last of its run)
//   k_dirty_climb   ONE launch for the whole climb of every replica (round 5): a lane per changed leaf
//                   writes the new leaf digest and climbs with the node's digest in registers, reading
//                   only clean siblings from HBM; where both children are dirty the two lanes meet on the
//                   parent's bit (write-through stores + an agent-scope fetch_or: the second arriver goes
//                   on). Parents outside the shard's owned range (sharded trees) stop the
//                   climb: their seam is recomputed by the fringe all-gather + mkv_shard_combine exactly as
//                   after a full build. The rendezvous bitmap is all-zero again when the launch ends.

#include "common.hpp"
#include "dev_util.hpp"
#include "kernels.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

__device__ __forceinline__ const uint8_t *tree_key(const DiffSide &T, uint64_t i, uint64_t *len) {
    const uint32_t o = T.perm[i];
    if (T.klen) {  // fixed-length keys: arithmetic offsets (koff[0] is one uniform read)
        *len = T.klen;
        return T.kb + T.koff[0] + (uint64_t)o * T.klen;
    }
    const uint64_t a = T.koff[o];
    *len = T.koff[o + 1] - a;
    return T.kb + a;
}

__device__ __forceinline__ uint64_t locate_run(const uint8_t *k, uint64_t len, uint64_t c0, const DiffSide &T,
                                               uint64_t lo);
constexpr int LOCATE_ILP = 2;  // batch keys per lane in k_locate / k_locate_multi
#ifndef MKV_LOCATE_BLOCKS
#define MKV_LOCATE_BLOCKS 128
#endif
constexpr uint64_t LOCATE_MAX_BLOCKS = MKV_LOCATE_BLOCKS;  // per tree (k_locate_multi grid.x)

// Sorted positions of K batch keys in tree T (found[j] = UINT64_MAX when key j is not a leaf), K keys per
// lane. ps[j] = T.pfx[LOC_STRIDE * j] (ns samples, a 1/64 copy that stays in the MALL / L2): the lower
// bound is first narrowed on the samples to a window of LOC_STRIDE prefixes (one or two HBM lines)
// instead of ~log2(n / LOC_STRIDE) random HBM reads into the full prefix array. Both lower bounds take
// the branchless fixed-trip form, so the K dependent load chains advance together (K misses in flight
// per lane instead of one), and the common single-candidate tail (one leaf holds the prefix) is
// straight-line loads; longer equal-prefix runs take locate_run.
template <int K>
__device__ __forceinline__ void locate_k(const uint8_t *const kp[K], const uint64_t len[K], const bool v[K],
                                         const DiffSide &T, const uint64_t *__restrict__ ps, uint64_t ns,
                                         uint64_t found[K]) {
    uint64_t c0[K], lo[K], w[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        c0[j] = v[j] ? key_chunk(kp[j], len[j], 0) : 0;
        lo[j] = 0;
    }
    if (ns) {  // first sample >= c0
        uint64_t n = ns;
        while (n > 1) {
            const uint64_t half = n >> 1;
#pragma unroll
            for (int j = 0; j < K; ++j) lo[j] = ps[lo[j] + half] < c0[j] ? lo[j] + half : lo[j];
            n -= half;
        }
#pragma unroll
        for (int j = 0; j < K; ++j) lo[j] += ps[lo[j]] < c0[j] ? 1 : 0;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {  // window of at most LOC_STRIDE prefixes
        const uint64_t j0 = lo[j];
        const uint64_t a = j0 ? (j0 - 1) * LOC_STRIDE + 1 : 0;
        const uint64_t b = j0 * LOC_STRIDE < T.n ? j0 * LOC_STRIDE : T.n;
        lo[j] = a;
        w[j] = b > a ? b - a : 0;
    }
    static_assert(LOC_STRIDE <= 64, "window search unrolled for <= 64 prefixes");
#pragma unroll
    for (int it = 0; it < 6; ++it) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (w[j] > 1) {
                const uint64_t half = w[j] >> 1;
                lo[j] = T.pfx[lo[j] + half] < c0[j] ? lo[j] + half : lo[j];
                w[j] -= half;
            }
    }
    bool hit[K], run[K];
    uint32_t o[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (w[j] == 1) lo[j] += T.pfx[lo[j]] < c0[j] ? 1 : 0;
        hit[j] = v[j] && lo[j] < T.n && T.pfx[lo[j]] == c0[j];
        run[j] = hit[j] && lo[j] + 1 < T.n && T.pfx[lo[j] + 1] == c0[j];
        o[j] = hit[j] && !run[j] ? T.perm[lo[j]] : 0;
    }
    uint64_t ka[K], kl[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (T.klen) {
            ka[j] = T.koff[0] + (uint64_t)o[j] * T.klen;
            kl[j] = T.klen;
        } else {
            ka[j] = hit[j] && !run[j] ? T.koff[o[j]] : 0;
            kl[j] = hit[j] && !run[j] ? T.koff[o[j] + 1] - ka[j] : 0;
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (!hit[j]) found[j] = UINT64_MAX;
        else if (run[j]) found[j] = locate_run(kp[j], len[j], c0[j], T, lo[j]);
        else found[j] = key_cmp(kp[j], len[j], c0[j], T.kb + ka[j], kl[j], c0[j]) == 0 ? lo[j] : UINT64_MAX;
    }
}

// Equal-prefix run starting at lo (T.pfx[lo] == c0): the sorted position of key k, UINT64_MAX if absent.
__device__ __forceinline__ uint64_t locate_run(const uint8_t *k, uint64_t len, uint64_t c0, const DiffSide &T,
                                               uint64_t lo) {
    uint64_t found = UINT64_MAX;
    {
        // Equal-prefix run [lo, e): keys sharing >= 8 leading bytes ("tenant/0001/obj/...") can make
        // it the whole tree, so it is binary-searched on the full key (lower_bound with key_cmp),
        // never walked: O(log n) full-key compares per batch key.
        uint64_t e = lo + 1;
        if (e < T.n && T.pfx[e] == c0) {
            uint64_t a = e, b = T.n;  // first position with pfx > c0
            while (a < b) {
                const uint64_t mid = (a + b) >> 1;
                if (T.pfx[mid] <= c0) a = mid + 1;
                else b = mid;
            }
            e = a;
        }
        uint64_t a = lo, b = e;
        while (a < b) {
            const uint64_t mid = (a + b) >> 1;
            uint64_t tl;
            const uint8_t *tk = tree_key(T, mid, &tl);
            if (key_cmp(tk, tl, c0, k, len, c0) < 0) a = mid + 1;
            else b = mid;
        }
        if (a < e) {
            uint64_t tl;
            const uint8_t *tk = tree_key(T, a, &tl);
            if (key_cmp(k, len, c0, tk, tl, c0) == 0) found = a;
        }
    }
    return found;
}

__global__ __launch_bounds__(256) void k_locate(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                uint64_t m, DiffSide T, const uint64_t *__restrict__ ps, uint64_t ns,
                                                uint64_t *__restrict__ pos, uint32_t *__restrict__ idx,
                                                uint32_t *__restrict__ missing) {
    const uint64_t i0 = (uint64_t)blockIdx.x * (LOCATE_ILP * blockDim.x) + threadIdx.x;
    const uint8_t *kp[LOCATE_ILP];
    uint64_t len[LOCATE_ILP], found[LOCATE_ILP];
    bool v[LOCATE_ILP];
#pragma unroll
    for (int j = 0; j < LOCATE_ILP; ++j) {
        const uint64_t i = i0 + (uint64_t)j * blockDim.x;
        v[j] = i < m;
        const uint64_t a = v[j] ? koff[i] : 0;
        kp[j] = kb + a;
        len[j] = v[j] ? koff[i + 1] - a : 0;
    }
    locate_k<LOCATE_ILP>(kp, len, v, T, ps, ns, found);
    uint32_t nmiss = 0;
#pragma unroll
    for (int j = 0; j < LOCATE_ILP; ++j) {
        const uint64_t i = i0 + (uint64_t)j * blockDim.x;
        const bool miss = v[j] && found[j] == UINT64_MAX;
        if (v[j]) {
            pos[i] = found[j];
            idx[i] = (uint32_t)i;
        }
        nmiss += (uint32_t)__popcll(__ballot(miss));
    }
    if ((threadIdx.x & 63) == 0 && nmiss) atomicAdd(missing, nmiss);
}

// ---- hash index (round 5): batch key -> sorted position in ~1.5 table probes + one full-key check ----
// The sample search above costs ~20 fabric requests per key at 125M leaves (PMC: 17M TCC_EA0_RDREQ for
// 875K keys, 0.34 ms): ~11 sample probes beyond L2 plus the prefix window and the key check. The index
// is keyed by a hash of the whole key, so keys sharing long prefixes spread like any others; a found
// entry is always confirmed on the tree's own key bytes, so a tag collision can never locate the wrong
// leaf, and a key that is not a leaf meets an empty slot (or the probe bound: then it counts as missing
// and the batch takes the exact merge path).
__device__ __forceinline__ uint64_t hix_mix(uint64_t z) {
    z ^= z >> 31;
    z *= 0x7FB5D329728EA185ull;
    z ^= z >> 27;
    z *= 0x81DADEF4BC2DD44Dull;
    z ^= z >> 33;
    return z;
}
__device__ __forceinline__ uint64_t hix_hash(const uint8_t *k, uint64_t len, uint64_t c0) {
    uint64_t h = hix_mix(c0 ^ (len * 0x9E3779B97F4A7C15ull));
    for (uint64_t off = 8; off < len; off += 8) h = hix_mix(h ^ key_chunk(k, len, off));
    return h;
}
constexpr uint32_t HIX_MAX_PROBES = 4096;

__global__ __launch_bounds__(256) void k_hix_build(DiffSide T, unsigned long long *__restrict__ tab, uint64_t mask) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t len;
        const uint8_t *k = tree_key(T, i, &len);
        const uint64_t h = hix_hash(k, len, key_chunk(k, len, 0));
        const unsigned long long e = ((h >> 32) | 1ull) << 32 | i;
        uint64_t s = h & mask;
        for (uint32_t q = 0; q <= mask; ++q) {  // the table has >= 2n slots: an empty one is always found
            if (atomicCAS(&tab[s], 0ull, e) == 0ull) break;
            s = (s + 1) & mask;
        }
    }
}

template <int K>
__device__ __forceinline__ void locate_hix(const uint8_t *const kp[K], const uint64_t len[K], const bool v[K],
                                           const DiffSide &T, const uint64_t *__restrict__ tab, uint64_t mask,
                                           uint64_t found[K]) {
    uint64_t c0[K], slot[K], tag[K];
    bool live[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        c0[j] = v[j] ? key_chunk(kp[j], len[j], 0) : 0;
        const uint64_t h = v[j] ? hix_hash(kp[j], len[j], c0[j]) : 0;
        slot[j] = h & mask;
        tag[j] = (h >> 32) | 1ull;
        live[j] = v[j];
        found[j] = UINT64_MAX;
    }
    for (uint32_t q = 0; q < HIX_MAX_PROBES; ++q) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < K; ++j) any |= live[j];
        if (!any) break;
        uint64_t e[K];
#pragma unroll
        for (int j = 0; j < K; ++j) e[j] = live[j] ? tab[slot[j]] : 0;  // the K probes in flight together
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (!live[j]) continue;
            if (e[j] == 0) {  // empty slot: not a leaf
                live[j] = false;
                continue;
            }
            if ((e[j] >> 32) == tag[j]) {  // a 32-bit tag match: confirm on the tree's key bytes (no
                const uint64_t p = e[j] & 0xFFFFFFFFull;  // prefix pre-check: one dependent read fewer)
                uint64_t tl;
                const uint8_t *tk = tree_key(T, p, &tl);
                if (tl == len[j] && key_cmp(kp[j], len[j], c0[j], tk, tl, key_chunk(tk, tl, 0)) == 0) {
                    found[j] = p;
                    live[j] = false;
                    continue;
                }
            }
            slot[j] = (slot[j] + 1) & mask;
        }
    }
}

__global__ __launch_bounds__(256) void k_locate_multi(LeafBatches B, LocateMulti L, int pbits,
                                                      uint64_t *__restrict__ pos, uint32_t *__restrict__ idx) {
    const uint32_t t = blockIdx.y;
    const uint64_t m = B.m[t];
    uint32_t nmiss = 0;
    for (uint64_t i0 = (uint64_t)blockIdx.x * (LOCATE_ILP * blockDim.x) + threadIdx.x; i0 < m;
         i0 += (uint64_t)gridDim.x * (LOCATE_ILP * blockDim.x)) {
    const uint8_t *kp[LOCATE_ILP];
    uint64_t len[LOCATE_ILP], found[LOCATE_ILP];
    bool v[LOCATE_ILP];
#pragma unroll
    for (int j = 0; j < LOCATE_ILP; ++j) {
        const uint64_t i = i0 + (uint64_t)j * blockDim.x;
        v[j] = i < m;
        const uint64_t a = v[j] ? B.koff[t][i] : 0;
        kp[j] = B.kb[t] + a;
        len[j] = v[j] ? B.koff[t][i + 1] - a : 0;
    }
    if (L.hix[t]) locate_hix<LOCATE_ILP>(kp, len, v, L.T[t], L.hix[t], L.hmask[t], found);  // uniform per tree
    else locate_k<LOCATE_ILP>(kp, len, v, L.T[t], L.ps[t], L.ns[t], found);
#pragma unroll
    for (int j = 0; j < LOCATE_ILP; ++j) {
        const uint64_t i = i0 + (uint64_t)j * blockDim.x;
        const bool miss = v[j] && found[j] == UINT64_MAX;
        if (v[j]) {
            const uint64_t g = B.base[t] + i;
            pos[g] = ((uint64_t)t << pbits) | (miss ? (1ull << pbits) - 1ull : found[j]);
            idx[g] = (uint32_t)g;
        }
        nmiss += (uint32_t)__popcll(__ballot(miss));
    }
    }
    if ((threadIdx.x & 63) == 0 && nmiss) atomicAdd(L.missing[t], nmiss);
}

// ---------------------------------------------------------------------------------------------------
// k_dirty_climb (round 5): the sparse part of the dirty-path rehash of k replicas, one wave per batch of 64
// consecutive entries, climbing level-synchronously with the batch's dirty nodes compacted in the wave's
// lanes; the dense part above it is the ordinary reduction (see the end of this comment).
//
// Entries: the batch positions sorted by (tree << pbits | leaf) — a run of equal keys is one leaf written
// several times; its LAST entry is the last write (merkle.rs:54). Lane k of a wave holds the batch's k-th
// dirty node (l, x) in key order: tree, the index range [lo, hi] of the entries under it with the
// neighbouring entries pn = key[hi + 1], pp = key[lo - 1], its digest and its sibling's digest read one
// level ahead, kept in the wave's LDS slots between levels (round 6: read whole at the top of a level, so
// no register state crosses the level's branches) together with the node's class, computed with that
// read-ahead. Per level (classify):
//   * parent not owned (root, or a shard's seam): store the digest, done;
//   * x is an odd level's last node: store it, the parent is the digest unchanged (R5 promotion);
//   * sibling clean (no entry inside its leaf range: one compare of pn or pp): store the digest, parent =
//     SHA-256(left || right) (R4) with the sibling's 32 B, read one level ahead (it lands while the
//     previous level hashes): 32 B read + 32 B written per rehashed node, the dirty child is never re-read;
//   * sibling dirty and held by lane k +/- 1 (the entries are sorted, so a dirty sibling's entries are the
//     neighbouring lane's): the left lane stores and stops, the right one hashes the parent with the left
//     lane's digest slots — no memory round trip, no barrier;
//   * sibling dirty beyond the batch (first / last lane only): a rendezvous with the other wave through a
//     mailbox per entry boundary — both sides publish {digest, outer entry bound, its neighbour}
//     write-through (sc1), drain, then fetch_or the boundary's bit at agent scope; the first arriver stops,
//     the second clears the bit, reads the other side with sc1 loads (the hand-off form of
//     MI355X_MICROARCH.md: sc1 payload -> vmcnt(0) -> atomic; consumer: returned atomic -> sc1 loads) and
//     goes on (the partner's digest goes into its own sibling slots). The bits are all-zero again when the
//     launch ends.
// After each level the survivors are compacted into the low slots (lane k of the next level = slot k). A wave's
// lanes thin out as its batch merges, so the climb stops at level `lstop`, the first level whose nodes span
// the mean gap between dirty leaves (about half of its nodes are dirty): it stores its dirty nodes there,
// and every level above is rehashed whole by the build's reduction kernels (run_reduce from lstop, all k
// trees in one launch per step, full waves, a few % more hashes than the dirty ones). Round 5 measured the
// alternative — more climb passes over the survivors packed across waves — at 0.47 ms for the levels above
// lstop of configs[4]; the waves still thinned out within each pass. Per-level dirty counts
// (mkv_tree_update_counts) are kept in LDS and added to the trees' counters once per workgroup.
// ---------------------------------------------------------------------------------------------------
constexpr int CW_THREADS = 256;  // four independent waves
// Launch cap: 2,048 workgroups (two per resident slot at 4 waves per SIMD), so a wave whose batches merge
// early leaves its slot to a later workgroup instead of taking a fixed share of a grid-stride loop (round 6,
// configs[4] climb: 1,024 resident workgroups 0.78 ms, 2,048 0.75-0.76, one batch per wave 0.75-0.75; 5 waves
// per SIMD, 95 VGPRs since the level state moved to LDS: 0.75-0.77. Round 5 with the register-carried
// state: 3 waves 0.82-0.84, 4 waves 0.81, 5 spilled).
constexpr uint32_t CW_MAX_BLOCKS = 2048;

// Tree node arrays are addressed through GLOBAL-address-space pointers: a pointer read back from LDS is a
// generic (flat) pointer, and a flat load also counts in lgkmcnt — every LDS wait of the level would then
// wait for the sibling read issued one level ahead, serialising what the read-ahead overlaps.
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) u4v g_u4v;
__device__ __forceinline__ g_u8 *gptr(uint64_t a) { return (g_u8 *)a; }
__device__ __forceinline__ void g_load_raw(const g_u8 *p, uint4 &a, uint4 &b) {
    const g_u4v *q = (const g_u4v *)p;
    const u4v x = q[0], y = q[1];
    a = make_uint4(x.x, x.y, x.z, x.w);
    b = make_uint4(y.x, y.y, y.z, y.w);
}
__device__ __forceinline__ void g_store_digest(g_u8 *p, const uint32_t w[8]) {
    g_u4v *q = (g_u4v *)p;
    q[0] = u4v{bswap32(w[0]), bswap32(w[1]), bswap32(w[2]), bswap32(w[3])};
    q[1] = u4v{bswap32(w[4]), bswap32(w[5]), bswap32(w[6]), bswap32(w[7])};
}
__device__ __forceinline__ void load_raw(const uint8_t *p, uint4 &a, uint4 &b) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    a = q[0];
    b = q[1];
}
__device__ __forceinline__ void raw_to_words(const uint4 &a, const uint4 &b, uint32_t w[8]) {
    w[0] = bswap32(a.x); w[1] = bswap32(a.y); w[2] = bswap32(a.z); w[3] = bswap32(a.w);
    w[4] = bswap32(b.x); w[5] = bswap32(b.y); w[6] = bswap32(b.z); w[7] = bswap32(b.w);
}

struct ClimbPlan {
    const uint64_t *base, *cnt, *off, *S;
    int L;
    uint64_t goff, N;
    int pbits;
};
enum : int { CL_TOP = 0, CL_PROMO = 1, CL_CLEAN = 2, CL_DIRTY = 3 };
// What node (l, x) of tree t does at this level; sib = its sibling's node slot (the dirty test compares
// the neighbouring entries with the sibling's leaf range).
__device__ __forceinline__ int classify(const ClimbPlan &P, uint32_t t, int l, uint64_t x, uint64_t pn, uint64_t pp1,
                                        uint64_t *sib) {
    const uint64_t qg = x >> 1;
    if (l + 1 >= P.L || !(qg >= P.base[l + 1] && qg < P.base[l + 1] + P.cnt[l + 1])) return CL_TOP;
    if (!(x & 1) && x + 1 >= P.S[l]) return CL_PROMO;
    const uint64_t tb = (uint64_t)t << P.pbits;
    *sib = P.off[l] + ((x ^ 1) - P.base[l]);
    if (!(x & 1)) {  // right sibling covers leaves [(x+1) << l, min((x+2) << l, N))
        const uint64_t e = ((x + 2) << l) < P.N ? ((x + 2) << l) : P.N;
        return pn < tb + (e - P.goff) ? CL_DIRTY : CL_CLEAN;
    }
    return pp1 > tb + (((x - 1) << l) - P.goff) ? CL_DIRTY : CL_CLEAN;  // left sibling: [(x-1) << l, x << l)
}

// Mailbox of entry boundary b (between entries b-1 and b): side 0 = the left subtree's {digest, lo, pp1},
// side 1 = the right subtree's {digest, hi, pn}; 8-B words, written with sc1 atomic stores.
constexpr uint64_t MBOX_SIDE_WORDS = 6, MBOX_WORDS = 2 * MBOX_SIDE_WORDS;

__global__ __launch_bounds__(CW_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_dirty_climb(ClimbArgs A) {
    __shared__ uint32_t s_lc[DIRTY_MAX_TREES * MKV_MAXLEV];
    __shared__ uint64_t s_nodes[DIRTY_MAX_TREES];  // addresses: used as global pointers (gptr)
    __shared__ uint32_t s_done;
    // per wave: the batch's dirty nodes in key order (slot k = dirty node k), rewritten every level
    __shared__ uint64_t s_qx[CW_THREADS / 64][64], s_qpn[CW_THREADS / 64][64], s_qpp[CW_THREADS / 64][64];
    __shared__ uint32_t s_qlo[CW_THREADS / 64][64], s_qhi[CW_THREADS / 64][64], s_qt[CW_THREADS / 64][64];
    __shared__ uint32_t s_qd[CW_THREADS / 64][8][64], s_qs[CW_THREADS / 64][8][64];
    const int L = A.P.L;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint64_t *q_x = s_qx[wv], *q_pn = s_qpn[wv], *q_pp = s_qpp[wv];
    uint32_t *q_lo = s_qlo[wv], *q_hi = s_qhi[wv], *q_t = s_qt[wv];
    uint32_t(*q_d)[64] = s_qd[wv];
    uint32_t(*q_s)[64] = s_qs[wv];
    __shared__ uint64_t s_base[MKV_MAXLEV], s_cnt[MKV_MAXLEV], s_off[MKV_MAXLEV], s_S[MKV_MAXLEV];
    for (int i = tid; i < L; i += CW_THREADS) {
        s_base[i] = A.P.base[i];
        s_cnt[i] = A.P.cnt[i];
        s_off[i] = A.P.off[i];
        s_S[i] = A.P.S[i];
    }
    for (uint32_t i = tid; i < A.k * (uint32_t)L; i += CW_THREADS) s_lc[i] = 0;
    __shared__ uint32_t s_miss[DIRTY_MAX_TREES];
    __shared__ uint32_t *s_cntp[DIRTY_MAX_TREES];
    if (tid < A.k) {
        s_nodes[tid] = reinterpret_cast<uint64_t>(A.nodes[tid]);
        s_miss[tid] = *A.missing[tid];
        s_cntp[tid] = A.cnt[tid];
    }
    if (tid == 0) s_done = 0;
    if (blockIdx.x == 0 && tid < A.k && A.ztab) A.ztab[tid] = (uint64_t)(A.nodes[tid] - A.nodes[0]);
    __syncthreads();  // the only barrier: the waves work on their own batches from here on
    const ClimbPlan P{s_base, s_cnt, s_off, s_S, L, s_base[0], s_S[0], A.pbits};
    const uint64_t pmask = (1ull << A.pbits) - 1ull;
    const uint32_t n = A.M;
    const uint64_t *__restrict__ keys = A.pos;
    const uint32_t nb_cap = (n + 63) / 64, nwaves = gridDim.x * (CW_THREADS / 64);
    // Survivor k -> slot k (key order kept): the level's state lives in the wave's LDS slots, read back
    // whole at the top of every level. No per-lane state crosses a level in registers, so the level body
    // needs no register copies to merge its branches (round 6: ~80 v_mov per level before).
    auto compact = [&](bool sv, uint32_t t_, int cls_, uint64_t x_, uint64_t pn_, uint64_t pp_, uint32_t lo_,
                       uint32_t hi_, const uint32_t *d_, const uint4 &a_, const uint4 &b_) -> uint32_t {
        const uint64_t m = __ballot(sv);
        if (sv) {
            const uint32_t k = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            q_x[k] = x_;
            q_pn[k] = pn_;
            q_pp[k] = pp_;
            q_lo[k] = lo_;
            q_hi[k] = hi_;
            q_t[k] = t_ | ((uint32_t)cls_ << 30);
#pragma unroll
            for (int i = 0; i < 8; ++i) q_d[i][k] = d_[i];
            uint32_t w[8];
            raw_to_words(a_, b_, w);
#pragma unroll
            for (int i = 0; i < 8; ++i) q_s[i][k] = w[i];
        }
        return (uint32_t)__popcll(m);
    };
    for (uint32_t bt = blockIdx.x * (CW_THREADS / 64) + (tid >> 6); bt < nb_cap; bt += nwaves) {
        // ---- the batch's entries: the last write of each key starts a climb ----
        uint32_t c;
        int l = 0;
        {
            const uint32_t s = bt * 64 + lane;
            bool surv = false;
            uint32_t t = 0, lo = 0, hi = 0;
            int cls = CL_TOP;
            uint64_t x = 0, pn = 0, pp1 = 0;
            uint32_t d[8];
            uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0;
            if (s < n) {
                const uint64_t key = keys[s];
                t = (uint32_t)(key >> A.pbits);
                if ((s + 1 == n || keys[s + 1] != key) && t < A.k && s_miss[t] == 0) {
                    // earlier writes of the same key: the run's start by galloping back, then a binary search
                    // (a serial walk was O(run length) dependent loads on one lane: a hot key written 1e5 times
                    // stalled its wave and with it the whole climb launch)
                    lo = s;
                    uint32_t step = 1;
                    while (lo >= step && keys[lo - step] == key) {
                        lo -= step;
                        step <<= 1;
                    }
                    uint32_t a = lo >= step ? lo - step + 1 : 0;  // keys[a - 1] != key (or a == 0); keys[lo] == key
                    while (a < lo) {
                        const uint32_t mid = (a + lo) >> 1;
                        if (keys[mid] == key) lo = mid;
                        else a = mid + 1;
                    }
                    load_digest(A.bdig + 32ull * A.bidx[s], d);
                    surv = true;
                }
                if (surv) {
                    hi = s;
                    pn = s + 1 < n ? keys[s + 1] : ~0ull;
                    pp1 = lo > 0 ? keys[lo - 1] + 1 : 0;
                    x = P.goff + (key & pmask);
                    uint64_t sib = 0;
                    cls = classify(P, t, 0, x, pn, pp1, &sib);
                    if (cls == CL_CLEAN) g_load_raw(gptr(s_nodes[t]) + 32 * sib, n0, n1);
                }
            }
            c = compact(surv, t, cls, x, pn, pp1, lo, hi, d, n0, n1);
        }
        for (; c != 0; ++l) {
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            // ---- this level: lane k holds dirty node k (slots >= c are stale; every use is under act) ----
            const bool act = lane < c;
            uint64_t x = q_x[lane], pn = q_pn[lane], pp1 = q_pp[lane];
            uint32_t lo = q_lo[lane], hi = q_hi[lane];
            const uint32_t tq = q_t[lane];
            const uint32_t t = tq & 0x3FFFFFFFu;
            int cls = (int)(tq >> 30);  // classified one level ahead (with the sibling read)
            uint32_t d[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) d[i] = q_d[i][lane];
            g_u8 *const nodes = gptr(s_nodes[act ? t : 0]);
            if (l == A.lstop) {  // dense from here: the reduction rehashes the levels above whole
                if (act) {
                    g_store_digest(nodes + 32 * (P.off[l] + (x - P.base[l])), d);
                    atomicAdd(&s_lc[t * L + l], 1u);
                }
                break;
            }
            bool surv = false, hash = false;
            // the sibling's words for the hash: slots q_s of this lane (clean sibling read one level ahead,
            // or a rendezvous partner's digest) or the digest slots of lane - 1 (dirty sibling in the wave);
            // one read path, so no sibling registers are carried between branches or levels
            const uint32_t *sp = &q_s[0][lane];
            g_u8 *ra = nodes;  // the next level's read: the parent's sibling when it is clean, else any valid line
            if (act) {
                g_u8 *np = nodes + 32 * (P.off[l] + (x - P.base[l]));
                atomicAdd(&s_lc[t * L + l], 1u);  // node (l, x) is dirty: stored in every case
                g_store_digest(np, d);
                if (cls == CL_TOP) {
                    // parent not owned: done
                } else if (cls == CL_PROMO) {
                    surv = true;
                } else if (cls == CL_CLEAN) {  // the sibling was read one level ahead (slots q_s)
                    hash = surv = true;
                } else if ((x & 1) && lane > 0) {  // right sibling of lane - 1, which stops: merge here
                    sp = &q_d[0][lane - 1];
                    lo = q_lo[lane - 1];
                    pp1 = q_pp[lane - 1];
                    hash = surv = true;
                } else if (!(x & 1) && lane + 1 < c) {
                    // left sibling of lane + 1, which goes on
                } else {
                    // the sibling's entries belong to another batch: rendezvous at entry boundary b
                    const bool right = x & 1;
                    const uint64_t b = right ? lo : (uint64_t)hi + 1;
                    uint64_t *mb = reinterpret_cast<uint64_t *>(A.mbox) + b * MBOX_WORDS;
                    uint64_t *mine = mb + (right ? MBOX_SIDE_WORDS : 0), *other = mb + (right ? 0 : MBOX_SIDE_WORDS);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        __hip_atomic_store(mine + i, ((uint64_t)d[2 * i + 1] << 32) | d[2 * i], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(mine + 4, right ? (uint64_t)hi : (uint64_t)lo, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(mine + 5, right ? pn : pp1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    // The hand-off form of MI355X_MICROARCH.md (valid forms, hand-off table row 1): the one lane
                    // that stored its payload with agent-scope (sc1, write-through) atomic stores drains them, then
                    // signals with an agent-scope atomic; the consumer is the lane told by its atomic's return
                    // value and reads the payload with sc1 (agent atomic) loads. gfx950 / ROCm 7.2 behaviour, not
                    // the C++ model's release/acquire: an ACQ_REL fetch_or (buffer_wbl2 sc1 + buffer_inv sc1 per
                    // merge) measured climb 0.81 -> 1.42 ms at configs[4] (round 6).
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    uint32_t *bw = A.bflags + (b >> 5);
                    const uint32_t bit = 1u << (b & 31);
                    const uint32_t old = __hip_atomic_fetch_or(bw, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (old & bit) {  // second arriver: the other side's data is complete
                        __hip_atomic_fetch_and(bw, ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the atomic
#pragma unroll
                        for (int i = 0; i < 4; ++i) {  // into this lane's own sibling slots (sp)
                            const uint64_t v = __hip_atomic_load(other + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            q_s[2 * i][lane] = (uint32_t)v;
                            q_s[2 * i + 1][lane] = (uint32_t)(v >> 32);
                        }
                        const uint64_t oi = __hip_atomic_load(other + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint64_t ok = __hip_atomic_load(other + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (right) {
                            lo = (uint32_t)oi;
                            pp1 = ok;
                        } else {
                            hi = (uint32_t)oi;
                            pn = ok;
                        }
                        hash = surv = true;
                    }
                }
                // the parent's class and, when its sibling is clean, the sibling itself (below), read now: it
                // lands while this level hashes (the next level's stop needs neither)
                cls = CL_TOP;
                if (surv && l + 1 != A.lstop) {
                    uint64_t sib2 = 0;
                    cls = classify(P, t, l + 1, x >> 1, pn, pp1, &sib2);
                    if (cls == CL_CLEAN) ra = nodes + 32 * sib2;
                }
            }
            // issued by every lane (a valid line where the sibling is not clean), so no branch merges n0 / n1
            uint4 n0, n1;
            g_load_raw(ra, n0, n1);
            if (hash) {
                const bool right = x & 1;
                uint32_t lw[8], rw[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t sw = sp[64 * i];
                    lw[i] = right ? sw : d[i];
                    rw[i] = right ? d[i] : sw;
                }
                sha_node<false>(lw, rw, d);
            }
            x >>= 1;
            __builtin_amdgcn_wave_barrier();  // this level's slot reads come before the compaction's writes
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            c = compact(surv, t, cls, x, pn, pp1, lo, hi, d, n0, n1);
        }
    }
    // ---- level counts: the last wave of the workgroup adds them to the trees' counters ----
    uint32_t done = 0;
    if (lane == 0) done = atomicAdd(&s_done, 1u);
    done = __builtin_amdgcn_readfirstlane(done);
    if (done == CW_THREADS / 64 - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (uint32_t i = lane; i < A.k * (uint32_t)L; i += 64) {
            const uint32_t v = __hip_atomic_load(&s_lc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (v) atomicAdd(s_cntp[i / L] + i % L, v);
        }
    }
}

constexpr int UM_THREADS = 256, UM_ITEMS = 8, UM_TILE = UM_THREADS * UM_ITEMS;

__device__ __forceinline__ int cmp_sides(const DiffSide &A, uint64_t i, const DiffSide &B, uint64_t j) {
    const uint64_t pa = A.pfx[i], pb = B.pfx[j];
    if (pa != pb) return pa < pb ? -1 : 1;
    uint64_t la, lb;
    const uint8_t *ka = tree_key(A, i, &la), *kb = tree_key(B, j, &lb);
    return key_cmp(ka, la, pa, kb, lb, pb);
}

// Number of A elements among the first d outputs of the merge (A first on equal keys).
__device__ uint64_t um_split(const DiffSide &A, const DiffSide &B, uint64_t d, uint64_t lo, uint64_t hi) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (cmp_sides(A, mid, B, d - 1 - mid) <= 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void k_umerge_partition(DiffSide A, DiffSide B, uint64_t ntiles, uint64_t *__restrict__ split) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t M = A.n + B.n;
    const uint64_t d = t * UM_TILE < M ? t * UM_TILE : M;
    split[t] = um_split(A, B, d, d > B.n ? d - B.n : 0, d < A.n ? d : A.n);
}

struct UmLane {
    uint64_t i, j;   // cursors at the lane's first output
    uint32_t fromA, keep, cnt;
};

__device__ __forceinline__ UmLane um_lane(const DiffSide &A, const DiffSide &B, const uint8_t *tomb,
                                          const uint64_t *split) {
    UmLane r{0, 0, 0, 0, 0};
    const uint64_t M = A.n + B.n;
    const uint64_t t = blockIdx.x;
    const uint64_t d0 = t * UM_TILE + (uint64_t)threadIdx.x * UM_ITEMS;
    if (d0 >= M) return r;
    const uint64_t a0 = split[t], a1 = split[t + 1];
    const uint64_t b0 = t * UM_TILE - a0;
    const uint64_t dt1 = (t + 1) * UM_TILE < M ? (t + 1) * UM_TILE : M;
    const uint64_t b1 = dt1 - a1;
    // lane diagonal inside the tile window [a0, a1) x [b0, b1)
    const uint64_t dl = d0 - t * UM_TILE, na = a1 - a0, nb = b1 - b0;
    const uint64_t lo = dl > nb ? dl - nb : 0, hi = dl < na ? dl : na;
    uint64_t l = lo, h = hi;
    while (l < h) {
        const uint64_t mid = (l + h) >> 1;
        if (cmp_sides(A, a0 + mid, B, b0 + dl - 1 - mid) <= 0) l = mid + 1;
        else h = mid;
    }
    uint64_t i = a0 + l, j = b0 + (dl - l);
    r.i = i;
    r.j = j;
    for (int s = 0; s < UM_ITEMS; ++s) {
        if (d0 + s >= M) break;
        bool takeA;
        int c = 1;
        if (i >= A.n) takeA = false;
        else if (j >= B.n) takeA = true;
        else {
            c = cmp_sides(A, i, B, j);
            takeA = c <= 0;
        }
        bool keep;
        if (takeA) {
            keep = !(j < B.n && c == 0);  // B holds the same key: replaced or removed
            r.fromA |= 1u << s;
            ++i;
        } else {
            keep = !(tomb && tomb[B.perm[j]]);
            ++j;
        }
        if (keep) r.keep |= 1u << s;
    }
    r.cnt = (uint32_t)__popc(r.keep);
    return r;
}

__global__ __launch_bounds__(UM_THREADS) void k_umerge_count(DiffSide A, DiffSide B, const uint8_t *__restrict__ tomb,
                                                            const uint64_t *__restrict__ split,
                                                            uint64_t *__restrict__ tilecnt) {
    __shared__ uint64_t lds[16];
    const UmLane r = um_lane(A, B, tomb, split);
    uint64_t tot;
    (void)block_excl_scan<uint64_t>((uint64_t)r.cnt, lds, &tot);
    if (threadIdx.x == 0) tilecnt[blockIdx.x] = tot;
}

// Outputs: pfx_out / perm_out (storage index; batch records stored after the tree's nstore_a) and the
// new leaf level dig_out (32 B per leaf).
__global__ __launch_bounds__(UM_THREADS) void k_umerge_write(DiffSide A, DiffSide B, const uint8_t *__restrict__ tomb,
                                                            const uint64_t *__restrict__ split,
                                                            const uint64_t *__restrict__ tileoff, uint32_t nstore_a,
                                                            uint64_t *__restrict__ pfx_out,
                                                            uint32_t *__restrict__ perm_out,
                                                            uint8_t *__restrict__ dig_out) {
    __shared__ uint64_t lds[16];
    const UmLane r = um_lane(A, B, tomb, split);
    uint64_t o = block_excl_scan<uint64_t>((uint64_t)r.cnt, lds, nullptr) + tileoff[blockIdx.x];
    uint64_t i = r.i, j = r.j;
    for (int s = 0; s < UM_ITEMS; ++s) {
        const bool fa = (r.fromA >> s) & 1u;
        const bool kp = (r.keep >> s) & 1u;
        if (kp) {
            const uint4 *src;
            if (fa) {
                pfx_out[o] = A.pfx[i];
                perm_out[o] = A.perm[i];
                src = reinterpret_cast<const uint4 *>(A.dig + 32 * i);
            } else {
                const uint32_t bs = B.perm[j];
                pfx_out[o] = B.pfx[j];
                perm_out[o] = nstore_a + bs;
                src = reinterpret_cast<const uint4 *>(B.dig + 32ull * bs);
            }
            uint4 *dst = reinterpret_cast<uint4 *>(dig_out + 32 * o);
            dst[0] = src[0];
            dst[1] = src[1];
            ++o;
        }
        if (fa) ++i;
        else ++j;
    }
}

inline dim3 grid1d(uint64_t n, uint32_t bs = 256) { return dim3((uint32_t)ceil_div(n ? n : 1, bs)); }

}  // namespace

void launch_locate(const uint8_t *kb, const uint64_t *koff, uint64_t m, const DiffSide &T, const uint64_t *ps,
                   uint64_t ns, uint64_t *pos, uint32_t *idx, uint32_t *missing, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_locate, dim3((uint32_t)ceil_div(m, 256 * LOCATE_ILP)), dim3(256), 0, st, kb, koff, m, T, ps, ns,
                       pos, idx, missing);
    MKV_LAUNCH_CHECK();
}

__global__ void k_strided_u64(const uint64_t *__restrict__ src, uint64_t ns, uint64_t *__restrict__ dst) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < ns) dst[j] = src[j * LOC_STRIDE];
}
void launch_locate_samples(const uint64_t *pfx, uint64_t n, uint64_t *ps, hipStream_t st) {
    const uint64_t ns = locate_samples(n);
    if (!ns) return;
    hipLaunchKernelGGL(k_strided_u64, grid1d(ns), dim3(256), 0, st, pfx, ns, ps);
    MKV_LAUNCH_CHECK();
}

void launch_locate_multi(const LeafBatches &B, const LocateMulti &L, uint32_t k, uint64_t mmax, int pbits,
                         uint64_t *pos, uint32_t *idx, hipStream_t st) {
    if (!k || !mmax) return;
    // A bounded grid (the blocks loop over their tree's keys): the locate's waves wait on memory most of
    // the time, and a wave per 128 keys (6,860 at configs[4]) held the CUs' wave slots that the batch hash
    // running beside it needs. configs[4] step per cap (interleaved A/B): 32 blocks per tree 1.98-2.06 ms,
    // 64 1.87, 128 1.80-1.84, uncapped (245) 1.86-1.87; locate and hash serialised on one stream 1.91-1.98
    const uint32_t gx = (uint32_t)std::min<uint64_t>(ceil_div(mmax, 256 * LOCATE_ILP), LOCATE_MAX_BLOCKS);
    hipLaunchKernelGGL(k_locate_multi, dim3(gx, k), dim3(256), 0, st, B, L, pbits, pos, idx);
    MKV_LAUNCH_CHECK();
}

void launch_hix_build(const DiffSide &T, uint64_t *tab, uint64_t mask, hipStream_t st) {
    if (!T.n) return;
    hipLaunchKernelGGL(k_hix_build, dim3((uint32_t)std::min<uint64_t>(ceil_div(T.n, 256), 65536)), dim3(256), 0, st, T,
                       reinterpret_cast<unsigned long long *>(tab), mask);
    MKV_LAUNCH_CHECK();
}

uint32_t climb_grid(uint64_t m) {
    return (uint32_t)std::min<uint64_t>(ceil_div(ceil_div(m ? m : 1, 64), CW_THREADS / 64), CW_MAX_BLOCKS);
}
size_t climb_mbox_bytes(uint64_t m) { return (m + 2) * MBOX_WORDS * 8; }

void launch_dirty_climb(const ClimbArgs &A, hipStream_t st) {
    if (!A.M || !A.k) return;
    hipLaunchKernelGGL(k_dirty_climb, dim3(climb_grid(A.M)), dim3(CW_THREADS), 0, st, A);
    MKV_LAUNCH_CHECK();
}

size_t umerge_scratch_bytes(uint64_t M) {
    const uint64_t nt = ceil_div(M ? M : 1, UM_TILE);
    return (nt + 2) * sizeof(uint64_t) * 2 + scan_scratch_bytes(nt + 1) + 1024;
}

void launch_umerge(const DiffSide &A, const DiffSide &B, const uint8_t *tomb, uint32_t nstore_a, void *scratch,
                   uint64_t *pfx_out, uint32_t *perm_out, uint8_t *dig_out, uint64_t *count, hipStream_t st) {
    const uint64_t M = A.n + B.n;
    if (M == 0) {
        MKV_HIP(hipMemsetAsync(count, 0, sizeof(uint64_t), st));
        return;
    }
    const uint64_t nt = ceil_div(M, UM_TILE);
    uint64_t *split = reinterpret_cast<uint64_t *>(scratch);
    uint64_t *tcnt = split + (nt + 2);
    void *sc = tcnt + (nt + 2);
    hipLaunchKernelGGL(k_umerge_partition, grid1d(nt + 1), dim3(256), 0, st, A, B, nt, split);
    hipLaunchKernelGGL(k_umerge_count, dim3((uint32_t)nt), dim3(UM_THREADS), 0, st, A, B, tomb, split, tcnt);
    MKV_LAUNCH_CHECK();
    exclusive_scan_u64(tcnt, tcnt, nt, count, sc, st);
    hipLaunchKernelGGL(k_umerge_write, dim3((uint32_t)nt), dim3(UM_THREADS), 0, st, A, B, tomb, split, tcnt, nstore_a,
                       pfx_out, perm_out, dig_out);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
