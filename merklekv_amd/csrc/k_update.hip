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
//                   back to the full rebuild for those batches).
//   (radix sort of (position, batch index); stable, so the last write of a key is the last of its run)
//   k_dirty_leaves  last write per position wins (merkle.rs:54); scatters the new leaf digests into
//                   level 0, sets the node's dirty bit and appends it to the level's dirty list.
//   k_dirty_level   one launch per level: every dirty node whose parent is owned hashes that parent
//                   unless its left sibling is also dirty (the left one owns the pair), promotes it
//                   unchanged past an odd level end (R5), marks the parent dirty and appends it. The
//                   level-l launch also clears the level-(l-1) bits of its entries' children, so the
//                   bitmap is all-zero again after the last level and no clearing pass is needed.
//
// Dirty lists are unordered (block-aggregated atomic append); the dirty bitmap (one bit per stored
// node) is what deduplicates parents, so no per-level sort or scan is needed. Parents outside the
// shard's owned range (sharded trees) stop the climb: their seam is recomputed by the
// fringe all-gather + mkv_shard_combine exactly as after a full build.
#include "common.hpp"
#include "dev_util.hpp"
#include "kernels.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

__device__ __forceinline__ const uint8_t *tree_key(const DiffSide &T, uint64_t i, uint64_t *len) {
    const uint32_t o = T.perm[i];
    const uint64_t a = T.koff[o];
    *len = T.koff[o + 1] - a;
    return T.kb + a;
}

__device__ __forceinline__ uint64_t locate_run(const uint8_t *k, uint64_t len, uint64_t c0, const DiffSide &T,
                                               uint64_t lo);
constexpr int LOCATE_ILP = 2;  // batch keys per lane in k_locate / k_locate_multi

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
        ka[j] = hit[j] && !run[j] ? T.koff[o[j]] : 0;
        kl[j] = hit[j] && !run[j] ? T.koff[o[j] + 1] - ka[j] : 0;
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

__global__ __launch_bounds__(256) void k_locate_multi(LeafBatches B, LocateMulti L, int pbits,
                                                      uint64_t *__restrict__ pos, uint32_t *__restrict__ idx) {
    const uint32_t t = blockIdx.y;
    const uint64_t m = B.m[t];
    const uint64_t i0 = (uint64_t)blockIdx.x * (LOCATE_ILP * blockDim.x) + threadIdx.x;
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
    locate_k<LOCATE_ILP>(kp, len, v, L.T[t], L.ps[t], L.ns[t], found);
    uint32_t nmiss = 0;
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
    if ((threadIdx.x & 63) == 0 && nmiss) atomicAdd(L.missing[t], nmiss);
}

__device__ __forceinline__ void set_bit(uint32_t *bm, uint64_t b) { atomicOr(bm + (b >> 5), 1u << (b & 31)); }
__device__ __forceinline__ void clear_bit(uint32_t *bm, uint64_t b) { atomicAnd(bm + (b >> 5), ~(1u << (b & 31))); }
__device__ __forceinline__ bool get_bit(const uint32_t *bm, uint64_t b) {
    return (__atomic_load_n(bm + (b >> 5), __ATOMIC_RELAXED) >> (b & 31)) & 1u;
}

// Level 0: sorted (position, batch index) pairs; the last entry of each equal-position run is the last
// write of that key. nodes0: local leaf level; bm bit index of leaf p = p (level 0 starts the bitmap).
__device__ __forceinline__ void dirty_leaves_block(const uint64_t *__restrict__ pos, const uint32_t *__restrict__ bidx,
                                                   uint64_t m, const uint8_t *__restrict__ bdig,
                                                   uint8_t *__restrict__ nodes0, uint32_t *__restrict__ bm,
                                                   uint32_t *__restrict__ list, uint32_t *__restrict__ count,
                                                   uint64_t pmask, uint32_t *sapp) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool act = false;
    uint32_t p = 0;
    if (s < m) {
        const uint64_t q = pos[s];
        act = (s + 1 == m) || pos[s + 1] != q;
        p = (uint32_t)(q & pmask);
        if (act) {
            const uint4 *src = reinterpret_cast<const uint4 *>(bdig + 32ull * bidx[s]);
            uint4 *dst = reinterpret_cast<uint4 *>(nodes0 + 32ull * p);
            dst[0] = src[0];
            dst[1] = src[1];
            set_bit(bm, p);
        }
    }
    block_append<uint32_t>(act, p, list, count, sapp);
}

__global__ __launch_bounds__(256) void k_dirty_leaves(const uint64_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ bidx, uint64_t m,
                                                      const uint8_t *__restrict__ bdig, uint8_t *__restrict__ nodes0,
                                                      uint32_t *__restrict__ bm, uint32_t *__restrict__ list,
                                                      uint32_t *__restrict__ count, const uint32_t *__restrict__ missing,
                                                      uint64_t pmask) {
    __shared__ uint32_t sapp[17];
    if (*missing) return;  // some batch key is not a leaf: the caller takes the merge path, tree untouched
    dirty_leaves_block(pos, bidx, m, bdig, nodes0, bm, list, count, pmask, sapp);
}

// k trees' level-0 scatters in one launch (grid.y = tree): tree q's sorted entries are
// pos[S.base[q], S.base[q] + S.m[q]).
__global__ __launch_bounds__(256) void k_dirty_leaves_multi(const uint64_t *__restrict__ pos,
                                                            const uint32_t *__restrict__ bidx, DirtySegs S,
                                                            const uint8_t *__restrict__ bdig, DirtyTrees T,
                                                            uint64_t pmask) {
    __shared__ uint32_t sapp[17];
    const DirtyTree &D = T.t[blockIdx.y];
    const uint64_t m = S.m[blockIdx.y], b = S.base[blockIdx.y];
    if (*D.missing || (uint64_t)blockIdx.x * blockDim.x >= m) return;  // workgroup-uniform exits
    dirty_leaves_block(pos + b, bidx + b, m, bdig, D.nodes, D.bm, D.l0, D.cnt, pmask, sapp);
}

// One dirty entry x (local index at level l): clears its children's bits, and, when its parent is owned
// and its left sibling is not dirty (the left one owns the pair), rehashes the parent (or promotes past
// an odd level end, R5), marks it dirty and returns true with the parent's local index in *qloc.
// SHORT: the short-chain round form (latency-bound fused top); the per-level launches are throughput-bound
// and take the plain form (fewer instructions).
template <bool SHORT>
__device__ __forceinline__ bool dirty_step(const DirtyLevel &L, uint64_t x, uint8_t *nodes, uint32_t *bm,
                                           uint32_t *qloc) {
    const uint64_t xg = L.a + x;
    // children of this entry at level l-1: their bits are no longer read by anyone
    if (L.has_child) {
        const uint64_t c0 = 2 * xg - L.a_child;
        if (c0 < L.c_child) clear_bit(bm, L.off_child + c0);
        if (c0 + 1 < L.c_child) clear_bit(bm, L.off_child + c0 + 1);
    }
    const uint64_t qg = xg >> 1;
    const bool owned = L.has_parent && qg >= L.a_par && qg < L.a_par + L.c_par;
    if (!owned) {
        clear_bit(bm, L.off + x);  // top of the local climb (root, or a seam parent)
        return false;
    }
    if ((xg & 1) && get_bit(bm, L.off + x - 1)) return false;
    const uint64_t lg = 2 * qg;  // left child (global); owned because the parent is
    const uint8_t *lp = nodes + 32 * (L.off + (lg - L.a));
    uint32_t lw[8], ow[8];
    load_digest(lp, lw);
    if (lg + 1 < L.S) {
        uint32_t rw[8];
        load_digest(lp + 32, rw);
        sha_node<SHORT>(lw, rw, ow);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) ow[q] = lw[q];  // R5 promotion
    }
    *qloc = (uint32_t)(qg - L.a_par);
    store_digest(nodes + 32 * (L.off_par + *qloc), ow);
    set_bit(bm, L.off_par + *qloc);
    return true;
}

__global__ __launch_bounds__(256) void k_dirty_level(DirtyLevel L, int l, DirtyTrees T) {
    __shared__ uint32_t sapp[17];
    const DirtyTree &D = T.t[blockIdx.y];
    if (*D.missing) return;
    const uint32_t *lin = (l & 1) ? D.l1 : D.l0;
    uint32_t *lout = (l & 1) ? D.l0 : D.l1;
    const uint32_t cnt = D.cnt[l];
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((uint64_t)blockIdx.x * blockDim.x >= cnt) return;  // whole workgroup idle (wave-uniform exit)
    bool act = false;
    uint32_t qloc = 0;
    if (i < cnt) act = dirty_step<false>(L, lin[i], D.nodes, D.bm, &qloc);
    block_append<uint32_t>(act, qloc, lout, D.cnt + l + 1, sapp);
}

__device__ __forceinline__ DirtyLevel level_of(const LevelPlan &P, int l) {
    DirtyLevel D{};
    D.a = P.base[l];
    D.c = P.cnt[l];
    D.off = P.off[l];
    D.S = P.S[l];
    D.has_parent = l + 1 < P.L && P.cnt[l + 1] > 0;
    if (D.has_parent) {
        D.a_par = P.base[l + 1];
        D.c_par = P.cnt[l + 1];
        D.off_par = P.off[l + 1];
    }
    D.has_child = l > 0 && !P.keep_bits;
    if (l > 0) {
        D.a_child = P.base[l - 1];
        D.c_child = P.cnt[l - 1];
        D.off_child = P.off[l - 1];
    }
    return D;
}

// All levels from l0 up in one workgroup, once a level's dirty set fits DIRTY_TOP_CAP (it never grows
// going up): the dirty lists live in LDS, levels are separated by a device-scope fence + barrier instead
// of a kernel boundary. Replaces the ~13 latency-bound single-workgroup launches at the top of a 1e8-leaf
// tree, and every launch above level 0 for batches of at most DIRTY_TOP_CAP keys.
__global__ __launch_bounds__(DIRTY_TOP_THREADS) void k_dirty_top(LevelPlan P, int l0, DirtyTrees T) {
    const DirtyTree &Dt = T.t[blockIdx.x];  // one workgroup per tree
    uint8_t *nodes = Dt.nodes;
    uint32_t *bm = Dt.bm;
    const uint32_t *lin = (l0 & 1) ? Dt.l1 : Dt.l0;
    const uint32_t *nin = Dt.cnt + l0;
    const uint32_t *missing = Dt.missing;
    __shared__ uint32_t list[2][DIRTY_TOP_CAP];
    __shared__ uint32_t ncnt[2];
    if (*missing) return;
    uint32_t n = *nin;
    if (n > DIRTY_TOP_CAP) n = DIRTY_TOP_CAP;  // cannot happen: the host bounds the level's dirty count
    for (uint32_t e = threadIdx.x; e < n; e += DIRTY_TOP_THREADS) list[0][e] = lin[e];
    if (threadIdx.x == 0) ncnt[1] = 0;
    __syncthreads();
    int cur = 0;
    for (int l = l0; l < P.L; ++l) {
        const DirtyLevel D = level_of(P, l);
        for (uint32_t e = threadIdx.x; e < n; e += DIRTY_TOP_THREADS) {
            uint32_t q;
            if (dirty_step<true>(D, list[cur][e], nodes, bm, &q)) list[cur ^ 1][atomicAdd(&ncnt[cur ^ 1], 1u)] = q;
        }
        // parents' digests and bits visible to every wave of the next level: one workgroup, one CU, so a
        // workgroup-scope fence (its stores complete) instead of an agent-scope one
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        if (!D.has_parent) break;
        n = ncnt[cur ^ 1];
        cur ^= 1;
        __syncthreads();
        if (threadIdx.x == 0) ncnt[cur ^ 1] = 0;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Batch merge (key-set changes): the tree's sorted leaves A and a sorted unique batch B
// (last write per key already chosen, tombstones flagged) merged into the new sorted leaf set. An A
// leaf survives unless B's cursor holds the same key (replaced or removed, merkle.rs:52-62); a B
// record survives unless it is a remove. Same merge-path tiling as the diff (k_diff.hip): one binary
// search per 2048-output tile, 8 outputs per lane, two passes around a scan of the kept counts.
// ---------------------------------------------------------------------------------------------
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

void launch_dirty_leaves_multi(const uint64_t *pos, const uint32_t *bidx, const DirtySegs &S, uint64_t mmax,
                               const uint8_t *bdig, const DirtyTrees &T, uint32_t k, hipStream_t st, uint64_t pmask) {
    if (!mmax || !k) return;
    hipLaunchKernelGGL(k_dirty_leaves_multi, dim3((uint32_t)ceil_div(mmax, 256), k), dim3(256), 0, st, pos, bidx, S,
                       bdig, T, pmask);
    MKV_LAUNCH_CHECK();
}

void launch_dirty_leaves(const uint64_t *pos, const uint32_t *bidx, uint64_t m, const uint8_t *bdig, uint8_t *nodes0,
                         uint32_t *bm, uint32_t *list, uint32_t *count, const uint32_t *missing, hipStream_t st,
                         uint64_t pmask) {
    if (!m) return;
    hipLaunchKernelGGL(k_dirty_leaves, grid1d(m), dim3(256), 0, st, pos, bidx, m, bdig, nodes0, bm, list, count,
                       missing, pmask);
    MKV_LAUNCH_CHECK();
}

void launch_locate_multi(const LeafBatches &B, const LocateMulti &L, uint32_t k, uint64_t mmax, int pbits,
                         uint64_t *pos, uint32_t *idx, hipStream_t st) {
    if (!k || !mmax) return;
    hipLaunchKernelGGL(k_locate_multi, dim3((uint32_t)ceil_div(mmax, 256 * LOCATE_ILP), k), dim3(256), 0, st, B, L, pbits,
                       pos, idx);
    MKV_LAUNCH_CHECK();
}

void launch_dirty_level(const DirtyLevel &L, int l, uint64_t max_entries, const DirtyTrees &T, uint32_t k,
                        hipStream_t st) {
    if (!max_entries || !k) return;
    hipLaunchKernelGGL(k_dirty_level, dim3((uint32_t)ceil_div(max_entries, 256), k), dim3(256), 0, st, L, l, T);
    MKV_LAUNCH_CHECK();
}

void launch_dirty_top(const LevelPlan &P, int l0, const DirtyTrees &T, uint32_t k, hipStream_t st) {
    if (!k) return;
    hipLaunchKernelGGL(k_dirty_top, dim3(k), dim3(DIRTY_TOP_THREADS), 0, st, P, l0, T);
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
