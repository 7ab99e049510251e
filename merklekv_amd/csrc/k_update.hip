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
// Dirty lists are unordered (wave-aggregated atomic append); the dirty bitmap (one bit per stored
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

__global__ __launch_bounds__(256) void k_locate(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                uint64_t m, DiffSide T, uint64_t *__restrict__ pos,
                                                uint32_t *__restrict__ idx, uint32_t *__restrict__ missing) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool miss = false;
    if (i < m) {
        const uint64_t a = koff[i], len = koff[i + 1] - a;
        const uint8_t *k = kb + a;
        const uint64_t c0 = key_chunk(k, len, 0);
        uint64_t lo = 0, hi = T.n;  // first position with pfx >= c0
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (T.pfx[mid] < c0) lo = mid + 1;
            else hi = mid;
        }
        uint64_t found = UINT64_MAX;
        for (uint64_t j = lo; j < T.n && T.pfx[j] == c0; ++j) {
            uint64_t tl;
            const uint8_t *tk = tree_key(T, j, &tl);
            const int c = key_cmp(k, len, c0, tk, tl, c0);
            if (c == 0) {
                found = j;
                break;
            }
            if (c < 0) break;
        }
        miss = found == UINT64_MAX;
        pos[i] = found;
        idx[i] = (uint32_t)i;
    }
    const uint64_t b = __ballot(miss);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(missing, (uint32_t)__popcll(b));
}

__device__ __forceinline__ void set_bit(uint32_t *bm, uint64_t b) { atomicOr(bm + (b >> 5), 1u << (b & 31)); }
__device__ __forceinline__ void clear_bit(uint32_t *bm, uint64_t b) { atomicAnd(bm + (b >> 5), ~(1u << (b & 31))); }
__device__ __forceinline__ bool get_bit(const uint32_t *bm, uint64_t b) {
    return (__atomic_load_n(bm + (b >> 5), __ATOMIC_RELAXED) >> (b & 31)) & 1u;
}

// Wave-aggregated append of `v` (when `act`) to list/count.
__device__ __forceinline__ void wave_append(bool act, uint32_t v, uint32_t *list, uint32_t *count) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t b = __ballot(act);
    uint32_t base = 0;
    if (lane == 0 && b) base = atomicAdd(count, (uint32_t)__popcll(b));
    base = __shfl(base, 0);
    if (act) list[base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = v;
}

// Level 0: sorted (position, batch index) pairs; the last entry of each equal-position run is the last
// write of that key. nodes0: local leaf level; bm bit index of leaf p = p (level 0 starts the bitmap).
__global__ __launch_bounds__(256) void k_dirty_leaves(const uint64_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ bidx, uint64_t m,
                                                      const uint8_t *__restrict__ bdig, uint8_t *__restrict__ nodes0,
                                                      uint32_t *__restrict__ bm, uint32_t *__restrict__ list,
                                                      uint32_t *__restrict__ count) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool act = false;
    uint32_t p = 0;
    if (s < m) {
        const uint64_t q = pos[s];
        act = (s + 1 == m) || pos[s + 1] != q;
        p = (uint32_t)q;
        if (act) {
            const uint4 *src = reinterpret_cast<const uint4 *>(bdig + 32ull * bidx[s]);
            uint4 *dst = reinterpret_cast<uint4 *>(nodes0 + 32ull * p);
            dst[0] = src[0];
            dst[1] = src[1];
            set_bit(bm, p);
        }
    }
    wave_append(act, p, list, count);
}

__global__ __launch_bounds__(256) void k_dirty_level(DirtyLevel L, uint8_t *__restrict__ nodes,
                                                     uint32_t *__restrict__ bm, const uint32_t *__restrict__ lin,
                                                     const uint32_t *__restrict__ nin, uint32_t *__restrict__ lout,
                                                     uint32_t *__restrict__ nout) {
    const uint32_t cnt = *nin;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((uint64_t)blockIdx.x * blockDim.x >= cnt) return;  // whole workgroup idle (wave-uniform exit)
    bool act = false;
    uint32_t qloc = 0;
    uint32_t ow[8];
    if (i < cnt) {
        const uint64_t x = lin[i];  // local index at level l
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
        } else if (!((xg & 1) && get_bit(bm, L.off + x - 1))) {
            const uint64_t lg = 2 * qg;  // left child (global); owned because the parent is
            const uint8_t *lp = nodes + 32 * (L.off + (lg - L.a));
            uint32_t lw[8];
            load_digest(lp, lw);
            if (lg + 1 < L.S) {
                uint32_t rw[8];
                load_digest(lp + 32, rw);
                sha_node<true>(lw, rw, ow);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) ow[q] = lw[q];  // R5 promotion
            }
            qloc = (uint32_t)(qg - L.a_par);
            store_digest(nodes + 32 * (L.off_par + qloc), ow);
            set_bit(bm, L.off_par + qloc);
            act = true;
        }
    }
    wave_append(act, qloc, lout, nout);
}

inline dim3 grid1d(uint64_t n, uint32_t bs = 256) { return dim3((uint32_t)ceil_div(n ? n : 1, bs)); }

}  // namespace

void launch_locate(const uint8_t *kb, const uint64_t *koff, uint64_t m, const DiffSide &T, uint64_t *pos,
                   uint32_t *idx, uint32_t *missing, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_locate, grid1d(m), dim3(256), 0, st, kb, koff, m, T, pos, idx, missing);
    MKV_LAUNCH_CHECK();
}

void launch_dirty_leaves(const uint64_t *pos, const uint32_t *bidx, uint64_t m, const uint8_t *bdig, uint8_t *nodes0,
                         uint32_t *bm, uint32_t *list, uint32_t *count, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_dirty_leaves, grid1d(m), dim3(256), 0, st, pos, bidx, m, bdig, nodes0, bm, list, count);
    MKV_LAUNCH_CHECK();
}

void launch_dirty_level(const DirtyLevel &L, uint64_t max_entries, uint8_t *nodes, uint32_t *bm, const uint32_t *lin,
                        const uint32_t *nin, uint32_t *lout, uint32_t *nout, hipStream_t st) {
    if (!max_entries) return;
    hipLaunchKernelGGL(k_dirty_level, grid1d(max_entries), dim3(256), 0, st, L, nodes, bm, lin, nin, lout, nout);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
