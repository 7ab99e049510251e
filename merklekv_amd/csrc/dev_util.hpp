// dev_util.hpp — device helpers shared by the sort, diff and reduce kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mkv {

// Big-endian word of the 4 bytes at p, never touching a 4-byte-aligned chunk wholly at/after `end`
// (an aligned dword that holds a valid byte lies in a mapped page, so no over-read can fault).
__device__ __forceinline__ uint32_t be_word_guarded(const uint8_t *p, const uint8_t *end) {
    uintptr_t ad = reinterpret_cast<uintptr_t>(p);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(ad & 3);
    uint32_t lo = (reinterpret_cast<const uint8_t *>(a) < end) ? a[0] : 0u;
    uint32_t hi = (reinterpret_cast<const uint8_t *>(a + 1) < end) ? a[1] : 0u;
    return __builtin_amdgcn_perm(hi, lo, 0x00010203u + sh * 0x01010101u);
}

// Bytes [off, off+8) of a key of length len as a big-endian u64, zero padded past len.
// Zero padding + a final length tie-break reproduces Rust String Ord (R3, merkle.rs:80-81) because
// 0x00 is the smallest byte.
__device__ __forceinline__ uint64_t key_chunk(const uint8_t *k, uint64_t len, uint64_t off) {
    if (off >= len) return 0;
    if (off + 8 <= len && (reinterpret_cast<uintptr_t>(k + off) & 3) == 0) {  // whole, 4-B aligned: 2 loads
        const uint32_t *q = reinterpret_cast<const uint32_t *>(k + off);
        return ((uint64_t)__builtin_bswap32(q[0]) << 32) | __builtin_bswap32(q[1]);
    }
    const uint8_t *end = k + len;
    uint64_t v = ((uint64_t)be_word_guarded(k + off, end) << 32) | be_word_guarded(k + off + 4, end);
    uint64_t rem = len - off;
    if (rem < 8) v &= ~0ull << (8 * (8 - rem));
    return v;
}

// Rust `str` Ord on raw bytes: <0, 0, >0. c0a/c0b: precomputed chunk 0 (prefix) of each key.
__device__ __forceinline__ int key_cmp(const uint8_t *ka, uint64_t la, uint64_t c0a, const uint8_t *kb, uint64_t lb,
                                       uint64_t c0b) {
    if (c0a != c0b) return c0a < c0b ? -1 : 1;
    uint64_t mx = la > lb ? la : lb;
    for (uint64_t off = 8; off < mx; off += 8) {
        uint64_t a = key_chunk(ka, la, off), b = key_chunk(kb, lb, off);
        if (a != b) return a < b ? -1 : 1;
    }
    return (la > lb) - (la < lb);
}

template <class T> __device__ __forceinline__ T wave_incl_scan(T x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}

// Exclusive scan over the block (blockDim.x multiple of 64, <= 1024). lds: >= 16 entries.
template <class T> __device__ __forceinline__ T block_excl_scan(T x, T *lds, T *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T inc = wave_incl_scan(x);
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    T pre = 0, tot = 0;
    for (int i = 0; i < nw; ++i) {
        T v = lds[i];
        pre += (i < w) ? v : T(0);
        tot += v;
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + inc - x;
}

// Block-aggregated append of v (when act) to out/count: one device-scope atomic per workgroup call.
// Same-address atomics serialize across the XCDs, so per-wave appends of large frontiers / dirty lists
// were bound by that one counter. Every thread of the block must call it (block-uniform control flow);
// lds: >= 17 u32 of shared scratch. Order within the block follows wave then lane order.
template <class T>
__device__ __forceinline__ void block_append(bool act, T v, T *out, uint32_t *count, uint32_t *lds) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const uint64_t m = __ballot(act);
    if (lane == 0) lds[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t i = 0; i < nw; ++i) {
            const uint32_t c = lds[i];
            lds[i] = tot;
            tot += c;
        }
        lds[16] = tot ? atomicAdd(count, tot) : 0u;
    }
    __syncthreads();
    if (act) out[lds[16] + lds[w] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = v;
    __syncthreads();  // lds is reused by the next call
}

}  // namespace mkv
