// k_sort.hip — Kernel C: leaf ordering (R3, merkle.rs:80-81) plus the scans / compactions / gathers
// the build needs.
//
// Ordering is Rust String Ord on raw key bytes. It is reproduced bit-exactly as:
//   1. stable LSD radix sort of (u64 big-endian 8-byte key prefix, input index), 8-bit digits;
//   2. for runs of equal prefix only: segmented refinement by the next 8-byte chunk (and finally by key
//      length), each round a stable chunk sort followed by a stable group-id sort (tree.cpp);
// zero padding + length tie-break == shorter-prefix-first. Stability keeps equal keys in insertion
// order so dedup keeps the last write (merkle.rs:54).
//
// Radix sort: tile = 4096 pairs per 256-thread workgroup (1024 per wave, 16 per lane, striped so each
// wave-load is 64 consecutive pairs). Pass = per-tile 256-bin histogram -> exclusive scan of the
// digit-major count matrix -> stable scatter, with in-wave ranks from 8 ballots (peer mask of lanes
// with the same digit) and per-wave LDS digit counters.
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.hpp"
#include "dev_util.hpp"
#include "kernels.hpp"

namespace mkv {

namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_IPT = 16;
constexpr int RS_TILE = RS_THREADS * RS_IPT;

constexpr int SC_THREADS = 256;
constexpr int SC_IPT = 8;
constexpr int SC_TILE = SC_THREADS * SC_IPT;

// Issue priority of the ordering kernels against co-resident leaf-hash waves: the highest, 3 (at 0, the
// leaf hash's, the co-running sort starves: 1.56 vs 0.92 ms beside the leaf hash, build 2.26-2.49 vs
// 2.17-2.22 ms/step).
__device__ __forceinline__ void sort_prio() { __builtin_amdgcn_s_setprio(3); }

__global__ __launch_bounds__(256) void k_prefix64(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                 uint64_t n, uint64_t *__restrict__ pfx, uint32_t *__restrict__ idx) {
    sort_prio();
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t a = koff[i], b = koff[i + 1];
    pfx[i] = key_chunk(kb + a, b - a, 0);
    idx[i] = (uint32_t)i;
}

// Prefix extraction fused with the digit histograms (one read of the keys): pfx[i] = big-endian first
// 8 key bytes (zero padded), counts[p*256 + d] += keys whose byte p (0 = least significant) is d. The
// input index is not written: the first radix pass generates it (k_os_pass with vin == nullptr).
// Sort window = the 8 key bytes at byte offset `off` (zero-padded): off = 0 is the key prefix; the host
// moves the window past the bytes every key shares (tree.cpp sort_unique). The pass also leaves, in
// onesweep control words the radix passes never touch (they use 8 * 256 + 0..31): the longest key length
// (PH_MAXLEN_WORD) and, with `lcp`, the complement of the shortest zero-padded common prefix of any key
// with key 0 (PH_NLCP_WORD; bounded by the longer of the two keys, capped at PH_LCP_CAP) and key 0's
// first 8 bytes (PH_K0_WORD, PH_K0_WORD + 1: high, low half); the complement of the shortest key length
// (PH_NMINLEN_WORD).
constexpr uint64_t PH_LCP_CAP = 1u << 16;
// zero2 (optional): eight counter words zeroed for the tie marker and refinement that follow. (No "last workgroup hands
// the words to the host" tail: its per-workgroup agent-scope fence + same-address arrival atomic made
// this pass 3x slower (161 -> 515 us) and, at sort priority, the co-running leaf hash 20 % slower.)
__global__ __launch_bounds__(RS_THREADS) void k_prefix_hist(const uint8_t *__restrict__ kb,
                                                           const uint64_t *__restrict__ koff, uint64_t n,
                                                           uint64_t off, bool lcp, uint64_t *__restrict__ pfx,
                                                           uint32_t *__restrict__ counts, uint32_t *__restrict__ zero2) {
    sort_prio();
    if (zero2 && blockIdx.x == 0 && threadIdx.x < 12) zero2[threadIdx.x] = 0;
    __shared__ uint32_t h[8][256];
    __shared__ uint32_t lmax, lmin, lshort;
    for (int i = threadIdx.x; i < 8 * 256; i += RS_THREADS) (&h[0][0])[i] = 0;
    if (threadIdx.x == 0) {
        lmax = 0;
        lmin = 0xFFFFFFFFu;
        lshort = 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * RS_THREADS;
    const uint64_t a0 = koff[0], l0 = koff[1] - a0;
    const uint64_t k0w = key_chunk(kb + a0, l0, 0);
    // key 0's chunks 1..3, once per thread: the common-prefix test below loads a key's chunks 1..3 in
    // one go (independent loads, one memory latency) instead of one dependent chunk per iteration
    const uint64_t k01 = lcp ? key_chunk(kb + a0, l0, 8) : 0, k02 = lcp ? key_chunk(kb + a0, l0, 16) : 0;
    const uint64_t k03 = lcp ? key_chunk(kb + a0, l0, 24) : 0;
    uint64_t mx = 0, mn = PH_LCP_CAP, sh = 0xFFFFFFFFull;
    // PH_ILP keys per thread and iteration, their offsets and first chunks loaded together: the pass runs
    // on a few workgroups beside the leaf hash, so each iteration is a chain of dependent memory round
    // trips (offsets -> key chunk), and ragged keys made it the build's critical path (10M: 673 us)
    constexpr int PH_ILP = 4;
    for (uint64_t i0 = (uint64_t)blockIdx.x * RS_THREADS + threadIdx.x; i0 < n; i0 += PH_ILP * stride) {
        uint64_t ka[PH_ILP], kl[PH_ILP], kc[PH_ILP];
#pragma unroll
        for (int j = 0; j < PH_ILP; ++j) {
            const uint64_t i = i0 + (uint64_t)j * stride;
            const bool v = i < n;
            const uint64_t a = v ? koff[i] : 0, b = v ? koff[i + 1] : 0;
            ka[j] = a;
            kl[j] = b - a;
        }
#pragma unroll
        for (int j = 0; j < PH_ILP; ++j) kc[j] = i0 + (uint64_t)j * stride < n ? key_chunk(kb + ka[j], kl[j], off) : 0;
#pragma unroll
        for (int j = 0; j < PH_ILP; ++j) {
            const uint64_t i = i0 + (uint64_t)j * stride;
            if (i >= n) break;
            const uint64_t a = ka[j], len = kl[j];
            const uint64_t k = kc[j];
            mx = len > mx ? len : mx;
            sh = len < sh ? len : sh;
            pfx[i] = k;
#pragma unroll
            for (int p = 0; p < 8; ++p) atomicAdd(&h[p][(uint32_t)(k >> (8 * p)) & 255u], 1u);
            if (lcp && mn) {  // common prefix with key 0, from the key's first chunk
                uint64_t lim = len > l0 ? len : l0;
                lim = lim < PH_LCP_CAP ? lim : PH_LCP_CAP;
                uint64_t L = 0, x = (off == 0 ? k : key_chunk(kb + a, len, 0)) ^ k0w;
                if (x == 0 && 8 < lim) {
                    const uint64_t x1 = key_chunk(kb + a, len, 8) ^ k01, x2 = key_chunk(kb + a, len, 16) ^ k02;
                    const uint64_t x3 = key_chunk(kb + a, len, 24) ^ k03;
                    L = 8;
                    x = x1;
                    if (x == 0 && L + 8 < lim) {
                        L = 16;
                        x = x2;
                        if (x == 0 && L + 8 < lim) {
                            L = 24;
                            x = x3;
                        }
                    }
                }
                while (x == 0 && L + 8 < lim) {
                    L += 8;
                    x = key_chunk(kb + a, len, L) ^ key_chunk(kb + a0, l0, L);
                }
                L += x ? (uint64_t)(__builtin_clzll(x) >> 3) : 8;
                L = L < lim ? L : lim;
                mn = L < mn ? L : mn;
            }
        }
    }
    atomicMax(&lmax, (uint32_t)(mx > 0xFFFFFFFFull ? 0xFFFFFFFFull : mx));
    atomicMin(&lshort, (uint32_t)sh);
    if (lcp) atomicMin(&lmin, (uint32_t)mn);
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * 256; i += RS_THREADS) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&counts[i], c);
    }
    if (threadIdx.x == 0) {
        if (lmax) atomicMax(&counts[PH_MAXLEN_WORD], lmax);
        atomicMax(&counts[PH_NMINLEN_WORD], ~lshort);  // max of ~x = min of x
        if (lcp) atomicMax(&counts[PH_NLCP_WORD], ~lmin);  // the words start at 0: max of ~x = min of x
        if (lcp && blockIdx.x == 0) {
            counts[PH_K0_WORD] = (uint32_t)(k0w >> 32);
            counts[PH_K0_WORD + 1] = (uint32_t)k0w;
        }
    }
}

// Sorted set prefixes from sort windows at byte offset win > 0 (bytes [0, win) are shared by every key;
// c = those bytes, big-endian at the top): the key prefix is c alone once win >= 8, else c followed by
// the window's first 8 - win bytes.
__global__ void k_pfx_from_window(uint64_t *__restrict__ pk, uint64_t n, uint64_t c, uint32_t win) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pk[i] = win >= 8 ? c : (c | (pk[i] >> (8 * win)));
}

// ---- onesweep LSD radix pass ----
// Look-back word per (tile, digit), 64 bits: [63:32] epoch of the pass that wrote it, [31:30] status (1
// aggregate, 2 inclusive), [29:0] count. A word of another epoch reads as "not ready", so a buffer that
// only ever holds look-back words needs no zeroing between passes or sorts (the build's sort keeps one
// per tree, zeroed once when allocated; every pass draws a fresh epoch).
constexpr uint32_t LB_AGG = 1u << 30, LB_INC = 2u << 30, LB_VAL = (1u << 30) - 1u;
constexpr uint32_t LB_SPIN_LIMIT = 1u << 26;  // bounded spin: sets an error flag instead of hanging

// Global digit counts of every pass in one read of the keys (counts[p*256 + d]).
__global__ __launch_bounds__(RS_THREADS) void k_os_hist(const uint64_t *__restrict__ keys, uint64_t n, int bit0,
                                                       int npass, uint32_t *__restrict__ counts) {
    sort_prio();
    __shared__ uint32_t h[8][256];
    for (int i = threadIdx.x; i < 8 * 256; i += RS_THREADS) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * RS_THREADS;
    for (uint64_t i = (uint64_t)blockIdx.x * RS_THREADS + threadIdx.x; i < n; i += stride) {
        const uint64_t k = keys[i];
        for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(uint32_t)(k >> (bit0 + 8 * p)) & 255u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * 256; i += RS_THREADS) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&counts[i], c);
    }
}

// One stable pass over 4096-pair tiles. Tiles take logical ids from an atomic counter in dispatch
// order, so a tile only ever waits on tiles that are already running or done (no deadlock whatever
// the hardware dispatch order). Ranks: 8 ballots per slot give each lane its peers with the same
// digit; per-wave LDS counters make them tile ranks. The tile publishes its digit counts, looks back
// over predecessors' words (agent-scope atomics: coherent across XCD L2s and CU L1s), sorts itself
// in LDS by digit and writes each digit run contiguously (coalesced) to its global slot.
// In-wave stable ranks: LDS_RANK = one ds_add_rtn_u32 per item on the wave's digit counter (gfx950 returns
// the pre-add values of lanes hitting one address in lane order — verified at first use by
// rank_selftest, tools/lds_atomic_order.hip); otherwise 8 ballots build each lane's peer mask.
// HALF: the local reorder goes through one key-sized LDS tile twice (keys, then values) instead of key
// and value tiles side by side; the sorted digits of the thread's output slots stay in registers
// between the two phases. IPT: items per thread (tile = 256 x IPT pairs).
template <bool LDS_RANK, bool HALF, int IPT = RS_IPT>
__global__ __launch_bounds__(RS_THREADS) void k_os_pass(const uint64_t *__restrict__ kin,
                                                       const uint32_t *__restrict__ vin,
                                                       uint64_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                       uint64_t n, int shift, const uint32_t *__restrict__ gcount,
                                                       uint64_t *__restrict__ lookback, uint32_t *__restrict__ ctl,
                                                       uint32_t epoch) {
    static_assert(IPT % 4 == 0, "the local reorder packs 4 output digits per word (dig[IPT / 4])");
    sort_prio();
    // The scan scratch and the tile id live in the first 260 B of the key tile (written only by the local
    // sort, after the barrier that follows them): 56,320 B at IPT 24 = 55 KiB, so one tile fits beside
    // three 34.25-KiB ragged-hash workgroups with 1-KiB LDS allocation granules (56,520 B did not).
    __shared__ uint64_t sk[(RS_THREADS * IPT)];
    uint32_t *sv;
    if constexpr (HALF) {
        sv = reinterpret_cast<uint32_t *>(sk);
    } else {
        __shared__ uint32_t sv_full[RS_THREADS * IPT];
        sv = sv_full;
    }
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t dstart[256];
    __shared__ uint64_t gofs[256];
    uint32_t *scan_lds = reinterpret_cast<uint32_t *>(sk);                 // 16 words
    uint64_t *scan_lds64 = sk + 8;                                          // 16 words
    uint32_t &sbid = reinterpret_cast<uint32_t *>(sk + 24)[0];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) sbid = atomicAdd(&ctl[0], 1u);
    for (int i = threadIdx.x; i < 1024; i += RS_THREADS) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t bid = sbid;
    const uint64_t tile0 = (uint64_t)bid * (RS_THREADS * IPT);
    const uint64_t base = tile0 + (uint64_t)w * (64 * IPT) + lane;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t key[IPT];
    uint32_t val[IPT];
    uint32_t rk[IPT];
#pragma unroll
    for (int s = 0; s < IPT; ++s) {
        const uint64_t i = base + (uint64_t)s * 64;
        const bool ok = i < n;
        key[s] = ok ? kin[i] : 0ull;
        val[s] = ok ? (vin ? vin[i] : (uint32_t)i) : 0u;  // vin == nullptr: values are the input indices
    }
#pragma unroll
    for (int s = 0; s < IPT; ++s) {
        const uint64_t i = base + (uint64_t)s * 64;
        const bool ok = i < n;
        const uint32_t d = (uint32_t)(key[s] >> shift) & 255u;
        if constexpr (LDS_RANK) {
            rk[s] = ok ? atomicAdd(&wcnt[w][d], 1u) : 0u;
            continue;
        }
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t before = wcnt[w][d];
        const uint32_t r = (uint32_t)__popcll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        if (ok && r == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        rk[s] = before + r;
    }
    __syncthreads();
    // ---- per digit (thread d): tile count, wave prefixes, publish, look back ----
    const uint32_t d = threadIdx.x;
    uint32_t c = 0;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
        const uint32_t x = wcnt[ww][d];
        wcnt[ww][d] = c;  // exclusive prefix over waves
        c += x;
    }
    const uint64_t ep = (uint64_t)epoch << 32;
    if (bid == 0) __hip_atomic_exchange(&lookback[d], ep | LB_INC | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_exchange(&lookback[(uint64_t)bid * 256 + d], ep | LB_AGG | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ds = block_excl_scan<uint32_t>(c, scan_lds, nullptr);
    const uint64_t gb = block_excl_scan<uint64_t>((uint64_t)gcount[d], scan_lds64, nullptr);
    dstart[d] = ds;
    uint64_t excl = 0;
    if (bid > 0) {
        int64_t j = (int64_t)bid - 1;
        uint32_t spins = 0;
        // Look back LB_WIN predecessors per step: their coherent (agent-scope) loads are issued together,
        // so a walk over k aggregate-only tiles costs ~k / LB_WIN load latencies instead of k.
        constexpr int LB_WIN = 4;
        while (j >= 0) {
            uint32_t v[LB_WIN];
#pragma unroll
            for (int q = 0; q < LB_WIN; ++q) {
                const uint64_t x = j - q >= 0 ? __hip_atomic_load(&lookback[(uint64_t)(j - q) * 256 + d], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT)
                                              : ep | LB_INC;  // before tile 0: an inclusive zero
                v[q] = (x & ~0xFFFFFFFFull) == ep ? (uint32_t)x : 0u;  // another epoch: not ready
            }
            int used = 0;
            bool done = false;
#pragma unroll
            for (int q = 0; q < LB_WIN; ++q) {
                if (done || used < q) break;  // stopped at an inclusive or a not-ready tile
                const uint32_t stt = v[q] >> 30;
                if (stt == 0) break;
                excl += v[q] & LB_VAL;
                ++used;
                done = stt == 2;
            }
            if (done) break;
            j -= used;
            if (used == 0) {  // j not ready yet
                if (++spins > LB_SPIN_LIMIT) {
                    atomicOr(&ctl[1], 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __hip_atomic_exchange(&lookback[(uint64_t)bid * 256 + d], ep | LB_INC | (uint32_t)(excl + c), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    }
    gofs[d] = gb + excl - ds;  // output position = gofs[digit] + local sorted position
    __syncthreads();
    // ---- local sort in LDS (stable: wave-major, slot, lane order) ----
    const uint32_t cnt = (uint32_t)(n - tile0 < (RS_THREADS * IPT) ? n - tile0 : (RS_THREADS * IPT));
    if constexpr (!HALF) {
#pragma unroll
        for (int s = 0; s < IPT; ++s) {
            const uint64_t i = base + (uint64_t)s * 64;
            if (i < n) {
                const uint32_t dd = (uint32_t)(key[s] >> shift) & 255u;
                const uint32_t lp = dstart[dd] + wcnt[w][dd] + rk[s];
                sk[lp] = key[s];
                sv[lp] = val[s];
            }
        }
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < cnt; p += RS_THREADS) {
            const uint64_t k = sk[p];
            const uint64_t pos = gofs[(uint32_t)(k >> shift) & 255u] + p;
            kout[pos] = k;
            vout[pos] = sv[p];
        }
    } else {
        uint32_t lpos[IPT];
#pragma unroll
        for (int s = 0; s < IPT; ++s) {
            const uint64_t i = base + (uint64_t)s * 64;
            const uint32_t dd = (uint32_t)(key[s] >> shift) & 255u;
            lpos[s] = dstart[dd] + wcnt[w][dd] + rk[s];
            if (i < n) sk[lpos[s]] = key[s];
        }
        __syncthreads();
        uint32_t dig[IPT / 4] = {};  // the digits of this thread's output slots, 8 bits each
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const uint32_t p = threadIdx.x + (uint32_t)m * RS_THREADS;
            if (p < cnt) {
                const uint64_t k = sk[p];
                const uint32_t dd = (uint32_t)(k >> shift) & 255u;
                dig[m >> 2] |= dd << (8 * (m & 3));
                kout[gofs[dd] + p] = k;
            }
        }
        __syncthreads();  // every key has left the tile: reuse it for the values
#pragma unroll
        for (int s = 0; s < IPT; ++s) {
            const uint64_t i = base + (uint64_t)s * 64;
            if (i < n) sv[lpos[s]] = val[s];
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < IPT; ++m) {
            const uint32_t p = threadIdx.x + (uint32_t)m * RS_THREADS;
            if (p < cnt) vout[gofs[(dig[m >> 2] >> (8 * (m & 3))) & 255u] + p] = sv[p];
        }
    }
}

// ---- exclusive scan (reduce-then-scan) ----
template <class T>
__global__ __launch_bounds__(SC_THREADS) void k_scan_reduce(const T *__restrict__ in, uint64_t n,
                                                           T *__restrict__ partial) {
    __shared__ T lds[16];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_IPT;
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_IPT; ++j)
        if (base + j < n) s += in[base + j];
    T tot;
    block_excl_scan<T>(s, lds, &tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

template <class T>
__global__ __launch_bounds__(1024) void k_scan_partials(T *__restrict__ partial, uint64_t nb, T *__restrict__ total) {
    __shared__ T lds[16];
    T carry = 0;
    for (uint64_t base = 0; base < nb; base += 1024) {
        uint64_t i = base + threadIdx.x;
        T x = i < nb ? partial[i] : T(0);
        T tot;
        T ex = block_excl_scan<T>(x, lds, &tot);
        if (i < nb) partial[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

template <class T>
__global__ __launch_bounds__(SC_THREADS) void k_scan_down(const T *in, T *out, uint64_t n,
                                                         const T *__restrict__ partial) {
    __shared__ T lds[16];
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_IPT;
    T v[SC_IPT];
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_IPT; ++j) {
        v[j] = (base + j < n) ? in[base + j] : T(0);
        s += v[j];
    }
    T ex = block_excl_scan<T>(s, lds, nullptr) + partial[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SC_IPT; ++j) {
        if (base + j < n) out[base + j] = ex;
        ex += v[j];
    }
}

template <class T> void scan_impl(const T *in, T *out, uint64_t n, T *total, void *scratch, hipStream_t st) {
    uint64_t nb = ceil_div(n ? n : 1, SC_TILE);
    T *partial = reinterpret_cast<T *>(scratch);
    if (n == 0) {
        if (total) MKV_HIP(hipMemsetAsync(total, 0, sizeof(T), st));
        return;
    }
    hipLaunchKernelGGL(k_scan_reduce<T>, dim3((uint32_t)nb), dim3(SC_THREADS), 0, st, in, n, partial);
    hipLaunchKernelGGL(k_scan_partials<T>, dim3(1), dim3(1024), 0, st, partial, nb, total);
    hipLaunchKernelGGL(k_scan_down<T>, dim3((uint32_t)nb), dim3(SC_THREADS), 0, st, in, out, n, partial);
    MKV_LAUNCH_CHECK();
}

// ---- ties / refinement ----
// tie[i] = prefix of i equals prefix of i-1 (count[0] += ties). Run heads (positions starting a tie
// run) are appended to heads[] (count[1] = number of heads), so the refinement visits only the runs
// instead of scanning all n flags. Same-address device atomics serialize across the XCDs (~10 ns each):
// a per-wave append cost ~0.5 ms at 46K heads, so each 1024-thread block walks a contiguous span,
// buffers its heads in LDS and publishes them with one atomic per 4,096 heads (plus one for its ties).
constexpr int MT_THREADS = 1024;
constexpr uint32_t MT_BUF = 4096;
__global__ __launch_bounds__(MT_THREADS) void k_mark_ties(const uint64_t *__restrict__ pfx, uint64_t n, int shift,
                                                         uint8_t *__restrict__ tie, uint32_t *__restrict__ count,
                                                         uint32_t *__restrict__ heads, uint32_t *__restrict__ zero,
                                                         uint32_t nzero) {
    sort_prio();
    if (blockIdx.x == 0) {
        // A pass whose look-back hit the spin limit flagged ctl[4p + 1] (words 2048 + 4p + 1) and went on with
        // a partial prefix: fold those flags into count[7] (read back with the tie counts; the host throws)
        // before the words are cleared for the next sort.
        if (threadIdx.x < 8 && nzero >= 8 * 256 + 32 && zero[8 * 256 + 4 * threadIdx.x + 1])
            atomicOr(&count[7], 1u);
        __syncthreads();
        // the sort's histogram / control words, ready (zero) for the next sort
        for (uint32_t i = threadIdx.x; i < nzero; i += MT_THREADS) zero[i] = 0;
    }
    __shared__ uint32_t buf[MT_BUF];
    __shared__ uint32_t wcnt[MT_THREADS / 64];
    __shared__ uint32_t sbase;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t tot_n = n + 1;  // position n writes the tie[n] = 0 sentinel
    const uint64_t per = ((tot_n + gridDim.x - 1) / gridDim.x + MT_THREADS - 1) / MT_THREADS * MT_THREADS;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < tot_n ? lo + per : tot_n;
    uint32_t nt = 0, nb = 0;  // nb: block-uniform count of buffered heads
    uint64_t fsum = 0, fxor = 0;  // key-set fingerprint: sum and xor of the sort keys (count[8..11])
    auto flush = [&]() {
        if (threadIdx.x == 0) sbase = atomicAdd(&count[1], nb);
        __syncthreads();
        const uint32_t b = sbase;
        for (uint32_t j = threadIdx.x; j < nb; j += MT_THREADS) heads[b + j] = buf[j];
        __syncthreads();
        nb = 0;
    };
    for (uint64_t i0 = lo; i0 < hi; i0 += MT_THREADS) {
        const uint64_t i = i0 + threadIdx.x;
        bool t = false, h = false;
        if (i < n) {
            const uint64_t full = pfx[i];
            fsum += full;
            fxor ^= full;
            const uint64_t p = full >> shift;
            t = i > 0 && p == (pfx[i - 1] >> shift);
            h = !t && i + 1 < n && (pfx[i + 1] >> shift) == p;
            tie[i] = t;
        } else if (i == n && i < hi) {
            tie[n] = 0;
        }
        nt += t;
        const uint64_t hm = __ballot(h);
        if (lane == 0) wcnt[w] = (uint32_t)__popcll(hm);
        __syncthreads();
        uint32_t off = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < MT_THREADS / 64; ++k) {
            const uint32_t c = wcnt[k];
            off += k < (int)w ? c : 0u;
            tot += c;
        }
        if (tot && nb + tot > MT_BUF) flush();
        if (h) buf[nb + off + (uint32_t)__popcll(hm & lt)] = (uint32_t)i;
        nb += tot;
        __syncthreads();  // wcnt is rewritten by the next iteration
    }
    if (nb) flush();
    // key-set fingerprint: wave sums, one atomic each per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        fsum += (uint64_t)__shfl_xor((long long)fsum, o);
        fxor ^= (uint64_t)__shfl_xor((long long)fxor, o);
    }
    if (lane == 0 && (fsum | fxor)) {
        atomicAdd(reinterpret_cast<unsigned long long *>(count + 8), (unsigned long long)fsum);
        atomicXor(&count[10], (uint32_t)fxor);
        atomicXor(&count[11], (uint32_t)(fxor >> 32));
    }
    // ties: wave sums, then one atomic per block
    uint32_t x = nt;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) wcnt[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tt = 0;
        for (int k = 0; k < MT_THREADS / 64; ++k) tt += wcnt[k];
        if (tt) atomicAdd(&count[0], tt);
    }
}

__global__ void k_active_flags(const uint8_t *__restrict__ tie, uint64_t n, uint32_t *__restrict__ flags) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flags[i] = (tie[i] | tie[i + 1]) ? 1u : 0u;
}

__global__ void k_compact_positions(const uint32_t *__restrict__ flags, const uint32_t *__restrict__ scan, uint64_t n,
                                    uint32_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flags[i]) out[scan[i]] = (uint32_t)i;
}

__global__ void k_max_keylen(const uint32_t *__restrict__ pos, uint64_t m, const uint32_t *__restrict__ perm,
                             const uint64_t *__restrict__ koff, uint32_t *__restrict__ out) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t o = perm[pos[k]];
    uint64_t len = koff[o + 1] - koff[o];
    atomicMax(out, (uint32_t)(len > 0xFFFFFFFFull ? 0xFFFFFFFFull : len));
}

__global__ void k_refine_keys(const uint32_t *__restrict__ pos, uint64_t m, const uint32_t *__restrict__ perm,
                              const uint8_t *__restrict__ tie, const uint8_t *__restrict__ kb,
                              const uint64_t *__restrict__ koff, uint32_t depth, int use_len,
                              uint64_t *__restrict__ chunk, uint32_t *__restrict__ kidx,
                              uint32_t *__restrict__ perm_act, uint32_t *__restrict__ headflag) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t p = pos[k];
    uint32_t o = perm[p];
    uint64_t a = koff[o], len = koff[o + 1] - a;
    uint64_t c = use_len ? len : key_chunk(kb + a, len, 8ull * depth);
    chunk[k] = c;            // sort key (overwritten by the sort)
    chunk[m + k] = c;        // kept copy, indexed by k
    kidx[k] = (uint32_t)k;
    perm_act[k] = o;
    headflag[k] = tie[p] ? 0u : 1u;
}

// key2[k'] = group id of element kidx[k'] = inclusive scan of head flags - 1
__global__ void k_gid_keys(const uint32_t *__restrict__ kidx, const uint32_t *__restrict__ excl,
                           const uint32_t *__restrict__ head, uint64_t m, uint64_t *__restrict__ key2) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint32_t e = kidx[k];
    key2[k] = (uint64_t)(excl[e] + head[e] - 1u);
}

__global__ void k_refine_apply(const uint32_t *__restrict__ pos, uint64_t m, const uint32_t *__restrict__ sorted_k,
                               const uint32_t *__restrict__ perm_act, const uint64_t *__restrict__ chunk_keep,
                               uint32_t *__restrict__ perm, uint8_t *__restrict__ tie, uint32_t *__restrict__ count) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool t = false;
    if (k < m) {
        uint32_t p = pos[k];
        uint32_t e = sorted_k[k];
        perm[p] = perm_act[e];
        // same group as the previous position (old tie) and equal on this round's chunk
        t = tie[p] && k > 0 && chunk_keep[e] == chunk_keep[sorted_k[k - 1]];
        tie[p] = t ? 1 : 0;
    }
    uint64_t bm = __ballot(t);
    if ((threadIdx.x & 63) == 0 && bm) atomicAdd(count, (uint32_t)__popcll(bm));
}

// Tie runs of at most RS_SMALL_RUN positions (the common case: a few keys sharing every sorted digit)
// are ordered by one thread each, in place: insertion sort on (8-byte prefix, full key, input index).
// The input index keeps equal keys in insertion order (stability, merkle.rs:54 last write wins).
// tie[] becomes full-key equality for those runs; count[0] += equal-key positions (duplicates),
// count[1] += longer runs, which are left untouched for the general refinement.
constexpr uint32_t RS_SMALL_RUN = 16;
// One run, starting at head i (tie[i] == 0, tie[i + 1] == 1).
__device__ void refine_small_run(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff, uint64_t n,
                                 uint32_t *__restrict__ perm, uint64_t *__restrict__ pfx, uint8_t *__restrict__ tie,
                                 uint32_t *__restrict__ count, uint64_t i) {
    uint64_t j = i + 1;
    while (j < n && tie[j] && j - i <= RS_SMALL_RUN) ++j;
    if (j - i > RS_SMALL_RUN) {
        atomicAdd(&count[1], 1u);
        return;
    }
    auto less = [&](uint64_t pa, uint32_t oa, uint64_t pb, uint32_t ob) {
        if (pa != pb) return pa < pb;
        const uint64_t a0 = koff[oa], b0 = koff[ob];
        const int c = key_cmp(kb + a0, koff[oa + 1] - a0, pa, kb + b0, koff[ob + 1] - b0, pb);
        return c != 0 ? c < 0 : oa < ob;
    };
    for (uint64_t x = i + 1; x < j; ++x) {
        const uint64_t px = pfx[x];
        const uint32_t ox = perm[x];
        uint64_t y = x;
        while (y > i && less(px, ox, pfx[y - 1], perm[y - 1])) {
            pfx[y] = pfx[y - 1];
            perm[y] = perm[y - 1];
            --y;
        }
        pfx[y] = px;
        perm[y] = ox;
    }
    uint32_t dups = 0;
    for (uint64_t x = i + 1; x < j; ++x) {
        const uint32_t oa = perm[x - 1], ob = perm[x];
        const uint64_t pa = pfx[x - 1], pb = pfx[x];
        bool eq = pa == pb;
        if (eq) {
            const uint64_t a0 = koff[oa], b0 = koff[ob];
            eq = key_cmp(kb + a0, koff[oa + 1] - a0, pa, kb + b0, koff[ob + 1] - b0, pb) == 0;
        }
        tie[x] = eq ? 1 : 0;
        dups += eq;
    }
    if (dups) atomicAdd(&count[0], dups);
}

__global__ __launch_bounds__(256) void k_refine_small(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                     uint64_t n, uint32_t *__restrict__ perm,
                                                     uint64_t *__restrict__ pfx, uint8_t *__restrict__ tie,
                                                     uint32_t *__restrict__ count,
                                                     const uint32_t *__restrict__ heads,
                                                     const uint32_t *__restrict__ nheads) {
    const uint64_t nh = *nheads;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nh; t += (uint64_t)gridDim.x * blockDim.x)
        refine_small_run(kb, koff, n, perm, pfx, tie, count, heads[t]);
}

// After a refinement that started at chunk 0: the prefixes of re-ordered tie-run positions follow.
__global__ void k_fix_pfx(const uint32_t *__restrict__ pos, uint64_t m, const uint32_t *__restrict__ perm,
                          const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff, uint64_t *__restrict__ pfx) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint32_t p = pos ? pos[k] : (uint32_t)k, o = perm[p];  // pos null: every position
    const uint64_t a = koff[o];
    pfx[p] = key_chunk(kb + a, koff[o + 1] - a, 0);
}

__global__ void k_keep_flags(const uint8_t *__restrict__ tie, const uint32_t *__restrict__ perm, uint64_t n,
                             uint64_t n_live, uint32_t *__restrict__ flags) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flags[i] = (!tie[i + 1] && perm[i] < n_live) ? 1u : 0u;
}

__global__ void k_compact_u32(const uint32_t *__restrict__ src, const uint32_t *__restrict__ flags,
                              const uint32_t *__restrict__ scan, uint64_t n, uint32_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flags[i]) dst[scan[i]] = src[i];
}

__global__ void k_compact_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ flags,
                              const uint32_t *__restrict__ scan, uint64_t n, uint64_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flags[i]) dst[scan[i]] = src[i];
}

// ---- gathers ----
__global__ void k_gather_digests(const uint32_t *__restrict__ perm, const uint8_t *__restrict__ dig, uint64_t n,
                                 uint8_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 *s = reinterpret_cast<const uint4 *>(dig + 32ull * perm[i]);
    uint4 *d = reinterpret_cast<uint4 *>(out + 32ull * i);
    uint4 x = s[0], y = s[1];
    d[0] = x;
    d[1] = y;
}

__global__ void k_gather_keylens(const uint32_t *__restrict__ perm, const uint64_t *__restrict__ koff, uint64_t n,
                                 uint64_t *__restrict__ lens) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t o = perm[i];
    lens[i] = koff[o + 1] - koff[o];
}

__global__ void k_gather_keys(const uint32_t *__restrict__ perm, const uint8_t *__restrict__ kb,
                              const uint64_t *__restrict__ koff, const uint64_t *__restrict__ koff_out, uint64_t n,
                              uint8_t *__restrict__ kb_out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t o = perm[i];
    uint64_t a = koff[o], len = koff[o + 1] - a;
    const uint8_t *s = kb + a;
    uint8_t *d = kb_out + koff_out[i];
    uintptr_t al = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)len;
    if ((al & 15) == 0) {
        for (uint64_t j = 0; j < len; j += 16)
            *reinterpret_cast<uint4 *>(d + j) = *reinterpret_cast<const uint4 *>(s + j);
    } else if ((al & 3) == 0) {
        for (uint64_t j = 0; j < len; j += 4)
            *reinterpret_cast<uint32_t *>(d + j) = *reinterpret_cast<const uint32_t *>(s + j);
    } else {
        for (uint64_t j = 0; j < len; ++j) d[j] = s[j];
    }
}

__global__ void k_gather_u64(const uint32_t *__restrict__ perm, const uint64_t *__restrict__ src, uint64_t n,
                             uint64_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

__global__ void k_gather_u32_to_u64(const uint32_t *__restrict__ src, const uint32_t *__restrict__ idx, uint64_t m,
                                    uint64_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) dst[i] = src[idx[i]];
}

__global__ void k_gather_u64_by_u32(const uint64_t *__restrict__ src, const uint32_t *__restrict__ idx, uint64_t m,
                                    uint64_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) dst[i] = src[idx[i]];
}

__global__ void k_add_offset_u64(const uint64_t *__restrict__ src, uint64_t n, uint64_t add,
                                 uint64_t *__restrict__ dst) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i] + add;
}

__global__ void k_iota_u32(uint32_t *__restrict__ dst, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (uint32_t)i;
}

inline dim3 grid1d(uint64_t n, uint32_t bs = 256) { return dim3((uint32_t)ceil_div(n ? n : 1, bs)); }

}  // namespace

__global__ __launch_bounds__(256) void k_rank_selftest(uint32_t trials, uint32_t *bad) {
    __shared__ uint32_t cnt[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t t = blockIdx.x; t < trials; t += gridDim.x) {
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) (&cnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t x = (t * 2654435761u) ^ (threadIdx.x * 40503u + 12345u);
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t mode = t & 3;  // uniform 8-bit, 4 distinct, all equal, 2 distinct
        const uint32_t d = mode == 0 ? (x & 255u) : mode == 1 ? (x & 3u) * 37u : mode == 2 ? 7u : (x & 1u) * 200u;
        uint64_t peers = ~0ull;
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t ref = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (atomicAdd(&cnt[w][d], 1u) != ref) atomicAdd(bad, 1u);
        __syncthreads();
    }
}

// Decided once per process on the first sort (one small kernel + readback).
static bool lds_rank_ok(hipStream_t st) {
    static int ok = -1;
    if (ok >= 0) return ok == 1;
    uint32_t *bad = nullptr;
    uint32_t hbad = 1;
    if (hipMalloc(&bad, 4) == hipSuccess) {
        (void)hipMemsetAsync(bad, 0, 4, st);
        hipLaunchKernelGGL(k_rank_selftest, dim3(256), dim3(256), 0, st, 8192u, bad);
        if (hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, st) == hipSuccess) (void)hipStreamSynchronize(st);
        (void)hipFree(bad);
    }
    ok = hbad == 0 ? 1 : 0;
    return ok == 1;
}

// Items per thread of the tree builds' prefix-sort passes: 24 (6,144 pairs per tile through the half-LDS
// reorder, ~53 KiB — the LDS footprint of the 4,096-pair tile with separate key and value tiles, 1.5x the
// pairs per look-back and 1.5x longer digit runs per write: the build's ordering stage 1.27 -> 1.11 ms
// beside the leaf hash; 32 no longer fits beside it). 12 / 16 / 20 (30-46 KiB) fit beside three leaf-hash
// workgroups per CU.
#ifndef MKV_SORT_IPT
#define MKV_SORT_IPT 24
#endif

void launch_prefix64(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint64_t *pfx, uint32_t *idx,
                     hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_prefix64, grid1d(n), dim3(256), 0, st, kb, koff, n, pfx, idx);
    MKV_LAUNCH_CHECK();
}

size_t scan_scratch_bytes(uint64_t n) { return (ceil_div(n ? n : 1, SC_TILE) + 16) * sizeof(uint64_t); }

size_t radix_scratch_bytes(uint64_t n) {
    // look-back words for the smallest tile any pass may use (12 items per thread)
    const uint64_t nb = ceil_div(n ? n : 1, (uint64_t)RS_THREADS * 12);
    // digit counts (8 x 256) + control words (8 passes x 4) + u64 look-back words (8 passes x tiles x 256)
    return (8 * 256 + 64) * sizeof(uint32_t) + 8ull * nb * 256 * sizeof(uint64_t) + 1024 + scan_scratch_bytes(n);
}

bool radix_sort_pairs(uint64_t *k, uint32_t *v, uint64_t *k2, uint32_t *v2, uint64_t n, int bit0, int bit1,
                      void *scratch, hipStream_t st) {
    if (n <= 1 || bit1 <= bit0) return false;
    if (n >= (1ull << 30)) throw Error(ST_EINVAL, "radix sort: more than 2^30 - 1 keys per device");
    const uint32_t nb = (uint32_t)ceil_div(n, RS_TILE);
    const int npass = (bit1 - bit0 + 7) / 8;
    uint32_t *counts = reinterpret_cast<uint32_t *>(scratch);
    uint32_t *ctl = counts + 8 * 256;
    uint64_t *lookback = reinterpret_cast<uint64_t *>(ctl + 64);  // byte offset 8448: 8-B aligned
    // this scratch is shared with other kernels (scans): zeroed look-back words, epoch 1
    MKV_HIP(hipMemsetAsync(counts, 0, (8 * 256 + 64) * sizeof(uint32_t) + (size_t)npass * nb * 256 * sizeof(uint64_t), st));
    const uint32_t hist_blocks = (uint32_t)std::min<uint64_t>(ceil_div(n, RS_THREADS * 16), 2048);
    hipLaunchKernelGGL(k_os_hist, dim3(hist_blocks), dim3(RS_THREADS), 0, st, k, n, bit0, npass, counts);
    MKV_LAUNCH_CHECK();
    uint64_t *ki = k, *ko = k2;
    uint32_t *vi = v, *vo = v2;
    bool swapped = false;
    for (int p = 0; p < npass; ++p) {
        if (lds_rank_ok(st))
            hipLaunchKernelGGL((k_os_pass<true, false>), dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n, bit0 + 8 * p,
                               counts + 256 * p, lookback + (size_t)p * nb * 256, ctl + 4 * p, 1u);
        else
            hipLaunchKernelGGL((k_os_pass<false, false>), dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n, bit0 + 8 * p,
                               counts + 256 * p, lookback + (size_t)p * nb * 256, ctl + 4 * p, 1u);
        MKV_LAUNCH_CHECK();
        std::swap(ki, ko);
        std::swap(vi, vo);
        swapped = !swapped;
    }
    return swapped;
}

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *scratch,
                        hipStream_t st) {
    scan_impl<uint32_t>(in, out, n, total, scratch, st);
}
void exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, void *scratch,
                        hipStream_t st) {
    scan_impl<uint64_t>(in, out, n, total, scratch, st);
}

void launch_mark_ties(const uint64_t *pfx, uint64_t n, uint8_t *tie, uint32_t *count, uint32_t *heads,
                      hipStream_t st, int shift, uint32_t *zero, uint32_t nzero) {
    // 128 workgroups: the tie marker runs beside the VALU-bound leaf hash of a build, and every resident
    // wave of it takes issue slots from the hash (10M build: 512 -> 128 workgroups, 2.25 -> 2.18 ms/step;
    // 2,048 / 8,192: 2.76 / 3.02; 64 equal, 32 slower: the marker then outlasts the hash)
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceil_div(n + 1, (uint64_t)MT_THREADS * 4), 128);
    hipLaunchKernelGGL(k_mark_ties, dim3(blocks), dim3(MT_THREADS), 0, st, pfx, n, shift, tie, count, heads, zero,
                       zero ? nzero : 0u);
    MKV_LAUNCH_CHECK();
}
void launch_refine_small(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint32_t *perm, uint64_t *pfx,
                         uint8_t *tie, uint32_t *count, const uint32_t *heads, const uint32_t *nheads,
                         uint64_t max_heads, hipStream_t st) {
    if (!n || !max_heads) return;
    // grid-stride over the device-side head count: a bounded grid however loose max_heads is
    const dim3 g((uint32_t)std::min<uint64_t>(ceil_div(max_heads, 256), 512));
    hipLaunchKernelGGL(k_refine_small, g, dim3(256), 0, st, kb, koff, n, perm, pfx, tie, count, heads, nheads);
    MKV_LAUNCH_CHECK();
}
void launch_fix_pfx(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint8_t *kb, const uint64_t *koff,
                    uint64_t *pfx, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_fix_pfx, grid1d(m), dim3(256), 0, st, pos, m, perm, kb, koff, pfx);
    MKV_LAUNCH_CHECK();
}

void launch_prefix_hist(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint64_t *pfx, void *scratch,
                        hipStream_t st, uint64_t off, bool lcp, bool zeroed, uint32_t *zero2) {
    uint32_t *counts = reinterpret_cast<uint32_t *>(scratch);
    if (!zeroed) MKV_HIP(hipMemsetAsync(counts, 0, (8 * 256 + 64) * sizeof(uint32_t), st));
    if (!n) {
        if (zero2) MKV_HIP(hipMemsetAsync(zero2, 0, 48, st));
        return;
    }
    // 256 workgroups for the same reason as the tie marker (beside the leaf hash: 2.18 -> 2.16 ms/step at 10M)
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceil_div(n, RS_THREADS * 8), 256);
    hipLaunchKernelGGL(k_prefix_hist, dim3(blocks), dim3(RS_THREADS), 0, st, kb, koff, n, off, lcp, pfx,
                       counts, zero2);
    MKV_LAUNCH_CHECK();
}

void launch_pfx_from_window(uint64_t *pk, uint64_t n, uint64_t shared, uint32_t win, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_pfx_from_window, grid1d(n), dim3(256), 0, st, pk, n, shared, win);
    MKV_LAUNCH_CHECK();
}

void radix_prefix_hist(const uint64_t *k, uint64_t n, void *scratch, hipStream_t st) {
    uint32_t *counts = reinterpret_cast<uint32_t *>(scratch);
    MKV_HIP(hipMemsetAsync(counts, 0, (8 * 256 + 64) * sizeof(uint32_t), st));
    if (!n) return;
    const uint32_t hist_blocks = (uint32_t)std::min<uint64_t>(ceil_div(n, RS_THREADS * 16), 2048);
    hipLaunchKernelGGL(k_os_hist, dim3(hist_blocks), dim3(RS_THREADS), 0, st, k, n, 0, 8, counts);
    MKV_LAUNCH_CHECK();
}

uint64_t radix_prefix_lookback_words(uint64_t n) { return ceil_div(n ? n : 1, (uint64_t)RS_THREADS * MKV_SORT_IPT) * 256; }

bool radix_prefix_passes(uint64_t *k, uint32_t *v, uint64_t *k2, uint32_t *v2, uint64_t n, uint32_t digit_mask,
                         void *scratch, uint64_t *lookback, uint32_t *epoch, hipStream_t st, bool v_identity) {
    if (n <= 1 || !digit_mask) {
        if (v_identity && n) {
            hipLaunchKernelGGL(k_iota_u32, grid1d(n), dim3(256), 0, st, v, n);
            MKV_LAUNCH_CHECK();
        }
        return false;
    }
    if (n >= (1ull << 30)) throw Error(ST_EINVAL, "radix sort: more than 2^30 - 1 keys per device");
    const uint32_t nb = (uint32_t)ceil_div(n, (uint64_t)RS_THREADS * MKV_SORT_IPT);
    uint32_t *counts = reinterpret_cast<uint32_t *>(scratch);
    uint32_t *ctl = counts + 8 * 256;
    uint64_t *ki = k, *ko = k2;
    uint32_t *vi = v_identity ? nullptr : v, *vo = v2;
    uint32_t *valt = v;  // the ping-pong partner of vo once the first pass has produced real values
    bool swapped = false;
    for (int p = 0; p < 8; ++p) {
        if (!((digit_mask >> p) & 1u)) continue;
        const bool lr = lds_rank_ok(st);
        // every pass a fresh epoch (0 is never drawn: the buffer starts zeroed); one region serves every
        // pass, since the previous pass's words read as not ready
        if (++*epoch == 0) ++*epoch;
        uint64_t *lb = lookback;
        if (lr)
            hipLaunchKernelGGL((k_os_pass<true, true, MKV_SORT_IPT>), dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n,
                               8 * p, counts + 256 * p, lb, ctl + 4 * p, *epoch);
        else  // same tile size (nb tiles of 256 x MKV_SORT_IPT), ballot ranks
            hipLaunchKernelGGL((k_os_pass<false, true, MKV_SORT_IPT>), dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n,
                               8 * p, counts + 256 * p, lb, ctl + 4 * p, *epoch);
        MKV_LAUNCH_CHECK();
        std::swap(ki, ko);
        uint32_t *written = vo;
        vo = vi ? vi : valt;
        vi = written;
        swapped = !swapped;
    }
    return swapped;
}
void launch_active_flags(const uint8_t *tie, uint64_t n, uint32_t *flags, hipStream_t st) {
    hipLaunchKernelGGL(k_active_flags, grid1d(n), dim3(256), 0, st, tie, n, flags);
    MKV_LAUNCH_CHECK();
}
void launch_compact_positions(const uint32_t *flags, const uint32_t *scan, uint64_t n, uint32_t *out,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_compact_positions, grid1d(n), dim3(256), 0, st, flags, scan, n, out);
    MKV_LAUNCH_CHECK();
}
void launch_max_keylen(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint64_t *koff, uint32_t *out,
                       hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_max_keylen, grid1d(m), dim3(256), 0, st, pos, m, perm, koff, out);
    MKV_LAUNCH_CHECK();
}
void launch_refine_keys(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint8_t *tie, const uint8_t *kb,
                        const uint64_t *koff, uint32_t depth, int use_len, uint64_t *chunk, uint32_t *kidx,
                        uint32_t *perm_act, uint32_t *headflag, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_refine_keys, grid1d(m), dim3(256), 0, st, pos, m, perm, tie, kb, koff, depth, use_len, chunk,
                       kidx, perm_act, headflag);
    MKV_LAUNCH_CHECK();
}
void launch_gid_keys(const uint32_t *kidx, const uint32_t *excl, const uint32_t *head, uint64_t m, uint64_t *key2,
                     hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_gid_keys, grid1d(m), dim3(256), 0, st, kidx, excl, head, m, key2);
    MKV_LAUNCH_CHECK();
}
void launch_gather_u64_by_u32(const uint64_t *src, const uint32_t *idx, uint64_t m, uint64_t *dst, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_gather_u64_by_u32, grid1d(m), dim3(256), 0, st, src, idx, m, dst);
    MKV_LAUNCH_CHECK();
}
void launch_gather_u32_to_u64(const uint32_t *src, const uint32_t *idx, uint64_t m, uint64_t *dst, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_gather_u32_to_u64, grid1d(m), dim3(256), 0, st, src, idx, m, dst);
    MKV_LAUNCH_CHECK();
}
void launch_refine_apply(const uint32_t *pos, uint64_t m, const uint32_t *sorted_k, const uint32_t *perm_act,
                         const uint64_t *chunk, uint32_t *perm, uint8_t *tie, uint32_t *count, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_refine_apply, grid1d(m), dim3(256), 0, st, pos, m, sorted_k, perm_act, chunk, perm, tie,
                       count);
    MKV_LAUNCH_CHECK();
}
void launch_keep_flags(const uint8_t *tie, const uint32_t *perm, uint64_t n, uint64_t n_live, uint32_t *flags,
                       hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_keep_flags, grid1d(n), dim3(256), 0, st, tie, perm, n, n_live, flags);
    MKV_LAUNCH_CHECK();
}
void launch_compact_u32(const uint32_t *src, const uint32_t *flags, const uint32_t *scan, uint64_t n, uint32_t *dst,
                        hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_compact_u32, grid1d(n), dim3(256), 0, st, src, flags, scan, n, dst);
    MKV_LAUNCH_CHECK();
}
void launch_compact_u64(const uint64_t *src, const uint32_t *flags, const uint32_t *scan, uint64_t n, uint64_t *dst,
                        hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_compact_u64, grid1d(n), dim3(256), 0, st, src, flags, scan, n, dst);
    MKV_LAUNCH_CHECK();
}
void launch_gather_digests(const uint32_t *perm, const uint8_t *dig_in, uint64_t n, uint8_t *out, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_gather_digests, grid1d(n), dim3(256), 0, st, perm, dig_in, n, out);
    MKV_LAUNCH_CHECK();
}
void launch_gather_keylens(const uint32_t *perm, const uint64_t *koff, uint64_t n, uint64_t *lens, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_gather_keylens, grid1d(n), dim3(256), 0, st, perm, koff, n, lens);
    MKV_LAUNCH_CHECK();
}
void launch_gather_keys(const uint32_t *perm, const uint8_t *kb, const uint64_t *koff, const uint64_t *koff_out,
                        uint64_t n, uint8_t *kb_out, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_gather_keys, grid1d(n), dim3(256), 0, st, perm, kb, koff, koff_out, n, kb_out);
    MKV_LAUNCH_CHECK();
}
void launch_gather_u64(const uint32_t *perm, const uint64_t *src, uint64_t n, uint64_t *dst, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_gather_u64, grid1d(n), dim3(256), 0, st, perm, src, n, dst);
    MKV_LAUNCH_CHECK();
}
void launch_add_offset_u64(const uint64_t *src, uint64_t n, uint64_t add, uint64_t *dst, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_add_offset_u64, grid1d(n), dim3(256), 0, st, src, n, add, dst);
    MKV_LAUNCH_CHECK();
}
void launch_iota_u32(uint32_t *dst, uint64_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_iota_u32, grid1d(n), dim3(256), 0, st, dst, n);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
