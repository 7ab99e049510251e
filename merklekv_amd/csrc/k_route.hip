// k_route.hip — redistribution of unpartitioned records into key-range shards (SURVEY §8e "sampled
// splitters when the distribution is unknown", §8f-3 "optional RCCL all-to-all redistribution").
//
// The sharded build (mkv_shard_*) needs rank r to hold every key of range r, ranges ordered by rank.
// Records that arrive on each rank in no particular key order (a store snapshot per GPU) are moved there
// by one all-to-all: ranges are cut on the 8-byte big-endian key prefix (zero-padded, so prefix order is
// consistent with Rust String order and equal prefixes never straddle two ranks) at splitters chosen from
// samples of every rank's prefixes. Per record this path is byte movement only: one prefix read for the
// destination, a stable one-digit radix pass that groups records by destination (source order kept, so
// "last write wins" keeps its meaning), and a gather of key / value bytes into the send buffers.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"

namespace mkv {

namespace {

__device__ __forceinline__ uint64_t be_prefix8(const uint8_t *k, uint64_t len) {
    uint64_t p = 0;
    const uint64_t m = len < 8 ? len : 8;
    for (uint64_t j = 0; j < m; ++j) p |= (uint64_t)k[j] << (56 - 8 * j);
    return p;
}

// Evenly spaced samples: sample i is the prefix of record ((2i + 1) n) / (2m).
__global__ void k_route_sample(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff, uint64_t n,
                               uint32_t m, uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t r = ((2 * (uint64_t)i + 1) * n) / (2 * (uint64_t)m);
    out[i] = be_prefix8(kb + koff[r], koff[r + 1] - koff[r]);
}

// Destination of every record = number of splitters <= its prefix (splitters non-decreasing), written as
// the radix key; per-destination record / key-byte / value-byte counts accumulate in LDS, then once per
// workgroup into counts[3 x world] (zeroed by the host).
__global__ __launch_bounds__(256) void k_route_dest(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                    const uint64_t *__restrict__ voff, uint64_t n,
                                                    const uint64_t *__restrict__ spl, uint32_t world,
                                                    uint64_t *__restrict__ dkey,
                                                    unsigned long long *__restrict__ counts) {
    __shared__ uint64_t s_spl[ROUTE_MAX_WORLD];
    __shared__ unsigned long long s_cnt[3 * ROUTE_MAX_WORLD];
    for (uint32_t j = threadIdx.x; j < world - 1; j += blockDim.x) s_spl[j] = spl[j];
    for (uint32_t j = threadIdx.x; j < 3 * world; j += blockDim.x) s_cnt[j] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a = koff[i], kl = koff[i + 1] - a;
        const uint64_t p = be_prefix8(kb + a, kl);
        uint32_t lo = 0, hi = world - 1;  // upper_bound over s_spl[0, world - 1)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_spl[mid] <= p) lo = mid + 1;
            else hi = mid;
        }
        dkey[i] = lo;
        atomicAdd(&s_cnt[lo], 1ull);
        atomicAdd(&s_cnt[world + lo], (unsigned long long)kl);
        atomicAdd(&s_cnt[2 * world + lo], (unsigned long long)(voff[i + 1] - voff[i]));
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 3 * world; j += blockDim.x)
        if (s_cnt[j]) atomicAdd(&counts[j], s_cnt[j]);
}

// u32 length of record perm[i]; lengths of 4 GiB or more raise *bad (the all-to-all carries u32 lengths).
__global__ void k_route_lens(const uint32_t *__restrict__ perm, const uint64_t *__restrict__ off, uint64_t n,
                             uint32_t *__restrict__ out, uint32_t *__restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = perm ? perm[i] : (uint32_t)i;
    const uint64_t len = off[o + 1] - off[o];
    if (len > 0xFFFFFFFFull) atomicOr(bad, 1u);
    out[i] = (uint32_t)len;
}

__global__ void k_u32_to_u64(const uint32_t *__restrict__ in, uint64_t n, uint64_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

}  // namespace

void launch_route_sample(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint32_t m, uint64_t *out,
                         hipStream_t st) {
    if (!m || !n) return;
    hipLaunchKernelGGL(k_route_sample, dim3((uint32_t)ceil_div(m, 256)), dim3(256), 0, st, kb, koff, n, m, out);
    MKV_LAUNCH_CHECK();
}

void launch_route_dest(const uint8_t *kb, const uint64_t *koff, const uint64_t *voff, uint64_t n, const uint64_t *spl,
                       uint32_t world, uint64_t *dkey, uint64_t *counts, hipStream_t st) {
    if (!n) return;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(ceil_div(n, 256 * 8), 2048);
    hipLaunchKernelGGL(k_route_dest, dim3(blocks), dim3(256), 0, st, kb, koff, voff, n, spl, world, dkey,
                       reinterpret_cast<unsigned long long *>(counts));
    MKV_LAUNCH_CHECK();
}

void launch_route_lens(const uint32_t *perm, const uint64_t *off, uint64_t n, uint32_t *out, uint32_t *bad,
                       hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_route_lens, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, perm, off, n, out, bad);
    MKV_LAUNCH_CHECK();
}

void launch_u32_to_u64(const uint32_t *in, uint64_t n, uint64_t *out, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_u32_to_u64, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, in, n, out);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
