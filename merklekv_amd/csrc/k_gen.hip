// k_gen.hip — on-device synthetic record generator (bench / test utility; not a reference API).
// Same definition as orc_gen_records (oracle/merkle_oracle.c) and gen_records (oracle/merkle_oracle.py):
//   word(seed, idx, field, j) = mix64(seed + GOLD * (((idx << 12) | (field << 6) | j) + 1))
//   char c of a field = SORTED_ALPHA[(word(.., c/10) >> 6*(c%10)) & 63]; key char 0 restricted to shard.
// Fixed-length records only (the configs' 32-byte keys / 100-byte values).
#include "common.hpp"
#include "kernels.hpp"

namespace mkv {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t gen_word(uint64_t seed, uint64_t idx, uint32_t field, uint32_t j) {
    return mix64(seed + 0x9E3779B97F4A7C15ull * (((idx << 12) | ((uint64_t)field << 6) | j) + 1));
}

__constant__ char kAlpha[65] = "-0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ_abcdefghijklmnopqrstuvwxyz";

__device__ void gen_field(uint64_t seed, uint64_t idx, uint32_t field, uint32_t len, uint32_t shard, uint32_t nshards,
                          uint8_t *out) {
    uint64_t w = 0;
    for (uint32_t c = 0; c < len; c += 4) {
        uint32_t packed = 0;
        for (uint32_t b = 0; b < 4 && c + b < len; ++b) {
            uint32_t cc = c + b;
            if (cc % 10 == 0 || b == 0) w = gen_word(seed, idx, field, cc / 10);
            uint32_t x = (uint32_t)(w >> (6 * (cc % 10))) & 63u;
            if (cc == 0 && field == 0 && nshards > 1) {
                const uint32_t lo = shard * 64 / nshards, hi = (shard + 1) * 64 / nshards;
                x = lo + x % (hi - lo);  // == shard*per + (x & (per-1)) when nshards | 64
            }
            packed |= (uint32_t)(uint8_t)kAlpha[x] << (8 * b);
        }
        if (c + 4 <= len && ((reinterpret_cast<uintptr_t>(out + c) & 3) == 0)) {
            *reinterpret_cast<uint32_t *>(out + c) = packed;
        } else {
            for (uint32_t b = 0; b < 4 && c + b < len; ++b) out[c + b] = (uint8_t)(packed >> (8 * b));
        }
    }
}

__global__ void k_gen_records(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, uint32_t shard,
                              uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb,
                              uint64_t *voff) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    koff[i] = i * klen;
    voff[i] = i * vlen;
    if (i == n) return;
    gen_field(seed, idx0 + i, 0, klen, shard, nshards, kb + i * klen);
    gen_field(seed, idx0 + i, vfield, vlen, 0, 1, vb + i * vlen);
}

// Ragged mode 2 of orc_gen_records ("store-like"): keys of [max(1, klen/8), klen] bytes, values of
// [vlen/16, vlen] bytes, packed back to back (so every record starts at an arbitrary byte offset).
// Pass 1 writes the lengths into koff[i] / voff[i] (scanned in place by the host side), pass 2 fills.
__global__ void k_gen_ragged_lens(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen,
                                  uint64_t *koff, uint64_t *voff) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t kmin = klen / 8 ? klen / 8 : 1, vmin = vlen / 16;
    koff[i] = kmin + gen_word(seed, idx0 + i, 62, 0) % (klen - kmin + 1);
    voff[i] = vmin + gen_word(seed, idx0 + i, 62, 1) % (vlen - vmin + 1);
}

__global__ void k_gen_ragged_fill(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t shard, uint32_t nshards,
                                  uint32_t vfield, uint8_t *kb, const uint64_t *koff, uint8_t *vb,
                                  const uint64_t *voff) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gen_field(seed, idx0 + i, 0, (uint32_t)(koff[i + 1] - koff[i]), shard, nshards, kb + koff[i]);
    gen_field(seed, idx0 + i, vfield, (uint32_t)(voff[i + 1] - voff[i]), 0, 1, vb + voff[i]);
}

}  // namespace

void launch_gen_records_ragged(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, uint32_t shard,
                               uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb,
                               uint64_t *voff, void *scan_scratch, hipStream_t st) {
    if (n) {
        hipLaunchKernelGGL(k_gen_ragged_lens, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, seed, idx0, n, klen,
                           vlen, koff, voff);
        MKV_LAUNCH_CHECK();
    }
    exclusive_scan_u64(koff, koff, n, koff + n, scan_scratch, st);
    exclusive_scan_u64(voff, voff, n, voff + n, scan_scratch, st);
    if (n) {
        hipLaunchKernelGGL(k_gen_ragged_fill, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, seed, idx0, n, shard,
                           nshards, vfield, kb, koff, vb, voff);
        MKV_LAUNCH_CHECK();
    }
}

void launch_gen_records(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, uint32_t shard,
                        uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb, uint64_t *voff,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_gen_records, dim3((uint32_t)ceil_div(n + 1, 256)), dim3(256), 0, st, seed, idx0, n, klen, vlen,
                       shard, nshards, vfield, kb, koff, vb, voff);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
