// Does ds_add_rtn_u32 return pre-add values in lane order for lanes hitting the same LDS address?
// (If so, one LDS atomic per item gives stable in-wave ranks for a radix pass.) Checks many random digit
// patterns per wave against the ballot-computed stable ranks; prints mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_test(const uint32_t *digits, uint32_t trials, uint32_t *bad) {
    __shared__ uint32_t cnt[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t t = blockIdx.x; t < trials; t += gridDim.x) {
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) (&cnt[0][0])[i] = 0;
        __syncthreads();
        const uint32_t d = digits[(uint64_t)t * 256 + threadIdx.x] & 255u;
        // reference: stable rank via ballots
        uint64_t peers = ~0ull;
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t ref = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        const uint32_t got = atomicAdd(&cnt[w][d], 1u);
        if (got != ref) atomicAdd(bad, 1u);
        __syncthreads();
    }
}

int main() {
    const uint32_t trials = 200000;
    std::vector<uint32_t> h((size_t)trials * 256);
    uint64_t x = 88172645463325252ull;
    for (size_t i = 0; i < h.size(); ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint32_t mode = (uint32_t)((i / 256) % 4);
        // modes: uniform 8-bit, few distinct (4), all equal, 2 distinct
        uint32_t v = (uint32_t)x;
        h[i] = mode == 0 ? (v & 255) : mode == 1 ? (v & 3) * 37 : mode == 2 ? 7 : (v & 1) * 200;
    }
    uint32_t *d, *bad;
    hipMalloc(&d, h.size() * 4);
    hipMalloc(&bad, 4);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_test, dim3(2048), dim3(256), 0, 0, d, trials, bad);
    uint32_t hb = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("lanes checked %llu, mismatches %u\n", (unsigned long long)trials * 256ull, hb);
    return 0;
}
