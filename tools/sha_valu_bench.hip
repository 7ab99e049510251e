// sha_valu_bench.hip — register-only SHA-256 compression throughput vs occupancy (waves/SIMD).
// Measures what the VALU can sustain for the exact compression code of sha256.hpp with no memory,
// to separate instruction-mix / latency limits from the leaf kernel's staging and LDS costs.
// Build: hipcc -O3 --offload-arch=gfx950 -I../merklekv_amd/csrc tools/sha_valu_bench.hip -o /tmp/svb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "sha256.hpp"

using namespace mkv;

template <bool SHORT>
__global__ __launch_bounds__(256) void k_bench(uint32_t *out, int iters) {
    extern __shared__ uint32_t pad[];  // dynamic LDS only limits occupancy
    uint32_t s[8], w[16];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    sha_init(s);
    for (int i = 0; i < 16; ++i) w[i] = t * 0x9E3779B9u + i;
    for (int it = 0; it < iters; ++it) {
        sha_compress<SHORT>(s, w);
        w[it & 15] ^= s[it & 7];
    }
    uint32_t x = s[0] ^ s[1] ^ s[2] ^ s[3] ^ s[4] ^ s[5] ^ s[6] ^ s[7];
    if (x == 0x12345678u) pad[0] = x;  // keep the LDS live
    out[t] = x;
}

int main() {
    const int iters = 200;
    uint32_t *out;
    hipMalloc(&out, 256 * 256 * 64 * sizeof(uint32_t));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int lds_for[] = {160 * 1024, 80 * 1024, 40 * 1024, 20 * 1024, 0};
    int wps[] = {1, 2, 4, 8, 8};
    for (int variant = 0; variant < 2; ++variant) {
        for (int c = 0; c < 5; ++c) {
            int lds = lds_for[c];
            int blocks = 256 * (c < 4 ? wps[c] : 8) * 4;  // 4 rounds of full residency
            auto kern = variant ? k_bench<true> : k_bench<false>;
            if (lds > 64 * 1024) hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, out, iters);
            hipDeviceSynchronize();
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            double comps = (double)blocks * 256 * iters;
            printf("variant %d  lds/WG %6d  ~waves/SIMD %d  %.3f ms  %.2f G compressions/s  (%.1f ns/comp/lane-slot)\n",
                   variant, lds, wps[c], ms, comps / ms / 1e6, ms * 1e6 / comps * 256 * 1024 / 64);
        }
    }
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
