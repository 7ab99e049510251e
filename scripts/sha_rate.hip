// Register-only SHA-256 throughput on gfx950: the ceiling the leaf / reduce / climb kernels are held
// against. k_node<SHORT> hashes 64-B nodes (sha_node: one scheduled block + the constant padding block)
// in a dependent loop per lane, no memory traffic; `waves` = resident waves per SIMD (grid sized so
// every SIMD holds that many, LDS caps the blocks per CU). Prints one JSON line: node hashes/s, compressions/s, and the VALU
// wave-instruction count per node from the kernel itself is left to the ISA dump.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../merklekv_amd/csrc/sha256.hpp"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

using namespace mkv;

constexpr int ITERS = 64;

template <bool SHORT>
__global__ __launch_bounds__(256) void k_node(uint32_t *out, uint32_t seed) {
    uint32_t l[8], r[8], o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        l[i] = threadIdx.x * 0x9E3779B9u + i + seed;
        r[i] = blockIdx.x * 0x85EBCA6Bu + i;
    }
    for (int it = 0; it < ITERS; ++it) {
        sha_node<SHORT>(l, r, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            r[i] = l[i];
            l[i] = o[i];
        }
    }
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v ^= l[i];
    if (v == 0x12345678u) out[0] = v;
}

int main() {
    uint32_t *out = nullptr;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("{");
    bool first = true;
    for (int sh = 0; sh < 2; ++sh) {
        for (int waves : {3, 4, 6, 8}) {
            // 256 CUs x 4 SIMDs x `waves` resident waves: 4 waves per block (one per SIMD), the block count
            // per CU capped by dynamic LDS (160 KiB per CU); 8 rounds of residency
            const uint32_t blocks = 256 * waves * 8;
            const size_t lds = 160 * 1024 / waves - 512;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(e0));
                if (sh)
                    hipLaunchKernelGGL(k_node<true>, dim3(blocks), dim3(256), lds, 0, out, 3u + rep);
                else
                    hipLaunchKernelGGL(k_node<false>, dim3(blocks), dim3(256), lds, 0, out, 3u + rep);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep && ms < best) best = ms;
            }
            const double nodes = (double)blocks * 256 * ITERS;
            std::printf("%s\"%s_w%d\": {\"ms\": %.4f, \"nodes_per_s\": %.4g, \"compressions_per_s\": %.4g}",
                        first ? "" : ", ", sh ? "short" : "plain", waves, best, nodes / (best * 1e-3),
                        2 * nodes / (best * 1e-3));
            first = false;
        }
    }
    std::printf("}\n");
    CK(hipFree(out));
    return 0;
}
