// PMC calibration for the access widths of the dirty climb (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE
// are calibrated only for 16-B-per-lane streaming; "other access widths are uncalibrated"). Each kernel
// touches a known number of bytes of a 4 GiB array (far beyond the 256 MiB Infinity Cache), every lane at
// a distinct 64-B slot (odd-multiplier scramble: a bijection mod 2^k, no slot twice):
//   rd32     32 B read per lane (the climb's sibling read: two 16-B loads of one 32-B digest)
//   wr32     32 B written per lane (the climb's node store)
//   rd64     64 B read per lane (a node + its sibling)
//   rdstream 16 B per lane, coalesced (the guide's calibrated case)
// Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) and divide by the printed byte counts.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t slot(uint64_t i, uint64_t mask) { return (i * 0x9E3779B97F4A7C15ull) & mask; }

__global__ void rd32(const uint4 *__restrict__ a, uint64_t mask, uint32_t *out) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x, s = slot(i, mask);
    const uint4 x = a[4 * s], y = a[4 * s + 1];
    const uint32_t v = x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w;
    if (v == 0x9E3779B9u) out[0] = v;  // keeps the loads
}
__global__ void rd64(const uint4 *__restrict__ a, uint64_t mask, uint32_t *out) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x, s = slot(i, mask);
    const uint4 x = a[4 * s], y = a[4 * s + 1], z = a[4 * s + 2], w = a[4 * s + 3];
    const uint32_t v = x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.w ^ w.y ^ w.z;
    if (v == 0x9E3779B9u) out[0] = v;
}
__global__ void wr32(uint4 *__restrict__ a, uint64_t mask) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x, s = slot(i, mask);
    a[4 * s] = make_uint4((uint32_t)i, 1, 2, 3);
    a[4 * s + 1] = make_uint4(4, 5, 6, (uint32_t)s);
}
__global__ void rdstream(const uint4 *__restrict__ a, uint32_t *out) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    const uint4 x = a[i];
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x9E3779B9u) out[0] = 1;
}

int main() {
    const uint64_t slots = 1ull << 26, bytes = slots * 64;  // 4 GiB of 64-B slots
    const uint64_t lanes = 1ull << 24;                       // 16M lanes
    uint4 *a = nullptr;
    uint32_t *out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipDeviceSynchronize());
    const dim3 g((uint32_t)(lanes / 256)), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd32, g, b, 0, 0, a, slots - 1, out);
        hipLaunchKernelGGL(rd64, g, b, 0, 0, a, slots - 1, out);
        hipLaunchKernelGGL(wr32, g, b, 0, 0, a, slots - 1);
        hipLaunchKernelGGL(rdstream, g, b, 0, 0, a, out);
        CK(hipDeviceSynchronize());
    }
    std::printf("{\"lanes\": %llu, \"rd32_bytes\": %llu, \"rd64_bytes\": %llu, \"wr32_bytes\": %llu, "
                "\"rdstream_bytes\": %llu}\n",
                (unsigned long long)lanes, (unsigned long long)(lanes * 32), (unsigned long long)(lanes * 64),
                (unsigned long long)(lanes * 32), (unsigned long long)(lanes * 16));
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
