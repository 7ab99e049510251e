// PCIe write ceiling (diagnostic): 3.2 MB (100K x 32-B keys, the 100M value-only diff's result) from HBM into
// mapped pinned host memory — kernel stores of 16 B per thread at different grid sizes, and one SDMA copy —
// timed with HIP events over 50 repetitions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
__global__ void k_copy16_nt(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        __builtin_nontemporal_store(v.x, &dst[i].x);
        __builtin_nontemporal_store(v.y, &dst[i].y);
        __builtin_nontemporal_store(v.z, &dst[i].z);
        __builtin_nontemporal_store(v.w, &dst[i].w);
    }
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
    const uint64_t sizes[3] = {800000, 3200000, 32000000};
    for (uint64_t bytes : sizes) {
        uint8_t *d, *h, *hd;
        CK(hipMalloc(&d, bytes));
        CK(hipMemset(d, 1, bytes));
        CK(hipHostMalloc(&h, bytes, hipHostMallocMapped));
        CK(hipHostGetDevicePointer((void **)&hd, h, 0));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        const uint64_t n16 = bytes / 16;
        const int grids[4] = {256, 1024, 2048, (int)((n16 + 255) / 256)};
        for (int nt = 0; nt < 2; ++nt)
            for (int g : grids) {
                for (int w = 0; w < 3; ++w) {
                    if (nt) hipLaunchKernelGGL(k_copy16_nt, dim3(g), dim3(256), 0, 0, (const uint4 *)d, (uint4 *)hd, n16);
                    else hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, 0, (const uint4 *)d, (uint4 *)hd, n16);
                }
                CK(hipEventRecord(a, 0));
                for (int r = 0; r < 50; ++r) {
                    if (nt) hipLaunchKernelGGL(k_copy16_nt, dim3(g), dim3(256), 0, 0, (const uint4 *)d, (uint4 *)hd, n16);
                    else hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, 0, (const uint4 *)d, (uint4 *)hd, n16);
                }
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                printf("bytes %9llu kernel%s grid %6d: %7.2f us  %6.1f GB/s\n", (unsigned long long)bytes, nt ? "-nt" : "   ", g,
                       ms * 1e3 / 50, bytes / (ms * 1e-3 / 50) / 1e9);
            }
        for (int w = 0; w < 3; ++w) CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0));
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < 50; ++r) CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("bytes %9llu memcpy D2H      : %7.2f us  %6.1f GB/s\n", (unsigned long long)bytes, ms * 1e3 / 50,
               bytes / (ms * 1e-3 / 50) / 1e9);
        CK(hipFree(d));
        CK(hipHostFree(h));
    }
    return 0;
}
