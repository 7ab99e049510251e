// valu_op_bench.hip — per-instruction VALU throughput on gfx950 (8 independent chains per lane,
// 8 waves/SIMD). Reports wave-instructions per SIMD-cycle at the effective clock (s_memtime).
#include <hip/hip_runtime.h>

#include <cstdio>

#define OP_LOOP(ASM)                                                                     \
    for (int it = 0; it < iters; ++it) {                                                 \
        _Pragma("unroll") for (int r = 0; r < 8; ++r) {                                  \
            asm volatile(ASM : "+v"(x0) : "v"(x1), "v"(x2));                             \
            asm volatile(ASM : "+v"(x1) : "v"(x2), "v"(x3));                             \
            asm volatile(ASM : "+v"(x2) : "v"(x3), "v"(x4));                             \
            asm volatile(ASM : "+v"(x3) : "v"(x4), "v"(x5));                             \
            asm volatile(ASM : "+v"(x4) : "v"(x5), "v"(x6));                             \
            asm volatile(ASM : "+v"(x5) : "v"(x6), "v"(x7));                             \
            asm volatile(ASM : "+v"(x6) : "v"(x7), "v"(x0));                             \
            asm volatile(ASM : "+v"(x7) : "v"(x0), "v"(x1));                             \
        }                                                                                \
    }

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t *out, int iters, unsigned long long *clk) {
    uint32_t t = threadIdx.x + blockIdx.x * 256;
    uint32_t x0 = t, x1 = t * 3, x2 = t * 5, x3 = t * 7, x4 = t * 11, x5 = t * 13, x6 = t * 17, x7 = t * 19;
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    if (OP == 0) OP_LOOP("v_add_u32_e32 %0, %1, %0")
    if (OP == 1) OP_LOOP("v_xor_b32_e32 %0, %1, %0")
    if (OP == 2) OP_LOOP("v_alignbit_b32 %0, %1, %0, 7")
    if (OP == 3) OP_LOOP("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96")
    if (OP == 4) OP_LOOP("v_add3_u32 %0, %1, %2, %0")
    if (OP == 5) OP_LOOP("v_lshrrev_b32_e32 %0, 3, %0")
    if (OP == 6) OP_LOOP("v_fma_f32 %0, %1, %2, %0")
    if (OP == 7) OP_LOOP("v_xad_u32 %0, %1, %2, %0")
    if (OP == 8) OP_LOOP("v_perm_b32 %0, %1, %2, %0")
    if (OP == 9) OP_LOOP("v_bfi_b32 %0, %1, %2, %0")
    if (OP == 10) OP_LOOP("v_pk_add_u16 %0, %1, %0")
    if (OP == 11) OP_LOOP("v_lshl_add_u32 %0, %1, 3, %0")
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    out[t] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (threadIdx.x == 0 && blockIdx.x == 0) *clk = c1 - c0;
}

static const char *names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_add3_u32",
                              "v_lshrrev_b32", "v_fma_f32", "v_xad_u32", "v_perm_b32", "v_bfi_b32",
                              "v_pk_add_u16", "v_lshl_add_u32"};

template <int OP> void run(uint32_t *out, unsigned long long *clk) {
    const int iters = 400, blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves/SIMD
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c;
    hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    double winstr = (double)blocks * 4 * iters * 64;  // wave-instructions
    double per_simd = winstr / 1024;
    printf("%-16s %8.3f ms  %.3f T lane-ops/s  %.2f SIMD-cycles/wave-instr @2.4GHz  (wave0 %.0f cyc/instr)\n",
           names[OP], ms, winstr * 64 / ms / 1e9, ms * 1e-3 * 2.4e9 / per_simd, (double)c / (iters * 64));
}

int main() {
    uint32_t *out;
    unsigned long long *clk;
    hipMalloc(&out, 256 * 256 * 8 * 4);
    hipMalloc(&clk, 8);
    run<0>(out, clk); run<1>(out, clk); run<2>(out, clk); run<3>(out, clk); run<4>(out, clk); run<5>(out, clk);
    run<6>(out, clk); run<7>(out, clk); run<8>(out, clk); run<9>(out, clk); run<10>(out, clk); run<11>(out, clk);
    printf("status %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
