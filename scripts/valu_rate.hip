// Integer VALU issue rate on gfx950, per instruction kind (the SHA-256 kernels' whole diet: the leaf kernel
// is v_alignbit_b32 38 %, v_bitop3_b32 23 %, v_add3_u32 16 %, v_add_u32 8 %, v_lshrrev_b32 6 %): is the
// 78.6 T lane-ops/s figure (256 CU x 128 lanes x 2.4 GHz, the f32 FMA rate) reachable for v_bitop3 /
// v_add3 / v_alignbit, or do the 3-operand integer forms issue at a lower rate? Each lane runs 8
// independent chains (no dependency stall with >= 2 waves per SIMD); 8 waves per SIMD.
// Prints one JSON line: lane-ops/s per kind and the fraction of 78.6 T.
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

constexpr int ITERS = 2048;

#define OP8(INS)                                                                               \
    asm volatile(INS " %0, %0, %8, %9\n" INS " %1, %1, %8, %9\n" INS " %2, %2, %8, %9\n" INS    \
                 " %3, %3, %8, %9\n" INS " %4, %4, %8, %9\n" INS " %5, %5, %8, %9\n" INS        \
                 " %6, %6, %8, %9\n" INS " %7, %7, %8, %9\n"                                   \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(b), "v"(c))
#define OP8_2(INS)                                                                             \
    asm volatile(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                 INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(b))

#define OP8_B3(IMM)                                                                            \
    asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:" IMM "\n v_bitop3_b32 %1, %1, %8, %9 bitop3:" IMM \
                 "\n v_bitop3_b32 %2, %2, %8, %9 bitop3:" IMM "\n v_bitop3_b32 %3, %3, %8, %9 bitop3:" IMM \
                 "\n v_bitop3_b32 %4, %4, %8, %9 bitop3:" IMM "\n v_bitop3_b32 %5, %5, %8, %9 bitop3:" IMM \
                 "\n v_bitop3_b32 %6, %6, %8, %9 bitop3:" IMM "\n v_bitop3_b32 %7, %7, %8, %9 bitop3:" IMM "\n" \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(b), "v"(c))

// 64-bit operand forms: 4 independent register pairs
#define OP4_64(INS)                                                                            \
    asm volatile(INS " %0, %4, %0\n" INS " %1, %4, %1\n" INS " %2, %4, %2\n" INS " %3, %4, %3\n" \
                 : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3)                                      \
                 : "v"(b))

#define KERNEL(NAME, BODY)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                \
        uint32_t r0 = threadIdx.x ^ seed, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,  \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                                        \
        const uint32_t b = seed * 3 + blockIdx.x, c = seed ^ 0x5bd1e995u;                      \
        for (int i = 0; i < ITERS; ++i) { BODY; }                                              \
        const uint32_t v = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;                              \
        if (v == 0x12345678u) out[0] = v;                                                      \
    }

KERNEL(k_add, OP8_2("v_add_u32"))
KERNEL(k_xor, OP8_2("v_xor_b32"))
KERNEL(k_xor3, OP8_B3("0x96"))
KERNEL(k_add3, OP8("v_add3_u32"))
KERNEL(k_alignbit, OP8("v_alignbit_b32"))
KERNEL(k_bfi, OP8_B3("0xca"))
KERNEL(k_fma, OP8("v_fma_f32"))
KERNEL(k_lshr, OP8_2("v_lshrrev_b32"))
KERNEL(k_lshl_or, OP8("v_lshl_or_b32"))
KERNEL(k_lshl_add, OP8("v_lshl_add_u32"))
KERNEL(k_perm, OP8("v_perm_b32"))
KERNEL(k_xad, OP8("v_xad_u32"))
KERNEL(k_and_or, OP8("v_and_or_b32"))
KERNEL(k_alignbyte, OP8("v_alignbyte_b32"))

// 64-bit shifts: lo word of (x:x) >> n is rotr(x, n); 4 pairs = 8 dwords per iteration, counted as 4 ops
__global__ __launch_bounds__(256) void k_lshr64(uint32_t *out, uint32_t seed) {
    uint64_t q0 = threadIdx.x ^ seed, q1 = q0 + 1, q2 = q0 + 2, q3 = q0 + 3;
    const uint32_t b = (seed & 7) + 1;
    for (int i = 0; i < ITERS; ++i) {
        OP4_64("v_lshrrev_b64");
        OP4_64("v_lshrrev_b64");
    }
    const uint64_t v = q0 ^ q1 ^ q2 ^ q3;
    if (v == 0x12345678u) out[0] = (uint32_t)v;
}

int main() {
    uint32_t *out = nullptr;
    CK(hipMalloc(&out, 64));
    const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD: 256 CU x 4 SIMD x 8 waves / 4 waves per block
    void (*ks[])(uint32_t *, uint32_t) = {k_add,     k_xor,      k_xor3, k_add3, k_alignbit, k_bfi,       k_fma,
                                          k_lshr,    k_lshl_or,  k_lshl_add, k_perm, k_xad, k_and_or, k_alignbyte,
                                          k_lshr64};
    const char *names[] = {"v_add_u32",     "v_xor_b32",      "v_bitop3_b32 (xor3)", "v_add3_u32",
                           "v_alignbit_b32", "v_bitop3_b32 (ch)", "v_fma_f32",         "v_lshrrev_b32",
                           "v_lshl_or_b32",  "v_lshl_add_u32", "v_perm_b32",          "v_xad_u32",
                           "v_and_or_b32",   "v_alignbyte_b32", "v_lshrrev_b64 (per 64-bit op)"};
    const int nk = (int)(sizeof(ks) / sizeof(ks[0]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("{");
    for (int k = 0; k < nk; ++k) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[k], dim3(blocks * 4), dim3(256), 0, 0, out, 7u + rep);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep && ms < best) best = ms;
        }
        const double ops = (double)blocks * 4 * 256 * ITERS * 8;
        const double rate = ops / (best * 1e-3);
        std::printf("%s\"%s\": {\"ms\": %.4f, \"lane_ops_per_s\": %.4g, \"frac_of_78.6T\": %.3f}", k ? ", " : "",
                    names[k], best, rate, rate / 78.6e12);
    }
    std::printf("}\n");
    CK(hipFree(out));
    return 0;
}
