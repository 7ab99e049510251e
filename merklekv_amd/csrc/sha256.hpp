// sha256.hpp — FIPS 180-4 SHA-256 compression for gfx950, one message per lane.
//
// The digest is the one the reference takes from sha2 0.10.9 (merkle.rs:1, :45-49, :99-103;
// Cargo.lock:1227-1230). Everything is 32-bit integer VALU work: rotates lower to v_alignbit_b32,
// Ch/Maj to v_bfi_b32, the three-way sums to v_add3_u32 / v_xor3_b32. No MFMA: SHA-256 has no
// GEMM structure.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mkv {

__host__ __device__ constexpr uint32_t k256(int t) {
    constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    return K[t];
}

__host__ __device__ constexpr uint32_t h256(int i) {
    constexpr uint32_t H[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    return H[i];
}

__host__ __device__ constexpr uint32_t crotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// K[t] + W[t] for the constant second block of a 64-byte message (0x80, zeros, bit length 512):
// every internal node (R4) hashes exactly 64 bytes, so its padding block's schedule is known at
// compile time and costs no schedule ops.
struct Sched64 {
    uint32_t v[64];
};
__host__ __device__ constexpr Sched64 make_pad64_kw() {
    Sched64 s{};
    uint32_t w[64] = {};
    w[0] = 0x80000000u;
    w[15] = 512u;
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = crotr(w[t - 15], 7) ^ crotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = crotr(w[t - 2], 17) ^ crotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    for (int t = 0; t < 64; ++t) s.v[t] = k256(t) + w[t];
    return s;
}

// Constant-amount rotate: clang emits llvm.fshr, which lowers to one v_alignbit_b32.
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return (x >> n) | (x << (32 - n)); }

// gfx950 v_bitop3_b32: D = LUT[4*S0 + 2*S1 + S2] per bit. hipcc does not fold x^y^z, Ch or Maj into
// it (it emits two v_xor_b32 per three-way xor), so the three-input functions are written directly:
// XOR3 = 0x96, Ch(e,f,g) = e ? f : g = 0xCA, Maj = 0xE8. One VALU op each.
__device__ __forceinline__ uint32_t bitop3_96(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t bitop3_ca(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t bitop3_e8(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return bitop3_96(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return bitop3_96(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t w) { return bitop3_96(rotr(w, 7), rotr(w, 18), w >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t w) { return bitop3_96(rotr(w, 17), rotr(w, 19), w >> 10); }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return bitop3_ca(e, f, g); }
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return bitop3_e8(a, b, c); }

__device__ __forceinline__ void sha_init(uint32_t s[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = h256(i);
}

__device__ __forceinline__ uint32_t add3_asm(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t add3_asm_s(uint32_t a, uint32_t k, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t add_asm(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// One SHA-256 round. Variant SHORT (true): hkw = h + K + W and dhkw = d + hkw depend only on values
// known a round earlier, so new e = Σ1(e) + Ch(e,f,g) + dhkw and new a = T1 + Σ0(a) + Maj(a,b,c) are
// alignbit -> bitop3 -> add3 (3 dependent VALU levels) from the previous state; the association is
// pinned with inline asm because LLVM re-associates the sums back into a 5-level chain
// (add3(w,h,Σ1) -> add3(.,Ch,K) -> +d). Variant false: plain C, LLVM's own association.
// Registers rotate by renaming: the new a goes into h's slot and the new e into d's slot.
template <bool SHORT>
__device__ __forceinline__ void sha_round(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                          uint32_t &f, uint32_t &g, uint32_t &h, uint32_t k, uint32_t w) {
    if constexpr (SHORT) {
        const uint32_t hkw = add3_asm_s(h, k, w);
        const uint32_t dhkw = add_asm(d, hkw);
        const uint32_t s1 = bsig1(e), c1 = ch(e, f, g);
        const uint32_t t1 = add3_asm(s1, c1, hkw);
        d = add3_asm(s1, c1, dhkw);
        h = add3_asm(t1, bsig0(a), maj(a, b, c));
    } else {
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + k + w;
        d = d + t1;
        h = t1 + bsig0(a) + maj(a, b, c);
    }
}

#ifndef MKV_SHA_SHORT_DEFAULT
#define MKV_SHA_SHORT_DEFAULT true
#endif

// One compression over the 16 big-endian message words in w (w is clobbered: rolling schedule).
template <bool SHORT = MKV_SHA_SHORT_DEFAULT>
__device__ __forceinline__ void sha_compress(uint32_t s[8], uint32_t w[16]) {
    uint32_t v[8] = {s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
            w[t & 15] = wt;
        }
        const int A = (64 - t) & 7;  // slot of a at round t
        sha_round<SHORT>(v[A], v[(A + 1) & 7], v[(A + 2) & 7], v[(A + 3) & 7], v[(A + 4) & 7], v[(A + 5) & 7],
                         v[(A + 6) & 7], v[(A + 7) & 7], k256(t), wt);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += v[i];  // 64 % 8 == 0: the renaming is back at the origin
}

// The constant padding block of a 64-byte message (schedule folded into K+W immediates).
template <bool SHORT = MKV_SHA_SHORT_DEFAULT>
__device__ __forceinline__ void sha_compress_pad64(uint32_t s[8]) {
    constexpr Sched64 KW = make_pad64_kw();
    uint32_t v[8] = {s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        const int A = (64 - t) & 7;
        sha_round<SHORT>(v[A], v[(A + 1) & 7], v[(A + 2) & 7], v[(A + 3) & 7], v[(A + 4) & 7], v[(A + 5) & 7],
                         v[(A + 6) & 7], v[(A + 7) & 7], KW.v[t], 0u);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += v[i];
}

// R4 (merkle.rs:99-103): parent = SHA-256(left32 || right32). l/r are the children's digest words
// already in big-endian word form (i.e. bswapped from the canonical byte order).
template <bool SHORT = MKV_SHA_SHORT_DEFAULT>
__device__ __forceinline__ void sha_node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        w[i] = l[i];
        w[8 + i] = r[i];
    }
    sha_init(out);
    sha_compress<SHORT>(out, w);
    sha_compress_pad64<SHORT>(out);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Load / store a 32-byte digest kept in canonical byte order in HBM, converting to/from BE words.
__device__ __forceinline__ void load_digest(const uint8_t *p, uint32_t w[8]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 x = q[0], y = q[1];
    w[0] = bswap32(x.x); w[1] = bswap32(x.y); w[2] = bswap32(x.z); w[3] = bswap32(x.w);
    w[4] = bswap32(y.x); w[5] = bswap32(y.y); w[6] = bswap32(y.z); w[7] = bswap32(y.w);
}
__device__ __forceinline__ void store_digest(uint8_t *p, const uint32_t w[8]) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
    q[0] = make_uint4(bswap32(w[0]), bswap32(w[1]), bswap32(w[2]), bswap32(w[3]));
    q[1] = make_uint4(bswap32(w[4]), bswap32(w[5]), bswap32(w[6]), bswap32(w[7]));
}

}  // namespace mkv
