// sha256.hpp — FIPS 180-4 SHA-256 compression for gfx950, one message per lane.
//
// The digest is the one the reference takes from sha2 0.10.9 (merkle.rs:1, :45-49, :99-103;
// Cargo.lock:1227-1230). Everything is 32-bit integer VALU work: rotates lower to v_alignbit_b32,
// Ch/Maj to v_bfi_b32, the three-way sums to v_add3_u32 / v_xor3_b32. No MFMA: SHA-256 has no
// GEMM structure.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

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

// Round whose message word is a compile-time constant: kw = K[t] + W[t] is one literal, so h + K + W is a
// plain v_add (fast) instead of a v_add3 with a materialised zero or constant.
template <bool SHORT>
__device__ __forceinline__ void sha_round_kw(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                             uint32_t &f, uint32_t &g, uint32_t &h, uint32_t kw) {
    if constexpr (SHORT) {
        const uint32_t hkw = h + kw;
        const uint32_t dhkw = add_asm(d, hkw);
        const uint32_t s1 = bsig1(e), c1 = ch(e, f, g);
        const uint32_t t1 = add3_asm(s1, c1, hkw);
        d = add3_asm(s1, c1, dhkw);
        h = add3_asm(t1, bsig0(a), maj(a, b, c));
    } else {
        const uint32_t t1 = h + bsig1(e) + ch(e, f, g) + kw;
        d = d + t1;
        h = t1 + bsig0(a) + maj(a, b, c);
    }
}

// Plain-C round (no inline asm): the compiler folds it completely when the state and W are constants,
// e.g. round 0 of a message's first block when the first word (a length field) is known.
__host__ __device__ constexpr void sha_round_c(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                               uint32_t &f, uint32_t &g, uint32_t &h, uint32_t k, uint32_t w) {
    const uint32_t t1 = h + (crotr(e, 6) ^ crotr(e, 11) ^ crotr(e, 25)) + ((e & f) ^ (~e & g)) + k + w;
    const uint32_t t2 = (crotr(a, 2) ^ crotr(a, 13) ^ crotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    d = d + t1;
    h = t1 + t2;
}

__host__ __device__ constexpr uint32_t cssig0(uint32_t w) { return crotr(w, 7) ^ crotr(w, 18) ^ (w >> 3); }
__host__ __device__ constexpr uint32_t cssig1(uint32_t w) { return crotr(w, 17) ^ crotr(w, 19) ^ (w >> 10); }

// Compile-time knowledge of a message block: which of its 16 words are constants (length fields,
// terminator, zero padding, bit length of a fixed-shape record) and their values, expanded through the
// message schedule (W[t] is known iff its four inputs are).
struct MsgKnown {
    uint32_t mask;  // bit i: word i is known
    uint32_t val[16];
};
struct SchedKnown {
    bool known[64];
    uint32_t val[64];
};
__host__ __device__ constexpr SchedKnown expand_known(const MsgKnown &m) {
    SchedKnown s{};
    for (int t = 0; t < 16; ++t) {
        s.known[t] = (m.mask >> t) & 1u;
        s.val[t] = s.known[t] ? m.val[t] : 0u;
    }
    for (int t = 16; t < 64; ++t) {
        s.known[t] = s.known[t - 2] && s.known[t - 7] && s.known[t - 15] && s.known[t - 16];
        s.val[t] = s.known[t] ? cssig1(s.val[t - 2]) + s.val[t - 7] + cssig0(s.val[t - 15]) + s.val[t - 16] : 0u;
    }
    return s;
}

// One round of a partly known block. Known schedule terms are summed at compile time (one literal);
// a known W[t] folds into the round constant; unknown words come from the rolling ring w[16].
template <bool SHORT, class KS, int T>
__device__ __forceinline__ void sha_step_known(uint32_t v[8], uint32_t w[16]) {
    constexpr SchedKnown S = KS::value;
    constexpr int A = (64 - T) & 7;
    if constexpr (S.known[T]) {
        sha_round_kw<SHORT>(v[A], v[(A + 1) & 7], v[(A + 2) & 7], v[(A + 3) & 7], v[(A + 4) & 7], v[(A + 5) & 7],
                            v[(A + 6) & 7], v[(A + 7) & 7], k256(T) + S.val[T]);
    } else {
        uint32_t wt;
        if constexpr (T < 16) {
            wt = w[T];
        } else {
            constexpr uint32_t cs = (S.known[T - 2] ? cssig1(S.val[T - 2]) : 0u) + (S.known[T - 7] ? S.val[T - 7] : 0u) +
                                    (S.known[T - 15] ? cssig0(S.val[T - 15]) : 0u) + (S.known[T - 16] ? S.val[T - 16] : 0u);
            uint32_t x = cs;
            if constexpr (!S.known[T - 2]) x += ssig1(w[(T - 2) & 15]);
            if constexpr (!S.known[T - 7]) x += w[(T - 7) & 15];
            if constexpr (!S.known[T - 15]) x += ssig0(w[(T - 15) & 15]);
            if constexpr (!S.known[T - 16]) x += w[T & 15];
            wt = x;
            w[T & 15] = wt;
        }
        sha_round<SHORT>(v[A], v[(A + 1) & 7], v[(A + 2) & 7], v[(A + 3) & 7], v[(A + 4) & 7], v[(A + 5) & 7],
                         v[(A + 6) & 7], v[(A + 7) & 7], k256(T), wt);
    }
}

template <bool SHORT, class KS, int... T>
__device__ __forceinline__ void sha_steps_known(uint32_t v[8], uint32_t w[16], std::integer_sequence<int, T...>) {
    (sha_step_known<SHORT, KS, T>(v, w), ...);
}

// Compression of a partly known block. FIRST: s holds the initial hash value H0 (a message's first
// block) — with a known W[0], rounds 0 and 1 then run in plain C, which the compiler folds to constants
// (round 0) and two adds (round 1).
template <bool SHORT, class KS, bool FIRST>
__device__ __forceinline__ void sha_compress_known(uint32_t s[8], uint32_t w[16]) {
    constexpr SchedKnown S = KS::value;
    uint32_t v[8] = {s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
    if constexpr (FIRST && S.known[0]) {
        // rounds 0 and 1 with the renaming of sha_compress (slot of a at round t = (64 - t) & 7)
        sha_round_c(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], k256(0), S.val[0]);
        uint32_t w1 = S.known[1] ? S.val[1] : w[1];
        sha_round_c(v[7], v[0], v[1], v[2], v[3], v[4], v[5], v[6], k256(1), w1);
        sha_steps_known<SHORT, KS>(v, w, std::integer_sequence<int, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17,
                                                            18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
                                                            35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51,
                                                            52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63>{});
    } else {
        sha_steps_known<SHORT, KS>(v, w, std::make_integer_sequence<int, 64>{});
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += v[i];
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
        sha_round_kw<SHORT>(v[A], v[(A + 1) & 7], v[(A + 2) & 7], v[(A + 3) & 7], v[(A + 4) & 7], v[(A + 5) & 7],
                            v[(A + 6) & 7], v[(A + 7) & 7], KW.v[t]);
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
