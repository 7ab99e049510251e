// k_leaf.hip — Kernel A: batched leaf hashing (R1 + R2), fixed-shape path and update batches.
//
// Restates merkle.rs:7-16 (encode_leaf) fused into merkle.rs:45-49 (compute_leaf_hash): the digest of
// u32_be(|k|) || k || u32_be(|v|) || v, computed without ever materialising the encoding.
//
// Records arrive as two packed blobs with u64 offsets (keys kb/koff, values vb/voff), exactly the mkv_blob
// pair of the C ABI. A leaf stage is two kernels on one stream:
//   k_leaf_direct (here) — the configs' record shape (32-B keys / 100-B values, 4-B aligned): one lane per
//       record, the message loaded straight into VGPRs, every constant word folded at compile time. The
//       first wave that meets a chunk of any other shape stops the kernel's chunk hand-out (leaf.hpp);
//   k_leaf_ragged (k_ragged.hip) — every chunk k_leaf_direct did not hash, any shape.
// k_leaf_multi hashes the (small) value batches of several replicas' dirty-path updates in one launch:
// LDS-staged 64-record tiles, a runtime-uniform fast path or byte-range assembly.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "leaf.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

constexpr int LEAF_WAVES = 4;                 // waves per workgroup
// LDS per wave of k_leaf_multi's staging: 64 x 132-B records + alignment slack (8,512 B) fit.
constexpr uint32_t LEAF_LDS_WAVE = 9216;

// Big-endian word of the 4 bytes at byte offset `off` of an LDS byte region starting at `base` (bytes).
__device__ __forceinline__ uint32_t lds_be_word(const uint32_t *lds, uint32_t byte) {
    uint32_t a = byte >> 2, sh = byte & 3;
    uint32_t lo = lds[a], hi = lds[a + 1];
    return __builtin_amdgcn_perm(hi, lo, 0x00010203u + sh * 0x01010101u);
}

// Same from global memory, never touching a 4-byte chunk that lies wholly past `end`.
__device__ __forceinline__ uint32_t glb_be_word(const uint8_t *p, const uint8_t *end) {
    uintptr_t ad = reinterpret_cast<uintptr_t>(p);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(ad & 3);
    uint32_t lo = (reinterpret_cast<const uint8_t *>(a) < end) ? a[0] : 0u;
    uint32_t hi = (reinterpret_cast<const uint8_t *>(a + 1) < end) ? a[1] : 0u;
    return __builtin_amdgcn_perm(hi, lo, 0x00010203u + sh * 0x01010101u);
}

// Mask of the first n (0..4) bytes of a big-endian word.
__device__ __forceinline__ uint32_t head_mask(int n) {
    return n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : ~(0xFFFFFFFFu >> (8 * n)));
}

struct LdsSrc {
    const uint32_t *lds;
    uint32_t kbyte, vbyte;  // byte offsets of this lane's key / value inside the wave's region
    __device__ __forceinline__ uint32_t key(uint32_t q, uint32_t) const { return lds_be_word(lds, kbyte + q); }
    __device__ __forceinline__ uint32_t val(uint32_t q, uint32_t) const { return lds_be_word(lds, vbyte + q); }
};

struct GlbSrc {
    const uint8_t *k, *v;
    const uint8_t *kend, *vend;
    __device__ __forceinline__ uint32_t key(uint32_t q, uint32_t) const { return glb_be_word(k + q, kend); }
    __device__ __forceinline__ uint32_t val(uint32_t q, uint32_t) const { return glb_be_word(v + q, vend); }
};

// Generic message word at byte position p (multiple of 4) of the padded encoding.
template <class Src>
__device__ __forceinline__ uint32_t msg_word(const Src &src, uint32_t p, uint32_t klen, uint32_t vlen, uint32_t L) {
    uint32_t w = 0;
    if (p == 0) w = klen;  // u32_be(|k|), bytes [0,4)
    // key bytes at [4, 4+klen): stream offset qk = p - 4 (multiple of 4, >= 0 once p >= 4)
    if (p >= 4 && p - 4 < klen) {
        uint32_t qk = p - 4;
        w |= src.key(qk, klen) & head_mask((int)(klen - qk));
    }
    // u32_be(|v|) at [4+klen, 8+klen)
    int d = (int)(4 + klen) - (int)p;
    if (d >= 0 && d < 4) w |= vlen >> (8 * d);
    else if (d < 0 && d > -4) w |= vlen << (8 * -d);
    // value bytes at [8+klen, L)
    int qv = (int)p - (int)(8 + klen);
    if (qv > -4 && qv < (int)vlen) {
        int s = qv < 0 ? -qv : 0;                     // first byte of the word that is value data
        uint32_t raw = src.val((uint32_t)(qv < 0 ? 0 : qv), vlen);
        raw = s ? (raw >> (8 * s)) : raw;
        int e = (int)vlen - qv;                       // one past the last value byte, word-relative
        uint32_t m = head_mask(e < 4 ? e : 4) & ~head_mask(s);
        w |= raw & m;
    }
    // 0x80 terminator at L
    int d2 = (int)L - (int)p;
    if (d2 >= 0 && d2 < 4) w |= 0x80000000u >> (8 * d2);
    return w;
}

template <bool SHORT, class Src>
__device__ __forceinline__ void hash_generic(const Src &src, uint32_t klen, uint32_t vlen, uint32_t out[8]) {
    uint32_t L = 8 + klen + vlen;
    uint32_t nb = (L + 9 + 63) >> 6;
    uint64_t bits = (uint64_t)L * 8;
    sha_init(out);
    for (uint32_t blk = 0; blk < nb; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = msg_word(src, blk * 64 + 4 * i, klen, vlen, L);
        if (blk == nb - 1) {
            w[14] |= (uint32_t)(bits >> 32);
            w[15] |= (uint32_t)bits;
        }
        sha_compress<SHORT>(out, w);
    }
}

// Fast path: K0 = |k|, V0 = |v| wave-uniform multiples of 4, data 4-aligned in LDS. Word g of the
// message is: 0 -> K0 | 1..K0/4 -> key | K0/4+1 -> V0 | .. -> value | L/4 -> 0x80000000 | 0.
template <bool SHORT>
__device__ __forceinline__ void hash_fast(const uint32_t *lds, uint32_t kword, uint32_t vword, uint32_t K0,
                                          uint32_t V0, uint32_t out[8]) {
    const uint32_t kw = K0 >> 2, vw = V0 >> 2;
    const uint32_t vbeg = kw + 2, vend = kw + 2 + vw, lw = vend;  // L/4 == vend
    const uint32_t L = 8 + K0 + V0;
    const uint32_t nb = (L + 9 + 63) >> 6;
    const uint64_t bits = (uint64_t)L * 8;
    sha_init(out);
    for (uint32_t blk = 0; blk < nb; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t g = blk * 16 + i;
            uint32_t x;
            if (g == 0) x = K0;
            else if (g <= kw) x = bswap32(lds[kword + g - 1]);
            else if (g == kw + 1) x = V0;
            else if (g < vend) x = bswap32(lds[vword + g - vbeg]);
            else if (g == lw) x = 0x80000000u;
            else x = 0;
            w[i] = x;
        }
        if (blk == nb - 1) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha_compress<SHORT>(out, w);
    }
}

// Compile-time record shape (the configs' 32-B keys / 100-B values): every message word's source is
// known while compiling — a constant (length fields, 0x80 terminator, zero padding, bit length) or one
// LDS word at a fixed offset. The constant words are folded at compile time (sha256.hpp
// sha_compress_known): K + W literals, schedule terms summed in advance, round 0 of the first block
// computed by the compiler. Block 3 of a 140-B leaf carries 13 constant words. No runtime selection
// chain, no scalar branches.
template <uint32_t K0, uint32_t V0>
struct LeafShape {
    static constexpr uint32_t kw = K0 / 4, vw = V0 / 4;
    static constexpr uint32_t vbeg = kw + 2, vend = kw + 2 + vw;  // value words [vbeg, vend); vend = L/4
    static constexpr uint32_t L = 8 + K0 + V0;
    static constexpr uint32_t NB = (L + 9 + 63) / 64;
    static constexpr uint64_t bits = (uint64_t)L * 8;
    // kind of message word g: 0 constant (value in *c), 1 key word g-1, 2 value word g-vbeg
    static constexpr int kind(uint32_t g, uint32_t *c) {
        if (g / 16 == NB - 1 && g % 16 == 14) return *c = (uint32_t)(bits >> 32), 0;
        if (g / 16 == NB - 1 && g % 16 == 15) return *c = (uint32_t)bits, 0;
        if (g == 0) return *c = K0, 0;
        if (g <= kw) return 1;
        if (g == kw + 1) return *c = V0, 0;
        if (g < vend) return 2;
        return *c = (g == vend ? 0x80000000u : 0u), 0;
    }
};
template <uint32_t K0, uint32_t V0, uint32_t BLK>
struct LeafBlockKnown {
    static constexpr MsgKnown msg() {
        MsgKnown m{};
        for (uint32_t i = 0; i < 16; ++i) {
            uint32_t c = 0;
            if (LeafShape<K0, V0>::kind(BLK * 16 + i, &c) == 0) {
                m.mask |= 1u << i;
                m.val[i] = c;
            }
        }
        return m;
    }
    static constexpr SchedKnown value = expand_known(msg());
};

template <bool SHORT, uint32_t K0, uint32_t V0, uint32_t BLK>
__device__ __forceinline__ void hash_regs_block(uint32_t *m, uint32_t out[8]);

// One workgroup tile (LEAF_WAVES x 64 records starting at record 256 x bx) of k_leaf_multi.
template <bool SHORT>
__device__ __forceinline__ void leaf_hash_tile(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                               const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                               uint64_t n, uint8_t *__restrict__ out, uint64_t bx, uint32_t *lds_all) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r0 = (bx * LEAF_WAVES + wave) * 64;
    const bool wave_live = r0 < n;
    const uint64_t r = r0 + lane;
    const bool valid = r < n;
    uint32_t *lds = lds_all + wave * (LEAF_LDS_WAVE / 4);

    uint64_t k0 = 0, v0 = 0, k1 = 0, v1 = 0;
    const uint8_t *kstart = kb, *vstart = vb;
    uint32_t kspan = 0, vspan = 0;
    bool staged = false;
    if (wave_live) {
        uint64_t rc = n - r0 < 64 ? n - r0 : 64;
        k0 = koff[r0]; k1 = koff[r0 + rc];
        v0 = voff[r0]; v1 = voff[r0 + rc];
        kstart = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(kb + k0) & ~uintptr_t(15));
        vstart = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(vb + v0) & ~uintptr_t(15));
        uint64_t ks = (uint64_t)((kb + k1) - kstart), vs = (uint64_t)((vb + v1) - vstart);
        ks = (ks + 15) & ~uint64_t(15);
        vs = (vs + 15) & ~uint64_t(15);
        staged = ks + vs + 32 <= LEAF_LDS_WAVE;
        if (staged) {
            kspan = (uint32_t)ks;
            vspan = (uint32_t)vs;
            const uint4 *gk = reinterpret_cast<const uint4 *>(kstart);
            const uint4 *gv = reinterpret_cast<const uint4 *>(vstart);
            uint4 *lk = reinterpret_cast<uint4 *>(lds);
            uint4 *lv = reinterpret_cast<uint4 *>(lds + kspan / 4);
            for (uint32_t i = lane; i < kspan / 16; i += 64) lk[i] = gk[i];
            for (uint32_t i = lane; i < vspan / 16; i += 64) lv[i] = gv[i];
        }
    }
    __syncthreads();
    if (!valid) return;

    const uint64_t kbeg = koff[r], kend = koff[r + 1], vbeg = voff[r], vend = voff[r + 1];
    const uint32_t klen = (uint32_t)(kend - kbeg), vlen = (uint32_t)(vend - vbeg);
    uint32_t st[8];
    if (staged) {
        const uint32_t kbyte = (uint32_t)((kb + kbeg) - kstart);
        const uint32_t vbyte = kspan + (uint32_t)((vb + vbeg) - vstart);
        // wave-uniform fast-path test over the live lanes
        const uint32_t K0 = __shfl(klen, 0), V0 = __shfl(vlen, 0);
        const bool mine = klen == K0 && vlen == V0 && ((K0 | V0 | kbyte | vbyte) & 3) == 0;
        if (__all(mine)) {
            const uint32_t k0u = __builtin_amdgcn_readfirstlane(K0), v0u = __builtin_amdgcn_readfirstlane(V0);
            if (k0u == 32 && v0u == 100) {  // the configs' shape: every constant word folded at compile time
                uint32_t m[33];
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) m[i] = bswap32(lds[(kbyte >> 2) + i]);
#pragma unroll
                for (uint32_t i = 0; i < 25; ++i) m[8 + i] = bswap32(lds[(vbyte >> 2) + i]);
                sha_init(st);
                hash_regs_block<SHORT, 32, 100, 0>(m, st);
            } else {
                hash_fast<SHORT>(lds, kbyte >> 2, vbyte >> 2, k0u, v0u, st);
            }
        } else {
            LdsSrc src{lds, kbyte, vbyte};
            hash_generic<SHORT>(src, klen, vlen, st);
        }
    } else {
        GlbSrc src{kb + kbeg, vb + vbeg, kb + kend, vb + vend};
        hash_generic<SHORT>(src, klen, vlen, st);
    }
    store_digest(out + 32 * r, st);
}

// k batches at once (grid.y = batch): batch b's digests go to out + 32 x base[b] (dirty-path updates of
// several replicas in one launch instead of one small launch per replica).
template <bool SHORT>
__global__ __launch_bounds__(256) void k_leaf_multi(LeafBatches B, uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[LEAF_WAVES * LEAF_LDS_WAVE / 4];
    const uint32_t b = blockIdx.y;
    if ((uint64_t)blockIdx.x * LEAF_WAVES * 64 >= B.m[b]) return;  // uniform per workgroup
    leaf_hash_tile<SHORT>(B.kb[b], B.koff[b], B.vb[b], B.voff[b], B.m[b], out + 32 * B.base[b], blockIdx.x, lds_all);
}

template <bool SHORT, uint32_t K0, uint32_t V0, uint32_t BLK>
__device__ __forceinline__ void hash_regs_block(uint32_t *m, uint32_t out[8]) {
    using Sh = LeafShape<K0, V0>;
    uint32_t w[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        uint32_t c = 0;
        const uint32_t g = BLK * 16 + i;
        const int kd = Sh::kind(g, &c);
        w[i] = kd == 1 ? m[g - 1] : kd == 2 ? m[Sh::kw + g - Sh::vbeg] : c;
    }
    sha_compress_known<SHORT, LeafBlockKnown<K0, V0, BLK>, BLK == 0>(out, w);
    if constexpr (BLK + 1 < Sh::NB) hash_regs_block<SHORT, K0, V0, BLK + 1>(m, out);
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

template <uint32_t NW>
__device__ __forceinline__ void load_words_a4(const uint8_t *p, uint32_t *w) {
    const u32x4_a4 *q = reinterpret_cast<const u32x4_a4 *>(p);
#pragma unroll
    for (uint32_t i = 0; i < NW / 4; ++i) {
        const u32x4_a4 x = q[i];
        w[4 * i] = x.x;
        w[4 * i + 1] = x.y;
        w[4 * i + 2] = x.z;
        w[4 * i + 3] = x.w;
    }
#pragma unroll
    for (uint32_t i = NW / 4 * 4; i < NW; ++i) w[i] = reinterpret_cast<const uint32_t *>(p)[i];
}

template <uint32_t NW>
__device__ __forceinline__ void store_words_a4(uint8_t *p, const uint32_t *w) {
    u32x4_a4 *q = reinterpret_cast<u32x4_a4 *>(p);
#pragma unroll
    for (uint32_t i = 0; i < NW / 4; ++i) q[i] = u32x4_a4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
#pragma unroll
    for (uint32_t i = NW / 4 * 4; i < NW; ++i) reinterpret_cast<uint32_t *>(p)[i] = w[i];
}

// Fixed-shape records (the configs' 32-B keys / 100-B values at 4-B alignment): each lane loads its own
// record's 33 message words straight from HBM into VGPRs with 16-B loads at 4-B alignment (gfx950 serves
// unaligned global loads; a wave's 64 records are contiguous, so it touches the cache lines a coalesced
// copy would), byte-swaps them and runs the three compressions with the constant words folded at compile
// time. No LDS: the ordering kernels co-running on the aux stream keep the CU's whole LDS. Wave w starts
// with chunk w, then takes LEAF_GRAIN chunks per atomic from a device counter, so waves on CUs that also
// run ordering workgroups simply take fewer. A chunk of any other shape ends the wave's work: it leaves
// that chunk and the rest of its range in its slot for k_leaf_ragged and raises the flag (leaf.hpp).
// KO: the key words already in registers go to the tree's own key buffer (and the offsets), so a build
// from borrowed buffers needs no separate key copy (leaf.hpp).
template <bool SHORT, uint32_t K0, uint32_t V0>
__global__ __launch_bounds__(256) void k_leaf_direct(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                    const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                    uint64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ ctr,
                                                    KeyOut KO) {
    using Sh = LeafShape<K0, V0>;
    constexpr uint32_t MW = Sh::kw + Sh::vw;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nch = (uint32_t)((n + 63) / 64);
    const uint32_t NW = gridDim.x * LEAF_WAVES;
    const uint32_t w = blockIdx.x * LEAF_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t b = w, e = std::min<uint32_t>(w + 1, nch);
    while (b < nch) {
        for (uint32_t c = b; c < e; ++c) {
            const uint64_t r = (uint64_t)c * 64 + lane;
            const bool valid = r < n;
            const uint64_t kbeg = valid ? koff[r] : 0, kend = valid ? koff[r + 1] : 0;
            const uint64_t vbeg = valid ? voff[r] : 0, vend = valid ? voff[r + 1] : 0;
            const uint8_t *kp = kb + kbeg, *vp = vb + vbeg;
            const bool fixed =
                __all(!valid || (kend - kbeg == K0 && vend - vbeg == V0 &&
                                 ((reinterpret_cast<uintptr_t>(kp) | reinterpret_cast<uintptr_t>(vp)) & 3) == 0));
            if (!fixed) {  // this chunk and the rest of the range go to the ragged stage
                if (lane == 0) {
                    ctr[CTR_STOP] = 1u;  // read by the ragged stage after this kernel
                    ctr[CTR_LIST + w] = (c << 5) | (e - c);
                }
                return;
            }
            if (!valid) continue;
            uint32_t m[MW];
            load_words_a4<Sh::kw>(kp, m);
            load_words_a4<Sh::vw>(vp, m + Sh::kw);
            if (KO.kdst && kend <= KO.kcap) store_words_a4<Sh::kw>(KO.kdst + kbeg, m);
            if (KO.odst) {
                KO.odst[r] = kbeg;
                if (r + 1 == n) KO.odst[n] = kend;
            }
#pragma unroll
            for (uint32_t i = 0; i < MW; ++i) m[i] = bswap32(m[i]);
            uint32_t st[8];
            sha_init(st);
            hash_regs_block<SHORT, K0, V0, 0>(m, st);
            store_digest(out + 32 * r, st);
        }
        // next range. (No look at the stop flag here: an agent-scope load of it beside every grab doubled
        // this kernel and slowed the co-running sort 3x; a wave simply stops at its own first chunk of
        // another shape.)
        uint32_t x = 0;
        if (lane == 0) x = atomicAdd(&ctr[CTR_FIXED], LEAF_GRAIN);
        b = NW + __builtin_amdgcn_readfirstlane(__shfl(x, 0));
        e = std::min<uint32_t>(b + LEAF_GRAIN, nch);
    }
}

int leaf_cus() {
    static int c = [] {
        int dev = 0, x = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&x, hipDeviceAttributeMultiprocessorCount, dev);
        return x > 0 ? x : 256;
    }();
    return c;
}

}  // namespace

void launch_leaf_hash_multi(const LeafBatches &B, uint32_t k, uint64_t mmax, uint8_t *out, hipStream_t st) {
    if (!k || !mmax) return;
    const dim3 grid((uint32_t)ceil_div(mmax, (uint64_t)LEAF_WAVES * 64), k);
    // small batches are latency-bound (the short dependency chain); large ones throughput-bound (fewer
    // instructions: configs[4]'s 7 x 125K records 438 -> ~150 us)
    if ((uint64_t)k * mmax >= (1u << 18))
        hipLaunchKernelGGL(k_leaf_multi<false>, grid, dim3(64 * LEAF_WAVES), 0, st, B, out);
    else
        hipLaunchKernelGGL(k_leaf_multi<true>, grid, dim3(64 * LEAF_WAVES), 0, st, B, out);
    MKV_LAUNCH_CHECK();
}

size_t leaf_ctr_words(uint64_t) { return CTR_LIST + LEAF_MAX_WAVES + 16; }

// Waves of the fixed-shape kernel for n records (the ragged kernel needs the same number).

// Two workgroups per CU (8 waves): room on every CU for the ordering kernels on the aux stream. Three
// speed the leaf hash alone but stretch the co-running sort past it (build 2.26-2.60 vs 2.18-2.23 ms).
constexpr int LEAF_WGS = 2;

uint32_t leaf_fixed_waves(uint64_t n) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(ceil_div(n, 64), LEAF_WAVES), (uint64_t)leaf_cus() * LEAF_WGS);
    return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(blocks, 1) * LEAF_WAVES, LEAF_MAX_WAVES);
}

void launch_leaf_fixed(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t *out, uint32_t *ctr, hipStream_t st, const KeyOut &KO) {
    const uint32_t nw = leaf_fixed_waves(n);
    MKV_HIP(hipMemsetAsync(ctr, 0, (CTR_LIST + nw) * sizeof(uint32_t), st));
    if (!n) return;
    hipLaunchKernelGGL((k_leaf_direct<false, 32, 100>), dim3(nw / LEAF_WAVES), dim3(64 * LEAF_WAVES), 0, st, kb, koff,
                       vb, voff, n, out, ctr, KO);
    MKV_LAUNCH_CHECK();
}

void launch_leaf_hash(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                      uint8_t *out, uint32_t *ctr, hipStream_t st, const KeyOut &KO) {
    // the key copy stores at the source's byte offsets: kb must share kdst's 16-B alignment
    const KeyOut K{(reinterpret_cast<uintptr_t>(kb) & 15) == 0 ? KO.kdst : nullptr, KO.odst, KO.kcap};
    launch_leaf_fixed(kb, koff, vb, voff, n, out, ctr, st, K);
    launch_leaf_ragged(kb, koff, vb, voff, n, out, ctr, st, K);
    launch_leaf_edges(kb, koff, vb, voff, n, out, st);  // the records near the blobs' ends it leaves
    if (K.kdst) launch_keycopy_ragged(kb, koff, n, ctr, K.kdst, K.kcap, st);
}

}  // namespace mkv
