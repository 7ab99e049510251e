// k_leaf.hip — Kernel A: batched leaf hashing (R1 + R2).
//
// Restates merkle.rs:7-16 (encode_leaf) fused into merkle.rs:45-49 (compute_leaf_hash): the digest of
// u32_be(|k|) || k || u32_be(|v|) || v, computed without ever materialising the encoding.
//
// Layout: records arrive as two packed blobs with u64 offsets (keys kb/koff, values vb/voff), exactly
// the mkv_blob pair of the C ABI. One lane owns one record; one wave owns 64 consecutive records, so
// the wave's key bytes and value bytes are each one contiguous span. The wave copies both spans into
// its private LDS region with coalesced 16-byte loads, then every lane builds its message words from
// LDS (ds_read_b32 + v_perm_b32 for the byte-swap / unaligned extract) and runs the compressions with
// state and the rolling schedule in VGPRs.
//
// Paths (chosen per wave, uniformly):
//   fast    — every record in the wave has the same |k| and |v|, both multiples of 4, 4-aligned in
//             LDS: every message word is one whole LDS word or a constant (the bench/config path).
//   generic — any lengths / alignments: words are assembled from byte-range masks.
//   global  — the wave's spans do not fit its LDS region: generic assembly straight from HBM.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

constexpr int LEAF_WAVES = 4;                 // waves per workgroup
// LDS per wave: 64 x 132-B records + alignment slack (8,512 B) fit; 4 waves -> 36 KiB per WG, so four
// leaf workgroups (144 KiB) leave room on the CU for a sort workgroup running on the aux stream.
constexpr uint32_t LEAF_LDS_WAVE = 9216;

// Block-count class of a record for the ragged leaf path: min(SHA blocks of its encoding, 32) - 1.
constexpr uint32_t RG_CLASSES = 32;
// Counter block layout (leaf_ctr_words): [0] leaf chunk counter, [1] listed chunks, [2] ragged chunk
// counter, [3] spare, [CTR_CLS, +32) listed records per block-count class (k_leaf_direct),
// [CTR_CUR, +32) class cursors (k_ragged_scatter), [CTR_FLAGS ..) one listed flag per chunk. The head
// (CTR_FLAGS words) is zeroed before every leaf stage.
constexpr uint32_t CTR_CLS = 4, CTR_CUR = CTR_CLS + RG_CLASSES, CTR_FLAGS = CTR_CUR + RG_CLASSES;
__device__ __forceinline__ uint32_t rg_class(uint64_t klen, uint64_t vlen) {
    const uint64_t nb = (8 + klen + vlen + 9 + 63) >> 6;
    return nb >= RG_CLASSES ? RG_CLASSES - 1 : (uint32_t)nb - 1;
}

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
__device__ __forceinline__ void hash_fixed_block(const uint32_t *lds, uint32_t kword, uint32_t vword, uint32_t out[8]) {
    using Sh = LeafShape<K0, V0>;
    uint32_t w[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        uint32_t c = 0;
        const uint32_t g = BLK * 16 + i;
        const int kd = Sh::kind(g, &c);
        w[i] = kd == 1 ? bswap32(lds[kword + g - 1]) : kd == 2 ? bswap32(lds[vword + g - Sh::vbeg]) : c;
    }
    sha_compress_known<SHORT, LeafBlockKnown<K0, V0, BLK>, BLK == 0>(out, w);
    if constexpr (BLK + 1 < Sh::NB) hash_fixed_block<SHORT, K0, V0, BLK + 1>(lds, kword, vword, out);
}

template <bool SHORT, uint32_t K0, uint32_t V0>
__device__ __forceinline__ void hash_fixed(const uint32_t *lds, uint32_t kword, uint32_t vword, uint32_t out[8]) {
    static_assert(K0 % 4 == 0 && V0 % 4 == 0, "fast-path shapes are word multiples");
    sha_init(out);
    hash_fixed_block<SHORT, K0, V0, 0>(lds, kword, vword, out);
}

// Wave-uniform dispatch of the fast path: specialised shapes first, the runtime-shape loop otherwise.
template <bool SHORT>
__device__ __forceinline__ void hash_fast_any(const uint32_t *lds, uint32_t kword, uint32_t vword, uint32_t K0,
                                              uint32_t V0, uint32_t out[8]) {
    if (K0 == 32 && V0 == 100) hash_fixed<SHORT, 32, 100>(lds, kword, vword, out);
    else hash_fast<SHORT>(lds, kword, vword, K0, V0, out);
}

// One workgroup tile (LEAF_WAVES x 64 records starting at record 256 x bx) of k_leaf_hash / k_leaf_multi.
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
            hash_fast<SHORT>(lds, kbyte >> 2, vbyte >> 2, __builtin_amdgcn_readfirstlane(K0),
                      __builtin_amdgcn_readfirstlane(V0), st);
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

template <bool SHORT>
__global__ __launch_bounds__(256) void k_leaf_hash(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                  const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                  uint64_t n, uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[LEAF_WAVES * LEAF_LDS_WAVE / 4];
    leaf_hash_tile<SHORT>(kb, koff, vb, voff, n, out, blockIdx.x, lds_all);
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

// ---------------------------------------------------------------------------------------------
// Persistent variant: each wave loops over 64-record chunks (grid sized to the device), and while it
// hashes chunk c from LDS the next chunk's spans (<= 9 x 16 B per lane) and per-lane offsets are
// already in flight into registers. Staging latency disappears behind the VALU work, LDS regions are
// wave-private (no workgroup barrier), and the bounded grid leaves CU slots for the ordering kernels
// running concurrently on the aux stream.
// ---------------------------------------------------------------------------------------------
constexpr int PF = LEAF_LDS_WAVE / (16 * 64);  // uint4 prefetch registers per lane

struct ChunkPlan {
    const uint8_t *kstart, *vstart;
    uint32_t kspan, vspan;
    uint64_t kcopy_end;  // byte offset (from kb) one past the chunk's 16-B-rounded key span
    bool staged;
};

// Optional key-ownership copy fused into the leaf hash (tree builds from borrowed device inputs): the
// wave already holds its chunk's key span in registers on the way to LDS, so it also stores it to the
// tree's own key buffer at the same offsets (16-B stores; neighbouring chunks may both write the
// granule they share, with identical bytes), and every lane stores its key offset. Chunks whose span
// ends past kcap (a buffer sized for a smaller earlier build) are skipped; the host then falls back
// to a plain copy.
struct KeyOut {
    uint8_t *kdst;    // null: no copy
    uint64_t *odst;   // null: offsets not copied
    uint64_t kcap;    // bytes available at kdst
    uint8_t *cls;     // k_leaf_direct: block-count class of every record of a listed chunk (null: none)
    uint32_t listed_keys_later;  // k_leaf_direct: listed chunks' keys are copied by k_leaf_ragged
};

template <uint32_t CAP = LEAF_LDS_WAVE>
__device__ __forceinline__ ChunkPlan plan_chunk(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                                                const uint64_t *voff, uint64_t n, uint64_t r0) {
    ChunkPlan P;
    const uint64_t rc = n - r0 < 64 ? n - r0 : 64;
    const uint64_t k0 = koff[r0], k1 = koff[r0 + rc], v0 = voff[r0], v1 = voff[r0 + rc];
    P.kstart = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(kb + k0) & ~uintptr_t(15));
    P.vstart = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(vb + v0) & ~uintptr_t(15));
    const uint64_t ks = ((uint64_t)((kb + k1) - P.kstart) + 15) & ~uint64_t(15);
    const uint64_t vs = ((uint64_t)((vb + v1) - P.vstart) + 15) & ~uint64_t(15);
    P.staged = ks + vs + 32 <= CAP;
    P.kcopy_end = (uint64_t)(P.kstart - kb) + ks;
    P.kspan = P.staged ? (uint32_t)ks : 0;
    P.vspan = P.staged ? (uint32_t)vs : 0;
    return P;
}

__device__ __forceinline__ void load_chunk(const ChunkPlan &P, uint32_t lane, uint4 R[PF]) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        const uint32_t byte = (lane + 64u * i) * 16u;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (byte < P.kspan) x = *reinterpret_cast<const uint4 *>(P.kstart + byte);
        else if (byte - P.kspan < P.vspan) x = *reinterpret_cast<const uint4 *>(P.vstart + (byte - P.kspan));
        R[i] = x;
    }
}

// The key-ownership copy of chunk P (see KeyOut): from the staged registers, or straight from HBM when
// the chunk is not staged.
__device__ __forceinline__ void copy_keys_out(const ChunkPlan &P, uint32_t lane, const uint4 R[PF], const uint8_t *kb,
                                              const KeyOut &KO) {
    if (P.kcopy_end > KO.kcap) return;
    uint8_t *d = KO.kdst + (P.kstart - kb);
    if (P.staged) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint32_t idx = lane + 64u * i;
            if (idx * 16u < P.kspan) reinterpret_cast<uint4 *>(d)[idx] = R[i];
        }
    } else {
        const uint64_t span = P.kcopy_end - (uint64_t)(P.kstart - kb);
        for (uint64_t b = 16ull * lane; b < span; b += 16ull * 64)
            *reinterpret_cast<uint4 *>(d + b) = *reinterpret_cast<const uint4 *>(P.kstart + b);
    }
}

__device__ __forceinline__ void store_chunk(const ChunkPlan &P, uint32_t lane, const uint4 R[PF], uint32_t *lds) {
    uint4 *l4 = reinterpret_cast<uint4 *>(lds);
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        const uint32_t idx = lane + 64u * i;
        if (idx * 16u < P.kspan + P.vspan) l4[idx] = R[i];
    }
}

// One record of a chunk planned by plan_chunk: from the wave's LDS copy when staged (fixed / runtime
// uniform shape, else the generic byte-range assembly), straight from HBM otherwise.
template <bool SHORT>
__device__ __forceinline__ void hash_record(const ChunkPlan &P, const uint32_t *lds, const uint8_t *kb,
                                            const uint8_t *vb, uint64_t kbeg, uint64_t kend, uint64_t vbeg,
                                            uint64_t vend, uint32_t st[8]) {
    const uint32_t klen = (uint32_t)(kend - kbeg), vlen = (uint32_t)(vend - vbeg);
    if (P.staged) {
        const uint32_t kbyte = (uint32_t)((kb + kbeg) - P.kstart);
        const uint32_t vbyte = P.kspan + (uint32_t)((vb + vbeg) - P.vstart);
        const uint32_t K0 = __shfl(klen, 0), V0 = __shfl(vlen, 0);
        const bool mine = klen == K0 && vlen == V0 && ((K0 | V0 | kbyte | vbyte) & 3) == 0;
        if (__all(mine)) {
            hash_fast_any<SHORT>(lds, kbyte >> 2, vbyte >> 2, __builtin_amdgcn_readfirstlane(K0),
                                 __builtin_amdgcn_readfirstlane(V0), st);
        } else {
            LdsSrc src{lds, kbyte, vbyte};
            hash_generic<SHORT>(src, klen, vlen, st);
        }
    } else {
        GlbSrc src{kb + kbeg, vb + vbeg, kb + kend, vb + vend};
        hash_generic<SHORT>(src, klen, vlen, st);
    }
}

// DYN: chunks are handed out by a device counter (`grain` chunks per atomic) instead of the static
// round-robin, so waves on CUs that also run the ordering kernels simply take fewer chunks (no tail of
// slow CUs). Every wave exits once the counter passes the last chunk.
template <bool DYN>
struct ChunkSource {
    uint64_t next, left, stride;
    uint32_t *ctr;
    uint32_t grain;
    __device__ __forceinline__ uint64_t get(uint32_t lane) {
        if constexpr (DYN) {
            if (left == 0) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(ctr, grain);
                next = __builtin_amdgcn_readfirstlane(__shfl(b, 0));
                left = grain;
            }
            --left;
            return next++;
        } else {
            const uint64_t c = next;
            next += stride;
            return c;
        }
    }
};

template <bool SHORT, bool DYN>
__global__ __launch_bounds__(256) void k_leaf_persist(const uint8_t *__restrict__ kb,
                                                     const uint64_t *__restrict__ koff,
                                                     const uint8_t *__restrict__ vb,
                                                     const uint64_t *__restrict__ voff, uint64_t n,
                                                     uint8_t *__restrict__ out, uint32_t *__restrict__ ctr,
                                                     uint32_t grain, KeyOut KO) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[LEAF_WAVES * LEAF_LDS_WAVE / 4];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *lds = lds_all + wave * (LEAF_LDS_WAVE / 4);
    const uint64_t nchunks = (n + 63) / 64;
    ChunkSource<DYN> src{(uint64_t)blockIdx.x * LEAF_WAVES + wave, 0, (uint64_t)gridDim.x * LEAF_WAVES, ctr, grain};
    uint64_t c = src.get(lane);
    if (c >= nchunks) return;  // wave-private work: no workgroup barrier anywhere

    ChunkPlan P = plan_chunk(kb, koff, vb, voff, n, c * 64);
    uint4 R[PF];
    load_chunk(P, lane, R);
    uint64_t r = c * 64 + lane;
    bool valid = r < n;
    uint64_t kbeg = valid ? koff[r] : 0, kend = valid ? koff[r + 1] : 0;
    uint64_t vbeg = valid ? voff[r] : 0, vend = valid ? voff[r + 1] : 0;
    while (true) {
        if (P.staged) store_chunk(P, lane, R, lds);
        if (KO.kdst) copy_keys_out(P, lane, R, kb, KO);
        if (KO.odst && valid) {
            KO.odst[r] = kbeg;
            if (r + 1 == n) KO.odst[n] = kend;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes land before its reads
        // ---- prefetch the next chunk (registers only; consumed next iteration) ----
        const uint64_t cn = src.get(lane);
        ChunkPlan Pn = P;
        uint64_t nkb = 0, nke = 0, nvb = 0, nve = 0;
        const bool more = cn < nchunks;
        if (more) {
            Pn = plan_chunk(kb, koff, vb, voff, n, cn * 64);
            load_chunk(Pn, lane, R);
            const uint64_t rn = cn * 64 + lane;
            if (rn < n) {
                nkb = koff[rn];
                nke = koff[rn + 1];
                nvb = voff[rn];
                nve = voff[rn + 1];
            }
        }
        // ---- hash chunk c ----
        if (valid) {
            uint32_t st[8];
            hash_record<SHORT>(P, lds, kb, vb, kbeg, kend, vbeg, vend, st);
            store_digest(out + 32 * r, st);
        }
        if (!more) break;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of chunk c done before it is overwritten
        c = cn;
        P = Pn;
        r = c * 64 + lane;
        valid = r < n;
        kbeg = nkb;
        kend = nke;
        vbeg = nvb;
        vend = nve;
    }
}

// ---------------------------------------------------------------------------------------------
// DMA variant (round 2, MKV_LEAF_KERNEL=2): the next chunk goes global -> LDS with LDS-DMA loads
// (global_load_lds_dwordx4: no VGPR destination) instead of the register prefetch, and on the
// fixed-shape path (K0 / V0 = the configs' 32-B keys / 100-B values) every lane pulls its whole message
// (kw + vw big-endian words) from LDS into registers at the start of a chunk, so the wave's LDS region is
// free again before the compressions start and the DMA of the next chunk lands behind them. Without the
// 36 prefetch VGPRs and with 8.5 KiB of LDS per wave, three workgroups per CU fit beside an ordering
// workgroup (3 x 34 KiB + 55 KiB <= 160 KiB; 101 VGPRs). Chunks of any other shape are only listed
// (ctr[1] = count, ctr[CTR_FLAGS..] = chunk flags) and hashed by k_leaf_list right after, so the general paths'
// registers do not weigh on this kernel.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t LEAF_LDS_DMA = 8704;  // 64 x 132-B records + 2 x 16-B alignment slack + 32

__device__ __forceinline__ void dma_chunk(const ChunkPlan &P, uint32_t lane, uint32_t *lds) {
    const uint32_t tot = P.kspan + P.vspan;
    const uint32_t ninst = (tot + 1023) / 1024;
    for (uint32_t i = 0; i < ninst; ++i) {
        const uint32_t byte = (lane + 64u * i) * 16u;
        if (byte < tot) {
            const uint8_t *g = byte < P.kspan ? P.kstart + byte : P.vstart + (byte - P.kspan);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), lds + 256u * i, 16, 0, 0);
        }
    }
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

template <bool SHORT, uint32_t K0, uint32_t V0>
__global__ __launch_bounds__(256) void k_leaf_dma(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                 const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                 uint64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ ctr,
                                                 uint32_t grain, KeyOut KO) {
    using Sh = LeafShape<K0, V0>;
    constexpr uint32_t MW = Sh::kw + Sh::vw;
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[LEAF_WAVES * LEAF_LDS_DMA / 4];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *lds = lds_all + wave * (LEAF_LDS_DMA / 4);
    const uint64_t nchunks = (n + 63) / 64;
    ChunkSource<true> src{0, 0, 0, ctr, grain};
    uint64_t c = src.get(lane);
    if (c >= nchunks) return;  // wave-private work: no workgroup barrier anywhere

    ChunkPlan P = plan_chunk<LEAF_LDS_DMA>(kb, koff, vb, voff, n, c * 64);
    if (P.staged) dma_chunk(P, lane, lds);
    uint64_t r = c * 64 + lane;
    bool valid = r < n;
    uint64_t kbeg = valid ? koff[r] : 0, kend = valid ? koff[r + 1] : 0;
    uint64_t vbeg = valid ? voff[r] : 0, vend = valid ? voff[r + 1] : 0;
    while (true) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c has landed in LDS
        if (KO.kdst && P.kcopy_end <= KO.kcap) {  // key-ownership copy from the staged span
            uint8_t *d = KO.kdst + (P.kstart - kb);
            if (P.staged) {
                const uint4 *l4 = reinterpret_cast<const uint4 *>(lds);
                for (uint32_t i = lane; i * 16u < P.kspan; i += 64) reinterpret_cast<uint4 *>(d)[i] = l4[i];
            } else {
                const uint64_t span = P.kcopy_end - (uint64_t)(P.kstart - kb);
                for (uint64_t b = 16ull * lane; b < span; b += 16ull * 64)
                    *reinterpret_cast<uint4 *>(d + b) = *reinterpret_cast<const uint4 *>(P.kstart + b);
            }
        }
        if (KO.odst && valid) {
            KO.odst[r] = kbeg;
            if (r + 1 == n) KO.odst[n] = kend;
        }
        const uint32_t klen = (uint32_t)(kend - kbeg), vlen = (uint32_t)(vend - vbeg);
        const uint32_t kbyte = (uint32_t)((kb + kbeg) - P.kstart);
        const uint32_t vbyte = P.kspan + (uint32_t)((vb + vbeg) - P.vstart);
        const bool fixed = P.staged && __all(!valid || (klen == K0 && vlen == V0 && ((kbyte | vbyte) & 3) == 0));
        if (lane == 0) ctr[CTR_FLAGS + c] = fixed ? 0u : 1u;  // chunk flags for k_leaf_list
        if (!fixed && lane == 0) atomicAdd(&ctr[1], 1u);
        uint32_t m[MW];
        if (fixed) {
#pragma unroll
            for (uint32_t i = 0; i < Sh::kw; ++i) m[i] = bswap32(lds[(kbyte >> 2) + i]);
#pragma unroll
            for (uint32_t i = 0; i < Sh::vw; ++i) m[Sh::kw + i] = bswap32(lds[(vbyte >> 2) + i]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the region's reads are done: it may be refilled
        // ---- next chunk: plan, offsets, and (fixed path) its DMA behind this chunk's compressions ----
        const uint64_t cn = src.get(lane);
        const bool more = cn < nchunks;
        ChunkPlan Pn = P;
        uint64_t nkb = 0, nke = 0, nvb = 0, nve = 0;
        if (more) {
            Pn = plan_chunk<LEAF_LDS_DMA>(kb, koff, vb, voff, n, cn * 64);
            if (Pn.staged) dma_chunk(Pn, lane, lds);
            const uint64_t rn = cn * 64 + lane;
            if (rn < n) {
                nkb = koff[rn];
                nke = koff[rn + 1];
                nvb = voff[rn];
                nve = voff[rn + 1];
            }
        }
        if (fixed && valid) {
            uint32_t st[8];
            sha_init(st);
            hash_regs_block<SHORT, K0, V0, 0>(m, st);
            store_digest(out + 32 * r, st);
        }
        if (!more) break;
        c = cn;
        P = Pn;
        r = c * 64 + lane;
        valid = r < n;
        kbeg = nkb;
        kend = nke;
        vbeg = nvb;
        vend = nve;
    }
}

// ---------------------------------------------------------------------------------------------
// Direct variant (round 2, MKV_LEAF_KERNEL=3): no LDS at all. On the fixed-shape path every lane loads
// its own record's message straight from HBM into registers (16-B loads at 4-B alignment: gfx950 serves
// unaligned global loads; the 64 lanes' spans are contiguous, so the L1/L2 lines a wave touches are the
// ones a coalesced copy would fetch). Without an LDS region the leaf hash no longer competes with the
// co-running ordering kernels for LDS, and at ~70 VGPRs several more waves fit per SIMD to hide the
// load latency. Non-fixed chunks are listed for k_leaf_list as in k_leaf_dma.
// ---------------------------------------------------------------------------------------------
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

constexpr uint32_t LIST_GRAIN = 16;  // k_leaf_direct: chunks per counter grab while a wave lists

template <bool SHORT, uint32_t K0, uint32_t V0>
__global__ __launch_bounds__(256) void k_leaf_direct(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                    const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                    uint64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ ctr,
                                                    uint32_t grain, KeyOut KO) {
    using Sh = LeafShape<K0, V0>;
    constexpr uint32_t MW = Sh::kw + Sh::vw;
    __shared__ uint32_t hist_all[4][RG_CLASSES];  // per wave: listed records per block-count class
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *hist = hist_all[(threadIdx.x >> 6) & 3];
    if (lane < RG_CLASSES) hist[lane] = 0;
    const uint64_t nchunks = (n + 63) / 64;
    ChunkSource<true> src{0, 0, 0, ctr, grain};
    uint32_t listed = 0;  // this wave's listed chunks: one atomic at the end, not one per chunk
    for (uint64_t c = src.get(lane); c < nchunks; c = src.get(lane)) {
        const uint64_t r = c * 64 + lane;
        const bool valid = r < n;
        const uint64_t kbeg = valid ? koff[r] : 0, kend = valid ? koff[r + 1] : 0;
        const uint64_t vbeg = valid ? voff[r] : 0, vend = valid ? voff[r + 1] : 0;
        const uint64_t cc = c;
        const uint8_t *kp = kb + kbeg, *vp = vb + vbeg;
        const bool fixed =
            __all(!valid || (kend - kbeg == K0 && vend - vbeg == V0 &&
                             ((reinterpret_cast<uintptr_t>(kp) | reinterpret_cast<uintptr_t>(vp)) & 3) == 0));
        if (lane == 0) ctr[CTR_FLAGS + cc] = fixed ? 0u : 1u;  // chunk flags: listed chunks are hashed afterwards
        if (!fixed) {
            ++listed;
            // a listed chunk costs a few stores, so grabs of `grain` chunks would make the shared chunk
            // counter the bottleneck (same-address atomics serialise in L2: 0.5 ms for 10M ragged
            // records at grain 4); while this wave lists, it grabs LIST_GRAIN chunks at a time (back to
            // `grain` at its next fixed-shape chunk, so a grab of fixed chunks stays small at the end)
            src.grain = LIST_GRAIN;
            if (KO.cls && valid) {
                const uint32_t k = rg_class(kend - kbeg, vend - vbeg);
                KO.cls[r] = (uint8_t)k;
                atomicAdd(&hist[k], 1u);
            }
            if (KO.kdst && !KO.listed_keys_later) {  // key-ownership copy of the chunk's span
                const ChunkPlan P = plan_chunk(kb, koff, vb, voff, n, cc * 64);
                if (P.kcopy_end <= KO.kcap) {
                    uint8_t *d = KO.kdst + (P.kstart - kb);
                    const uint64_t span = P.kcopy_end - (uint64_t)(P.kstart - kb);
                    for (uint64_t b = 16ull * lane; b < span; b += 16ull * 64)
                        *reinterpret_cast<uint4 *>(d + b) = *reinterpret_cast<const uint4 *>(P.kstart + b);
                }
            }
            if (KO.odst && valid) {
                KO.odst[r] = kbeg;
                if (r + 1 == n) KO.odst[n] = kend;
            }
            continue;
        }
        src.grain = grain;
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
    if (listed && lane == 0) atomicAdd(&ctr[1], listed);
    if (listed && KO.cls && lane < RG_CLASSES) {  // the wave's class counts into the block totals
        const uint32_t h = hist[lane];
        if (h) atomicAdd(&ctr[CTR_CLS + lane], h);
    }
}

// The chunks k_leaf_dma / k_leaf_direct listed (any shape but the fixed one): one wave per listed chunk, staged through
// the wave's private LDS region exactly like k_leaf_persist.
template <bool SHORT>
__global__ __launch_bounds__(256) void k_leaf_list(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                  const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                  uint64_t n, uint8_t *__restrict__ out,
                                                  const uint32_t *__restrict__ ctr) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[LEAF_WAVES * LEAF_LDS_WAVE / 4];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *lds = lds_all + wave * (LEAF_LDS_WAVE / 4);
    if (ctr[1] == 0) return;
    const uint64_t nchunks = (n + 63) / 64;
    for (uint64_t c = (uint64_t)blockIdx.x * LEAF_WAVES + wave; c < nchunks; c += (uint64_t)gridDim.x * LEAF_WAVES) {
        if (!ctr[CTR_FLAGS + c]) continue;  // flagged by k_leaf_direct / k_leaf_dma
        const ChunkPlan P = plan_chunk(kb, koff, vb, voff, n, c * 64);
        if (P.staged) {
            uint4 R[PF];
            load_chunk(P, lane, R);
            store_chunk(P, lane, R, lds);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        const uint64_t r = c * 64 + lane;
        if (r < n) {
            uint32_t st[8];
            hash_record<SHORT>(P, lds, kb, vb, koff[r], koff[r + 1], voff[r], voff[r + 1], st);
            store_digest(out + 32 * r, st);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the region is refilled
    }
}

// ---------------------------------------------------------------------------------------------
// Ragged records (round 3): the chunks k_leaf_direct lists (any key / value lengths, any byte
// alignment) — the shape of a real store snapshot (sync.rs:109-115 hashes arbitrary &str pairs).
//
// A 64-lane wave only computes at full width when its 64 records need the same number of SHA blocks,
// so the listed records are first bucketed by block count (class = min(blocks, 32) - 1): a per-
// workgroup LDS histogram (k_ragged_count), one exclusive scan of the class-major (class, workgroup)
// counts, and a scatter of record ids into class order (k_ragged_scatter; LDS cursors, no global
// atomics). k_leaf_ragged then hands out 64-entry chunks of that list: within a chunk every lane runs
// the same number of compressions.
//
// Per lane the padded encoding (R1 + SHA padding) is materialised as big-endian words in the wave's
// private LDS region, three blocks (48 words) at a time: all the byte shifting happens once per message
// word on the way in — one v_perm_b32 extracts (and byte-swaps) a word at any byte offset from two
// aligned source dwords — instead of per-word region tests in the compression loop:
//   words 1 .. ceil(k/4)      key bytes (the key starts word-aligned, at stream byte 4);
//   words b1+1 .. b3          value bytes shifted by c = k & 3 (b1 = (4+k)/4, b3 = L/4);
//   then three read-modify-writes fix the only words that mix fields: b1 (key tail | vlen head),
//   b1+1 (vlen tail | value head) and b3 (value tail | 0x80); word 0 = klen, the last word = 8L, and
//   everything else was zero-filled first.
// Layout: quad q (words 4q..4q+3) of lane l at uint4 index q * 64 + l: the b32 writes of 64 lanes hit
// 32 different banks per half-wave whatever each lane's word index, and the hash reads whole quads.
// The source loads are aligned dwords (16 B at a time), kept inside [floor4(first byte), ceil4(last
// byte)) of each blob so that reading past a record never leaves the blob's pages.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t RG_WIN = 3;                   // blocks materialised per window
constexpr uint32_t RG_WQ = 4 * RG_WIN;           // uint4 quads per lane per window
constexpr int RG_WAVES = 4;
constexpr uint32_t RG_SCATTER_CHUNKS = 256;      // listed chunks per workgroup of k_ragged_scatter


// Bucketing of the listed records by class, one launch: the class totals came from k_leaf_direct, so a
// workgroup takes its classes' bases from their exclusive scan (32 values) plus one atomic per class on
// the class cursors, then scatters its records through LDS cursors. RG_SCATTER_CHUNKS chunks per
// workgroup keep those same-address atomics few (at 16 chunks per workgroup they serialised to
// 0.44 ms for 10M ragged records). Order inside a class is arbitrary
// (every digest goes to its own record's slot).
__global__ __launch_bounds__(256) void k_ragged_scatter(const uint8_t *__restrict__ cls, uint64_t n,
                                                       uint32_t *__restrict__ ctr, uint64_t *__restrict__ total,
                                                       uint32_t *__restrict__ list) {
    __shared__ uint32_t cur[RG_CLASSES];
    if (ctr[1] == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *total = 0;
        return;
    }
    if (threadIdx.x < RG_CLASSES) cur[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t nchunks = (n + 63) / 64;
    // each wave takes RG_SCATTER_CHUNKS / 4 consecutive chunks, 8 at a time with their flags and
    // classes loaded together (one memory latency per 8 chunks)
    const uint64_t c0 = (uint64_t)blockIdx.x * RG_SCATTER_CHUNKS + wave * (RG_SCATTER_CHUNKS / 4);
    for (uint32_t q = 0; q < RG_SCATTER_CHUNKS / 4; q += 8) {
        uint32_t k[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t c = c0 + q + u, r = c * 64 + lane;
            k[u] = (c < nchunks && r < n && ctr[CTR_FLAGS + c]) ? cls[r] : RG_CLASSES;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k[u] < RG_CLASSES) atomicAdd(&cur[k[u]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < RG_CLASSES) {
        const uint32_t k = threadIdx.x;
        uint32_t cb = 0;
        for (uint32_t j = 0; j < k; ++j) cb += ctr[CTR_CLS + j];
        const uint32_t cnt = cur[k];
        cur[k] = cb + (cnt ? atomicAdd(&ctr[CTR_CUR + k], cnt) : 0u);
        if (blockIdx.x == 0 && k == RG_CLASSES - 1) *total = (uint64_t)cb + ctr[CTR_CLS + k];
    }
    __syncthreads();
    for (uint32_t q = 0; q < RG_SCATTER_CHUNKS / 4; q += 8) {
        uint32_t k[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t c = c0 + q + u, r = c * 64 + lane;
            k[u] = (c < nchunks && r < n && ctr[CTR_FLAGS + c]) ? cls[r] : RG_CLASSES;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k[u] < RG_CLASSES) list[atomicAdd(&cur[k[u]], 1u)] = (uint32_t)((c0 + q + u) * 64 + lane);
    }
}

typedef uint32_t rg_u32x4 __attribute__((ext_vector_type(4), aligned(4)));

// Four aligned dwords at a (4-B aligned), zero where a dword is outside [lo, hi).
__device__ __forceinline__ rg_u32x4 rg_load4(const uint8_t *a, const uint8_t *lo, const uint8_t *hi) {
    if (a >= lo && a + 16 <= hi) return *reinterpret_cast<const rg_u32x4 *>(a);
    rg_u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (a + 4 * j >= lo && a + 4 * j + 4 <= hi) r[j] = reinterpret_cast<const uint32_t *>(a)[j];
    return r;
}
__device__ __forceinline__ uint32_t rg_load1(const uint8_t *a, const uint8_t *lo, const uint8_t *hi) {
    return (a >= lo && a + 4 <= hi) ? *reinterpret_cast<const uint32_t *>(a) : 0u;
}
// big-endian word of the 4 bytes at byte offset s (0..3) of the little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t rg_be(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t rg_head_mask(uint32_t nbytes) {  // first nbytes (0..3) of a BE word
    return nbytes ? ~(0xFFFFFFFFu >> (8 * nbytes)) : 0u;
}

// 16 stream words of one field: w = BE word of the source bytes at (src + 4 (w - fw)), for the words of
// [w, w1] (at most 16), from 17 aligned source dwords.
struct RgField {
    const uint8_t *A;  // floor4(src)
    uint32_t sel;      // v_perm selector of the source's byte alignment
    uint32_t fw;       // stream word of the field's first word
};
__device__ __forceinline__ RgField rg_field(const uint8_t *src, uint32_t fw) {
    RgField f;
    f.A = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(src) & ~uintptr_t(3));
    f.sel = 0x00010203u + (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3) * 0x01010101u;
    f.fw = fw;
    return f;
}
__device__ __forceinline__ void rg_load16(const RgField &f, uint32_t w, uint32_t w1, const uint8_t *lo,
                                          const uint8_t *hi, uint32_t d[17]) {
    const uint8_t *a = f.A + 4 * (w - f.fw);
    const uint32_t nw = w <= w1 ? w1 - w + 1 : 0;  // words of this step: they need dwords 0 .. nw
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
        rg_u32x4 x = {0u, 0u, 0u, 0u};
        if (nw && 4 * g <= nw) x = rg_load4(a + 16 * g, lo, hi);
        d[4 * g] = x.x;
        d[4 * g + 1] = x.y;
        d[4 * g + 2] = x.z;
        d[4 * g + 3] = x.w;
    }
    d[16] = nw > 15 ? rg_load1(a + 64, lo, hi) : 0u;
}
__device__ __forceinline__ void rg_store16(const RgField &f, uint32_t w, uint32_t w1, const uint32_t d[17],
                                           uint32_t *lw, uint32_t lane, uint32_t W0) {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        if (w + j <= w1) {
            const uint32_t u = w + j - W0;
            lw[((u >> 2) * 64 + lane) * 4 + (u & 3)] = rg_be(d[j + 1], d[j], f.sel);
        }
    }
}

// The key-ownership copy of a ragged record (builds from borrowed buffers): the aligned source dwords
// just loaded for its key words go to the tree's key store at the same byte offsets. Dwords shared with a
// neighbouring key carry the same bytes from every writer; none leaves the blob's dword range or kcap.
__device__ __forceinline__ void rg_copy_out(const RgField &f, uint32_t w, uint32_t w1, const uint32_t d[17],
                                            const uint8_t *kb, const uint8_t *lo, const uint8_t *hi,
                                            const KeyOut &KO) {
    if (w > w1) return;
    const uint8_t *a = f.A + 4 * (w - f.fw);
    const uint32_t nd = w1 - w + 2;  // source dwords that carry this step's words
#pragma unroll
    for (uint32_t j = 0; j < 17; ++j) {
        const uint8_t *p = a + 4 * j;
        if (j < nd && p >= lo && p + 4 <= hi && p >= kb && (uint64_t)(p + 4 - kb) <= KO.kcap)
            *reinterpret_cast<uint32_t *>(KO.kdst + (p - kb)) = d[j];
    }
}

template <bool SHORT>
__global__ __launch_bounds__(64 * RG_WAVES) void k_leaf_ragged(const uint8_t *__restrict__ kb,
                                                              const uint64_t *__restrict__ koff,
                                                              const uint8_t *__restrict__ vb,
                                                              const uint64_t *__restrict__ voff, uint64_t n,
                                                              uint8_t *__restrict__ out,
                                                              const uint32_t *__restrict__ list,
                                                              const uint64_t *__restrict__ total,
                                                              uint32_t *__restrict__ gctr, uint32_t grain,
                                                              KeyOut KO) {
    __shared__ __attribute__((aligned(16))) uint4 lds_all[RG_WAVES * RG_WQ * 64];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 *lq = lds_all + wave * (RG_WQ * 64);
    uint32_t *lw = reinterpret_cast<uint32_t *>(lq);
    // the blobs' byte ranges, rounded out to whole dwords: no source load leaves them
    const uint8_t *klo = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(kb + koff[0]) & ~uintptr_t(3));
    const uint8_t *khi =
        reinterpret_cast<const uint8_t *>((reinterpret_cast<uintptr_t>(kb + koff[n]) + 3) & ~uintptr_t(3));
    const uint8_t *vlo = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(vb + voff[0]) & ~uintptr_t(3));
    const uint8_t *vhi =
        reinterpret_cast<const uint8_t *>((reinterpret_cast<uintptr_t>(vb + voff[n]) + 3) & ~uintptr_t(3));
    const uint64_t T = *total;
    const uint64_t nch = (T + 63) / 64;
    if (nch == 0) return;  // nothing listed (every chunk had the fixed shape): no chunk counter traffic
    ChunkSource<true> src{0, 0, 0, gctr, grain};
    for (uint64_t c = src.get(lane); c < nch; c = src.get(lane)) {
        const uint64_t p = c * 64 + lane;
        const bool valid = p < T;
        const uint32_t r = valid ? list[p] : 0u;
        uint64_t k0 = 0, k1 = 0, v0 = 0, v1 = 0;
        if (valid) {
            k0 = koff[r];
            k1 = koff[r + 1];
            v0 = voff[r];
            v1 = voff[r + 1];
        }
        const uint32_t k = (uint32_t)(k1 - k0), v = (uint32_t)(v1 - v0);
        const uint32_t L = 8 + k + v;
        const uint32_t nb = valid ? (L + 9 + 63) >> 6 : 0u;
        const uint32_t W = 16 * nb;                     // message words
        const uint32_t b1 = (4 + k) >> 2, c4 = k & 3;   // key ends in word b1; value shift c4
        const uint32_t b3 = L >> 2, e4 = L & 3;         // value ends / 0x80 in word b3
        const uint32_t nk = (k + 3) >> 2;               // key words 1..nk
        const uint8_t *kp = kb + k0, *vp = vb + v0;
        uint32_t st[8];
        sha_init(st);
        for (uint32_t win = 0; __any(win * RG_WIN < nb); ++win) {
            const uint32_t blo = win * RG_WIN;
            const uint32_t nbw = blo < nb ? min(RG_WIN, nb - blo) : 0u;  // this lane's blocks in the window
            const uint32_t W0 = 16 * blo, W1 = W0 + 16 * nbw;            // words [W0, W1)
            for (uint32_t q = 0; q < 4 * nbw; ++q) lq[q * 64 + lane] = make_uint4(0, 0, 0, 0);
            if (nbw) {
                // key words [kw0, kw1] and value words [vw0, vw1] of the window, 16 of each per step with
                // both fields' loads in flight together (one memory latency per step)
                const uint32_t kw0 = max(1u, W0), kw1 = min(nk, W1 - 1);
                const uint32_t vw0 = max(b1 + 1, W0), vw1 = min(b3, W1 - 1);
                const RgField fk = rg_field(kp, 1), fv = rg_field(vp - c4, b1 + 1);
                for (uint32_t kw = kw0, vw = vw0; kw <= kw1 || vw <= vw1; kw += 16, vw += 16) {
                    uint32_t dk[17], dv[17];
                    rg_load16(fk, kw, kw1, klo, khi, dk);
                    rg_load16(fv, vw, vw1, vlo, vhi, dv);
                    if (KO.kdst) rg_copy_out(fk, kw, kw1, dk, kb, klo, khi, KO);  // key ownership, same offsets
                    rg_store16(fk, kw, kw1, dk, lw, lane, W0);
                    rg_store16(fv, vw, vw1, dv, lw, lane, W0);
                }
                // the words that mix fields (read-modify-write, in this order)
                const uint32_t hc = rg_head_mask(c4);
                auto at = [&](uint32_t w) -> uint32_t & {
                    const uint32_t u = w - W0;
                    return lw[((u >> 2) * 64 + lane) * 4 + (u & 3)];
                };
                if (W0 == 0) at(0) = k;
                if (b1 >= W0 && b1 < W1) {
                    uint32_t &x = at(b1);
                    x = (x & hc) | (v >> (8 * c4));
                }
                if (b1 + 1 >= W0 && b1 + 1 < W1) {
                    uint32_t &x = at(b1 + 1);
                    x = ((c4 ? v << (32 - 8 * c4) : 0u) & hc) | (x & ~hc);
                }
                if (b3 >= W0 && b3 < W1) {
                    uint32_t &x = at(b3);
                    const uint32_t he = rg_head_mask(e4);
                    x = (x & he) | (0x80000000u >> (8 * e4));
                }
                if (W - 1 >= W0 && W - 1 < W1) at(W - 1) = L * 8;  // bit length (high word stays 0)
            }
            for (uint32_t b = 0; b < nbw; ++b) {
                uint32_t w[16];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint4 x = lq[(4 * b + j) * 64 + lane];
                    w[4 * j] = x.x;
                    w[4 * j + 1] = x.y;
                    w[4 * j + 2] = x.z;
                    w[4 * j + 3] = x.w;
                }
                sha_compress<SHORT>(st, w);
            }
        }
        if (valid) store_digest(out + 32 * (uint64_t)r, st);
    }
}

// ---------------------------------------------------------------------------------------------
// Ragged records, register form (round 3, MKV_LEAF_RAGGED=2): the bucketed list of k_leaf_ragged, but
// no LDS. Per block each lane loads the 17 aligned source dwords that cover its 16 message words of the
// key field (stream words 1..b1, key at stream byte 4) and of the value field (stream words b1+1..b3,
// addressed from vp - (k & 3) so that it starts on a stream word), extracts every word with one v_perm
// (byte swap + byte offset), picks key or value word by a per-lane compare, and patches the few words
// that mix fields — b1 (key tail | vlen head), b1+1 (vlen tail | value head), b3 (value tail | 0x80),
// the words past b3 (zero) and the bit length — only in the blocks where some lane of the wave has them
// (wave-uniform tests: for a record class these are the first and the last one or two blocks; the
// middle blocks are plain value words). The next block's source dwords are loaded before the current
// block is compressed, so their latency hides behind the 64 rounds. Lanes of one chunk share the block
// count (the list is bucketed by it), except in the open-ended last class, where lanes simply stop.
// ---------------------------------------------------------------------------------------------
// Dwords [d0, d1] (0 <= d0, d1 <= 16) of the 17 at a (4-B aligned), zero elsewhere: only the 16-B
// groups that meet [d0, d1] are loaded (a lane's words of one field rarely fill the block, and every
// address a wave-wide load carries costs the texture path a cycle). safe: every group this lane can
// touch lies inside the blob (decided once per record), else each dword is range-checked.
__device__ __forceinline__ void rr_load17(const uint8_t *a, int32_t d0, int32_t d1, bool safe, const uint8_t *lo,
                                          const uint8_t *hi, uint32_t d[17]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        rg_u32x4 x = {0u, 0u, 0u, 0u};
        const uint8_t *q = a + 16 * g;
        if (4 * g + 3 >= d0 && 4 * g <= d1) {
            if (safe) x = *reinterpret_cast<const rg_u32x4 *>(q);
            else x = rg_load4(q, lo, hi);
        }
        d[4 * g] = x.x;
        d[4 * g + 1] = x.y;
        d[4 * g + 2] = x.z;
        d[4 * g + 3] = x.w;
    }
    d[16] = 0u;
    if (d1 >= 16) d[16] = safe ? reinterpret_cast<const uint32_t *>(a)[16] : rg_load1(a + 64, lo, hi);
}

// One lane's record in the register form: the two field sources and the stream positions of the
// words that mix fields (b1: key tail | vlen head, b1 + 1: vlen tail | value head, b3: value tail | 0x80).
struct RrLane {
    const uint8_t *kp, *ka, *va;  // key start; floor4 of the key field / value field sources
    uint32_t ksel, vsel;          // v_perm selectors of their byte alignments
    uint32_t k, v, L, nb, b1, b3;
    uint32_t hc, vh, vt, he, term;
    bool ksafe, vsafe;
};

__device__ __forceinline__ RrLane rr_lane(const uint8_t *kb, const uint8_t *vb, uint64_t k0, uint64_t k1, uint64_t v0,
                                          uint64_t v1, bool valid, const uint8_t *klo, const uint8_t *khi,
                                          const uint8_t *vlo, const uint8_t *vhi) {
    RrLane R;
    R.k = (uint32_t)(k1 - k0);
    R.v = (uint32_t)(v1 - v0);
    R.L = 8 + R.k + R.v;
    R.nb = valid ? (R.L + 9 + 63) >> 6 : 0u;
    R.b1 = (4 + R.k) >> 2;
    R.b3 = R.L >> 2;
    const uint32_t c4 = R.k & 3, e4 = R.L & 3;
    R.hc = rg_head_mask(c4);
    R.vh = R.v >> (8 * c4);
    R.vt = c4 ? R.v << (32 - 8 * c4) : 0u;
    R.he = rg_head_mask(e4);
    R.term = 0x80000000u >> (8 * e4);
    R.kp = kb + k0;
    const uint8_t *vq = vb + v0 - c4;
    R.ka = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(R.kp) & ~uintptr_t(3));
    R.va = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(vq) & ~uintptr_t(3));
    R.ksel = 0x00010203u + (uint32_t)(reinterpret_cast<uintptr_t>(R.kp) & 3) * 0x01010101u;
    R.vsel = 0x00010203u + (uint32_t)(reinterpret_cast<uintptr_t>(vq) & 3) * 0x01010101u;
    // every group a block can load: key field [ka - 4, ka + 4 b1 + 68), value field
    // [va - 4 (b1 + 1) + 16 floor((b1 + 1) / 4) - 16, va + 4 (b3 - b1) + 68); generous bounds below
    R.ksafe = R.ka >= klo + 8 && R.ka + 4 * (uint64_t)R.b1 + 80 <= khi;
    R.vsafe = R.va >= vlo + 4 * (uint64_t)R.b1 + 24 && R.va + 4 * (uint64_t)(R.b3 - R.b1) + 80 <= vhi;
    return R;
}

// Source dwords of block b. Word j of the block (stream word 16b + j) takes dwords j and j + 1 of its
// field's 17; a field's words in the block are j in [1 (block 0) or 0, tb1] (key) and [tb1 + 1, tb3]
// (value); the second dword is needed only for a misaligned source.
__device__ __forceinline__ void rr_fetch(const RrLane &R, uint32_t b, bool fk, bool fv, const uint8_t *klo,
                                         const uint8_t *khi, const uint8_t *vlo, const uint8_t *vhi, uint32_t dk[17],
                                         uint32_t dv[17]) {
    const int32_t tb1 = (int32_t)R.b1 - (int32_t)(16 * b), tb3 = (int32_t)R.b3 - (int32_t)(16 * b);
    const bool act = R.nb > b;
    if (fk) {
        const int32_t j0 = b == 0 ? 1 : 0, j1 = min(tb1, 15);
        const int32_t d0 = act ? j0 : 99, d1 = act ? j1 + (R.ksel != 0x00010203u) : -1;
        rr_load17(R.ka + 4 * ((int64_t)(16 * b) - 1), d0, d1, R.ksafe, klo, khi, dk);
    }
    if (fv) {
        const int32_t j0 = max(tb1 + 1, 0), j1 = min(tb3, 15);
        const int32_t d0 = act ? j0 : 99, d1 = act ? j1 + (R.vsel != 0x00010203u) : -1;
        rr_load17(R.va + 4 * ((int64_t)(16 * b) - (int64_t)R.b1 - 1), d0, d1, R.vsafe, vlo, vhi, dv);
    }
}

// key field present in block b iff b1 >= 16b for some lane; value field iff b3 >= 16b and b1 + 1 <=
// 16b + 15 for some lane that still has block b
__device__ __forceinline__ bool rr_need_k(const RrLane &R, uint32_t b) { return __any(R.nb > b && R.b1 >= 16 * b); }
__device__ __forceinline__ bool rr_need_v(const RrLane &R, uint32_t b) {
    return __any(R.nb > b && R.b3 >= 16 * b && R.b1 + 1 <= 16 * b + 15);
}

template <bool SHORT>
__global__ __launch_bounds__(256) void k_leaf_rreg(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                   const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                   uint64_t n, uint8_t *__restrict__ out,
                                                   const uint32_t *__restrict__ list, const uint64_t *__restrict__ total,
                                                   uint32_t *__restrict__ gctr, uint32_t grain, KeyOut KO) {
    const uint32_t lane = threadIdx.x & 63;
    const uint8_t *klo = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(kb + koff[0]) & ~uintptr_t(3));
    const uint8_t *khi =
        reinterpret_cast<const uint8_t *>((reinterpret_cast<uintptr_t>(kb + koff[n]) + 3) & ~uintptr_t(3));
    const uint8_t *vlo = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(vb + voff[0]) & ~uintptr_t(3));
    const uint8_t *vhi =
        reinterpret_cast<const uint8_t *>((reinterpret_cast<uintptr_t>(vb + voff[n]) + 3) & ~uintptr_t(3));
    const uint64_t T = *total;
    const uint64_t nch = (T + 63) / 64;
    if (nch == 0) return;
    ChunkSource<true> src{0, 0, 0, gctr, grain};
    for (uint64_t c = src.get(lane); c < nch; c = src.get(lane)) {
        const uint64_t p = c * 64 + lane;
        const bool valid = p < T;
        const uint32_t r = list[valid ? p : c * 64];  // idle lanes shadow the chunk's first record
        const RrLane R = rr_lane(kb, vb, koff[r], koff[r + 1], voff[r], voff[r + 1], valid, klo, khi, vlo, vhi);
        uint32_t nbw = R.nb;  // wave-uniform block count
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nbw = max(nbw, (uint32_t)__shfl_xor((int)nbw, o));
        nbw = __builtin_amdgcn_readfirstlane(nbw);
        uint32_t dk[17], dv[17];
        bool fk = rr_need_k(R, 0), fv = rr_need_v(R, 0);
        rr_fetch(R, 0, fk, fv, klo, khi, vlo, vhi, dk, dv);
        uint32_t st[8];
        sha_init(st);
        for (uint32_t b = 0; b < nbw; ++b) {
            const int32_t tb1 = (int32_t)R.b1 - (int32_t)(16 * b), tb3 = (int32_t)R.b3 - (int32_t)(16 * b);
            const bool act = R.nb > b;
            uint32_t w[16];
            if (fk && KO.kdst) {  // key ownership: the key dwords just loaded, at the same offsets
                const uint8_t *a = R.ka + 4 * ((int64_t)(16 * b) - 1);
                const uint8_t *kend = R.kp + R.k;
#pragma unroll
                for (int j = 0; j < 17; ++j) {
                    const uint8_t *q = a + 4 * j;
                    if (act && q + 4 > R.kp && q < kend && q >= klo && q >= kb && q + 4 <= khi &&
                        (uint64_t)(q + 4 - kb) <= KO.kcap)
                        *reinterpret_cast<uint32_t *>(KO.kdst + (q - kb)) = dk[j];
                }
            }
            if (fk) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t kw = rg_be(dk[j + 1], dk[j], R.ksel);
                    const uint32_t vw = fv ? rg_be(dv[j + 1], dv[j], R.vsel) : 0u;
                    w[j] = j <= tb1 ? kw : vw;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) w[j] = rg_be(dv[j + 1], dv[j], R.vsel);
            }
            if (__any(act && tb1 >= -1 && tb1 <= 15)) {  // b1 / b1 + 1 in this block
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (j == tb1) w[j] = (w[j] & R.hc) | R.vh;
                    if (j == tb1 + 1) w[j] = (R.vt & R.hc) | (w[j] & ~R.hc);
                }
            }
            if (b == 0) w[0] = R.k;
            if (__any(act && tb3 <= 15)) {  // b3 (and the zero tail) in this block
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    if (j == tb3) w[j] = (w[j] & R.he) | R.term;
                    if (j > tb3) w[j] = 0u;
                }
                if (b + 1 == R.nb) w[15] = R.L * 8;  // bit length (L < 2^29: the high word stays 0)
            }
            if (b + 1 < nbw) {  // next block's sources in flight during this block's rounds
                fk = rr_need_k(R, b + 1);
                fv = rr_need_v(R, b + 1);
                rr_fetch(R, b + 1, fk, fv, klo, khi, vlo, vhi, dk, dv);
            }
            if (act) {
                uint32_t s2[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) s2[i] = st[i];
                sha_compress<SHORT>(s2, w);
#pragma unroll
                for (int i = 0; i < 8; ++i) st[i] = s2[i];
            }
        }
        if (valid) store_digest(out + 32 * (uint64_t)r, st);
    }
}

}  // namespace

void launch_leaf_hash_multi(const LeafBatches &B, uint32_t k, uint64_t mmax, uint8_t *out, hipStream_t st) {
    if (!k || !mmax) return;
    const dim3 grid((uint32_t)ceil_div(mmax, (uint64_t)LEAF_WAVES * 64), k);
    if (sha_variant() == 0)
        hipLaunchKernelGGL(k_leaf_multi<false>, grid, dim3(64 * LEAF_WAVES), 0, st, B, out);
    else
        hipLaunchKernelGGL(k_leaf_multi<true>, grid, dim3(64 * LEAF_WAVES), 0, st, B, out);
    MKV_LAUNCH_CHECK();
}

// The counter block (leaf_ctr_words): the head described at CTR_FLAGS, one flag per chunk; then, 16-B
// aligned, the ragged bucketing scratch: the list total (u64), the class-ordered record list (u32 per
// record) and the block-count class of every record (u8).
struct RaggedScratch {
    uint8_t *cls;  // block-count class per record (written for listed chunks by k_leaf_direct)
    uint64_t *total;
    uint32_t *list;
    uint32_t nwg;
};
static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
static RaggedScratch ragged_scratch(uint32_t *ctr, uint64_t n, size_t *bytes_out = nullptr) {
    const uint64_t nch = (n + 63) / 64;
    const uint32_t nwg = (uint32_t)std::max<uint64_t>(1, ceil_div(nch, RG_SCATTER_CHUNKS));
    size_t off = align16(4 * (CTR_FLAGS + (size_t)nch));
    RaggedScratch R;
    uint8_t *base = reinterpret_cast<uint8_t *>(ctr);
    R.total = reinterpret_cast<uint64_t *>(base + off);
    off = align16(off + 8);
    R.list = reinterpret_cast<uint32_t *>(base + off);
    off = align16(off + 4 * (size_t)n);
    R.cls = base + off;
    off = align16(off + (size_t)n + 64);
    R.nwg = nwg;
    if (bytes_out) *bytes_out = off;
    return R;
}

size_t leaf_ctr_words(uint64_t n) {
    size_t bytes = 0;
    (void)ragged_scratch(nullptr, n, &bytes);
    return bytes / 4 + 4;
}

// MKV_LEAF_RAGGED (A/B knob): listed chunks go through the bucketed ragged kernels — 1 (default) the LDS
// form k_leaf_ragged, 2 the register form k_leaf_rreg — or 0: the round-2 LDS chunk kernel k_leaf_list.
static int leaf_ragged_enabled() {
    static const int v = [] {
        const char *e = getenv("MKV_LEAF_RAGGED");
        return e ? atoi(e) : 1;
    }();
    return v;
}

// The listed chunks of ctr (k_leaf_direct): bucket their records by block count, then hash them.
// MKV_RAGGED_WGS (A/B knob): k_leaf_ragged workgroups per CU (48 KiB of LDS each). Default 3 (fills the
// CU's LDS, 3 waves per SIMD): 10M ragged build 4.06-4.09 -> 3.93 ms/step, the hash 2.70 -> 2.22 ms,
// although an ordering workgroup then finds no LDS beside it until the hash finishes; 2 leaves room.
static int ragged_wgs() {
    static const int v = [] {
        const char *e = getenv("MKV_RAGGED_WGS");
        const int x = e ? atoi(e) : 3;
        return x < 1 ? 1 : (x > 3 ? 3 : x);
    }();
    return v;
}

// MKV_RREG_WGS (A/B knob): k_leaf_rreg workgroups (4 waves, no LDS) per CU.
static int rreg_wgs() {
    static const int v = [] {
        const char *e = getenv("MKV_RREG_WGS");
        const int x = e ? atoi(e) : 4;
        return x < 1 ? 1 : (x > 8 ? 8 : x);
    }();
    return v;
}

template <bool SHORT>
static void launch_ragged_stage(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff,
                                uint64_t n, uint8_t *out, uint32_t *ctr, const KeyOut &KO, hipStream_t st) {
    static int cus = [] {
        int dev = 0, c = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c > 0 ? c : 256;
    }();
    const RaggedScratch R = ragged_scratch(ctr, n);
    hipLaunchKernelGGL(k_ragged_scatter, dim3(R.nwg), dim3(256), 0, st, R.cls, n, ctr, R.total, R.list);
    if (leaf_ragged_enabled() == 2) {
        const uint64_t grid = std::min<uint64_t>((uint64_t)cus * rreg_wgs(), ceil_div(ceil_div(n, 64), 4));
        hipLaunchKernelGGL(k_leaf_rreg<SHORT>, dim3((uint32_t)std::max<uint64_t>(grid, 1)), dim3(256), 0, st, kb, koff,
                           vb, voff, n, out, R.list, R.total, ctr + 2, 2u, KO);
        MKV_LAUNCH_CHECK();
        return;
    }
    const uint64_t grid = std::min<uint64_t>((uint64_t)cus * ragged_wgs(), ceil_div(ceil_div(n, 64), RG_WAVES));
    hipLaunchKernelGGL(k_leaf_ragged<SHORT>, dim3((uint32_t)std::max<uint64_t>(grid, 1)), dim3(64 * RG_WAVES), 0, st,
                       kb, koff, vb, voff, n, out, R.list, R.total, ctr + 2, 2u, KO);
    MKV_LAUNCH_CHECK();
}

// SHA round form of k_leaf_direct (MKV_LEAF_SHA, default 0 = plain association, fewer instructions):
// with the LDS-free kernel the short-chain form (1) measured slower (leaf 1.38 vs 1.32 ms beside the sort)
static int leaf_sha_variant() {
    static const int v = [] {
        const char *e = getenv("MKV_LEAF_SHA");
        return e ? atoi(e) : 0;
    }();
    return v;
}

static int leaf_kernel_variant() {
    static const int v = [] {
        // 3 = k_leaf_direct (default), 2 = k_leaf_dma, 1 = k_leaf_persist, 0 = k_leaf_hash
        const char *e = getenv("MKV_LEAF_KERNEL");
        return e ? atoi(e) : 3;
    }();
    return v;
}

static uint32_t leaf_dyn_grain() {
    static const uint32_t v = [] {
        const char *e = getenv("MKV_LEAF_DYN");  // chunks per atomic grab; 0 = static round-robin
        const int x = e ? atoi(e) : 4;
        return (uint32_t)(x < 0 ? 0 : x);
    }();
    return v;
}

bool launch_leaf_hash(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                      uint8_t *out, hipStream_t st, uint32_t *ctr, uint8_t *kcopy, uint64_t kcap, uint64_t *ocopy) {
    if (n == 0) return false;
    uint64_t waves = ceil_div(n, 64);
    uint64_t blocks = ceil_div(waves, LEAF_WAVES);
    if (leaf_kernel_variant() == 3 && ctr) {
        static int cus3 = [] {
            int dev = 0, c = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
            return c > 0 ? c : 256;
        }();
        static int wgs3 = [] {
            const char *e = getenv("MKV_LEAF_WGS");
            int v = e ? atoi(e) : 2;
            return v < 1 ? 1 : (v > 8 ? 8 : v);
        }();
        static const int grid3 = [] {  // MKV_LEAF_GRID (A/B knob): total workgroups instead of wgs per CU
            const char *e = getenv("MKV_LEAF_GRID");
            return e ? atoi(e) : 0;
        }();
        const uint64_t pblocks = std::min<uint64_t>(blocks, grid3 > 0 ? (uint64_t)grid3 : (uint64_t)cus3 * wgs3);
        const uint32_t grain = std::max<uint32_t>(leaf_dyn_grain(), 1u);
        // the span copy of listed chunks rounds to 16 B like the staged paths: kb must be 16-B aligned. With
        // the ragged stage, listed chunks' keys are copied by k_leaf_ragged instead (it loads them anyway)
        const bool rag = leaf_ragged_enabled() != 0;
        const RaggedScratch R = ragged_scratch(ctr, n);
        const KeyOut KO{(reinterpret_cast<uintptr_t>(kb) & 15) == 0 ? kcopy : nullptr, ocopy, kcap,
                        rag ? R.cls : nullptr, rag ? 1u : 0u};
        const KeyOut KOr{KO.kdst, nullptr, kcap, nullptr, 0u};
        MKV_HIP(hipMemsetAsync(ctr, 0, CTR_FLAGS * sizeof(uint32_t), st));
        if (leaf_sha_variant() == 0) {
            hipLaunchKernelGGL((k_leaf_direct<false, 32, 100>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb,
                               koff, vb, voff, n, out, ctr, grain, KO);
            if (rag)
                launch_ragged_stage<false>(kb, koff, vb, voff, n, out, ctr, KOr, st);
            else
                hipLaunchKernelGGL(k_leaf_list<false>, dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff,
                                   vb, voff, n, out, ctr);
        } else {
            hipLaunchKernelGGL((k_leaf_direct<true, 32, 100>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb,
                               koff, vb, voff, n, out, ctr, grain, KO);
            if (rag)
                launch_ragged_stage<true>(kb, koff, vb, voff, n, out, ctr, KOr, st);
            else
                hipLaunchKernelGGL(k_leaf_list<true>, dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff,
                                   vb, voff, n, out, ctr);
        }
        MKV_LAUNCH_CHECK();
        return KO.kdst != nullptr;
    }
    if (leaf_kernel_variant() == 2 && ctr) {
        static int cus2 = [] {
            int dev = 0, c = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
            return c > 0 ? c : 256;
        }();
        static int wgs2 = [] {
            // 2 per CU: with 3 the leaf hash runs 1.27 instead of 1.45 ms but the co-running ordering
            // stage stretches to 1.4-1.65 ms and becomes the critical path (build 2.32-2.60 vs 2.31 ms)
            const char *e = getenv("MKV_LEAF_WGS");
            int v = e ? atoi(e) : 2;
            return v < 1 ? 1 : (v > 4 ? 4 : v);
        }();
        const uint64_t pblocks = std::min<uint64_t>(blocks, (uint64_t)cus2 * wgs2);
        const uint32_t grain = std::max<uint32_t>(leaf_dyn_grain(), 1u);
        const KeyOut KO{(reinterpret_cast<uintptr_t>(kb) & 15) == 0 ? kcopy : nullptr, ocopy, kcap, nullptr, 0u};
        MKV_HIP(hipMemsetAsync(ctr, 0, 2 * sizeof(uint32_t), st));
        if (sha_variant() == 0) {
            hipLaunchKernelGGL((k_leaf_dma<false, 32, 100>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff,
                               vb, voff, n, out, ctr, grain, KO);
            hipLaunchKernelGGL(k_leaf_list<false>, dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff, vb,
                               voff, n, out, ctr);
        } else {
            hipLaunchKernelGGL((k_leaf_dma<true, 32, 100>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff,
                               vb, voff, n, out, ctr, grain, KO);
            hipLaunchKernelGGL(k_leaf_list<true>, dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff, vb,
                               voff, n, out, ctr);
        }
        MKV_LAUNCH_CHECK();
        return KO.kdst != nullptr;
    }
    if (leaf_kernel_variant() >= 1) {
        static int cus = [] {
            int dev = 0, c = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
            return c > 0 ? c : 256;
        }();
        // Bounded residency (default 2 workgroups = 8 waves per CU, 2 per SIMD): leaves VGPRs, LDS and
        // wave slots for the aux-stream sort workgroups (k_os_pass needs 165 VGPRs/wave + 56.5 KiB LDS).
        static int wgs = [] {
            const char *e = getenv("MKV_LEAF_WGS");
            int v = e ? atoi(e) : 2;
            return v < 1 ? 1 : (v > 4 ? 4 : v);
        }();
        // MKV_LEAF_GRID (A/B knob): total persistent workgroups instead of wgs per CU; with the dynamic
        // chunk hand-out an uneven grid no longer leaves CUs with an extra workgroup finishing last.
        static const int grid = [] {
            const char *e = getenv("MKV_LEAF_GRID");
            return e ? atoi(e) : 0;
        }();
        const uint64_t pblocks = std::min<uint64_t>(blocks, grid > 0 ? (uint64_t)grid : (uint64_t)cus * wgs);
        const uint32_t grain = ctr ? leaf_dyn_grain() : 0;
        // the fused copy needs kb 16-B aligned (same alignment as the destination)
        const KeyOut KO{(reinterpret_cast<uintptr_t>(kb) & 15) == 0 ? kcopy : nullptr, ocopy, kcap, nullptr, 0u};
        if (grain) {
            MKV_HIP(hipMemsetAsync(ctr, 0, sizeof(uint32_t), st));
            if (sha_variant() == 0)
                hipLaunchKernelGGL((k_leaf_persist<false, true>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st,
                                   kb, koff, vb, voff, n, out, ctr, grain, KO);
            else
                hipLaunchKernelGGL((k_leaf_persist<true, true>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st,
                                   kb, koff, vb, voff, n, out, ctr, grain, KO);
        } else if (sha_variant() == 0) {
            hipLaunchKernelGGL((k_leaf_persist<false, false>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st,
                               kb, koff, vb, voff, n, out, ctr, 0u, KO);
        } else {
            hipLaunchKernelGGL((k_leaf_persist<true, false>), dim3((uint32_t)pblocks), dim3(64 * LEAF_WAVES), 0, st,
                               kb, koff, vb, voff, n, out, ctr, 0u, KO);
        }
        MKV_LAUNCH_CHECK();
        return KO.kdst != nullptr;
    }
    if (sha_variant() == 0)
        hipLaunchKernelGGL(k_leaf_hash<false>, dim3((uint32_t)blocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff, vb, voff,
                           n, out);
    else
        hipLaunchKernelGGL(k_leaf_hash<true>, dim3((uint32_t)blocks), dim3(64 * LEAF_WAVES), 0, st, kb, koff, vb, voff,
                           n, out);
    MKV_LAUNCH_CHECK();
    return false;
}

}  // namespace mkv
