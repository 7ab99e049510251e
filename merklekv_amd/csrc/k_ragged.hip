// k_ragged.hip — Kernel A for store-shaped records: R1 + R2 (merkle.rs:7-16, :45-49) for any key / value
// lengths at any byte offsets, the records a real SYNC snapshot hands over (sync.rs:109-115 hashes
// arbitrary &str pairs).
//
// Work distribution: lane refill. A wave keeps one record per lane and runs one SHA-256 compression per
// step; a lane whose record ends takes the next record of the wave's queue (ballot + mbcnt over the lanes
// that need one), so records of 1..n blocks mix freely at full wave width with no bucketing pass. The
// queue hands out 64-record chunks from a device counter (RG_GRAIN per atomic). Everything a step needs
// is loaded one step ahead: the next record's offsets (koff/voff pairs) while the current block is
// compressed, and the next block's source dwords likewise.
//
// Message words. Block `blk` of a record covers stream words 16 blk .. 16 blk + 15 of
//   u32_be(k) || key || u32_be(v) || value || 0x80 || 0.. || u64_be(8L)
// The key occupies stream words 1 .. b1 (b1 = (4 + k) / 4; word b1 also carries the head of u32_be(v)),
// the value words b1 + 1 .. b3 (b3 = L / 4; word b1 + 1 starts with the tail of u32_be(v), word b3 ends
// with 0x80). Per lane the block is assembled in a private 16-dword LDS slot from three 16-word RUNS
// whose positions depend on the lane's record:
//   key run   — 16 key words ENDING at position tb1 = b1 - 16 blk (or the whole block when the key goes
//               on): its last word is word b1 at a static register index, spliced with the head of
//               u32_be(v) in registers;
//   value run — 16 value words STARTING at tb1 + 1: its first word (b1 + 1) is spliced with the tail of
//               u32_be(v), again at a static index;
//   zero run  — 16 zeros starting after word b3;
// then one read-modify-write puts 0x80 into word b3, and the first / last block get u32_be(k) / 8L.
// Runs are written at a dynamic base with static offsets (ds_write2_b32), so every source word costs one
// v_perm_b32 (byte-swap + byte offset from two aligned dwords) and no per-word compare. Positions outside
// the slot land in trash dwords: a lane's slot is followed by 20 dwords shared with the next lane's
// leading trash (the key run reaches 15 below, the value / zero runs 15 above); nobody reads them.
#include "common.hpp"
#include "kernels.hpp"
#include "leaf.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

constexpr int RG_WAVES = 4;                             // waves per workgroup
// Lane stride 34 dwords: slots 8-B aligned, read back as 8-B words — lanes 0-31 (and 32-63) of a
// ds_read_b64 then start on 32 distinct even banks of 64 (34 / 2 = 17 is odd), conflict-free — and a
// 4-wave workgroup takes 34.3 KiB: three of them (12 waves per CU) leave room for a 56.5-KiB sort tile,
// two of them (the default since round 6) for the sort's tiles to co-run at full width.
constexpr uint32_t RG_STRIDE = 34;                      // dwords per lane
constexpr uint32_t RG_FRONT = 16;                       // trash below lane 0's slot
constexpr uint32_t RG_WAVE_DW = RG_FRONT + 64 * RG_STRIDE;  // lane 63 reaches dword 16 + 63 x 34 + 30
static_assert(RG_FRONT + 63 * RG_STRIDE + 31 <= RG_WAVE_DW, "lane 63's trash fits the wave region");
static_assert(RG_STRIDE >= 31 && RG_STRIDE % 2 == 0 && (RG_STRIDE / 2) % 2 == 1,
              "trash shared with neighbours; 8-B aligned, conflict-free slots");
constexpr uint32_t RG_GRAIN = 4;                        // virtual chunks per hand-out atomic
constexpr uint32_t RG_INV = 0xFFFFFFFFu;
#ifndef MKV_RAGGED_WGS
// workgroups per CU (persistent grid). Round 6: 2 instead of 3 — with the faster leaf stage the radix
// passes beside it had become the ragged build's critical path (sort 2.0 vs hash 1.8 ms); at 2 the hash
// runs ~5 % slower but the sort ~0.25 ms faster: build 2.92-2.96 -> 2.80-2.85 ms (interleaved A/B, 4 reps)
#define MKV_RAGGED_WGS 2
#endif

typedef uint32_t rg4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t rg3 __attribute__((ext_vector_type(3), aligned(4)));

// 17 dwords at base + a (base and a 4-B aligned; gfx950 serves 16-B loads at 4-B alignment). Addresses
// stay pointer arithmetic on the kernel's blob arguments so the loads are global_load, not flat_load
// (a flat load also counts in lgkmcnt: every LDS wait would wait for it).
__device__ __forceinline__ void rg_ld17(const uint8_t *base, int64_t a, uint32_t d[17]) {
    const rg4 *q = reinterpret_cast<const rg4 *>(base + a);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const rg4 x = q[g];
        d[4 * g] = x.x;
        d[4 * g + 1] = x.y;
        d[4 * g + 2] = x.z;
        d[4 * g + 3] = x.w;
    }
    d[16] = reinterpret_cast<const uint32_t *>(base + a)[16];
}
// Big-endian word of the 4 bytes at byte offset sel (0..3, encoded as a v_perm selector) of (lo, hi).
__device__ __forceinline__ uint32_t rg_be(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// One lane's record: addresses and the constants of its boundary words.
struct RgRec {
    int64_t ka, va;       // floor4(key start), floor4(value start - (k & 3)) as offsets from the dword-aligned
                          // blob bases (value words align to stream words)
    uint32_t ksel, vsel;  // v_perm selectors of the two sources' byte offsets
    uint32_t k, L, b1, b3, nb, blk, r;
    uint32_t hc;          // head mask of word b1's key bytes (k & 3 of them)
    uint32_t vhl, vtl;    // u32_be(v) split across words b1 / b1 + 1
    uint32_t he, term;    // word b3: kept bytes (L & 3), 0x80 terminator
    bool live;
};

// kmis / vmis: byte misalignment of the key / value blob pointers (the bases are the blobs rounded down to
// a dword). k1, v1: the low words of the record's end offsets (a record is shorter than 4 GiB).
__device__ __forceinline__ void rg_take(RgRec &R, uint64_t k0, uint32_t k1, uint64_t v0, uint32_t v1, uint32_t r,
                                        uint32_t kmis, uint32_t vmis) {
    const uint32_t k = k1 - (uint32_t)k0, v = v1 - (uint32_t)v0;
    const uint32_t c4 = k & 3;
    R.k = k;
    R.L = 8 + k + v;
    R.nb = (R.L + 72) >> 6;
    R.b1 = (4 + k) >> 2;
    R.b3 = R.L >> 2;
    R.blk = 0;
    R.r = r;
    const int64_t kp = (int64_t)(kmis + k0), vq = (int64_t)(vmis + v0) - c4;  // vq < 0: unsafe (first record)
    R.ka = kp & ~int64_t(3);
    R.va = vq & ~int64_t(3);
    R.ksel = 0x00010203u + (uint32_t)(kp & 3) * 0x01010101u;
    R.vsel = 0x00010203u + (uint32_t)(vq & 3) * 0x01010101u;
    R.hc = ~(0xFFFFFFFFu >> (8 * c4));
    R.vhl = v >> (8 * c4);
    R.vtl = v << ((32 - 8 * c4) & 31);  // only its head c4 bytes are used (hc)
    const uint32_t e4 = R.L & 3;
    R.he = ~(0xFFFFFFFFu >> (8 * e4));
    R.term = 0x80000000u >> (8 * e4);
    R.live = true;
}

// Records near the blobs' ends (every record of a blob of empty or tiny keys) go to k_leaf_edges instead:
// no bounds checks in this kernel's loads (the checked form cost ~70 VGPRs). The split is an interval:
// record i is hashed here iff
//   koff[i] >= koff[0] + 67,  voff[i] >= voff[0] + 6,  koff[i+1] + 68 <= koff[n],  voff[i+1] + 136 <= voff[n]
// — each test monotone in i, so the records left over are a prefix and a suffix that k_leaf_edges finds by
// itself (two searches), runs on another stream beside this kernel and needs no list from it. The test
// keeps every source dword a block loads (key run: [ka - 60, ka + 4 b1 + 4], value run: [va, va + 4 (b3 -
// b1) + 64), ka / va the dword-aligned starts) inside the blobs' dword ranges [klo, khi) / [vlo, vhi):
//   ka >= kmis + k0 - 3 >= klo + 64;   ka + 4 b1 + 64 <= kmis + k0 + (4 + k) + 64 = kmis + k1 + 68 <= khi;
//   va >= vmis + v0 - (k & 3) - 3 >= vmis + voff[0] >= vlo;
//   va + 4 (b3 - b1) + 128 <= vmis + v0 + (v + 7) + 128 < vmis + v1 + 136 <= vhi
// (4 b1 <= 4 + k, 4 b1 >= k + 1, 4 b3 <= 8 + k + v). Round 6: this replaced a per-record bounds test kept
// beside it as a guard (~10 VALU instructions per step: a take runs in most steps of a wave).
struct RgSplit {
    uint64_t kA, vA, KN, VN;  // koff[0] + 67, voff[0] + 6, koff[n], voff[n]
};
__device__ __forceinline__ bool rg_inner(const RgSplit &X, uint64_t k0, uint64_t k1, uint64_t v0, uint64_t v1) {
    return k0 >= X.kA && v0 >= X.vA && k1 + 68 <= X.KN && v1 + 136 <= X.VN;
}
__device__ __forceinline__ void rg_take_or_leave(RgRec &R, uint64_t k0, uint32_t k1, uint64_t v0, uint32_t v1,
                                                 uint32_t r, uint32_t kmis, uint32_t vmis, const RgSplit &X) {
    rg_take(R, k0, k1, v0, v1, r, kmis, vmis);
    R.live = rg_inner(X, k0, k0 + R.k, v0, v0 + (R.L - 8 - R.k));
}

// The block's positions of the boundary words (block-relative, may lie outside 0..15).
struct RgPos {
    int32_t tb1, tb3;
    int32_t kend;   // key run ends here (min(tb1, 15))
    int32_t vbeg;   // value run starts here (max(tb1 + 1, 0))
    bool key_in, val_in;
};
__device__ __forceinline__ RgPos rg_pos(const RgRec &R) {
    RgPos P;
    P.tb1 = (int32_t)R.b1 - (int32_t)(16 * R.blk);
    P.tb3 = (int32_t)R.b3 - (int32_t)(16 * R.blk);
    P.kend = min(P.tb1, 15);
    P.vbeg = max(P.tb1 + 1, 0);
    P.key_in = R.live && P.tb1 >= 0;
    P.val_in = R.live && P.tb1 <= 14 && P.tb3 >= 0;
    return P;
}

// Source dwords of the lane's current (record, block): key run and value run.
__device__ __forceinline__ void rg_fetch(const RgRec &R, const uint8_t *kbase, const uint8_t *vbase, uint32_t dk[17],
                                         uint32_t dv[17]) {
    const RgPos P = rg_pos(R);
    const int64_t ak = R.ka + 4 * (int64_t)((int32_t)(16 * R.blk) + P.kend - 16);
    const int64_t av = R.va + 4 * (int64_t)((int32_t)(16 * R.blk) + P.vbeg - (int32_t)R.b1 - 1);
    if (P.key_in) rg_ld17(kbase, ak, dk);
    if (P.val_in) rg_ld17(vbase, av, dv);
}

// Virtual chunk ids -> chunks: the fixed-shape kernel's slots first (NW x LEAF_GRAIN ids: slot v / G,
// its (v % G)-th chunk; ids past a slot's count are skipped), then chunks [B, nch).
struct RgQueue {
    uint32_t qc, qn, qpos;  // current / next chunk, records of qc handed out
    uint32_t pv, pe;        // ids left in the current grab
    uint32_t pnext;         // first id of the next grab (its atomic was issued when this grab opened)
    uint32_t nv, nslot, B;  // ids in all, ids of the slot part, first chunk never handed to k_leaf_direct
};

// The fixed kernel's hand-off state (leaf.hpp): B, and whether any slot holds chunks.
__device__ __forceinline__ void rg_handoff(const uint32_t *ctr, uint32_t nch, uint32_t nw, uint32_t *B, uint32_t *nslot) {
    const uint64_t b = (uint64_t)nw + ctr[CTR_FIXED];
    *B = b < nch ? (uint32_t)b : nch;
    *nslot = ctr[CTR_STOP] ? nw * LEAF_GRAIN : 0u;
}
__device__ __forceinline__ uint32_t rg_slot_chunk(const uint32_t *ctr, uint32_t v) {  // RG_INV: empty id
    const uint32_t s = ctr[CTR_LIST + v / LEAF_GRAIN], off = v % LEAF_GRAIN;
    return off < (s & 31u) ? (s >> 5) + off : RG_INV;
}

__device__ __forceinline__ uint32_t rg_grab(uint32_t *ctr, uint32_t lane) {
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(&ctr[CTR_RAGGED], RG_GRAIN);
    return __builtin_amdgcn_readfirstlane(__shfl(b, 0));
}

__device__ __forceinline__ uint32_t rg_next_chunk(RgQueue &Q, uint32_t *ctr, uint32_t lane) {
    while (true) {
        if (Q.pv >= Q.pe) {
            if (Q.pnext >= Q.nv) return RG_INV;  // nothing left anywhere: no further atomics
            Q.pv = Q.pnext;
            Q.pe = Q.pnext + RG_GRAIN;
            Q.pnext = rg_grab(ctr, lane);
        }
        const uint32_t v = Q.pv++;
        if (v >= Q.nv) return RG_INV;
        if (v >= Q.nslot) return Q.B + (v - Q.nslot);
        const uint32_t c = __builtin_amdgcn_readfirstlane(rg_slot_chunk(ctr, v));
        if (c != RG_INV) return c;
    }
}

template <bool SHORT>
__global__ __launch_bounds__(64 * RG_WAVES) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_leaf_ragged(const uint8_t *__restrict__ kb,
                                                              const uint64_t *__restrict__ koff,
                                                              const uint8_t *__restrict__ vb,
                                                              const uint64_t *__restrict__ voff, uint64_t n,
                                                              uint8_t *__restrict__ out, uint32_t *__restrict__ ctr,
                                                              uint32_t nw, KeyOut KO) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[RG_WAVES * RG_WAVE_DW];  // 34.3 KiB
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *lb = lds_all + wave * RG_WAVE_DW + RG_FRONT + lane * RG_STRIDE;  // this lane's block slot

    const uint32_t nch = (uint32_t)((n + 63) / 64);
    RgQueue Q;
    rg_handoff(ctr, nch, nw, &Q.B, &Q.nslot);
    Q.nv = Q.nslot + (nch - Q.B);
    if (Q.nv == 0) return;  // k_leaf_direct hashed every chunk

    // dword-aligned blob bases; the blobs' byte ranges rounded out to whole dwords (as offsets from the
    // bases): no source load leaves them
    const uint32_t kmis = (uint32_t)(reinterpret_cast<uintptr_t>(kb) & 3), vmis = (uint32_t)(reinterpret_cast<uintptr_t>(vb) & 3);
    const uint8_t *kbase = kb - kmis, *vbase = vb - vmis;
    const RgSplit X{koff[0] + 67, voff[0] + 6, koff[n], voff[n]};

    Q.pnext = rg_grab(ctr, lane);
    Q.pv = Q.pe = 0;
    Q.qc = rg_next_chunk(Q, ctr, lane);
    if (Q.qc == RG_INV) return;
    Q.qn = rg_next_chunk(Q, ctr, lane);
    Q.qpos = 0;

    // next record of this lane (offsets in flight one step ahead)
    uint64_t nk0 = 0, nv0 = 0;
    uint32_t nk1 = 0, nv1 = 0;  // low words of koff[rec + 1] / voff[rec + 1]
    uint32_t nrec = 0;
    bool nok = false;
    auto refill = [&](bool need) {
        const uint64_t m = __ballot(need);
        const uint32_t cnt = (uint32_t)__popcll(m);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t pos = Q.qpos + rank;
        const uint32_t ch = pos < 64 ? Q.qc : Q.qn;
        const uint64_t rec = (uint64_t)ch * 64 + (pos & 63);
        if (need) {
            nok = ch != RG_INV && rec < n;
            if (nok) {
                nrec = (uint32_t)rec;
                // koff[rec] and the low word of koff[rec + 1] (lengths are < 4 GiB): 12-B loads, so no
                // loaded dword is dead — a dead destination register gets reused as a temporary, and the
                // write-after-write wait on it would stall the step on these loads
                const rg3 *kq = reinterpret_cast<const rg3 *>(koff + rec);
                const rg3 *vq = reinterpret_cast<const rg3 *>(voff + rec);
                const rg3 a = *kq, b = *vq;
                nk0 = ((uint64_t)a.y << 32) | a.x;
                nk1 = a.z;
                nv0 = ((uint64_t)b.y << 32) | b.x;
                nv1 = b.z;
            }
        }
        if (Q.qc != RG_INV) {
            Q.qpos += cnt;
            if (Q.qpos >= 64) {
                Q.qpos -= 64;
                Q.qc = Q.qn;
                Q.qn = Q.qc == RG_INV ? RG_INV : rg_next_chunk(Q, ctr, lane);
            }
        }
    };

    RgRec R;
    R.live = false;
    R.k = R.L = R.b1 = R.b3 = R.nb = R.blk = R.r = 0;
    R.ka = R.va = 0;
    R.ksel = R.vsel = R.hc = R.vhl = R.vtl = R.he = R.term = 0;
    // key ownership: every record of a ragged chunk is taken exactly once (leaf.hpp); its offsets are
    // stored then, from registers that were loaded a step earlier (a store in the refill itself would wait
    // for the offsets it just requested)
    auto take = [&]() {
        rg_take_or_leave(R, nk0, nk1, nv0, nv1, nrec, kmis, vmis, X);
        if (KO.odst) {
            KO.odst[nrec] = nk0;
            if ((uint64_t)nrec + 1 == n) KO.odst[n] = koff[n];
        }
    };
    refill(true);
    if (nok) take();
    nok = false;
    refill(true);

    uint32_t dk[17], dv[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) dk[j] = dv[j] = 0;
    rg_fetch(R, kbase, vbase, dk, dv);
    uint32_t st[8];
    sha_init(st);

    while (__any(R.live || nok)) {
        // Every load of the previous step (source dwords, next offsets) lands here, on every path: the
        // compiler's own waits sit inside the lane-conditional assembly branches, so on a path that skipped
        // them it waited again in the middle of the step, in front of the new loads.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
        // ---- assemble this step's block in the lane's LDS slot ----
        uint32_t w[16];
        {
            const RgPos P = rg_pos(R);
            uint32_t kr[16], vr[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) kr[m] = rg_be(dk[m + 1], dk[m], R.ksel);
            if (P.tb1 <= 15) kr[15] = (R.hc & kr[15]) | (~R.hc & R.vhl);  // word b1: key tail | head of u32_be(v)
#pragma unroll
            for (int m = 0; m < 16; ++m) vr[m] = rg_be(dv[m + 1], dv[m], R.vsel);
            if (P.tb1 >= -1) vr[0] = (R.hc & R.vtl) | (~R.hc & vr[0]);  // word b1 + 1: tail of u32_be(v) | value
            if (P.key_in) {
                uint32_t *p = lb + (P.kend - 15);
#pragma unroll
                for (int m = 0; m < 16; ++m) p[m] = kr[m];
            }
            if (P.val_in) {
                uint32_t *p = lb + P.vbeg;
#pragma unroll
                for (int m = 0; m < 16; ++m) p[m] = vr[m];
            }
            const int32_t z = min(max(P.tb3 + 1, 0), 16);
            if (R.live && z <= 15) {
                uint32_t *p = lb + z;
#pragma unroll
                for (int m = 0; m < 16; ++m) p[m] = 0u;
            }
            if (R.live && P.tb3 >= 0 && P.tb3 <= 15) {
                const uint32_t x = lb[P.tb3];
                lb[P.tb3] = (x & R.he) | R.term;
            }
            if (R.live && R.blk == 0) lb[0] = R.k;
            if (R.live && R.blk + 1 == R.nb) {  // 64-bit bit length 8L
                lb[14] = R.L >> 29;
                lb[15] = R.L << 3;
            }
            const uint2 *l2 = reinterpret_cast<const uint2 *>(lb);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint2 x = l2[j];
                w[2 * j] = x.x;
                w[2 * j + 1] = x.y;
            }
        }
        // ---- advance: next block, or the next record ----
        const bool was_live = R.live;
        const bool fin = R.live && R.blk + 1 == R.nb;
        const uint32_t rfin = R.r;
        if (R.live && !fin) {
            ++R.blk;
        } else {
            if (nok) take();
            else R.live = false;
            nok = false;
        }
        // both in flight during the rounds: the block's source dwords first, then the next record's offsets
        // (fetching after the refill made every step wait for the offsets before its source loads issued)
        rg_fetch(R, kbase, vbase, dk, dv);
        refill(!nok);
        // ---- compress ----
        sha_compress<SHORT>(st, w);
        if (fin) store_digest(out + 32 * (uint64_t)rfin, st);
        if (fin || !was_live) sha_init(st);
    }
}

// The records k_leaf_ragged leaves (the prefix and suffix outside rg_inner's interval): one record per lane,
// every message byte read inside the record's fields (no load outside them). A few hundred records
// normally; every record for blobs whose values (or keys) are all empty or tiny.
__device__ __forceinline__ uint32_t edge_byte(const uint8_t *kp, const uint8_t *vp, uint32_t k, uint32_t v, uint32_t L,
                                              uint32_t nb, uint32_t p) {
    if (p < 4) return (k >> (24 - 8 * p)) & 0xFFu;
    if (p < 4 + k) return kp[p - 4];
    if (p < 8 + k) return (v >> (24 - 8 * (p - 4 - k))) & 0xFFu;
    if (p < L) return vp[p - 8 - k];
    if (p == L) return 0x80u;
    if (p >= 64 * nb - 8) {  // the big-endian u64 bit length 8L in the last 8 bytes
        const uint32_t i = p - (64 * nb - 8);
        return (uint32_t)((((uint64_t)L << 3) >> (56 - 8 * i)) & 0xFFu);
    }
    return 0u;
}
// First i in [0, n) with pred(i) (n if none) for a predicate monotone false -> true: a 64-ary search by
// one wave (4 rounds for 16M records; the answer stays in [lo, hi], probes at or past hi count as true).
template <class Pred>
__device__ uint64_t edge_first(uint64_t n, uint32_t lane, Pred pred) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t step = (hi - lo + 63) / 64, idx = lo + lane * step;
        const uint64_t m = __ballot(idx >= hi || pred(idx));
        if (m == 0) {
            lo += 63 * step + 1;
            continue;
        }
        const uint32_t f = (uint32_t)__builtin_ctzll(m);
        if (f == 0) return lo;
        hi = std::min<uint64_t>(lo + f * step, hi);
        lo += (uint64_t)(f - 1) * step + 1;
    }
    return lo;
}
__global__ __launch_bounds__(256) void k_leaf_edges(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                   const uint8_t *__restrict__ vb, const uint64_t *__restrict__ voff,
                                                   uint64_t n, uint8_t *__restrict__ out) {
    __shared__ uint64_t s_ends[2];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave < 2) {
        const RgSplit X{koff[0] + 67, voff[0] + 6, koff[n], voff[n]};
        // P: first record past the prefix; S: first record of the suffix
        const uint64_t e = wave == 0 ? edge_first(n, lane, [&](uint64_t i) { return koff[i] >= X.kA && voff[i] >= X.vA; })
                                     : edge_first(n, lane, [&](uint64_t i) {
                                           return !(koff[i + 1] + 68 <= X.KN && voff[i + 1] + 136 <= X.VN);
                                       });
        if (lane == 0) s_ends[wave] = e;
    }
    __syncthreads();
    uint64_t P = s_ends[0], S = s_ends[1];
    if (P >= S) P = S = n;  // no interval: every record is an edge one
    const uint64_t m = P + (n - S);
    // one record per lane (round 6; it had been one wave per record, every lane assembling one byte): a
    // blob of empty values makes EVERY record an edge one (voff never moves off voff[0]), and 10M such
    // records then took ~30 ms through one wave each
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += nt) {
        const uint64_t r = i < P ? i : S + (i - P);
        const uint64_t k0 = koff[r], v0 = voff[r];
        const uint32_t k = (uint32_t)(koff[r + 1] - k0), v = (uint32_t)(voff[r + 1] - v0);
        const uint32_t L = 8 + k + v, nb = (L + 72) >> 6;
        const uint8_t *kp = kb + k0, *vp = vb + v0;
        uint32_t st[8];
        sha_init(st);
        for (uint32_t b = 0; b < nb; ++b) {
            uint32_t w[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t p = 64 * b + 4 * j;
                w[j] = (edge_byte(kp, vp, k, v, L, nb, p) << 24) | (edge_byte(kp, vp, k, v, L, nb, p + 1) << 16) |
                       (edge_byte(kp, vp, k, v, L, nb, p + 2) << 8) | edge_byte(kp, vp, k, v, L, nb, p + 3);
            }
            sha_compress<false>(st, w);
        }
        store_digest(out + 32 * r, st);
    }
}

// Key ownership of the chunks the ragged stage hashed (leaf.hpp; their offsets were stored by the
// ragged kernel's refill): the key bytes of every such chunk, copied in 16-B granules at their source
// offsets — chunks [B, nch) as one span (blockIdx.y 0), each fixed-kernel slot's chunks by one wave
// (blockIdx.y 1). It runs on a stream of its own as soon as k_leaf_direct is done, beside the VALU-bound
// ragged hash (a few VGPRs, no LDS). (Stores of the key-run dwords from inside k_leaf_ragged cost 10 % of
// the hash: 68 B of partial-line stores per record and key block; queued after the ragged kernels it
// stretched the sort's co-running passes.)
__global__ __launch_bounds__(256) void k_keycopy_ragged(const uint8_t *__restrict__ kb, const uint64_t *__restrict__ koff,
                                                        uint64_t n, const uint32_t *__restrict__ ctr, uint32_t nw,
                                                        uint8_t *__restrict__ kdst, uint64_t kcap) {
    const uint32_t nch = (uint32_t)((n + 63) / 64);
    uint32_t B, nslot;
    rg_handoff(ctr, nch, nw, &B, &nslot);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    auto copy_span = [&](uint64_t r0, uint64_t r1, uint64_t t0, uint64_t step) {  // records [r0, r1)
        const uint64_t g0 = koff[r0] & ~15ull, g1 = (koff[r1] + 15) & ~15ull;
        if (g1 <= kcap)
            for (uint64_t g = g0 + 16 * t0; g < g1; g += 16 * step)
                *reinterpret_cast<uint4 *>(kdst + g) = *reinterpret_cast<const uint4 *>(kb + g);
    };
    if (blockIdx.y == 0) {
        if (B < nch) copy_span((uint64_t)B * 64, n, t, stride);
    } else if (nslot) {
        const uint32_t lane = threadIdx.x & 63;
        for (uint64_t s = t / 64; s < nw; s += stride / 64) {
            const uint32_t v = ctr[CTR_LIST + s], c = v >> 5, cnt = v & 31u;
            if (cnt) copy_span((uint64_t)c * 64, std::min<uint64_t>((uint64_t)(c + cnt) * 64, n), lane, 64);
        }
    }
}

int device_cus() {
    static int c = [] {
        int dev = 0, x = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&x, hipDeviceAttributeMultiprocessorCount, dev);
        return x > 0 ? x : 256;
    }();
    return c;
}

}  // namespace

void launch_leaf_ragged(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                        uint8_t *out, uint32_t *ctr, hipStream_t st, const KeyOut &KO) {
    if (!n) return;
    const uint64_t grid = std::min<uint64_t>((uint64_t)device_cus() * MKV_RAGGED_WGS, ceil_div(ceil_div(n, 64), RG_WAVES));
    hipLaunchKernelGGL(k_leaf_ragged<false>, dim3((uint32_t)std::max<uint64_t>(grid, 1)), dim3(64 * RG_WAVES), 0, st,
                       kb, koff, vb, voff, n, out, ctr, leaf_fixed_waves(n), KO);
    MKV_LAUNCH_CHECK();
}

void launch_leaf_edges(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t *out, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_leaf_edges, dim3((uint32_t)std::min<uint64_t>(ceil_div(n, 256), 256)), dim3(256), 0, st, kb, koff,
                       vb, voff, n, out);
    MKV_LAUNCH_CHECK();
}

void launch_keycopy_ragged(const uint8_t *kb, const uint64_t *koff, uint64_t n, const uint32_t *ctr, uint8_t *kdst,
                           uint64_t kcap, hipStream_t st) {
    if (!n || !kdst) return;
    hipLaunchKernelGGL(k_keycopy_ragged, dim3(1024, 2), dim3(256), 0, st, kb, koff, n, ctr, leaf_fixed_waves(n), kdst, kcap);
    MKV_LAUNCH_CHECK();
}


}  // namespace mkv
