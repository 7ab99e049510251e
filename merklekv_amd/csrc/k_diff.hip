// k_diff.hip — Kernel D: two-tree key diff (R7, merkle.rs:171-196) and prefix bounds (HASH <prefix>).
//
// The reference builds a BTreeSet over the union of both leaf maps and looks every key up in both
// HashMaps. Both trees here already hold their leaves sorted by key (R3), so the same set is a
// merge-join of two sorted (key, digest) arrays:
//   pass 0  partition the merged sequence into 512-output wave tiles, one launch: a wave per 64 tiles
//           finds the group's two boundary splits by a cooperative 33-ary merge-path search, then each
//           lane the split of one tile between them (interpolation + galloping search);
//   pass 1  one wave per tile, no LDS: near-identical tiles (every A key paired in lockstep with a B key
//           of the same prefix) compare their digest pairs with coalesced loads and wave ballots; any
//           other tile runs the general per-lane 8-output merge: an A key is divergent unless the B
//           cursor holds the same key with the same leaf digest, a B key unless the previous A key is
//           equal. Lane results are packed to one u32 (split, from-A bits, divergent bits) plus a
//           per-tile count;
//   scan    exclusive scan of tile counts;
//   pass 2  wave-scan compaction writes (side, index) refs of divergent keys in merged = sorted order;
//           the same launch verifies the aligned path's deferred key checks.
// Ties on the 8-byte prefix fall back to a full-key compare in HBM (key_cmp), so any key set is exact.
#include <algorithm>

#include "common.hpp"
#include "dev_util.hpp"
#include "kernels.hpp"

namespace mkv {

namespace {

constexpr int DI = DIFF_ITEMS;
constexpr int WTILE = 64 * DI;  // merged outputs per wave tile

// Sorted key i of a side: storage record perm[i].
__device__ __forceinline__ const uint8_t *key_at(const DiffSide &S, uint64_t i, uint64_t *len) {
    const uint32_t o = S.perm[i];
    if (S.klen) {  // fixed-length keys: the offset is arithmetic (koff[0] is one uniform read)
        *len = S.klen;
        return S.kb + S.koff[0] + (uint64_t)o * S.klen;
    }
    const uint64_t a = S.koff[o];
    *len = S.koff[o + 1] - a;
    return S.kb + a;
}

__device__ __forceinline__ int cmp_ab(const DiffSide &A, uint64_t i, uint64_t pa, const DiffSide &B, uint64_t j,
                                      uint64_t pb) {
    if (pa != pb) return pa < pb ? -1 : 1;
    uint64_t la, lb;
    const uint8_t *ka = key_at(A, i, &la), *kb = key_at(B, j, &lb);
    return key_cmp(ka, la, pa, kb, lb, pb);
}

// Equal keys at sorted position i of both trees (the top-down leaf check). Prefixes and permutation
// entries of both sides load together, then both offset pairs, then every key word beyond the prefix
// at once (aligned keys up to 64 B), so a check is three dependent memory round trips; cmp_ab's
// chunk loop pays one per 8 bytes. Equal 8-byte prefixes + equal lengths = equal first 8 bytes.
__device__ __forceinline__ bool key_eq_at(const DiffSide &A, const DiffSide &B, uint64_t i) {
    const uint64_t pa = A.pfx[i], pb = B.pfx[i];
    const uint32_t oa = A.perm[i], ob = B.perm[i];
    uint64_t a0, a1, b0, b1;
    if (A.klen && B.klen) {  // fixed-length keys: arithmetic offsets
        a0 = A.koff[0] + (uint64_t)oa * A.klen;
        a1 = a0 + A.klen;
        b0 = B.koff[0] + (uint64_t)ob * B.klen;
        b1 = b0 + B.klen;
    } else {
        a0 = A.koff[oa];
        a1 = A.koff[oa + 1];
        b0 = B.koff[ob];
        b1 = B.koff[ob + 1];
    }
    const uint64_t len = a1 - a0;
    if (pa != pb || len != b1 - b0) return false;
    if (len <= 8) return true;
    const uint8_t *ka = A.kb + a0, *kb = B.kb + b0;
    if (((a0 | b0) & 3) == 0 && len <= 64) {
        const uint32_t *wa = reinterpret_cast<const uint32_t *>(ka), *wb = reinterpret_cast<const uint32_t *>(kb);
        const uint32_t nw = (uint32_t)(len >> 2);
        bool eq = true;
#pragma unroll
        for (uint32_t q = 2; q < 16; ++q)
            if (q < nw) eq &= wa[q] == wb[q];
        for (uint64_t x = (uint64_t)nw * 4; x < len; ++x) eq &= ka[x] == kb[x];
        return eq;
    }
    return key_cmp(ka, len, pa, kb, len, pb) == 0;
}

__device__ __forceinline__ bool digest_eq(const uint8_t *a, const uint8_t *b) {
    const uint4 *x = reinterpret_cast<const uint4 *>(a);
    const uint4 *y = reinterpret_cast<const uint4 *>(b);
    uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
    return x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w && x1.x == y1.x && x1.y == y1.y &&
           x1.z == y1.z && x1.w == y1.w;
}

__device__ __forceinline__ bool u4eq(uint4 a, uint4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }

// Key order between A[i] and B[j] for the merge. Equal 8-byte prefixes first try the leaf digests:
// equal digests mean equal encoded leaves (u32 |k| || k || u32 |v| || v), hence equal keys, unless
// SHA-256 collides — the same assumption the top-down walk and the reference's anti-entropy make when
// equal subtree hashes are taken as equal contents. Replicas agree on almost every key, so this skips
// the dependent perm -> koff -> key-bytes gathers for nearly every comparison; only keys whose
// prefixes tie and whose digests differ (changed values, or distinct keys sharing 8 bytes) pay the
// full compare.
__device__ __forceinline__ int cmp_merge(const DiffSide &A, uint64_t i, uint64_t pa, const DiffSide &B, uint64_t j,
                                         uint64_t pb) {
    if (pa != pb) return pa < pb ? -1 : 1;
    if (digest_eq(A.dig + 32 * i, B.dig + 32 * j)) return 0;
    return cmp_ab(A, i, pa, B, j, pb);
}

// Partition, one wave per group of PART_STRIDE tiles (one launch). The group's two boundary splits
// (tiles t0 and t1 = min(t0 + PART_STRIDE, ntiles)) by a cooperative search: lanes 0-31 search t0's
// diagonal, lanes 32-63 t1's, each half probing 32 points per round (below). Then lane l computes tile t0 + l's split inside that
// bracket: the split is monotone in the diagonal, so it lies between the two boundary splits; start at
// their linear interpolation (exact for near-identical replicas up to the few inserts/deletes in
// between), gallop outwards, then binary search the bracket — probes within a few cache lines that
// neighbouring tiles share.
constexpr uint64_t PART_STRIDE = 64;
// Probes per boundary and round: a half wave (the exponential first round needs all 32).
constexpr uint32_t PART_PROBES = 32;

// pred(a): A[a] precedes B[d-1-a] in the merge (A first on equal keys), i.e. the split of diagonal d is
// > a. Valid for max(0, d - B.n) <= a < min(d, A.n).
__device__ __forceinline__ bool part_pred(const DiffSide &A, const DiffSide &B, uint64_t d, uint64_t a) {
    const uint64_t jb = d - 1 - a;
    return cmp_merge(A, a, A.pfx[a], B, jb, B.pfx[jb]) <= 0;
}

__global__ __launch_bounds__(256) void k_diff_partition(DiffSide A, DiffSide B, uint64_t ntiles,
                                                        uint64_t *__restrict__ split, uint32_t *__restrict__ defer_count,
                                                        uint64_t *__restrict__ fail) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g == 0 && lane == 0) {  // this diff's deferred-check counter and fail word
        *defer_count = 0;
        fail[0] = 0;
    }
    const uint64_t ngroups = (ntiles + PART_STRIDE - 1) / PART_STRIDE;
    if (g >= ngroups) return;  // wave-uniform
    const uint64_t M = A.n + B.n;
    const uint64_t t0 = g * PART_STRIDE, t1 = t0 + PART_STRIDE < ntiles ? t0 + PART_STRIDE : ntiles;
    const uint32_t half = lane >> 5, k = lane & 31;
    // ---- boundary splits: half h searches diagonal dh; answer in [lo, hi] ----
    // Round 0: 32 probes at exponentially spaced offsets (0, +-1, +-3, ... +-65535) around the interpolated
    // split d * |A| / (|A| + |B|): replicas that agree on most keys have their split within a few hundred
    // positions of it, so the bracket shrinks to about that distance in one round; then 33-ary rounds. At
    // 100M mixed: ~3 dependent rounds instead of ~9 of the plain 9-ary search, and most probes away from the
    // split compare unequal prefixes (no digest reads).
    const uint64_t dh = half ? (t1 * WTILE < M ? t1 * WTILE : M) : t0 * WTILE;
    uint64_t lo = dh > B.n ? dh - B.n : 0, hi = dh < A.n ? dh : A.n;
    const uint64_t guess = (uint64_t)((double)dh * ((double)A.n / (double)(M ? M : 1)));
    bool first = true;
    while (__any(lo < hi)) {
        const uint64_t n = hi - lo;
        const bool act = lo < hi, expo = first && n > PART_PROBES;
        uint64_t p = 0;
        bool pv = false;
        if (act) {
            if (expo) {
                const int64_t off = k < 16 ? -(int64_t)((1u << (16 - k)) - 1u) : (int64_t)((1u << (k - 16)) - 1u);
                int64_t q = (int64_t)guess + off;
                q = q < (int64_t)lo ? (int64_t)lo : q;
                q = q > (int64_t)hi - 1 ? (int64_t)hi - 1 : q;
                p = (uint64_t)q;
            } else {
                p = n <= PART_PROBES ? lo + k : lo + ((uint64_t)(k + 1) * n) / (PART_PROBES + 1);
            }
            pv = (n > PART_PROBES || k < n) && part_pred(A, B, dh, p);
        }
        const uint32_t m = (uint32_t)(__ballot(pv) >> (32 * half));
        const uint32_t c = (uint32_t)__popc(m);  // preds are monotone in p: c leading trues
        const uint64_t pc1 = __shfl(p, (int)(32 * half + (c ? c - 1 : 0)));            // last true probe
        const uint64_t pc = __shfl(p, (int)(32 * half + (c < PART_PROBES ? c : 0)));  // first false probe
        if (act) {
            if (n <= PART_PROBES) {
                lo = hi = lo + c;
            } else {
                if (c) lo = pc1 + 1;
                if (c < PART_PROBES) hi = pc;
            }
        }
        first = false;
    }
    const uint64_t s0 = __shfl(lo, 0), s1 = __shfl(lo, 32);
    if (lane == 0) split[t0] = s0;
    if (lane == 32 && t1 == ntiles) split[ntiles] = s1;
    // ---- the group's other tiles ----
    const uint64_t t = t0 + lane;
    if (lane == 0 || t >= t1) return;
    const uint64_t d = t * WTILE, d0 = t0 * WTILE, d1 = t1 * WTILE < M ? t1 * WTILE : M;
    const uint64_t a0 = s0, a1 = s1;
    lo = a1 > d1 - d ? a1 - (d1 - d) : 0;
    hi = a0 + (d - d0);
    if (lo < a0) lo = a0;
    if (hi > a1) hi = a1;
    if (d > B.n && lo < d - B.n) lo = d - B.n;
    if (hi > A.n) hi = A.n;
    if (hi > d) hi = d;
    uint64_t gs = a0 + (uint64_t)((double)(a1 - a0) * (double)(d - d0) / (double)(d1 - d0) + 0.5);
    if (gs < lo) gs = lo;
    if (gs > hi) gs = hi;
    uint64_t L = lo, H = hi;  // answer in [L, H]
    // The split is gs exactly when pred(gs - 1) holds and pred(gs) does not: both tested at once (their
    // prefixes are two adjacent pairs, one round trip; unequal prefixes in the common case, so no digest
    // reads), else gallop from the side they point to.
    const uint64_t pa0 = gs > lo ? A.pfx[gs - 1] : 0, pa1 = gs < hi ? A.pfx[gs] : 0;
    const uint64_t pb0 = gs > lo ? B.pfx[d - gs] : 0, pb1 = gs < hi ? B.pfx[d - 1 - gs] : 0;
    const bool below = gs == lo || (pa0 != pb0 ? pa0 < pb0 : cmp_merge(A, gs - 1, pa0, B, d - gs, pb0) <= 0);
    const bool at = gs < hi && (pa1 != pb1 ? pa1 < pb1 : cmp_merge(A, gs, pa1, B, d - 1 - gs, pb1) <= 0);
    if (below && !at) {
        L = H = gs;
    } else if (at) {
        L = gs + 1;
        for (uint64_t step = 2;; step <<= 1) {
            const uint64_t q = gs + step - 1;
            if (q >= hi) break;
            if (!part_pred(A, B, d, q)) { H = q; break; }
            L = q + 1;
        }
    } else {  // pred(gs - 1) false: the split is below gs
        H = gs - 1;
        for (uint64_t step = 2;; step <<= 1) {
            if (gs < lo + step) break;
            const uint64_t q = gs - step;
            if (part_pred(A, B, d, q)) { L = q + 1; break; }
            H = q;
        }
    }
    while (L < H) {
        const uint64_t mid = (L + H) >> 1;
        if (part_pred(A, B, d, mid)) L = mid + 1;
        else H = mid;
    }
    split[t] = L;
}

struct TileCtx {
    uint64_t a0, a1, b0, b1;  // this tile's A range [a0,a1) and B range [b0,b1)
    uint64_t d0;              // first merged output of the tile
};

// One 512-output tile per wave: tile t covers merged outputs [t*WTILE, min((t+1)*WTILE, M)).
__device__ __forceinline__ TileCtx wave_tile(const DiffSide &A, const DiffSide &B, const uint64_t *split, uint64_t t) {
    TileCtx c;
    const uint64_t M = A.n + B.n;
    c.d0 = t * WTILE;
    uint64_t d1 = c.d0 + WTILE;
    if (d1 > M) d1 = M;
    c.a0 = split[t];
    c.a1 = split[t + 1];
    c.b0 = c.d0 - c.a0;
    c.b1 = d1 - c.a1;
    return c;
}

// General merge of one lane's 8 outputs; returns packed (isplit << 16) | (fromA << 8) | div and the div
// count. Prefixes come straight from HBM/L2 (the tile's slices were just touched by the aligned check):
// pa(0) = A[a0-1], pa(1+x) = A[a0+x], pb(x) = B[b0+x].
__device__ __forceinline__ uint32_t merge_lane(const DiffSide &A, const DiffSide &B, const TileCtx &c, uint32_t lane,
                                            uint32_t *ndiv) {
    const uint64_t na = c.a1 - c.a0, nb = c.b1 - c.b0;
    const uint64_t M = A.n + B.n;
    const uint64_t dl = (uint64_t)lane * DI;  // local diagonal
    if (c.d0 + dl >= M || dl >= na + nb) {
        *ndiv = 0;
        return 0;
    }
    auto pa = [&](uint64_t x) -> uint64_t { return x ? A.pfx[c.a0 + x - 1] : (c.a0 ? A.pfx[c.a0 - 1] : 0); };
    auto pb = [&](uint64_t x) -> uint64_t { return c.b0 + x < B.n ? B.pfx[c.b0 + x] : 0; };
    // local merge-path search
    uint64_t lo = dl > nb ? dl - nb : 0, hi = dl < na ? dl : na;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        uint64_t jb = dl - 1 - mid;
        if (cmp_merge(A, c.a0 + mid, pa(1 + mid), B, c.b0 + jb, pb(jb)) <= 0) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t isplit = (uint32_t)lo;
    uint64_t i = c.a0 + lo, j = c.b0 + (dl - lo);
    uint32_t fromA = 0, div = 0;
    // A key equal to B[j] is always emitted just before B[j] (A first on ties), so a B step right after
    // an A step with the same j reuses that comparison: nearly identical replicas (the anti-entropy
    // case) then pay one prefix compare + one digest compare per union key, not three.
    bool prevA_matched = false;
    for (int s = 0; s < DI; ++s) {
        if (dl + s >= na + nb) break;
        const uint64_t li = i - c.a0, lj = j - c.b0;
        bool takeA;
        int cab = 1;
        bool deq = false;
        if (i >= c.a1) takeA = false;
        else if (j >= B.n) takeA = true;
        else {
            const uint64_t xa = pa(1 + li), xb = pb(lj);
            if (xa != xb) cab = xa < xb ? -1 : 1;
            else if (digest_eq(A.dig + 32 * i, B.dig + 32 * j)) cab = 0, deq = true;  // see cmp_merge
            else cab = cmp_ab(A, i, xa, B, j, xb);
            takeA = (j >= c.b1) ? true : (cab <= 0);
            // j == b1 < B.n: the tile's B slice is exhausted, so A[i] < B[b1] or equal (then matched)
        }
        bool d;
        if (takeA) {
            const bool matched = (j < B.n) && cab == 0;
            d = !matched || !deq;
            prevA_matched = matched;
            fromA |= 1u << s;
            ++i;
        } else {
            bool matched;
            if (s > 0 && ((fromA >> (s - 1)) & 1u)) matched = prevA_matched;  // A[i-1] vs this B[j]: done
            else matched = i > 0 && cmp_merge(A, i - 1, pa(li), B, j, pb(lj)) == 0;
            prevA_matched = false;
            d = !matched;
            ++j;
        }
        if (d) div |= 1u << s;
    }
    *ndiv = (uint32_t)__popc(div);
    return (isplit << 16) | (fromA << 8) | div;
}

// Prefix-only merge of one lane's 8 outputs over the wave's LDS prefix slices (pa(0) = A[a0-1],
// pa(1+x) = A[a0+x], pb(x) = B[b0+x], B[b1] included), A first on equal prefixes. Cross-side pairs with
// equal prefixes are taken as the same key and verified afterwards with one batch of independent digest
// loads (full key compare only when the digests differ). The prefix-only merge is the true merge as long
// as the last A key and the first B key of every equal-prefix run are the same key, and that pair is
// always among the verified ones, so a failed verification (*bad) sends the wave to the exact merge.
constexpr int VMAX = 5;  // tentative pairs per lane: a B at output 0 plus at most 4 A/B pairs
__device__ __forceinline__ uint32_t merge_lane_pfx(const DiffSide &A, const DiffSide &B, const TileCtx &c,
                                                   uint32_t lane, const uint64_t *pa, const uint64_t *pb,
                                                   uint32_t *ndiv, bool *bad) {
    const uint64_t na = c.a1 - c.a0, nb = c.b1 - c.b0;
    const uint64_t M = A.n + B.n;
    const uint64_t dl = (uint64_t)lane * DI;
    *ndiv = 0;
    if (c.d0 + dl >= M || dl >= na + nb) return 0;
    uint64_t lo = dl > nb ? dl - nb : 0, hi = dl < na ? dl : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (pa[1 + mid] <= pb[dl - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t isplit = (uint32_t)lo;
    uint64_t i = c.a0 + lo, j = c.b0 + (dl - lo);
    uint32_t fromA = 0, div = 0;
    uint64_t vi[VMAX], vj[VMAX];
    uint32_t vs[VMAX];  // output bit of each tentative pair (A output: divergent if the digests differ)
    int nv = 0;
    bool prevA_tie = false;
#pragma unroll
    for (int s = 0; s < DI; ++s) {
        if (dl + s >= na + nb) break;
        const uint64_t li = i - c.a0, lj = j - c.b0;
        bool takeA, tie = false;
        if (i >= c.a1) takeA = false;
        else if (j >= B.n) takeA = true;
        else {
            const uint64_t xa = pa[1 + li], xb = pb[lj];
            tie = xa == xb;
            takeA = (j >= c.b1) || xa <= xb;
        }
        if (takeA) {
            if (tie) {
                if (nv == VMAX) { *bad = true; return 0; }
                vi[nv] = i, vj[nv] = j, vs[nv] = 1u << s, ++nv;
            } else {
                div |= 1u << s;  // no B key shares its prefix
            }
            prevA_tie = tie;
            fromA |= 1u << s;
            ++i;
        } else {
            bool tieB = prevA_tie && s > 0 && ((fromA >> (s - 1)) & 1u);  // pair recorded at that A step
            if (!tieB && i > 0 && pa[li] == pb[lj]) {
                if (nv == VMAX) { *bad = true; return 0; }
                vi[nv] = i - 1, vj[nv] = j, vs[nv] = 0, ++nv;  // B output: matched by key, never by digest
                tieB = true;
            }
            if (!tieB) div |= 1u << s;
            prevA_tie = false;
            ++j;
        }
    }
    // verification: all digest pairs loaded at once
    uint4 da[VMAX][2], db[VMAX][2];
#pragma unroll
    for (int v = 0; v < VMAX; ++v) {
        const uint64_t x = v < nv ? vi[v] : 0, y = v < nv ? vj[v] : 0;
        const uint4 *p = reinterpret_cast<const uint4 *>(A.dig + 32 * x);
        const uint4 *q = reinterpret_cast<const uint4 *>(B.dig + 32 * y);
        da[v][0] = p[0], da[v][1] = p[1], db[v][0] = q[0], db[v][1] = q[1];
    }
#pragma unroll
    for (int v = 0; v < VMAX; ++v) {
        if (v >= nv) break;
        if (u4eq(da[v][0], db[v][0]) && u4eq(da[v][1], db[v][1])) continue;
        const uint64_t p = A.pfx[vi[v]];
        if (cmp_ab(A, vi[v], p, B, vj[v], p) != 0) *bad = true;  // equal prefixes, different keys
        else div |= vs[v];                                        // same key, changed value: A divergent
    }
    *ndiv = (uint32_t)__popc(div);
    return (isplit << 16) | (fromA << 8) | div;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    return ((uint64_t)(uint32_t)__shfl((int)(v >> 32), src) << 32) | (uint32_t)__shfl((int)(uint32_t)v, src);
}
__device__ __forceinline__ uint4 shfl_u4(uint4 v, int src) {
    return make_uint4(__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src));
}

// Pass 1, one wave per 512-output tile, no LDS (high occupancy keeps enough loads in flight).
// Aligned fast path (near-identical replicas): when every A key of the tile has a partner B key with the
// same prefix in lockstep, the tile's merge is A0 B0 A1 B1 ... (phase 0) or, when the tile starts with
// the partner of the previous tile's last A, B0 A0 B1 A1 ... (phase 1). Pair x is read by lane x % 64
// (coalesced: consecutive lanes, consecutive digests), all prefixes and digests are loaded at once, the
// phase-1 partner comes from the neighbouring lane by shuffle, and per-pair results are gathered into
// each output lane's 8-output word through wave ballots. A pair with equal prefixes but different
// digests gets the full key compare; if those keys differ the tile is not aligned and the wave runs the
// general merge instead (which is exact for any key sets).
// One 512-output tile (the body of pass 1): aligned fast path for near-identical replicas, else the
// general merge. Returns this lane's packed (isplit << 16) | (fromA << 8) | div; *total = the tile's
// divergent count (wave-uniform). lp: the wave's LDS prefix slice (WTILE + 2 entries).
// Deferred key checks of the aligned path (round 3): a pair with equal 8-byte prefixes and different
// digests is taken as the same key with a changed value, and its (A index, B index) goes to this list;
// pass 2's verify blocks then compare all their keys at once, off pass 1's critical path (each inline check is
// three dependent random reads per side that hold the wave). A failed check or a full list makes the
// caller run the diff again without deferral (exact for any key sets).
struct DeferList {
    uint64_t *ent;    // (A index << 32) | B index
    uint32_t *count;  // entries appended (may exceed cap: overflow)
    uint32_t cap;
};

__device__ __forceinline__ void defer_pairs(const DeferList &V, bool want, uint64_t e, uint32_t lane) {
    const uint64_t bal = __ballot(want);
    if (!bal) return;
    const uint32_t leader = (uint32_t)__builtin_ctzll(bal);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(V.count, (uint32_t)__popcll(bal));
    base = __shfl(base, (int)leader);
    const uint32_t k = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (want && k < V.cap) V.ent[k] = e;
}

template <bool DEFER = false>
__device__ __forceinline__ uint32_t diff_tile(const DiffSide &A, const DiffSide &B, const TileCtx &c, uint32_t lane,
                                              uint64_t *lp, uint32_t *total, const DeferList &V = DeferList{}) {
    const uint64_t na = c.a1 - c.a0, nb = c.b1 - c.b0;
    uint32_t nd = 0, pk = 0;
    bool general = true;
    if (na == nb) {
        // slot q of lane l holds pair x = l + 64 q (q < 4), in two halves (q = 0, 1 then 2, 3) so that
        // only half of the tile's prefixes and digests are in registers at once; the phase-1 partner of
        // lane 63's last slot in a half is B[b0 + 128 (h + 1)] (loaded as the half's end element)
        uint64_t pA[4];
        bool ok0 = true, ok1 = true;
        uint32_t eq0 = 0, eq1 = 0;
        const int src = (int)((lane + 1) & 63);
        uint4 dB00[2];  // B[b0]'s digest (lane 0's slot 0): the phase-1 partner of A[a0 - 1]
        uint64_t pB00 = ~0ull;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint64_t pB[2];
            uint4 dA[2][2], dB[2][2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = 2 * h + u;
                const uint64_t x = lane + 64 * q;
                pA[q] = 0;
                pB[u] = ~0ull;
                dA[u][0] = dA[u][1] = dB[u][0] = dB[u][1] = make_uint4(0, 0, 0, 0);
                if (x < na) {
                    pA[q] = A.pfx[c.a0 + x];
                    const uint4 *p = reinterpret_cast<const uint4 *>(A.dig + 32 * (c.a0 + x));
                    dA[u][0] = p[0];
                    dA[u][1] = p[1];
                }
                if (x <= nb && c.b0 + x < B.n) {
                    pB[u] = B.pfx[c.b0 + x];
                    const uint4 *p = reinterpret_cast<const uint4 *>(B.dig + 32 * (c.b0 + x));
                    dB[u][0] = p[0];
                    dB[u][1] = p[1];
                }
            }
            const uint64_t xe = 128ull * (h + 1);
            uint64_t pEnd = ~0ull;
            uint4 dEnd[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
            if (xe <= nb && c.b0 + xe < B.n) {
                pEnd = B.pfx[c.b0 + xe];
                const uint4 *p = reinterpret_cast<const uint4 *>(B.dig + 32 * (c.b0 + xe));
                dEnd[0] = p[0];
                dEnd[1] = p[1];
            }
            if (h == 0) {
                dB00[0] = dB[0][0];
                dB00[1] = dB[0][1];
                pB00 = pB[0];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = 2 * h + u;
                const uint64_t x = lane + 64 * q;
                const uint64_t pn = shfl_u64(pB[u], src), pw = u < 1 ? shfl_u64(pB[u + 1], 0) : pEnd;
                const uint4 n0 = shfl_u4(dB[u][0], src), n1 = shfl_u4(dB[u][1], src);
                const uint4 w0 = u < 1 ? shfl_u4(dB[u + 1][0], 0) : dEnd[0];
                const uint4 w1 = u < 1 ? shfl_u4(dB[u + 1][1], 0) : dEnd[1];
                const uint64_t pN = lane == 63 ? pw : pn;
                const bool e0 = u4eq(dA[u][0], dB[u][0]) && u4eq(dA[u][1], dB[u][1]);
                const bool e1 = lane == 63 ? (u4eq(dA[u][0], w0) && u4eq(dA[u][1], w1))
                                           : (u4eq(dA[u][0], n0) && u4eq(dA[u][1], n1));
                if (x < na) {
                    ok0 &= pA[q] == pB[u];
                    ok1 &= (c.b0 + x + 1 < B.n) && pA[q] == pN;
                }
                eq0 |= (uint32_t)e0 << q;
                eq1 |= (uint32_t)e1 << q;
            }
            asm volatile("" ::: "memory");  // keep the second half's loads behind the first half's use
        }
        uint64_t pPrev = 0;  // A[a0-1], the phase-1 partner of B[b0]
        uint4 dPrev[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        if (c.a0 > 0) {
            pPrev = A.pfx[c.a0 - 1];
            const uint4 *p = reinterpret_cast<const uint4 *>(A.dig + 32 * (c.a0 - 1));
            dPrev[0] = p[0];
            dPrev[1] = p[1];
        }
        const uint64_t pB0 = pB00;
        const bool eqPrev = u4eq(dPrev[0], dB00[0]) && u4eq(dPrev[1], dB00[1]);  // meaningful in lane 0
        if (lane == 0) ok1 &= c.a0 > 0 && pPrev == pB0;
        int phase = -1;
        if (__ballot(!ok0) == 0) phase = 0;
        else if (__ballot(!ok1) == 0) phase = 1;
        if (phase >= 0) {
            // digest mismatches get the full key compare (equal keys: changed value -> divergent A)
            const uint32_t eq = phase ? eq1 : eq0;
            bool bad = false;
            uint64_t dm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t x = lane + 64 * q;
                bool dv = false;
                if (x < na && !((eq >> q) & 1u)) {
                    dv = true;
                    if (!DEFER && cmp_ab(A, c.a0 + x, pA[q], B, c.b0 + x + phase, pA[q]) != 0) bad = true;
                }
                if (DEFER) defer_pairs(V, dv, ((c.a0 + x) << 32) | (c.b0 + x + phase), lane);
                dm[q] = __ballot(dv);
            }
            // B[b0] must be the key of A[a0-1]
            if (DEFER) defer_pairs(V, phase == 1 && lane == 0 && !eqPrev, ((c.a0 - 1) << 32) | c.b0, lane);
            else if (phase == 1 && lane == 0 && !eqPrev && cmp_ab(A, c.a0 - 1, pPrev, B, c.b0, pPrev) != 0)
                bad = true;
            if (__ballot(bad) == 0) {
                general = false;
                // output lane L holds pairs 4L .. 4L+3: A outputs at even (phase 0) / odd (phase 1) bits
                const uint32_t w = lane >> 4;
                const uint64_t m = w == 0 ? dm[0] : w == 1 ? dm[1] : w == 2 ? dm[2] : dm[3];
                const uint32_t nib = (uint32_t)(m >> ((4 * lane) & 63)) & 0xFu;
                const uint32_t div =
                    ((nib & 1u) | ((nib & 2u) << 1) | ((nib & 4u) << 2) | ((nib & 8u) << 3)) << phase;
                const uint64_t dl = (uint64_t)lane * DI;
                if (dl < na + nb) pk = ((uint32_t)(dl / 2) << 16) | ((phase ? 0xAAu : 0x55u) << 8) | div;
                *total = (uint32_t)(__popcll(dm[0]) + __popcll(dm[1]) + __popcll(dm[2]) + __popcll(dm[3]));
            }
        }
    }
    if (general) {
        // stage the tile's prefixes in the wave's LDS slice: pa = lp[0 .. na], pb = lp[na+1 .. na+1+nb]
        const uint64_t tot = na + nb + 2;
#pragma unroll
        for (int r = 0; r < (WTILE + 2 + 63) / 64; ++r) {
            const uint64_t x = lane + 64 * r;
            if (x < tot) {
                uint64_t v;
                if (x == 0) v = c.a0 ? A.pfx[c.a0 - 1] : 0;
                else if (x <= na) v = A.pfx[c.a0 + x - 1];
                else v = c.b0 + (x - na - 1) < B.n ? B.pfx[c.b0 + (x - na - 1)] : ~0ull;
                lp[x] = v;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        bool bad = false;
        pk = merge_lane_pfx(A, B, c, lane, lp, lp + na + 1, &nd, &bad);
        if (__ballot(bad) != 0) pk = merge_lane(A, B, c, lane, &nd);  // exact merge (shared prefixes)
        uint32_t s = nd;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        *total = s;
    }
    return pk;
}

// Pass 1, one wave per 512-output tile (multi-pass form). Pinned to 3 waves per SIMD (the aligned path in
// two halves leaves 159 VGPRs, no spill): 100M identical replicas 1.49 -> 1.33 ms (6.0 TB/s of the
// algorithmic 80 B per key), mixed 1.64 -> 1.56 ms; at 4 waves the compiler spills 176 B per lane (1.95 ms).
template <bool DEFER>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_diff_pass1(DiffSide A, DiffSide B, const uint64_t *__restrict__ split,
                                                    uint64_t nt, uint32_t *__restrict__ packed,
                                                    uint64_t *__restrict__ tilecnt, DeferList V) {
    __shared__ uint64_t lds[4 * (WTILE + 2)];  // per-wave prefix slices for the general merge
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= nt) return;  // wave-uniform
    const uint32_t lane = threadIdx.x & 63;
    const TileCtx c = wave_tile(A, B, split, t);
    uint32_t total = 0;
    const uint32_t pk = diff_tile<DEFER>(A, B, c, lane, lds + (threadIdx.x >> 6) * (WTILE + 2), &total, V);
    if (lane == 0) tilecnt[t] = total;
    if (total) packed[t * 64 + lane] = pk;  // only tiles with divergent outputs are read again (pass 2)
}

// Pass 2, one wave per 64 tiles: lane offsets by a wave scan of the divergent counts, then refs in merged order.
// The deferred key checks ride in the same launch (blocks from nb2 on): fail[0] = 1 if any pair holds
// different keys or the list overflowed (the caller then reruns without deferral).
__global__ __launch_bounds__(256) void k_diff_pass2(DiffSide A, DiffSide B, const uint64_t *__restrict__ split,
                                                    uint64_t nt, const uint32_t *__restrict__ packed,
                                                    const uint64_t *__restrict__ tilecnt,
                                                    const uint64_t *__restrict__ tileoff, uint64_t *__restrict__ refs,
                                                    uint32_t nb2, DeferList V, uint64_t *__restrict__ fail) {
    if (blockIdx.x >= nb2) {
        const uint32_t cnt = *V.count;
        const uint64_t vb = blockIdx.x - nb2, nvb = gridDim.x - nb2;
        if (cnt > V.cap) {
            if (vb == 0 && threadIdx.x == 0) fail[0] = 1;
            return;
        }
        for (uint64_t k = vb * blockDim.x + threadIdx.x; k < cnt; k += nvb * blockDim.x) {
            const uint64_t e = V.ent[k], i = e >> 32, j = e & 0xFFFFFFFFull;
            if (cmp_ab(A, i, A.pfx[i], B, j, B.pfx[j]) != 0) fail[0] = 1;
        }
        return;
    }
    // one wave per 64 tiles: lane q reads tile (64 w + q)'s count, output offset and split in one round
    // trip, then the wave emits only the tiles with divergent outputs (~23 % at 0.1 % divergence), taking
    // a tile's offset / split from its lane (shuffles), the packed words of 8 live tiles loaded at once
    // (one workgroup per tile left ~100K mostly idle workgroups to dispatch; a dependent load chain per
    // live tile cost ~50 us at 100M)
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t t0 = w * 64;
    if (t0 >= nt) return;  // wave-uniform
    const bool tv = t0 + lane < nt;
    const uint64_t mycnt = tv ? tilecnt[t0 + lane] : 0, myoff = tv ? tileoff[t0 + lane] : 0,
                   mysplit = tv ? split[t0 + lane] : 0;
    uint64_t live = __ballot(mycnt != 0);
    while (live) {
        // the packed words of up to PASS2_AHEAD live tiles in flight at once, then their refs
        constexpr int PASS2_AHEAD = 8;
        uint32_t tq[PASS2_AHEAD], pk[PASS2_AHEAD];
#pragma unroll
        for (int u = 0; u < PASS2_AHEAD; ++u) {
            tq[u] = live ? (uint32_t)__builtin_ctzll(live) : 64u;
            pk[u] = live ? packed[(t0 + tq[u]) * 64 + lane] : 0u;
            live &= live - 1;
        }
#pragma unroll
        for (int u = 0; u < PASS2_AHEAD; ++u) {
            if (tq[u] == 64u) break;  // wave-uniform
            const uint32_t q = tq[u];
            const uint32_t div = pk[u] & 0xFF, fromA = (pk[u] >> 8) & 0xFF, isplit = pk[u] >> 16;
            const uint32_t cnt = __popc(div);
            uint64_t off = (uint64_t)__shfl((long long)myoff, (int)q) + (wave_incl_scan<uint32_t>(cnt) - cnt);
            const uint64_t a0 = (uint64_t)__shfl((long long)mysplit, (int)q), d0 = (t0 + q) * WTILE;
            if (!div) continue;
            const uint64_t dl = (uint64_t)lane * DI;
            uint64_t i = a0 + isplit, j = (d0 - a0) + (dl - isplit);
            for (int s = 0; s < DI; ++s) {
                const bool fa = (fromA >> s) & 1u;
                const uint64_t ref = fa ? i : (j | (1ull << 63));
                if (fa) ++i; else ++j;
                if ((div >> s) & 1u) refs[off++] = ref;
            }
        }
    }
}

__global__ void k_diff_keylens(const uint64_t *__restrict__ refs, uint64_t m, DiffSide A, DiffSide B,
                               uint64_t *__restrict__ lens) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint64_t r = refs[k];
    const DiffSide &S = (r >> 63) ? B : A;
    uint64_t i = r & ~(1ull << 63);
    uint64_t len;
    (void)key_at(S, i, &len);
    lens[k] = len;
}

__global__ void k_diff_keys(const uint64_t *__restrict__ refs, uint64_t m, DiffSide A, DiffSide B,
                            const uint64_t *__restrict__ off, uint8_t *__restrict__ out) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    uint64_t r = refs[k];
    const DiffSide &S = (r >> 63) ? B : A;
    uint64_t i = r & ~(1ull << 63);
    uint64_t len;
    const uint8_t *s = key_at(S, i, &len);
    uint8_t *d = out + off[k];
    // widest copy the alignments allow: fixed 16-B-multiple keys (configs' 32-B keys) move as 16-B words,
    // so a wave's stores cover one contiguous span (the destination may be mapped host memory)
    const uintptr_t al = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)len;
    if ((al & 15) == 0) {
        for (uint64_t x = 0; x < len; x += 16)
            *reinterpret_cast<uint4 *>(d + x) = *reinterpret_cast<const uint4 *>(s + x);
    } else if ((al & 3) == 0) {
        for (uint64_t x = 0; x < len; x += 4)
            *reinterpret_cast<uint32_t *>(d + x) = *reinterpret_cast<const uint32_t *>(s + x);
    } else {
        for (uint64_t x = 0; x < len; ++x) d[x] = s[x];
    }
}

// Fixed-length keys (klen % 16 == 0): one 16-B granule of the list per thread, key k at out + k x klen
// (the offsets are arithmetic: no offset array is read or written). Every wave's store covers 1 KiB of
// consecutive bytes and twice as many gathers are in flight as with a thread per key.
__global__ void k_diff_keys_g16(const uint64_t *__restrict__ refs, uint64_t m, DiffSide A, DiffSide B, uint32_t klen,
                                uint8_t *__restrict__ out) {
    const uint32_t gpk = klen >> 4;
    const uint64_t G = m * gpk;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < G; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = gpk == 2 ? t >> 1 : t / gpk, x = t - k * gpk;  // (32-B keys: a shift)
        const uint64_t r = refs[k];
        uint64_t len;
        const uint8_t *src = key_at((r >> 63) ? B : A, r & ~(1ull << 63), &len) + 16 * x;
        uint4 v;
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            v = *reinterpret_cast<const uint4 *>(src);
        } else {
            uint32_t w[4];
            for (int j = 0; j < 4; ++j)
                w[j] = (uint32_t)src[4 * j] | ((uint32_t)src[4 * j + 1] << 8) | ((uint32_t)src[4 * j + 2] << 16) |
                       ((uint32_t)src[4 * j + 3] << 24);
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4 *>(out + 16 * t) = v;
    }
}

// lohi[0] = lower_bound(prefix), lohi[1] = first index >= lo whose key does not start with prefix.
__global__ void k_prefix_bounds(DiffSide A, const uint8_t *__restrict__ prefix, uint32_t plen,
                                uint64_t *__restrict__ lohi) {
    if (threadIdx.x != 0) return;
    const uint64_t pp = key_chunk(prefix, plen, 0);
    uint64_t lo = 0, hi = A.n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        uint64_t la;
        const uint8_t *ka = key_at(A, mid, &la);
        if (key_cmp(ka, la, A.pfx[mid], prefix, plen, pp) < 0) lo = mid + 1;
        else hi = mid;
    }
    // keys with the prefix are exactly those >= prefix that start with it: binary search on "starts with"
    uint64_t l2 = lo, h2 = A.n;
    while (l2 < h2) {
        uint64_t mid = (l2 + h2) >> 1;
        uint64_t la;
        const uint8_t *ka = key_at(A, mid, &la);
        bool starts = la >= plen;
        for (uint32_t x = 0; starts && x < plen; ++x) starts = ka[x] == prefix[x];
        if (starts) l2 = mid + 1;
        else h2 = mid;
    }
    lohi[0] = lo;
    lohi[1] = l2;
}

constexpr int TD_THREADS = 1024;  // frontier kernels: one append atomic per 16 waves

// ---- top-down diff (equal leaf counts): expand the divergent frontier one level down ----
// frontier_in holds node indices of level l whose digests differ between the trees; children (l-1)
// whose digests differ are appended to frontier_out (wave-aggregated: one atomic per wave).
// One level of the top-down walk. fin: divergent parents (local indices of the owned parent range,
// global index = local + a_par); their children (global 2p, 2p+1, local = global - a_child) are
// compared and the divergent ones appended to fout. r0/r1: local child-level indices of owned nodes
// whose parent is not owned (the tree's own root at the top level; a shard's fringe roots below it),
// compared as extra frontier candidates (UINT64_MAX = none).
__global__ __launch_bounds__(TD_THREADS) void k_topdown_level(const uint8_t *__restrict__ ca, const uint8_t *__restrict__ cb,
                                                      uint64_t child_count, uint64_t a_par, uint64_t a_child,
                                                      uint64_t r0, uint64_t r1, const uint32_t *__restrict__ fin,
                                                      const uint32_t *__restrict__ nin, uint32_t *__restrict__ fout,
                                                      uint32_t *__restrict__ nout) {
    __shared__ uint32_t sapp[17];
    const uint32_t cnt = *nin;
    const uint64_t tot = 2ull * cnt + 2;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < tot; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = base + threadIdx.x;  // two candidate children per frontier node, then r0, r1
        bool d = false;
        uint64_t c = UINT64_MAX;
        if (t < 2ull * cnt) c = 2 * ((uint64_t)fin[t >> 1] + a_par) + (t & 1) - a_child;
        else if (t == 2ull * cnt) c = r0;
        else if (t == 2ull * cnt + 1) c = r1;
        if (c < child_count) d = !digest_eq(ca + 32ull * c, cb + 32ull * c);
        block_append<uint32_t>(d, (uint32_t)c, fout, nout, sapp);
    }
}

// Key-set screen before a top-down walk: compares the sorted 8-byte key prefixes of both trees at
// `samples` evenly spaced positions. Equal key sets never differ there; an insertion or deletion
// shifts every later position, so a handful of samples detect it (then the merge-join runs directly).
__global__ __launch_bounds__(256) void k_sample_pfx(const uint64_t *__restrict__ pa, const uint64_t *__restrict__ pb,
                                                   uint64_t n, uint32_t samples, uint32_t *__restrict__ count) {
    uint32_t bad = 0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < samples; k += gridDim.x * blockDim.x) {
        const uint64_t i = samples > 1 ? (uint64_t)((unsigned __int128)k * (n - 1) / (samples - 1)) : 0;
        bad += pa[i] != pb[i];
    }
    if (bad) atomicAdd(count, bad);
}
// ---- top-down walk in jumps of k levels (unsharded plans) ----
// A divergent node p at level l has its level-(l-k) descendants at [p << k, (p+1) << k) (clipped to the
// level: R5 promotion keeps the implicit arrays aligned). Comparing those 2^k nodes directly — they are
// contiguous, so the loads coalesce — replaces k dependent level launches: the walk is latency-bound,
// and a descendant can only differ when its ancestors do. One thread per (parent, descendant).
// gate != nullptr: the level-4 abort test of the one-wait pair diff, made by every workgroup before it
// starts (the jump from level 4): the key-set screen word gate[word] set, or a frontier over half the level
// (nin > level_count / 2) -> no descendant is compared and workgroup 0 sets bit 31 of the word (merge-join).
// Every workgroup reaches the same verdict: nin is not written here, and the word is nonzero either way.
// (k_topdown_jump_u below: the unrolled form of this jump)

// Sharded form (a shard's owned ranges per level): entry p of level l is global node p + a_par, its
// descendants at level l - k are global ((p + a_par) << k) + j, local minus a_desc (an owned node's leaves
// are all owned, so they are too). After the frontier's descendants come the seeds: the fringe roots of
// the levels this jump crosses, which no frontier entry covers, each as its span of descendants.
__global__ __launch_bounds__(TD_THREADS) void k_topdown_jump_sh(const uint8_t *__restrict__ ca, const uint8_t *__restrict__ cb,
                                                        uint64_t desc_count, int k, uint64_t a_par, uint64_t a_desc,
                                                        TdSeeds S, const uint32_t *__restrict__ fin,
                                                        const uint32_t *__restrict__ nin, uint32_t *__restrict__ fout,
                                                        uint32_t *__restrict__ nout) {
    __shared__ uint32_t sapp[17];
    const uint32_t cnt = *nin;
    const uint64_t totf = (uint64_t)cnt << k, tot = totf + S.total;
    const uint64_t mask = (1ull << k) - 1ull;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < tot; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = base + threadIdx.x;
        bool d = false;
        uint64_t c = UINT64_MAX;
        if (t < totf) {
            c = ((((uint64_t)fin[t >> k] + a_par) << k) | (t & mask)) - a_desc;
        } else if (t < tot) {
            uint32_t u = (uint32_t)(t - totf), i = 0;
            while (i + 1 < S.n && u >= S.span[i]) u -= S.span[i++];
            c = S.first[i] + u;
        }
        if (c < desc_count) d = !digest_eq(ca + 32ull * c, cb + 32ull * c);
        block_append<uint32_t>(d, (uint32_t)c, fout, nout, sapp);
    }
}

// Batched form (entries (variant << 32) | node): k_topdown_jump_batch_u below.

// ---- unrolled form of the jumps (round 6) ----
// Consecutive lanes keep consecutive descendants (a wave's 16-B loads cover whole 128-B lines: 4 lanes per
// line), but each thread takes JU descendants a block apart per grid-stride step and issues all their
// loads before comparing, then appends its divergent ones with ONE block-wide reservation per step. The
// form above pays a block barrier + a device atomic round trip for every 1,024 descendants with one
// dependent chain (entry -> two 32-B digests) in flight per thread. Interleaved A/B on one box (configs[4]
// walk per step / 100M value-only device ms): one per thread 0.333 / 0.197, JU = 2 0.285 / 0.194, JU = 3
// 0.325, JU = 4 0.332 / 0.206, JU = 8 0.557 / 0.273 (fewer waves per CU); grid cap 2,048 vs 1,024 workgroups
// 0.285 vs 0.295. Tried first: a thread per 4 consecutive descendants, 16 loads each — 20 % slower (every
// load instruction then touched 64 lines).
constexpr int JU = 2;
__device__ __forceinline__ bool u4_eq(const uint4 &x, const uint4 &y) {
    return ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) == 0;
}
// Block-wide reservation of `cnt` output slots per thread: returns the thread's first slot (one device
// atomic per call; every thread of the block calls it). lds: >= 17 u32.
__device__ __forceinline__ uint32_t block_reserve(uint32_t cnt, uint32_t *count, uint32_t *lds) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t inc = wave_incl_scan<uint32_t>(cnt);
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t i = 0; i < nw; ++i) {
            const uint32_t c = lds[i];
            lds[i] = tot;
            tot += c;
        }
        lds[16] = tot ? atomicAdd(count, tot) : 0u;
    }
    __syncthreads();
    const uint32_t r = lds[16] + lds[w] + inc - cnt;
    __syncthreads();  // lds is reused by the next call
    return r;
}

__global__ __launch_bounds__(TD_THREADS) void k_topdown_jump_u(const uint8_t *__restrict__ ca, const uint8_t *__restrict__ cb,
                                                       uint64_t desc_count, int k, const uint32_t *__restrict__ fin,
                                                       const uint32_t *__restrict__ nin, uint32_t *__restrict__ fout,
                                                       uint32_t *__restrict__ nout, uint32_t *__restrict__ gate,
                                                       uint32_t word, uint64_t level_count, uint32_t *__restrict__ bm,
                                                       const uint32_t *__restrict__ scr, TdScreen SC) {
    __shared__ uint32_t sapp[17];
    // SC.slots: this jump also takes the key-set screen (a jump before the gated one): the sampled prefix
    // loads issue first and are counted after the walk's work, one word per slot (plain stores)
    uint32_t sbad = 0;  // bit j: this thread's sample of the block's j-th slot differs
    if (SC.slots) {
        const uint32_t samples = (uint32_t)std::min<uint64_t>(SC.n, 256u * TD_SCREEN_SLOTS);
        uint32_t j = 0;
        for (uint32_t sl = blockIdx.x; sl < TD_SCREEN_SLOTS; sl += gridDim.x, ++j) {
            const uint32_t q = sl * 256 + threadIdx.x;
            if (threadIdx.x < 256 && q < samples) {
                // 64-bit (q < 2^12, n < 2^48); the 128-bit division of k_sample_pfx cost a jump ~6 us
                const uint64_t i = samples > 1 ? (uint64_t)q * (SC.n - 1) / (samples - 1) : 0;
                sbad |= (uint32_t)(SC.pa[i] != SC.pb[i]) << j;
            }
        }
    }
    const uint32_t cnt = *nin;
    uint32_t screen = 0;  // k_sample_pfx_slots' words (scr: TD_SCREEN_SLOTS of them), else the gate word's count
    if (gate && scr)
        for (int i = 0; i < TD_SCREEN_SLOTS; ++i) screen |= scr[i];
    if (gate && (screen != 0 || gate[word] != 0 || 2ull * cnt > level_count)) {  // the level-4 abort test of the pair walk
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(gate + word, 0x80000000u);
        return;
    }
    const uint64_t tot = (uint64_t)cnt << k;
    const uint64_t mask = (1ull << k) - 1ull;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * JU;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * JU; base < tot; base += step) {
        // branch-free: out-of-range slots load a clamped (valid) address and are masked afterwards, so the
        // JU entry loads and then the 4 x JU digest loads issue back to back (a conditional load per slot
        // made the compiler wait for each before the next)
        // (32-bit index arithmetic: node indices of a level fit u32 — the frontier is u32 — and a 64-bit
        // zero-extended shift made the compiler load every entry into the same register pair, one at a time)
        uint64_t c[JU];
        uint32_t f[JU];
        uint4 x[JU][2], y[JU][2];
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            const uint64_t t = base + (uint64_t)u * blockDim.x + threadIdx.x;
            f[u] = fin[(t < tot ? t : tot - 1) >> k];
        }
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            const uint64_t t = base + (uint64_t)u * blockDim.x + threadIdx.x;
            c[u] = t < tot ? (uint64_t)((f[u] << k) | ((uint32_t)t & (uint32_t)mask)) : UINT64_MAX;
        }
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            const uint64_t cc = c[u] < desc_count ? c[u] : desc_count - 1;
            const uint4 *pa = reinterpret_cast<const uint4 *>(ca + 32 * cc);
            const uint4 *pb = reinterpret_cast<const uint4 *>(cb + 32 * cc);
            x[u][0] = pa[0], x[u][1] = pa[1], y[u][0] = pb[0], y[u][1] = pb[1];
        }
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < JU; ++u)
            if (c[u] < desc_count && !(u4_eq(x[u][0], y[u][0]) && u4_eq(x[u][1], y[u][1]))) m |= 1u << u;
        uint32_t o = block_reserve((uint32_t)__popc(m), nout, sapp);
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            if (m & (1u << u)) {
                fout[o++] = (uint32_t)c[u];
                if (bm) atomicOr(bm + (c[u] >> 5), 1u << (c[u] & 31));  // landing on the leaves: position bitmap
            }
        }
    }
    if (SC.slots) {
        uint32_t j = 0;
        for (uint32_t sl = blockIdx.x; sl < TD_SCREEN_SLOTS; sl += gridDim.x, ++j) {
            const int c = __syncthreads_count((sbad >> j) & 1u);
            if (threadIdx.x == 0) SC.slots[sl] = (uint32_t)c;
        }
    }
}

__global__ __launch_bounds__(TD_THREADS) void k_topdown_jump_batch_u(const uint8_t *__restrict__ ca, TdVariants V,
                                                             uint64_t desc_off, uint64_t desc_count, int k,
                                                             const uint64_t *__restrict__ fin,
                                                             const uint32_t *__restrict__ nin,
                                                             uint64_t *__restrict__ fout, uint32_t *__restrict__ nout,
                                                             uint32_t *__restrict__ bm, uint64_t bn,
                                                             uint32_t *__restrict__ gate, uint32_t word,
                                                             uint64_t level_count) {
    __shared__ uint32_t sapp[17];
    // the variants' node arrays from LDS (a per-lane index into the kernel-argument array is a dependent
    // global load per descendant); used as global-address-space pointers, so the digest loads stay
    // global_load (a flat pointer would make every LDS wait wait for them too)
    __shared__ uint64_t s_vn[TD_MAX_VARIANTS];
    if (threadIdx.x < TD_MAX_VARIANTS) s_vn[threadIdx.x] = reinterpret_cast<uint64_t>(V.nodes[threadIdx.x]) + desc_off;
    __syncthreads();
    const uint32_t cnt = *nin;
    if (gate && (gate[word] != 0 || 2ull * cnt > level_count)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(gate + word, 0x80000000u);
        return;
    }
    const uint64_t tot = (uint64_t)cnt << k;
    const uint64_t mask = (1ull << k) - 1ull;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * JU;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * JU; base < tot; base += step) {
        uint64_t c[JU];
        uint32_t v[JU];
        uint4 x[JU][2], y[JU][2];
#pragma unroll
        for (int u = 0; u < JU; ++u) {  // branch-free, as in k_topdown_jump_u
            const uint64_t t = base + (uint64_t)u * blockDim.x + threadIdx.x;
            const uint64_t tc = t < tot ? t : tot - 1;
            const uint64_t e = fin[tc >> k];
            v[u] = (uint32_t)(e >> 32);
            c[u] = t < tot ? (((e & 0xFFFFFFFFull) << k) | (tc & mask)) : UINT64_MAX;
        }
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            const uint64_t cc = c[u] < desc_count ? c[u] : desc_count - 1;
            const uint4 *pa = reinterpret_cast<const uint4 *>(ca + 32 * cc);
            typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(1))) const u4v_t g_u4c;
            const g_u4c *pb = (const g_u4c *)(s_vn[v[u]] + 32 * cc);
            const u4v_t b0 = pb[0], b1 = pb[1];
            x[u][0] = pa[0], x[u][1] = pa[1];
            y[u][0] = make_uint4(b0.x, b0.y, b0.z, b0.w);
            y[u][1] = make_uint4(b1.x, b1.y, b1.z, b1.w);
        }
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < JU; ++u)
            if (c[u] < desc_count && !(u4_eq(x[u][0], y[u][0]) && u4_eq(x[u][1], y[u][1]))) m |= 1u << u;
        uint32_t o = block_reserve((uint32_t)__popc(m), nout, sapp);
#pragma unroll
        for (int u = 0; u < JU; ++u) {
            if (m & (1u << u)) {
                fout[o++] = ((uint64_t)v[u] << 32) | c[u];
                if (bm) {  // landing on the leaves: the (variant, position) bit of k_vpos_* directly
                    const uint64_t g = (uint64_t)v[u] * bn + c[u];
                    atomicOr(bm + (g >> 5), 1u << (g & 31));
                }
            }
        }
    }
}

// ---- the top of an unsharded walk in one workgroup (round 6) ----
// The first launches of a walk compare a handful of nodes each (configs[4]: 7 roots, 56, 896, 13K
// descendants) and cost ~4-8 us apiece plus ~5 us of dispatch gap: ~45 us per step for almost no bytes.
// One 1,024-thread workgroup walks them instead: frontier entries (v << 24 | node) in LDS (LDS atomics for
// the appends, a barrier per jump), the last target level's divergent nodes reserved block-wide in HBM.
constexpr uint32_t TOP_F = (uint32_t)TD_TOP_MAX_FRONTIER;  // LDS frontier entries (the host bounds k x nodes)
template <bool WIDE>
__global__ __launch_bounds__(1024) void k_topdown_top(const uint8_t *__restrict__ na, TdVariants V, uint32_t k, TdTop P,
                                                       void *__restrict__ fout_v, uint32_t *__restrict__ cnt,
                                                       uint32_t zero_n, uint32_t ff_from) {
    __shared__ uint32_t fa[TOP_F], fb[TOP_F];
    __shared__ uint32_t s_n[2], sapp[17];
    __shared__ uint64_t s_vn[TD_MAX_VARIANTS];
    const uint32_t tid = threadIdx.x;
    if (tid < TD_MAX_VARIANTS) s_vn[tid] = reinterpret_cast<uint64_t>(V.nodes[tid]);
    if (tid < 2) s_n[tid] = 0;
    // the walk's counters cnt[0 .. zero_n) zeroed here instead of by a fill launch before this one (the
    // barrier below waits for the stores before any count is added to)
    // (words [ff_from, zero_n) get 0xFFFFFFFF instead: the batched walk's per-variant segment starts)
    for (uint32_t i = tid; i < zero_n; i += blockDim.x) cnt[i] = i < ff_from ? 0u : 0xFFFFFFFFu;
    __syncthreads();
    typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const u4v_t g_u4c;
    auto differs = [&](uint32_t v, uint64_t node_off) {  // node at 32 x node_off in the base and variant v
        const g_u4c *pa = (const g_u4c *)(reinterpret_cast<uint64_t>(na) + 32 * node_off);
        const g_u4c *pb = (const g_u4c *)(s_vn[v] + 32 * node_off);
        const u4v_t a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
        const u4v_t x = (a0 ^ b0) | (a1 ^ b1);
        return (x.x | x.y | x.z | x.w) != 0;
    };
    // the roots (level T[0] = L - 1: one node)
    uint32_t *fin = fa, *fo = fb;
    if (tid < k && differs(tid, P.off[P.T[0]])) fin[atomicAdd(&s_n[0], 1u)] = tid << 24;
    __syncthreads();
    uint32_t nin = s_n[0];
    if (tid == 0) cnt[P.T[0]] = nin;
    for (uint32_t q = 1; q <= P.nt; ++q) {
        const uint32_t l = P.T[q - 1], lt = P.T[q], kk = l - lt;
        const bool last = q == P.nt;
        const uint64_t dc = P.cnt[lt], doff = P.off[lt];
        const uint32_t tot = nin << kk, mask = (1u << kk) - 1u;
        for (uint32_t b = 0; b < tot; b += 1024) {
            const uint32_t t = b + tid;
            bool d = false;
            uint32_t e = 0, c = 0;
            if (t < tot) {
                e = fin[t >> kk];
                c = ((e & 0xFFFFFFu) << kk) | (t & mask);
                d = c < dc && differs(e >> 24, doff + c);
            }
            if (!last) {
                if (d) fo[atomicAdd(&s_n[q & 1], 1u)] = (e & 0xFF000000u) | c;
            } else {  // block-wide reservation in the walk's next frontier (HBM)
                const uint64_t m = __ballot(d);
                const uint32_t lane = tid & 63, w = tid >> 6;
                if (lane == 0) sapp[w] = (uint32_t)__popcll(m);
                __syncthreads();
                if (tid == 0) {
                    uint32_t s = 0;
                    for (uint32_t i = 0; i < 16; ++i) {
                        const uint32_t x = sapp[i];
                        sapp[i] = s;
                        s += x;
                    }
                    sapp[16] = s ? atomicAdd(cnt + lt, s) : 0u;
                }
                __syncthreads();
                if (d) {
                    const uint32_t o = sapp[16] + sapp[w] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                    if (WIDE) reinterpret_cast<uint64_t *>(fout_v)[o] = ((uint64_t)(e >> 24) << 32) | c;
                    else reinterpret_cast<uint32_t *>(fout_v)[o] = c;
                }
                __syncthreads();
            }
        }
        if (last) break;
        __syncthreads();
        nin = s_n[q & 1];
        if (tid == 0) {
            cnt[lt] = nin;
            s_n[(q + 1) & 1] = 0;
        }
        uint32_t *sw = fin;
        fin = fo;
        fo = sw;
        __syncthreads();
    }
}

// ---- batched top-down walk: one base tree against k variants with the same level plan (configs[4]) ----
// Frontier entries are (variant << 32) | local node index; every level is one launch for all variants.
__global__ __launch_bounds__(TD_THREADS) void k_topdown_level_batch(const uint8_t *__restrict__ ca, TdVariants V,
                                                            uint64_t child_off, uint64_t child_count, uint64_t a_par,
                                                            uint64_t a_child, uint64_t r0, uint64_t r1, uint32_t k,
                                                            const uint64_t *__restrict__ fin,
                                                            const uint32_t *__restrict__ nin,
                                                            uint64_t *__restrict__ fout, uint32_t *__restrict__ nout) {
    __shared__ uint32_t sapp[17];
    const uint32_t cnt = *nin;
    const uint64_t tot = 2ull * cnt + 2ull * k;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < tot; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = base + threadIdx.x;
        bool d = false;
        uint64_t c = UINT64_MAX;
        uint32_t v = 0;
        if (t < 2ull * cnt) {
            const uint64_t e = fin[t >> 1];
            v = (uint32_t)(e >> 32);
            c = 2 * ((e & 0xFFFFFFFFull) + a_par) + (t & 1) - a_child;
        } else if (t < tot) {
            const uint64_t q = t - 2ull * cnt;
            v = (uint32_t)(q >> 1);
            c = (q & 1) ? r1 : r0;
        }
        if (c < child_count) d = !digest_eq(ca + 32ull * c, V.nodes[v] + child_off + 32ull * c);
        block_append<uint64_t>(d, ((uint64_t)v << 32) | c, fout, nout, sapp);
    }
}

// Sorted (variant, leaf position) entries: keys must be equal on both sides (else that variant's key
// set differs there: nbad[v]); refs[k] = the base's sorted index; count[v] = first entry of variant v
// (left untouched — the caller presets all-ones — when v has none).
// mdev (optional): the entry count on the device (grid-stride; m is then only the grid's bound).
__global__ void k_topdown_leaves_batch(const uint64_t *__restrict__ ent, uint64_t m, int pb, DiffSide A,
                                       const DiffSide *__restrict__ Bs, uint64_t check, uint64_t *__restrict__ refs,
                                       uint32_t *__restrict__ nbad, uint32_t *__restrict__ count,
                                       const uint32_t *__restrict__ mdev) {
    if (mdev) m = *mdev;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = ent[k];  // (variant << pb) | position
        const uint32_t v = (uint32_t)(e >> pb);
        const uint64_t i = e & ((1ull << pb) - 1ull);
        refs[k] = i;
        if (k == 0 || (uint32_t)(ent[k - 1] >> pb) != v) count[v] = (uint32_t)k;  // segment start of variant v
        if (((check >> v) & 1ull) && !key_eq_at(A, Bs[v], i)) atomicAdd(&nbad[v], 1u);
    }
}

// ---- batched walk: (variant, position) leaf entries in ascending order without a sort (round 5) ----
// One bit per (variant, position) over k x n bits (all-zero between calls): set from the level-0 frontier
// (device count), per-block popcounts, an exclusive scan of the block counts, then each block writes its
// entries in order and clears its words. Replaces a host readback of the frontier size + a 5-launch
// radix sort of the entries (configs[4]: ~0.15 ms per step).
// Round 6: 16 consecutive words per thread (4 uint4 loads in flight, 4x fewer blocks to scan); the
// variant of a set bit from one division per thread (a block spans at most two variants when n >= 2^17)
constexpr uint32_t VP_TW = 16;                 // words per thread
constexpr uint32_t VP_WORDS = 256 * VP_TW;     // bitmap words per block
__device__ __forceinline__ uint4 vp_words(const uint32_t *bm, uint64_t w0, uint64_t words) {
    if (w0 + 3 < words) return *reinterpret_cast<const uint4 *>(bm + w0);
    uint4 x = make_uint4(0, 0, 0, 0);
    if (w0 < words) x.x = bm[w0];
    if (w0 + 1 < words) x.y = bm[w0 + 1];
    if (w0 + 2 < words) x.z = bm[w0 + 2];
    return x;
}
__global__ void k_vpos_setbits(const uint64_t *__restrict__ f, const uint32_t *__restrict__ mdev, uint64_t n,
                               uint32_t *__restrict__ bm) {
    const uint64_t m = *mdev;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = f[i];  // (variant << 32) | position
        const uint64_t g = (e >> 32) * n + (e & 0xFFFFFFFFull);
        atomicOr(bm + (g >> 5), 1u << (g & 31));
    }
}
__device__ __forceinline__ uint32_t vp_load(const uint32_t *bm, uint64_t w0, uint64_t words, uint32_t x[VP_TW]) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < VP_TW / 4; ++j) {
        const uint4 v = vp_words(bm, w0 + 4 * j, words);
        x[4 * j] = v.x, x[4 * j + 1] = v.y, x[4 * j + 2] = v.z, x[4 * j + 3] = v.w;
        c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
    }
    return c;
}
__global__ __launch_bounds__(256) void k_vpos_count(const uint32_t *__restrict__ bm, uint64_t words,
                                                    uint32_t *__restrict__ bc) {
    __shared__ uint32_t red[4];
    const uint64_t w0 = (uint64_t)blockIdx.x * VP_WORDS + VP_TW * threadIdx.x;
    uint32_t x[VP_TW];
    uint32_t c = vp_load(bm, w0, words, x);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// DIRECT: boff holds the per-block counts and each block sums those before it itself (no scan launches;
// at most VP_DIRECT_BLOCKS blocks, a few thousand L2-resident words each); else boff = their exclusive scan.
constexpr uint64_t VP_DIRECT_BLOCKS = 8192;
template <bool DIRECT>
__global__ __launch_bounds__(256) void k_vpos_emit(uint32_t *__restrict__ bm, uint64_t words,
                                                   const uint32_t *__restrict__ boff, uint64_t n, int pb,
                                                   uint64_t *__restrict__ out) {
    if (DIRECT ? boff[blockIdx.x] == 0 : boff[blockIdx.x + 1] == boff[blockIdx.x]) return;  // no entry here
    __shared__ uint32_t tot_w[4], base_w[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t base = 0;
    if (DIRECT) {
        uint32_t sb = 0;
        for (uint32_t i = threadIdx.x; i < blockIdx.x; i += 256) sb += boff[i];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) sb += __shfl_xor(sb, d);
        if (lane == 0) base_w[wave] = sb;
    }
    const uint64_t w0 = (uint64_t)blockIdx.x * VP_WORDS + VP_TW * threadIdx.x;
    uint32_t x[VP_TW];
    const uint32_t c = vp_load(bm, w0, words, x);
    const uint32_t v = wave_incl_scan<uint32_t>(c);
    if (lane == 63) tot_w[wave] = v;
    __syncthreads();
    if (DIRECT) base = (uint64_t)base_w[0] + base_w[1] + base_w[2] + base_w[3];
    else base = boff[blockIdx.x];
    uint64_t o = base + (v - c);
    for (uint32_t w = 0; w < wave; ++w) o += tot_w[w];
    if (!c) return;
    // the thread's 512 bits span at most two variants (n >= 512) or any number (tiny n: divide per bit)
    const uint64_t g0 = w0 * 32;
    uint64_t vv = g0 / n, vend = (vv + 1) * n;
#pragma unroll
    for (uint32_t q = 0; q < VP_TW; ++q) {
        for (uint32_t b = x[q]; b; b &= b - 1) {
            const uint64_t g = (w0 + q) * 32 + (uint32_t)(__ffs(b) - 1);
            while (g >= vend) {
                ++vv;
                vend += n;
            }
            out[o++] = (vv << pb) | (g - (vend - n));
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < VP_TW / 4; ++j) {
        const uint64_t wj = w0 + 4 * j;
        if (wj + 3 < words) {
            *reinterpret_cast<uint4 *>(bm + wj) = make_uint4(0, 0, 0, 0);
        } else {
            for (int q = 0; q < 4; ++q)
                if (wj + q < words) bm[wj + q] = 0;
        }
    }
}

// Divergent leaf positions (sorted): refs of keys equal on both sides; counts positions whose keys
// differ (then the key sets differ there and the caller falls back to the merge-join).
__global__ void k_topdown_leaves(const uint64_t *__restrict__ pos, uint64_t m, DiffSide A, DiffSide B, int check,
                                 uint64_t *__restrict__ refs, uint32_t *__restrict__ nbad) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t i = pos[k];
    refs[k] = i;
    if (check && !key_eq_at(A, B, i)) atomicAdd(nbad, 1u);
}

// ---- one-wait tail of the unsharded top-down pair diff (round 3) ----
// The same steps as the round-2 tail (leaf-key check, key lengths, scan, key gather, copy into pinned
// host memory), but sized from the device's divergent count (*mdev) and a host capacity (cap_m keys,
// cap_b bytes) instead of a host readback between them, so the whole diff is queued before the host
// waits once. k_td_gate makes the walk's level-4 abort test on the device.
__global__ void k_td_gate(uint32_t *__restrict__ cnt, uint32_t word, uint32_t level, uint64_t level_count) {
    if (threadIdx.x != 0) return;
    if (cnt[word] != 0 || 2 * (uint64_t)cnt[level] > level_count) {
        cnt[word] |= 0x80000000u;  // screen failed or frontier over half the level: merge-join
        cnt[level] = 0;            // the jumps below see an empty frontier
    }
}

// refs[k] (k < *mdev, side-A positions) checked against B's keys (leaf-key check).
__global__ void k_td_check_dev(const uint64_t *__restrict__ refs, const uint32_t *__restrict__ mdev, DiffSide A,
                               DiffSide B, uint32_t *__restrict__ nbad) {
    const uint64_t m = *mdev;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x)
        if (!key_eq_at(A, B, refs[k])) atomicAdd(nbad, 1u);
}

// lens[k] = key length of refs[k] for k < min(*mdev, cap), 0 up to cap (the scan's padding).
__global__ void k_keylens_dev(const uint64_t *__restrict__ refs, const uint32_t *__restrict__ mdev, uint64_t cap,
                              DiffSide A, uint64_t *__restrict__ lens) {
    const uint64_t m = *mdev;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cap; k += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t len = 0;
        if (k < m) (void)key_at(A, refs[k], &len);
        lens[k] = len;
    }
}

// Key bytes of refs[k] at off[k]; nothing when the list outgrew the capacity (the host falls back).
__global__ void k_keys_dev(const uint64_t *__restrict__ refs, const uint32_t *__restrict__ mdev, uint64_t cap_m,
                           uint64_t cap_b, DiffSide A, const uint64_t *__restrict__ off, uint8_t *__restrict__ out) {
    const uint64_t m = *mdev;
    if (m > cap_m || off[cap_m] > cap_b) return;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t len;
        const uint8_t *src = key_at(A, refs[k], &len);
        uint8_t *d = out + off[k];
        const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)len;
        if ((al & 15) == 0) {
            for (uint64_t x = 0; x < len; x += 16)
                *reinterpret_cast<uint4 *>(d + x) = *reinterpret_cast<const uint4 *>(src + x);
        } else if ((al & 3) == 0) {
            for (uint64_t x = 0; x < len; x += 4)
                *reinterpret_cast<uint32_t *>(d + x) = *reinterpret_cast<const uint32_t *>(src + x);
        } else {
            for (uint64_t x = 0; x < len; ++x) d[x] = src[x];
        }
    }
}

// Offsets (m + 1) and key bytes into the mapped pinned block (16-B stores), unless over capacity.
__global__ __launch_bounds__(256) void k_tail_copy_dev(const uint64_t *__restrict__ off, const uint8_t *__restrict__ kout,
                                                       const uint32_t *__restrict__ mdev, uint64_t cap_m, uint64_t cap_b,
                                                       uint8_t *__restrict__ doff, uint8_t *__restrict__ dkeys,
                                                       int copy_offsets) {
    const uint64_t m = *mdev;
    if (m > cap_m) return;
    const uint64_t bytes = off[cap_m];
    if (bytes > cap_b) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x, t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t no = 8 * (m + 1), nvo = no / 16;
    const uint8_t *so = reinterpret_cast<const uint8_t *>(off);
    if (copy_offsets) {
        for (uint64_t v = t; v < nvo; v += stride)
            reinterpret_cast<uint4 *>(doff)[v] = reinterpret_cast<const uint4 *>(so)[v];
        if (t < no - nvo * 16) doff[nvo * 16 + t] = so[nvo * 16 + t];
    }
    const uint64_t nvk = bytes / 16;
    for (uint64_t v = t; v < nvk; v += stride)
        reinterpret_cast<uint4 *>(dkeys)[v] = reinterpret_cast<const uint4 *>(kout)[v];
    if (t < bytes - nvk * 16) dkeys[nvk * 16 + t] = kout[nvk * 16 + t];
}

inline dim3 grid1d(uint64_t n, uint32_t bs = 256) { return dim3((uint32_t)ceil_div(n ? n : 1, bs)); }

}  // namespace

static uint64_t defer_cap(uint64_t M) { return std::min<uint64_t>(M, 1ull << 21); }

size_t diff_scratch_bytes(uint64_t M) {
    uint64_t nt = ceil_div(M ? M : 1, WTILE);
    size_t b = 0;
    b += (nt + 2) * sizeof(uint64_t);             // split
    b += nt * 64 * sizeof(uint32_t);              // packed
    b += (nt + 2) * sizeof(uint64_t);             // tile counts
    b += (nt + 2) * sizeof(uint64_t);             // tile offsets
    b += scan_scratch_bytes(nt) + 1024;
    b += defer_cap(M) * sizeof(uint64_t) + 512;                     // deferred key checks + their count
    return b;
}

void launch_diff(const DiffSide &A, const DiffSide &B, void *scratch, uint64_t *refs, uint64_t *count,
                 hipStream_t st, bool defer) {
    const uint64_t M = A.n + B.n;
    if (M == 0) {
        MKV_HIP(hipMemsetAsync(count, 0, 2 * sizeof(uint64_t), st));
        return;
    }
    const uint64_t nt = ceil_div(M, WTILE);
    uint8_t *p = reinterpret_cast<uint8_t *>(scratch);
    auto carve = [&](size_t bytes) {
        uint8_t *r = p;
        p += (bytes + 255) & ~size_t(255);
        return r;
    };
    uint64_t *split = reinterpret_cast<uint64_t *>(carve((nt + 2) * sizeof(uint64_t)));
    uint32_t *packed = reinterpret_cast<uint32_t *>(carve(nt * 64 * sizeof(uint32_t)));
    uint64_t *tilecnt = reinterpret_cast<uint64_t *>(carve((nt + 2) * sizeof(uint64_t)));
    uint64_t *tileoff = reinterpret_cast<uint64_t *>(carve((nt + 2) * sizeof(uint64_t)));
    void *sc = carve(scan_scratch_bytes(nt));
    DeferList V{reinterpret_cast<uint64_t *>(carve(defer_cap(M) * sizeof(uint64_t))),
                reinterpret_cast<uint32_t *>(carve(256)), (uint32_t)defer_cap(M)};
    const uint32_t wg = (uint32_t)ceil_div(nt, 4);
    // partition + this diff's deferred-check reset (one launch)
    hipLaunchKernelGGL(k_diff_partition, dim3((uint32_t)ceil_div(ceil_div(nt, PART_STRIDE), 4)), dim3(256), 0, st, A, B,
                       nt, split, V.count, count + 1);
    if (defer)
        hipLaunchKernelGGL(k_diff_pass1<true>, dim3(wg), dim3(256), 0, st, A, B, split, nt, packed, tilecnt, V);
    else
        hipLaunchKernelGGL(k_diff_pass1<false>, dim3(wg), dim3(256), 0, st, A, B, split, nt, packed, tilecnt, V);
    MKV_LAUNCH_CHECK();
    exclusive_scan_u64(tilecnt, tileoff, nt, count, sc, st);
    // pass 2 + (defer) the key checks in the same launch
    const uint32_t nvb = defer ? (uint32_t)std::min<uint64_t>(ceil_div(defer_cap(M), 256), 1024) : 0;
    const uint32_t wg2 = (uint32_t)ceil_div(ceil_div(nt, 64), 4);  // one wave per 64 tiles
    hipLaunchKernelGGL(k_diff_pass2, dim3(wg2 + nvb), dim3(256), 0, st, A, B, split, nt, packed, tilecnt, tileoff, refs,
                       wg2, V, count + 1);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_level(const uint8_t *ca, const uint8_t *cb, uint64_t child_count, uint64_t a_par, uint64_t a_child,
                          uint64_t r0, uint64_t r1, const uint32_t *fin, const uint32_t *nin, uint32_t *fout,
                          uint32_t *nout, uint64_t max_frontier, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(2 * max_frontier + 2, TD_THREADS), 2048);
    hipLaunchKernelGGL(k_topdown_level, dim3((uint32_t)blocks), dim3(TD_THREADS), 0, st, ca, cb, child_count, a_par, a_child,
                       r0, r1, fin, nin, fout, nout);
    MKV_LAUNCH_CHECK();
}

void launch_sample_pfx(const uint64_t *pa, const uint64_t *pb, uint64_t n, uint32_t samples, uint32_t *count,
                       hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_sample_pfx, dim3((samples + 255) / 256), dim3(256), 0, st, pa, pb, n, samples, count);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_level_batch(const uint8_t *ca, const TdVariants &V, uint64_t child_off, uint64_t child_count,
                                uint64_t a_par, uint64_t a_child, uint64_t r0, uint64_t r1, uint32_t k,
                                const uint64_t *fin, const uint32_t *nin, uint64_t *fout, uint32_t *nout,
                                uint64_t max_frontier, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(2 * max_frontier + 2 * k, TD_THREADS), 2048);
    hipLaunchKernelGGL(k_topdown_level_batch, dim3((uint32_t)blocks), dim3(TD_THREADS), 0, st, ca, V, child_off, child_count,
                       a_par, a_child, r0, r1, k, fin, nin, fout, nout);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_leaves_batch(const uint64_t *ent, uint64_t m, int pb, const DiffSide &A, const DiffSide *Bs,
                                 uint64_t check, uint64_t *refs, uint32_t *nbad, uint32_t *count, hipStream_t st,
                                 const uint32_t *mdev) {
    if (!m) return;
    const dim3 g = mdev ? dim3((uint32_t)std::min<uint64_t>(ceil_div(m, 256), 2048)) : grid1d(m);
    hipLaunchKernelGGL(k_topdown_leaves_batch, g, dim3(256), 0, st, ent, m, pb, A, Bs, check, refs, nbad, count, mdev);
    MKV_LAUNCH_CHECK();
}

uint64_t vpos_scratch_words(uint64_t bits) { return 2 * (ceil_div((bits + 31) / 32, VP_WORDS) + 2); }

void launch_vpos_sorted_dev(const uint64_t *f, const uint32_t *mdev, uint64_t cap, uint64_t n, uint32_t k, int pb,
                            uint32_t *bm, uint32_t *bc, void *scan_scr, uint64_t *out, hipStream_t st, bool bits_set) {
    const uint64_t words = ((uint64_t)k * n + 31) / 32, nb = ceil_div(words, VP_WORDS);
    uint32_t *boff = bc + nb + 1;
    if (!bits_set) hipLaunchKernelGGL(k_vpos_setbits, dim3((uint32_t)std::min<uint64_t>(ceil_div(cap ? cap : 1, 256), 2048)), dim3(256),
                       0, st, f, mdev, n, bm);
    hipLaunchKernelGGL(k_vpos_count, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc);
    if (nb <= VP_DIRECT_BLOCKS) {  // round 6: configs[4]'s 6.7K blocks without the 3-launch scan (~15 us)
        hipLaunchKernelGGL(k_vpos_emit<true>, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc, n, pb, out);
    } else {
        exclusive_scan_u32(bc, boff, nb, boff + nb, scan_scr, st);
        hipLaunchKernelGGL(k_vpos_emit<false>, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, boff, n, pb, out);
    }
    MKV_LAUNCH_CHECK();
}

__global__ void k_pack_entries(const uint64_t *__restrict__ ent, uint64_t m, int pb, uint64_t *__restrict__ key,
                               uint32_t *__restrict__ val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t e = ent[k];
    key[k] = ((e >> 32) << pb) | (e & 0xFFFFFFFFull);
    val[k] = (uint32_t)k;
}
void launch_pack_entries(const uint64_t *ent, uint64_t m, int pb, uint64_t *key, uint32_t *val, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_pack_entries, grid1d(m), dim3(256), 0, st, ent, m, pb, key, val);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_jump(const uint8_t *ca, const uint8_t *cb, uint64_t desc_count, int k, const uint32_t *fin,
                         const uint32_t *nin, uint32_t *fout, uint32_t *nout, uint64_t max_desc, hipStream_t st,
                         uint32_t *gate, uint32_t word, uint64_t level_count, uint32_t *bm, const uint32_t *scr,
                         const TdScreen &SC) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(max_desc ? max_desc : 1, (uint64_t)TD_THREADS * JU), 2048);
    hipLaunchKernelGGL(k_topdown_jump_u, dim3((uint32_t)blocks), dim3(TD_THREADS), 0, st, ca, cb, desc_count, k, fin, nin,
                       fout, nout, gate, word, level_count, bm, scr, SC);
    MKV_LAUNCH_CHECK();
}
void launch_topdown_jump_sh(const uint8_t *ca, const uint8_t *cb, uint64_t desc_count, int k, uint64_t a_par,
                            uint64_t a_desc, const TdSeeds &S, const uint32_t *fin, const uint32_t *nin, uint32_t *fout,
                            uint32_t *nout, uint64_t max_desc, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(max_desc + S.total ? max_desc + S.total : 1, TD_THREADS), 2048);
    hipLaunchKernelGGL(k_topdown_jump_sh, dim3((uint32_t)blocks), dim3(TD_THREADS), 0, st, ca, cb, desc_count, k, a_par,
                       a_desc, S, fin, nin, fout, nout);
    MKV_LAUNCH_CHECK();
}
void launch_topdown_jump_batch(const uint8_t *ca, const TdVariants &V, uint64_t desc_off, uint64_t desc_count, int k,
                               const uint64_t *fin, const uint32_t *nin, uint64_t *fout, uint32_t *nout,
                               uint64_t max_desc, hipStream_t st, uint32_t *bm, uint64_t bn, uint32_t *gate,
                               uint32_t word, uint64_t level_count) {
    const uint64_t blocks = std::min<uint64_t>(ceil_div(max_desc ? max_desc : 1, (uint64_t)TD_THREADS * JU), 2048);
    hipLaunchKernelGGL(k_topdown_jump_batch_u, dim3((uint32_t)blocks), dim3(TD_THREADS), 0, st, ca, V, desc_off, desc_count,
                       k, fin, nin, fout, nout, bm, bn, gate, word, level_count);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_top(const uint8_t *na, const TdVariants &V, uint32_t k, const TdTop &P, void *fout, bool wide,
                        uint32_t *cnt, hipStream_t st, uint32_t zero_n, uint32_t ff_from) {
    ff_from = std::min(ff_from, zero_n);
    if (wide) hipLaunchKernelGGL(k_topdown_top<true>, dim3(1), dim3(1024), 0, st, na, V, k, P, fout, cnt, zero_n, ff_from);
    else hipLaunchKernelGGL(k_topdown_top<false>, dim3(1), dim3(1024), 0, st, na, V, k, P, fout, cnt, zero_n, ff_from);
    MKV_LAUNCH_CHECK();
}

// ---- anti-entropy exchange primitives: node digests by index, peer comparison ----
__global__ void k_node_digests(const uint8_t *__restrict__ lvl, uint64_t count, const uint64_t *__restrict__ idx,
                               uint64_t m, uint8_t *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t i = idx[k];
    uint4 x = make_uint4(0, 0, 0, 0), y = x;  // absent node: zero digest (the peer treats it as divergent)
    if (i < count) {
        const uint4 *src = reinterpret_cast<const uint4 *>(lvl + 32 * i);
        x = src[0];
        y = src[1];
    }
    uint4 *dst = reinterpret_cast<uint4 *>(out + 32 * k);
    dst[0] = x;
    dst[1] = y;
}
__global__ void k_compare_nodes(const uint8_t *__restrict__ lvl, uint64_t count, const uint64_t *__restrict__ idx,
                                const uint8_t *__restrict__ peer, uint64_t m, uint8_t *__restrict__ flag) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint64_t i = idx[k];
    flag[k] = (i >= count || !digest_eq(lvl + 32 * i, peer + 32 * k)) ? 1 : 0;
}
void launch_node_digests(const uint8_t *lvl, uint64_t count, const uint64_t *idx, uint64_t m, uint8_t *out,
                         hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_node_digests, grid1d(m), dim3(256), 0, st, lvl, count, idx, m, out);
    MKV_LAUNCH_CHECK();
}
void launch_compare_nodes(const uint8_t *lvl, uint64_t count, const uint64_t *idx, const uint8_t *peer, uint64_t m,
                          uint8_t *flag, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_compare_nodes, grid1d(m), dim3(256), 0, st, lvl, count, idx, peer, m, flag);
    MKV_LAUNCH_CHECK();
}

void launch_topdown_leaves(const uint64_t *pos, uint64_t m, const DiffSide &A, const DiffSide &B, bool check,
                           uint64_t *refs, uint32_t *nbad, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_topdown_leaves, grid1d(m), dim3(256), 0, st, pos, m, A, B, (int)check, refs, nbad);
    MKV_LAUNCH_CHECK();
}

__global__ void k_fill_stride_u64(uint64_t *__restrict__ off, uint64_t m, uint64_t stride) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= m) off[k] = k * stride;
}
void launch_fill_stride_u64(uint64_t *off, uint64_t m, uint64_t stride, hipStream_t st) {
    hipLaunchKernelGGL(k_fill_stride_u64, grid1d(m + 1), dim3(256), 0, st, off, m, stride);
    MKV_LAUNCH_CHECK();
}

void launch_diff_keylens(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, uint64_t *lens,
                         hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_diff_keylens, grid1d(m), dim3(256), 0, st, refs, m, A, B, lens);
    MKV_LAUNCH_CHECK();
}

void launch_diff_keys_fixed(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, uint64_t klen,
                            uint8_t *out, hipStream_t st) {
    if (!m) return;
    const uint64_t G = m * (klen / 16);
    hipLaunchKernelGGL(k_diff_keys_g16, dim3((uint32_t)std::min<uint64_t>(ceil_div(G, 256), 8192)), dim3(256), 0, st, refs, m,
                       A, B, (uint32_t)klen, out);
    MKV_LAUNCH_CHECK();
}

void launch_diff_keys(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, const uint64_t *off,
                      uint8_t *out, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_diff_keys, grid1d(m), dim3(256), 0, st, refs, m, A, B, off, out);
    MKV_LAUNCH_CHECK();
}

void launch_prefix_bounds(const DiffSide &A, const uint8_t *prefix, uint32_t plen, uint64_t *lohi, hipStream_t st) {
    hipLaunchKernelGGL(k_prefix_bounds, dim3(1), dim3(64), 0, st, A, prefix, plen, lohi);
    MKV_LAUNCH_CHECK();
}


void launch_td_gate(uint32_t *cnt, uint32_t word, uint32_t level, uint64_t level_count, hipStream_t st) {
    hipLaunchKernelGGL(k_td_gate, dim3(1), dim3(64), 0, st, cnt, word, level, level_count);
    MKV_LAUNCH_CHECK();
}

// off[k] = min(k, *mdev) x klen for k <= cap (fixed-length keys: the tail's offsets without a scan).
__global__ void k_fill_stride_dev(uint64_t *__restrict__ off, const uint32_t *__restrict__ mdev, uint64_t cap,
                                  uint64_t klen) {
    const uint64_t m = *mdev;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= cap; k += (uint64_t)gridDim.x * blockDim.x)
        off[k] = (k < m ? k : m) * klen;
}

// Fixed-length keys (every key of both trees klen bytes): the leaf-key check (check), the offsets
// min(k, *mdev) x klen for k <= cap_m and the key bytes at k x klen in one launch (the offsets are
// known per position, so no thread waits for another's).
__global__ void k_tail_fixed_dev(const uint64_t *__restrict__ refs, const uint32_t *__restrict__ mdev, uint64_t cap_m,
                                 uint64_t cap_b, DiffSide A, DiffSide B, int check, uint32_t *__restrict__ nbad,
                                 uint64_t klen, uint64_t *__restrict__ off, uint8_t *__restrict__ out) {
    const uint64_t m = *mdev;
    const bool fits = m <= cap_m && m * klen <= cap_b;
    const uint64_t end = m > cap_m + 1 ? m : cap_m + 1;  // every divergent position is checked, even past cap_m
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < end; k += (uint64_t)gridDim.x * blockDim.x) {
        if (k <= cap_m) off[k] = (k < m ? k : m) * klen;
        if (k >= m) continue;
        const uint64_t i = refs[k];
        if (check && !key_eq_at(A, B, i)) atomicAdd(nbad, 1u);
        if (!fits) continue;
        uint64_t len;
        const uint8_t *src = key_at(A, i, &len);
        uint8_t *d = out + k * klen;
        const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)len;
        if ((al & 15) == 0) {
            for (uint64_t x = 0; x < len; x += 16)
                *reinterpret_cast<uint4 *>(d + x) = *reinterpret_cast<const uint4 *>(src + x);
        } else if ((al & 3) == 0) {
            for (uint64_t x = 0; x < len; x += 4)
                *reinterpret_cast<uint32_t *>(d + x) = *reinterpret_cast<const uint32_t *>(src + x);
        } else {
            for (uint64_t x = 0; x < len; ++x) d[x] = src[x];
        }
    }
}

// The same for the mapped pinned block, one thread per 16-B granule of the output: every store
// instruction of a wave covers 1 KiB of consecutive host addresses (a thread per key stored 16 B at a
// 32-B stride, twice), so the PCIe writes leave in full lines. klen % 16 == 0, out 16-B aligned.
__global__ void k_tail_fixed_g16(const uint64_t *__restrict__ refs, const uint32_t *__restrict__ mdev, uint64_t cap_m,
                                 uint64_t cap_b, DiffSide A, DiffSide B, int check, uint32_t *__restrict__ nbad,
                                 uint32_t klen, uint64_t *__restrict__ off, uint8_t *__restrict__ out,
                                 uint64_t *__restrict__ hsmall) {
    const uint64_t m = *mdev;
    const bool fits = m <= cap_m && m * klen <= cap_b;
    // hsmall: the call's scalars go to the host from here, no copy launch after this one — the count, the key
    // bytes and the walk's screen / abort word are final when it starts (block 0 stores them); a leaf-key
    // mismatch found here stores 1 into hsmall[3] (zeroed by the host before the call)
    if (hsmall && blockIdx.x == 0 && threadIdx.x == 0) {
        hsmall[0] = m;
        hsmall[1] = *nbad;
        hsmall[2] = (m < cap_m ? m : cap_m) * klen;
    }
    const uint32_t gpk = klen >> 4;
    const uint64_t end = m > cap_m + 1 ? m : cap_m + 1;
    const uint64_t G = fits ? m * gpk : 0;
    const uint64_t tot = G > end ? G : end, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += stride) {
        if (t < end) {
            if (t <= cap_m) off[t] = (t < m ? t : m) * klen;
            if (t < m && check && !key_eq_at(A, B, refs[t])) {
                atomicAdd(nbad, 1u);
                if (hsmall) hsmall[3] = 1;
            }
        }
        if (t < G) {
            const uint64_t k = t / gpk, x = t - k * gpk;
            uint64_t len;
            const uint8_t *src = key_at(A, refs[k], &len) + 16 * x;
            uint4 v;
            if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
                v = *reinterpret_cast<const uint4 *>(src);
            } else {
                uint32_t w[4];
                for (int j = 0; j < 4; ++j)
                    w[j] = (uint32_t)src[4 * j] | ((uint32_t)src[4 * j + 1] << 8) | ((uint32_t)src[4 * j + 2] << 16) |
                           ((uint32_t)src[4 * j + 3] << 24);
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            *reinterpret_cast<uint4 *>(out + 16 * t) = v;
        }
    }
}

bool launch_diff_tail_dev(const uint64_t *refs, const uint32_t *mdev, const DiffSide &A, const DiffSide &B, bool check,
                          uint32_t *nbad, uint64_t cap_m, uint64_t cap_b, uint64_t *lens, uint64_t *off, void *scan_scr,
                          uint8_t *kout, uint8_t *doff, uint8_t *dkeys, hipStream_t st, uint64_t klen,
                          bool host_offsets, uint64_t *hsmall) {
    const dim3 g((uint32_t)std::min<uint64_t>(ceil_div(cap_m, 256), 2048));
    if (klen && host_offsets) {
        // the key bytes straight into the mapped pinned block, no device staging + copy kernel (round 6: 100M
        // value-only diff 0.185 -> 0.172 ms device; the gather's random reads now overlap the PCIe writes of
        // other workgroups instead of preceding one streaming copy)
        const bool g16 = klen % 16 == 0 && klen < (1u << 20) && (reinterpret_cast<uintptr_t>(dkeys) & 15) == 0;
        if (g16)
            hipLaunchKernelGGL(k_tail_fixed_g16,
                               dim3((uint32_t)std::min<uint64_t>(ceil_div(std::max(cap_m + 1, cap_m * (klen / 16)), 256), 2048)),
                               dim3(256), 0, st, refs, mdev, cap_m, cap_b, A, B, (int)check, nbad, (uint32_t)klen, off, dkeys,
                               hsmall);
        else
            hipLaunchKernelGGL(k_tail_fixed_dev, dim3((uint32_t)std::min<uint64_t>(ceil_div(cap_m + 1, 256), 2048)),
                               dim3(256), 0, st, refs, mdev, cap_m, cap_b, A, B, (int)check, nbad, klen, off, dkeys);
        MKV_LAUNCH_CHECK();
        return g16 && hsmall;
    }
    if (klen) {  // every key of both trees has length klen: check, offsets and key bytes in one launch
        hipLaunchKernelGGL(k_tail_fixed_dev, dim3((uint32_t)std::min<uint64_t>(ceil_div(cap_m + 1, 256), 2048)), dim3(256),
                           0, st, refs, mdev, cap_m, cap_b, A, B, (int)check, nbad, klen, off, kout);
    } else {
        if (check) hipLaunchKernelGGL(k_td_check_dev, g, dim3(256), 0, st, refs, mdev, A, B, nbad);
        hipLaunchKernelGGL(k_keylens_dev, g, dim3(256), 0, st, refs, mdev, cap_m, A, lens);
        exclusive_scan_u64(lens, off, cap_m, off + cap_m, scan_scr, st);
        hipLaunchKernelGGL(k_keys_dev, g, dim3(256), 0, st, refs, mdev, cap_m, cap_b, A, off, kout);
    }
    const uint64_t cb = std::min<uint64_t>(ceil_div(std::max(8 * (cap_m + 1), cap_b) / 16 + 1, 256), 2048);
    hipLaunchKernelGGL(k_tail_copy_dev, dim3((uint32_t)cb), dim3(256), 0, st, off, kout, mdev, cap_m, cap_b, doff, dkeys,
                       (int)!(klen && host_offsets));
    MKV_LAUNCH_CHECK();
    return false;
}

}  // namespace mkv
