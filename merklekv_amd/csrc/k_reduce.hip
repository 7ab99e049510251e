// k_reduce.hip — Kernel B: level-by-level internal-node reduction (R4/R5, merkle.rs:94-118).
//
// The reference materialises a pointer tree, deep-cloning both subtrees into every parent
// (merkle.rs:107-108). Here the tree is implicit: level l is a dense array of 32-byte digests and
// node (l, j) covers leaves [j*2^l, min((j+1)*2^l, n)). Parent j hashes children 2j and 2j+1; when
// 2j+1 falls off the end of an odd level the child is promoted unchanged (R5), so level sizes are
// n, ceil(n/2), ceil(n/4), ..., 1 and every level is kept in HBM (diff, level views, incremental).
//
// One launch fuses up to 4 levels (10 for the last, small launch): a 512-thread workgroup owns a
// tile of 512 first-level parents (1024 children read coalesced from HBM, 64 B per lane), keeps each
// produced level in LDS (BE words, ping-pong 2 x 16 KiB) and feeds the next level from there. Level k
// of the tile has 512>>(k-1) parents, so with 4 fused levels every wave is fully busy: 8+4+2+1
// wave-hashes for 960 hashes, no lane idles. The second compression of every node is the constant
// padding block (sha_compress_pad64), so a node costs ~1.65 compressions of VALU work.
//
// Ownership (sharded trees): a launch computes only nodes whose leaf span lies inside the shard
// [o, o+n); plan.a/plan.c give, per level, the owned global index range. With one shard this is the
// whole tree.
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "sha256.hpp"

namespace mkv {

namespace {

constexpr int RD_TILE = 512;

template <bool SHORT, int THREADS>
__global__ __launch_bounds__(THREADS) void k_reduce_fused(FusePlan p) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][RD_TILE * 8];
    const uint64_t t = p.tile0 + blockIdx.x;
    const uint64_t dz = p.ztab ? p.ztab[blockIdx.y] : 0;  // this tree's arrays (several trees: grid.y)
    for (int k = 1; k <= p.nl; ++k) {
      const uint64_t Tk = (uint64_t)RD_TILE >> (k - 1);
      // THREADS < RD_TILE: a thread takes several parents of the first fused levels, so the upper fused
      // levels keep a larger share of the workgroup's waves busy
      for (uint32_t i = threadIdx.x; i < (Tk < (uint64_t)THREADS ? (uint32_t)THREADS : (uint32_t)Tk); i += THREADS) {
        const uint64_t j = t * Tk + i;
        const bool own = i < Tk && j >= p.a[k] && j < p.a[k] + p.c[k];
        if (own) {
            uint32_t l[8], r[8], o[8];
            const uint64_t c0 = 2 * j;
            const bool pair = c0 + 1 < p.S[k - 1];
            if (k == 1 && p.perm) {
                // children of owned parents are owned leaves (local index c0 - a[0]); the <= 2 shard-edge
                // leaves without an owned parent are gathered by the host-side plan (run_reduce)
                const uint64_t lc = c0 - p.a[0];
                uint4 *dst0 = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(p.in) + 32 * lc);
                const uint4 *s0 = reinterpret_cast<const uint4 *>(p.dig + 32 * (uint64_t)p.perm[lc]);
                const uint4 x0 = s0[0], y0 = s0[1];
                uint4 x1 = make_uint4(0, 0, 0, 0), y1 = x1;
                if (pair) {
                    const uint4 *s1 = reinterpret_cast<const uint4 *>(p.dig + 32 * (uint64_t)p.perm[lc + 1]);
                    x1 = s1[0];
                    y1 = s1[1];
                    dst0[2] = x1;
                    dst0[3] = y1;
                }
                dst0[0] = x0;
                dst0[1] = y0;
                l[0] = bswap32(x0.x); l[1] = bswap32(x0.y); l[2] = bswap32(x0.z); l[3] = bswap32(x0.w);
                l[4] = bswap32(y0.x); l[5] = bswap32(y0.y); l[6] = bswap32(y0.z); l[7] = bswap32(y0.w);
                r[0] = bswap32(x1.x); r[1] = bswap32(x1.y); r[2] = bswap32(x1.z); r[3] = bswap32(x1.w);
                r[4] = bswap32(y1.x); r[5] = bswap32(y1.y); r[6] = bswap32(y1.z); r[7] = bswap32(y1.w);
            } else if (k == 1) {
                const uint8_t *src = p.in + dz + 32 * (c0 - p.a[0]);
                load_digest(src, l);
                if (pair) load_digest(src + 32, r);
            } else {
                const uint32_t *src = buf[(k - 1) & 1] + 16 * i;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    l[q] = src[q];
                    r[q] = src[8 + q];
                }
            }
            if (pair) {
                sha_node<SHORT>(l, r, o);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = l[q];  // R5: promote unchanged
            }
            uint32_t *dst = buf[k & 1] + 8 * i;
#pragma unroll
            for (int q = 0; q < 8; ++q) dst[q] = o[q];
            store_digest(p.out[k - 1] + dz + 32 * (j - p.a[k]), o);
        }
      }
      __syncthreads();
    }
}

// ---- top of the tree: every level from a <= RD_TOP_TILES-tile level to the root in ONE launch ----
// Phase 1: each workgroup fuses up to 10 levels of its 512-parent tile in LDS (the tile's
// subtree collapses to one node after 10 levels). Phase 2: the last workgroup to finish (agent-scope
// arrival counter; it resets the counter for the next launch) reads the <= ntiles + 2 nodes the tiles
// produced and climbs the remaining levels alone, in LDS. One cross-workgroup hand-off instead of one
// kernel launch (and its drain / ramp) per 4 levels: the top of a 10M-key tree was three launches of
// ~34 us each, almost all latency (a few hundred nodes per level, 2 dependent compressions per node).

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global
// stores (__syncthreads' release fence also drains the level's HBM stores, one memory round trip per
// level on this latency-bound path).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool SHORT>
__global__ __launch_bounds__(RD_TILE) void k_reduce_top(TopPlan p) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][RD_TILE * 8];
    __shared__ uint32_t last;
    const uint64_t t = p.tile0 + blockIdx.x;
    const uint64_t dz = p.ztab ? p.ztab[blockIdx.y] : 0;  // this tree's arrays (several trees: grid.y)
    uint32_t *const arrive = p.arrive + 16 * blockIdx.y;
    const int nf = p.nf;
    for (int k = 1; k <= nf; ++k) {
        const uint64_t Tk = (uint64_t)RD_TILE >> (k - 1);
        const uint32_t i = threadIdx.x;
        const uint64_t j = t * Tk + i;
        const bool own = i < Tk && j >= p.a[k] && j < p.a[k] + p.c[k];
        if (own) {
            uint32_t l[8], r[8], o[8];
            const uint64_t c0 = 2 * j;
            const bool pair = c0 + 1 < p.S[k - 1];
            if (k == 1 && p.perm) {
                const uint64_t lc = c0 - p.a[0];
                uint4 *dst0 = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(p.in) + 32 * lc);
                const uint4 *s0 = reinterpret_cast<const uint4 *>(p.dig + 32 * (uint64_t)p.perm[lc]);
                const uint4 x0 = s0[0], y0 = s0[1];
                uint4 x1 = make_uint4(0, 0, 0, 0), y1 = x1;
                if (pair) {
                    const uint4 *s1 = reinterpret_cast<const uint4 *>(p.dig + 32 * (uint64_t)p.perm[lc + 1]);
                    x1 = s1[0];
                    y1 = s1[1];
                    dst0[2] = x1;
                    dst0[3] = y1;
                }
                dst0[0] = x0;
                dst0[1] = y0;
                l[0] = bswap32(x0.x); l[1] = bswap32(x0.y); l[2] = bswap32(x0.z); l[3] = bswap32(x0.w);
                l[4] = bswap32(y0.x); l[5] = bswap32(y0.y); l[6] = bswap32(y0.z); l[7] = bswap32(y0.w);
                r[0] = bswap32(x1.x); r[1] = bswap32(x1.y); r[2] = bswap32(x1.z); r[3] = bswap32(x1.w);
                r[4] = bswap32(y1.x); r[5] = bswap32(y1.y); r[6] = bswap32(y1.z); r[7] = bswap32(y1.w);
            } else if (k == 1) {
                const uint8_t *src = p.in + dz + 32 * (c0 - p.a[0]);
                load_digest(src, l);
                if (pair) load_digest(src + 32, r);
            } else {
                const uint32_t *src = buf[(k - 1) & 1] + 16 * i;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    l[q] = src[q];
                    r[q] = src[8 + q];
                }
            }
            if (pair) {
                sha_node<SHORT>(l, r, o);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = l[q];  // R5: promote unchanged
            }
            uint32_t *dst = buf[k & 1] + 8 * i;
#pragma unroll
            for (int q = 0; q < 8; ++q) dst[q] = o[q];
            store_digest(p.out[k - 1] + dz + 32 * (j - p.a[k]), o);
        }
        lds_barrier();
    }
    if (nf >= p.nl) return;
    // ---- hand-off: the last tile to finish climbs the rest ----
    if (p.ntiles > 1) {
        __threadfence();  // this thread's level writes, visible device-wide before the arrival
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = prev + 1 == (uint32_t)p.ntiles;
            if (last) __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!last) return;
        __threadfence();
    } else {
        // one tile: phase 2 still reads level nf back from HBM, so every thread's stores of it must have
        // landed (lds_barrier waits for LDS operations only)
        __threadfence();
        __syncthreads();
    }
    // levels nf+1 .. nl: parents [a[k], a[k] + c[k]) (<= RD_TILE: level nf holds <= ntiles <= RD_TOP_TILES
    // nodes); the first of them reads its children (level nf, written by every tile) coherently from HBM,
    // the others from LDS
    for (int k = nf + 1; k <= p.nl; ++k) {
        const uint32_t i = threadIdx.x;
        const uint64_t j = p.a[k] + i;  // owned parents [a[k], a[k] + c[k]), children owned at level k-1
        if (i < p.c[k]) {
            uint32_t l[8], r[8], o[8];
            const uint64_t c0 = 2 * j;
            const bool pair = c0 + 1 < p.S[k - 1];
            if (k == nf + 1) {
                const uint32_t *src = reinterpret_cast<const uint32_t *>(p.out[nf - 1] + dz) + 8 * (c0 - p.a[nf]);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    l[q] = bswap32(__hip_atomic_load(src + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    r[q] = pair ? bswap32(__hip_atomic_load(src + 8 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0u;
                }
            } else {
                const uint32_t *src = buf[(k - 1) & 1] + 8 * (c0 - p.a[k - 1]);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    l[q] = src[q];
                    r[q] = pair ? src[8 + q] : 0u;
                }
            }
            if (pair) {
                sha_node<SHORT>(l, r, o);
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = l[q];
            }
            uint32_t *dst = buf[k & 1] + 8 * i;
#pragma unroll
            for (int q = 0; q < 8; ++q) dst[q] = o[q];
            store_digest(p.out[k - 1] + dz + 32 * i, o);
        }
        lds_barrier();
    }
}

// ---- seam combine ----
struct SeamEntry {
    uint32_t level;
    uint32_t valid;
    uint64_t idx;
    uint8_t h[32];
};
static_assert(sizeof(SeamEntry) == 48, "seam entry layout");

constexpr int SEAM_MAX = 64;

// Device-side fringe ordering (mkv_shard_combine_device): `world` all-gathered fringe blocks (block r at
// blocks + r * stride; up to max_e entries, valid ones first, each rank's sorted by (level, index), at
// most two per level) -> one array sorted by (level, index) plus its length. Ranks hold contiguous key
// ranges ordered by rank, so inside a level rank order is index order: the position of an entry is
// (entries of lower levels) + (entries of lower ranks at its level) + (0 or 1 within its rank).
constexpr uint32_t SEAM_PREP_THREADS = 256;
constexpr uint32_t SEAM_MAX_RANKS = 64;
__global__ __launch_bounds__(SEAM_PREP_THREADS) void k_seam_prep(const uint8_t *__restrict__ blocks, uint32_t world,
                                                                 uint64_t stride, uint32_t max_e,
                                                                 SeamEntry *__restrict__ out, uint32_t *__restrict__ count) {
    __shared__ uint32_t cnt[64 * SEAM_MAX_RANKS];  // [level][rank]
    const uint32_t tid = threadIdx.x, groups = 64 * world, tot = world * max_e;
    for (uint32_t i = tid; i < groups; i += SEAM_PREP_THREADS) cnt[i] = 0;
    __syncthreads();
    for (uint32_t s = tid; s < tot; s += SEAM_PREP_THREADS) {
        const uint32_t r = s / max_e, e = s - r * max_e;
        const SeamEntry *E = reinterpret_cast<const SeamEntry *>(blocks + r * stride) + e;
        if (E->valid && E->level < 64) atomicAdd(&cnt[E->level * world + r], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // <= 64 x world groups, LDS only
        uint32_t run = 0;
        for (uint32_t i = 0; i < groups; ++i) {
            const uint32_t c = cnt[i];
            cnt[i] = run;
            run += c;
        }
        *count = run;
    }
    __syncthreads();
    for (uint32_t s = tid; s < tot; s += SEAM_PREP_THREADS) {
        const uint32_t r = s / max_e, e = s - r * max_e;
        const SeamEntry *E = reinterpret_cast<const SeamEntry *>(blocks + r * stride) + e;
        if (!E->valid || E->level >= 64) continue;
        const uint32_t within = (e > 0 && E[-1].valid && E[-1].level == E->level) ? 1u : 0u;
        out[cnt[E->level * world + r] + within] = *E;
    }
}
constexpr uint32_t SEAM_STAGE = 1024;  // fringe entries staged in LDS (8 ranks x <= 130 fit)

// One wave. Loose nodes of level l (fringes handed over by the shards + seam nodes computed from
// level l-1) are kept sorted by index in LDS; each lane hashes at most one parent per level.
__global__ __launch_bounds__(64) void k_seam_combine(const SeamEntry *__restrict__ ent, uint32_t nent,
                                                    const uint32_t *__restrict__ nent_dev,
                                                    const uint64_t *__restrict__ S, uint32_t L,
                                                    uint8_t *__restrict__ root) {
    if (nent_dev) nent = *nent_dev;  // entries prepared on the device (k_seam_prep)
    __shared__ uint64_t cidx[SEAM_MAX];
    __shared__ uint32_t ch[SEAM_MAX][8];
    __shared__ uint64_t nidx[SEAM_MAX];
    __shared__ uint32_t nh[SEAM_MAX][8];
    __shared__ uint32_t ncnt, ccnt, epos;
    // the fringe entries and level sizes, staged once: the single-lane merge below then reads LDS
    // instead of issuing dependent global loads (which dominated the combine's latency)
    __shared__ uint32_t elev[SEAM_STAGE];
    __shared__ uint64_t eidx[SEAM_STAGE];
    __shared__ uint32_t eh[SEAM_STAGE][8];
    __shared__ uint64_t sS[64];
    const uint32_t lane = threadIdx.x;
    const bool staged = nent <= SEAM_STAGE;
    if (staged) {
        for (uint32_t e = lane; e < nent; e += 64) {
            elev[e] = ent[e].level;
            eidx[e] = ent[e].idx;
            const uint8_t *h = ent[e].h;
            for (int q = 0; q < 8; ++q)
                eh[e][q] = ((uint32_t)h[4 * q] << 24) | ((uint32_t)h[4 * q + 1] << 16) | ((uint32_t)h[4 * q + 2] << 8) |
                           (uint32_t)h[4 * q + 3];
        }
    }
    for (uint32_t i = lane; i < L && i < 64; i += 64) sS[i] = S[i];
    if (lane == 0) {
        ccnt = 0;
        epos = 0;
    }
    __syncthreads();
    for (uint32_t l = 0; l < L; ++l) {
        // computed parents of level l come from cur (level l-1) -> nidx/nh (sorted by construction)
        if (lane == 0) ncnt = 0;
        __syncthreads();
        if (l > 0) {
            const uint32_t cc = ccnt;
            bool act = false;
            uint64_t x = 0;
            uint32_t lw[8], rw[8], ow[8];
            bool pair = false;
            if (lane < cc) {
                x = cidx[lane];
                if ((x & 1) == 0) {
                    act = true;
                    pair = x + 1 < sS[l - 1];
                    for (int q = 0; q < 8; ++q) lw[q] = ch[lane][q];
                    if (pair) {
                        // sibling must be the next loose node
                        for (int q = 0; q < 8; ++q) rw[q] = (lane + 1 < cc) ? ch[lane + 1][q] : 0u;
                    }
                }
            }
            const uint64_t m = __ballot(act);
            if (act) {
                if (pair) sha_node(lw, rw, ow);
                else
                    for (int q = 0; q < 8; ++q) ow[q] = lw[q];
                const uint32_t slot = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                nidx[slot] = x >> 1;
                for (int q = 0; q < 8; ++q) nh[slot][q] = ow[q];
            }
            if (lane == 0) ncnt = (uint32_t)__popcll(m);
        }
        __syncthreads();
        // merge computed (nidx) with this level's fringe entries into cur. Staged: every lane places one
        // element by its rank in the other sorted list (computed and fringe indices never coincide:
        // computed nodes are seams, fringe nodes are owned); otherwise a single-lane merge from HBM.
        if (staged) {
            const uint32_t e0 = epos;
            uint32_t e1 = e0;
            while (e1 < nent && elev[e1] == l) ++e1;  // same bound in every lane (LDS reads)
            const uint32_t na = ncnt, nb = e1 - e0;
            if (lane < na + nb) {
                uint64_t x;
                const uint32_t *src;
                uint32_t r = 0;
                if (lane < na) {
                    x = nidx[lane];
                    src = nh[lane];
                    for (uint32_t j = 0; j < nb; ++j) r += eidx[e0 + j] < x;
                    r += lane;
                } else {
                    const uint32_t j = lane - na;
                    x = eidx[e0 + j];
                    src = eh[e0 + j];
                    for (uint32_t i = 0; i < na; ++i) r += nidx[i] < x;
                    r += j;
                }
                uint32_t w[8];
                for (int q = 0; q < 8; ++q) w[q] = src[q];
                if (r < SEAM_MAX) {
                    cidx[r] = x;
                    for (int q = 0; q < 8; ++q) ch[r][q] = w[q];
                }
            }
            __syncthreads();
            if (lane == 0) {
                ccnt = na + nb < SEAM_MAX ? na + nb : SEAM_MAX;
                epos = e1;
            }
        } else if (lane == 0) {
            uint32_t a = 0, na = ncnt, e = epos, c = 0;
            while (true) {
                const bool hasE = e < nent && ent[e].level == l;
                const bool hasA = a < na;
                if (!hasE && !hasA) break;
                const uint64_t ei = hasE ? ent[e].idx : 0;
                bool takeE = hasE && (!hasA || ei < nidx[a]);
                if (c < SEAM_MAX) {
                    if (takeE) {
                        cidx[c] = ei;
                        const uint8_t *h = ent[e].h;
                        for (int q = 0; q < 8; ++q)
                            ch[c][q] = ((uint32_t)h[4 * q] << 24) | ((uint32_t)h[4 * q + 1] << 16) |
                                       ((uint32_t)h[4 * q + 2] << 8) | (uint32_t)h[4 * q + 3];
                    } else {
                        cidx[c] = nidx[a];
                        for (int q = 0; q < 8; ++q) ch[c][q] = nh[a][q];
                    }
                }
                ++c;
                if (takeE) ++e; else ++a;
            }
            ccnt = c < SEAM_MAX ? c : SEAM_MAX;
            epos = e;
        }
        __syncthreads();
    }
    if (lane == 0) {
        if (ccnt >= 1) store_digest(root, ch[0]);
    }
}

}  // namespace

void launch_reduce_fused(const FusePlan &p, hipStream_t st) {
    if (p.ntiles == 0) return;
    // Few tiles = latency-bound (each fused level waits one full node hash): the short dependency chain
    // there; many tiles = throughput-bound: fewer instructions win (profiles/r01_valu_microbench.md).
    const dim3 g((uint32_t)p.ntiles, p.nz ? p.nz : 1);
    if (p.ntiles * g.y < 256)
        hipLaunchKernelGGL((k_reduce_fused<true, RD_TILE>), g, dim3(RD_TILE), 0, st, p);
    else
        hipLaunchKernelGGL((k_reduce_fused<false, RD_TILE>), g, dim3(RD_TILE), 0, st, p);
    MKV_LAUNCH_CHECK();
}

void launch_reduce_top(const TopPlan &p, hipStream_t st) {
    if (p.ntiles == 0) return;
    // Plain rounds: one wave per SIMD is bound by its own issue rate (~4 cycles per VALU instruction), not
    // by the round's dependency chain, so the form with fewer instructions wins even here (10M build: 110
    // vs 116 us for the short-chain form).
    hipLaunchKernelGGL(k_reduce_top<false>, dim3((uint32_t)p.ntiles, p.nz ? p.nz : 1), dim3(RD_TILE), 0, st, p);
    MKV_LAUNCH_CHECK();
}

void launch_seam_combine(const uint8_t *entries, uint32_t nent, const uint64_t *level_sizes, uint32_t nlevels,
                         uint8_t *scratch, uint8_t *root_out, hipStream_t st) {
    (void)scratch;
    hipLaunchKernelGGL(k_seam_combine, dim3(1), dim3(64), 0, st, reinterpret_cast<const SeamEntry *>(entries), nent,
                       static_cast<const uint32_t *>(nullptr), level_sizes, nlevels, root_out);
    MKV_LAUNCH_CHECK();
}

void launch_seam_prep_combine(const uint8_t *blocks, uint32_t world, uint64_t stride, uint32_t max_entries,
                              const uint64_t *level_sizes, uint32_t nlevels, uint8_t *scratch, uint32_t *count,
                              uint8_t *root_out, hipStream_t st) {
    SeamEntry *sorted = reinterpret_cast<SeamEntry *>(scratch);
    hipLaunchKernelGGL(k_seam_prep, dim3(1), dim3(SEAM_PREP_THREADS), 0, st, blocks, world, stride, max_entries, sorted,
                       count);
    hipLaunchKernelGGL(k_seam_combine, dim3(1), dim3(64), 0, st, sorted, 0u, count, level_sizes, nlevels, root_out);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
