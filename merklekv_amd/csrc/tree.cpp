// tree.cpp — native runtime behind include/mkv_merkle.h: device memory, stream, build / upsert / remove /
// diff orchestration over the HIP kernels, sharded-tree seams, profiling. No CPU compute fallback: every
// digest, sort, reduction and diff runs on the GPU; the host only plans launches and moves results.
#include "mkv_merkle.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

using namespace mkv;

static thread_local std::string g_err;
void mkv::set_last_error(const char *msg) { g_err = msg; }

// Host-side phase trace of the last API call on this thread (mkv_debug_trace): labelled timestamps
// (µs since the call started) at the call's blocking points, so a slow call names where its host time
// went (a device wait, a readback, a copy) next to the device time the HIP events report.
namespace {
struct HostTrace {
    std::chrono::steady_clock::time_point t0;
    int n = 0;
    const char *label[64];
    double us[64];
    void reset() {
        n = 0;
        t0 = std::chrono::steady_clock::now();
    }
    void mark(const char *l) {
        if (n < 64) {
            label[n] = l;
            us[n++] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
    }
};
thread_local HostTrace g_trace;
}  // namespace
#define HTRACE(l) g_trace.mark(l)

namespace {

struct EvPair {
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s = nullptr;
    std::string group;
    bool closed = false;
};

}  // namespace

// Key lists live in pinned host blocks that the device writes directly (no pageable staging, no extra
// host copy); a batched diff's per-variant lists are views sharing one block. Blocks are recycled
// through a small pool because pinning tens of MB costs milliseconds. The pool is bounded: at most
// POOL_MAX_BLOCKS blocks and MKV_POOL_MAX_MB (default 1024) MiB are kept, a request never takes a
// pooled block more than 4x its size (a one-key diff must not hold a multi-GB block), and the pool is
// emptied when the last tree handle is destroyed or on mkv_pool_trim(). Allocation counters
// (mkv_pool_stats) let a caller see whether a slow call paid for page pinning.
namespace {
std::mutex g_pool_mu;
// a free pinned block; fill_klen / fill_n: its first fill_n u64 words hold k x fill_klen (the offsets of a
// fixed-length key list, written by the host once and kept while the block cycles through the pool)
struct PoolEnt {
    uint8_t *first;
    size_t second;
    uint64_t fill_klen, fill_n;
};
std::vector<PoolEnt> g_pool;  // free pinned blocks
size_t g_pool_bytes = 0;
std::atomic<uint64_t> g_pin_allocs{0}, g_pin_frees{0}, g_pin_alloc_bytes{0};
std::atomic<uint64_t> g_pin_ns{0};  // host time spent in hipHostMalloc / hipHostFree
std::atomic<int64_t> g_live_trees{0};
constexpr size_t POOL_MAX_BLOCKS = 16;

size_t pool_max_bytes() {
    static const size_t v = [] {
        const char *e = getenv("MKV_POOL_MAX_MB");
        const double mb = e ? atof(e) : 1024.0;
        return (size_t)(mb > 0 ? mb : 0) << 20;
    }();
    return v;
}

void pin_free(uint8_t *p) {
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipHostFree(p);
    g_pin_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    ++g_pin_frees;
}

void pool_trim_locked() {
    for (auto &b : g_pool) pin_free(b.first);
    g_pool.clear();
    g_pool_bytes = 0;
}

struct PinnedBlock {
    uint8_t *p = nullptr;
    uint8_t *dp = nullptr;  // the same memory as the device sees it (written by k_copy_to_host)
    size_t cap = 0;
    // words [0, fill_n) hold k x fill_klen. Kept through the pool only for an owner that asks for it
    // (keep_fill) and writes that range through fill_offsets alone; every other acquisition clears it.
    uint64_t fill_klen = 0, fill_n = 0;
    explicit PinnedBlock(size_t bytes, bool keep_fill = false) {
        {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            const size_t limit = std::max<size_t>(4 * bytes, 1 << 20);
            size_t best = SIZE_MAX;
            for (size_t i = 0; i < g_pool.size(); ++i)
                if (g_pool[i].second >= bytes && g_pool[i].second <= limit &&
                    (best == SIZE_MAX || g_pool[i].second < g_pool[best].second))
                    best = i;
            if (best != SIZE_MAX) {
                p = g_pool[best].first;
                cap = g_pool[best].second;
                if (keep_fill) {
                    fill_klen = g_pool[best].fill_klen;
                    fill_n = g_pool[best].fill_n;
                }
                g_pool_bytes -= cap;
                g_pool.erase(g_pool.begin() + (long)best);
                map_device();
                return;
            }
        }
        cap = std::max<size_t>(bytes + bytes / 4, 4096);
        const auto t0 = std::chrono::steady_clock::now();
        MKV_HIP(hipHostMalloc(reinterpret_cast<void **>(&p), cap, hipHostMallocDefault));
        map_device();
        g_pin_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        ++g_pin_allocs;
        g_pin_alloc_bytes += cap;
    }
    // words [0, n) = k x klen, writing only what an earlier fill of this memory did not leave there
    void fill_offsets(uint64_t klen, uint64_t n) {
        uint64_t *o = reinterpret_cast<uint64_t *>(p);
        const uint64_t from = fill_klen == klen ? std::min(fill_n, n) : 0;
        for (uint64_t k = from; k < n; ++k) o[k] = k * klen;
        fill_klen = klen;
        fill_n = n;
    }
    void map_device() {
        void *d = nullptr;
        MKV_HIP(hipHostGetDevicePointer(&d, p, 0));
        dp = static_cast<uint8_t *>(d);
    }
    PinnedBlock(const PinnedBlock &) = delete;
    PinnedBlock &operator=(const PinnedBlock &) = delete;
    ~PinnedBlock() {
        // A full pool keeps its largest blocks (within the byte cap): small ones left by earlier calls
        // (level views, short key lists) must not force every large diff result through
        // hipHostMalloc/hipHostFree, whose page (un)pinning costs milliseconds.
        std::lock_guard<std::mutex> lk(g_pool_mu);
        const size_t maxb = pool_max_bytes();
        if (cap > maxb || g_live_trees.load() <= 0) {
            pin_free(p);
            return;
        }
        while (!g_pool.empty() && (g_pool.size() >= POOL_MAX_BLOCKS || g_pool_bytes + cap > maxb)) {
            size_t small = 0;
            for (size_t i = 1; i < g_pool.size(); ++i)
                if (g_pool[i].second < g_pool[small].second) small = i;
            if (g_pool[small].second >= cap) {  // every pooled block is at least as large: drop this one
                pin_free(p);
                return;
            }
            g_pool_bytes -= g_pool[small].second;
            pin_free(g_pool[small].first);
            g_pool.erase(g_pool.begin() + (long)small);
        }
        g_pool.push_back({p, cap, fill_klen, fill_n});
        g_pool_bytes += cap;
    }
};
}  // namespace

// Completion of an asynchronous device -> pinned copy (a key list still in flight).
struct KeyEvent {
    hipEvent_t e = nullptr;
    KeyEvent() { MKV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
    ~KeyEvent() {
        if (e) (void)hipEventDestroy(e);
    }
    KeyEvent(const KeyEvent &) = delete;
    KeyEvent &operator=(const KeyEvent &) = delete;
};

struct mkv_keylist {
    std::shared_ptr<PinnedBlock> blk;  // null for an empty list
    const uint8_t *bytes = nullptr;
    const uint64_t *offsets = nullptr;  // n+1 entries; offsets[0] may be nonzero (a view into a shared block)
    uint64_t n = 0;
    uint64_t zero = 0;
    // set while the bytes / offsets are still being copied (the batched diff's lists): mkv_keylist_get
    // with a bytes or offsets pointer waits for it, and so does the destructor (before blk goes back to
    // the pinned pool)
    std::shared_ptr<KeyEvent> ready;
    mkv_keylist() { offsets = &zero; }
    ~mkv_keylist() {
        if (ready) (void)hipEventSynchronize(ready->e);
    }
    void wait() {
        if (ready) {
            (void)hipEventSynchronize(ready->e);
            ready.reset();
        }
    }
};

// A key list over host bytes (the sharded diff's gathered global list, comm.cpp): one pinned block holding
// offsets[0..n] (offsets[0] == 0) and the key bytes.
mkv_keylist *mkv::keylist_from_host(const uint8_t *bytes, const uint64_t *offsets, uint64_t n) {
    auto *l = new mkv_keylist();
    if (!n) return l;
    const uint64_t kpos = (8 * (n + 1) + 15) & ~uint64_t(15), nb = offsets[n];
    auto blk = std::make_shared<PinnedBlock>(kpos + nb + 16);
    std::memcpy(blk->p, offsets, 8 * (n + 1));
    if (nb) std::memcpy(blk->p + kpos, bytes, nb);
    l->blk = blk;
    l->offsets = reinterpret_cast<const uint64_t *>(blk->p);
    l->bytes = blk->p + kpos;
    l->n = n;
    return l;
}

uint64_t mkv::tree_global_n(const mkv_tree *t);  // defined after mkv_tree

// Key-set identity: two trees with the same id hold the same sorted key sequence (a clone inherits its
// source's id; every build or merge draws a fresh one; value-only updates keep it), so a diff between
// them can skip checking that divergent leaf positions hold equal keys.
static std::atomic<uint64_t> g_keyset_ids{0};
static uint64_t next_keyset() { return g_keyset_ids.fetch_add(1, std::memory_order_relaxed) + 1; }

struct mkv_tree {
    int dev = 0;
    hipStream_t st = nullptr;   // main stream: leaf hashing, digest gather, reduction, diff
    hipStream_t st2 = nullptr;  // aux stream: key ownership copy, prefix sort, ties, dedup (overlaps st)
    hipEvent_t ev_in = nullptr, ev_join = nullptr, ev_wait = nullptr;
    hipStream_t st3 = nullptr;  // build: the ragged chunks' key copy, beside the ragged hash
    hipEvent_t ev_fixed = nullptr, ev_kc = nullptr, ev_edge = nullptr;

    // ---- contents (device) ----
    uint64_t n = 0;       // local leaves
    // Keys are owned in storage (input) order: kb/koff hold nstore records (kbytes bytes); perm[i] is the
    // storage index of sorted leaf i; pfx[i] its 8-byte big-endian key prefix. Keeping input order
    // avoids a random-access gather of every key on each build.
    uint64_t nstore = 0, kbytes = 0;
    DevBuf kb, koff, perm, pfx, nodes;
    uint64_t sort_win_hint = 0;            // shared key prefix length found by the last sort (sort_unique)
    DevBuf pfx_s;                          // locate samples of pfx (every LOC_STRIDE-th), built on demand
    DevBuf hix;                            // hash index of the sorted keys (locate_index_of), built on demand
    uint64_t hix_gen = 0, hix_mask = 0;
    uint64_t pfx_gen = 1, pfx_s_gen = 0;   // pfx_s is current while pfx_s_gen == pfx_gen
    uint64_t keyset = next_keyset();       // key-set identity (see next_keyset)
    // Key-set fingerprint of the last sort (sum and xor of the sorted key prefixes, k_mark_ties): two trees
    // whose fingerprints differ hold different key sets, so a diff goes straight to the merge-join instead
    // of first trying the top-down walk (which needs equal key sets). Equal fingerprints prove nothing: the
    // walk's own key-set screen and leaf-key checks decide as before. Cleared by key-set changes.
    uint64_t kfp[2] = {0, 0};
    bool kfp_ok = false;
    uint64_t klen_fixed = 0;               // every key has this length (0: unknown / mixed): key lists skip the length scan
    std::vector<uint64_t> lev_cnt, lev_off, lev_base, lev_S;  // per level: owned count, node offset, base, global size
    bool has_root = false;
    uint8_t root[32] = {0};
    // shard state
    uint64_t goff = 0, gN = 0;
    bool sharded = false;
    bool gather_pending = false;  // sorted leaf level not yet materialised (fused into the reduce)
    bool prepared = false;  // shard_prepare done, reduce pending
    bool combine_pending = false;  // sharded tree updated in place: global root stale until shard_combine

    // ---- scratch (device) ----
    DevBuf s_kb, s_koff, s_vb, s_voff, s_dig, s_tomb;
    DevBuf s_k1, s_k2, s_v1, s_v2;
    DevBuf s_tie, s_flags, s_scan, s_pos, s_pos0, s_lens;
    DevBuf s_radix, s_misc;
    // the build sort's own histogram / control words (zero between sorts: the tie marker clears them) and
    // epoch-tagged look-back words (zeroed once when allocated, never written by anything else)
    DevBuf s_sortctl, s_lb;
    uint32_t lb_epoch = 0;
    bool sortctl_dirty = true;  // a sort started and did not reach its clearing launch
    bool kc_pending = false;    // the ragged key copy on st3 is not yet joined into st2
    DevBuf rd_arrive;  // k_reduce_top's arrival counter (zeroed once; every launch leaves it 0)
    std::vector<DiffSide> tb_sides_host;  // what tb_sides holds (the batched walk's variant sides)
    const void *tb_sides_dev = nullptr;
    uint32_t walk_fused = 0;  // jumps of the last walk done inside the one-workgroup top launch
    uint64_t hix_skip_gen = 0;  // pfx_gen + 1 of a key set whose hash index did not fit (0: none)
    // introspection of the last batched walk (mkv_tree_walk_stats): (from level, to level) per launch
    std::vector<std::pair<uint32_t, uint32_t>> walk_jumps;
    uint32_t walk_L = 0, walk_k = 0;
    DevBuf r_chunk, r_chunk2, r_kidx, r_kidx2, r_permact, r_head, r_gexcl, r_key2, r_key22;
    DevBuf s_nodes2;  // prefix-root scratch levels
    DevBuf leaf_ctr;  // dynamic chunk counter of the leaf hash
    DevBuf d_refs, d_diffscr, d_out, d_outoff;
    DevBuf a_out, a_outoff, a_lens;    // staging of the batched diff's key list (copied out asynchronously)
    std::shared_ptr<KeyEvent> a_ev;    // that copy: the next use of a_out / a_outoff waits for it
    hipEvent_t ev_a = nullptr;         // gather done on st -> copy on st3
    DevBuf td_f0, td_f1, td_cnt, td_k1, td_k2, td_v1, td_v2;
    DevBuf td_bm, td_bc;            // divergent-position bitmap (all-zero between calls) + block counts
    uint64_t tail_cap_m = 0, tail_cap_b = 0;  // one-wait top-down tail: key-list capacity (keys, bytes)
    std::shared_ptr<PinnedBlock> tail_blk;      // its staging block (reused while no result holds it)
    uint64_t td_bm_words = 0;       // words of td_bm known to be zero
    DevBuf tb_f0, tb_f1, tb_sides, tb_screen;  // batched top-down walk
    DevBuf tb_bm, tb_bc;            // its (variant, position) bitmap (all-zero between calls) + block counts
    uint64_t tb_bm_words = 0;       // words of tb_bm known to be zero
    DevBuf x_idx, x_dig, x_flag;                // anti-entropy exchange requests
    DevBuf w_scan, w_gets, w_nl1, w_nl2, w_scr, w_ks, w_kl, w_vs, w_vl, w_found, w_rank;  // wire ingestion
    DevBuf d_seam, d_S, d_fr;
    // redistribution (mkv_route_*): splitters, per-destination counts, the destination-grouped permutation
    // (the permutation lives in a route-owned buffer: the sort scratch it comes from is reused by every
    // other entry point; the plan's blobs are recorded so a pack of different records is refused)
    DevBuf rt_spl, rt_cnt, rt_pbuf;
    const uint32_t *rt_perm = nullptr;
    uint64_t rt_n = 0;
    const uint8_t *rt_kb = nullptr, *rt_vb = nullptr;
    const uint64_t *rt_koff = nullptr, *rt_voff = nullptr;
    // incremental update: batch staging, positions, dirty lists, dirty-node bitmap (all-zero between calls)
    DevBuf u_kb, u_koff, u_vb, u_voff, u_dig, u_pos, u_pos2, u_idx, u_idx2, u_cnt, u_bf, u_mbox;
    DevBuf u_ztab;        // climb -> reduction: the group's node-array offsets from t0's
    int upd_dense_from = -1;  // last dirty update: levels above this one were rehashed whole
    // batch merge (key-set changes): batch tombstones, merged prefixes / permutation / levels, count
    DevBuf u_tomb, m_pfx, m_perm, m_nodes, m_cnt;
    uint64_t bf_words = 0;  // words of u_bf known to be zero (every climb leaves them all-zero)
    // words of u_cnt known to be zero: the end-of-update readback copies the counters to h_small + UCNT_HOST
    // and zeroes them, so the next update needs no zeroing launch (one at the start of the update ran beside
    // the previous step's key-list DMA, which stretched it from ~4 to 50-240 us)
    uint64_t ucnt_zero_words = 0;
    uint64_t *h_small = nullptr;  // pinned host scalars (1 KB: bytes [512, 1024) = batched-walk counters)
    uint8_t *h_small_dev = nullptr;  // h_small as the device sees it (readbacks are kernel stores)
    uint32_t *h_counts = nullptr;  // pinned host copy of the prefix digit histograms (8 x 256)
    uint32_t *h_counts_dev = nullptr;  // h_counts as the device sees it (k_prefix_hist stores there)
    uint8_t *h_seam = nullptr;     // pinned staging of seam-combine inputs
    size_t h_seam_cap = 0;

    // ---- profiling ----
    bool prof = false;
    std::vector<EvPair> evpool;
    std::vector<size_t> evfree, evdone;
    std::map<std::string, std::pair<double, uint64_t>> pg;

    // the device pointers of the current staged build input
    const uint8_t *in_kb = nullptr;
    const uint64_t *in_koff = nullptr;
    uint64_t in_n = 0;
    const uint8_t *in_tomb = nullptr;
    bool counted = false;  // counted in g_live_trees
};

uint64_t mkv::tree_global_n(const mkv_tree *t) { return t->sharded ? t->gN : t->n; }

// Same key-set id => same sorted keys. The id is a correctness input (the batched dirty path locates a
// replica's batch in another tree, the walks skip the leaf-key check), so the cheap host-side facts that
// must agree are checked every time: a mismatch means some key-changing path kept a stale id.
// Both trees' keys all have one length: key lists need no length gather (0 otherwise).
static uint64_t pair_klen(const mkv_tree *a, const mkv_tree *b) {
    return a->klen_fixed && a->klen_fixed == b->klen_fixed ? a->klen_fixed : 0;
}

// Different key-set fingerprints (see mkv_tree::kfp): the key sets differ for certain.
static bool keysets_differ(const mkv_tree *a, const mkv_tree *b) {
    return a->kfp_ok && b->kfp_ok && (a->kfp[0] != b->kfp[0] || a->kfp[1] != b->kfp[1]);
}

static bool same_keyset(const mkv_tree *a, const mkv_tree *b) {
    if (a->keyset != b->keyset) return false;
    if (a->n != b->n || a->nstore != b->nstore || a->kbytes != b->kbytes)
        throw Error(ST_ESTATE, "internal: trees share a key-set id but hold different keys");
    return true;
}

namespace {

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d) {
        (void)hipGetLastError();  // a stale error from an unrelated earlier call must not fail this one
        (void)hipGetDevice(&prev);
        MKV_HIP(hipSetDevice(d));
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

__global__ void k_clear_tomb(const uint8_t *__restrict__ tomb, const uint32_t *__restrict__ perm, uint64_t n,
                             uint32_t *__restrict__ flags) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && tomb[perm[i]]) flags[i] = 0;
}
// Device -> pinned host copy done by a kernel on the tree's stream (16-B stores straight into the
// mapped host block) instead of hipMemcpyAsync: the runtime's D2H path occasionally held the calling
// thread for ~10 ms inside hipMemcpyAsync itself (r02 bench: diff host trace, "copies-queued").
// src and dst 16-B aligned; the tail is copied bytewise.
__global__ __launch_bounds__(256) void k_copy_to_host(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                      uint64_t bytes) {
    const uint64_t nv = bytes / 16, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t v = t; v < nv; v += stride)
        reinterpret_cast<uint4 *>(dst)[v] = reinterpret_cast<const uint4 *>(src)[v];
    if (t < bytes - nv * 16) dst[nv * 16 + t] = src[nv * 16 + t];
}
// max_blocks: a PCIe-bound copy needs few waves in flight; an asynchronous one (beside other work) keeps
// its CU footprint small.
void copy_to_host(const void *src, uint8_t *dst_dev_view, uint64_t bytes, hipStream_t st, uint64_t max_blocks = 2048) {
    if (!bytes) return;
    const uint64_t blocks = std::min<uint64_t>(ceil_div(bytes / 16 + 1, 256), max_blocks);
    hipLaunchKernelGGL(k_copy_to_host, dim3((uint32_t)blocks), dim3(256), 0, st, static_cast<const uint8_t *>(src),
                       dst_dev_view, bytes);
    MKV_LAUNCH_CHECK();
}

// Several small device -> mapped-pinned copies in one launch (one workgroup per copy, <= 32 copies of
// <= 4 KiB): the per-tree scalar readbacks of a multi-tree call.
struct SmallCopies {
    const uint8_t *src[32];
    uint8_t *dst[32];
    uint32_t bytes[32];
    uint32_t zero;  // bit c: copy c also zeroes its source (a counter array read back and reset in one launch)
};
__global__ __launch_bounds__(64) void k_copy_small_many(SmallCopies C) {
    const uint32_t c = blockIdx.x;
    const bool z = (C.zero >> c) & 1u;
    for (uint32_t b = threadIdx.x; b < C.bytes[c]; b += 64) {
        const uint8_t v = C.src[c][b];
        C.dst[c][b] = v;
        if (z) const_cast<uint8_t *>(C.src[c])[b] = 0;
    }
}
constexpr size_t UCNT_HOST = 256;  // byte offset in h_small of the last update's counters (L + 2 words)

// Zero-fill of up to 32 device ranges in one launch (grid.y = range): a multi-replica update clears
// every replica's dirty bitmap and level counters with one launch instead of one memset call each
// (each ~10 µs of host enqueue and ~5 µs of device time, serialised).
constexpr int ZERO_MAX_RANGES = 40;
struct ZeroRanges {
    uint8_t *p[ZERO_MAX_RANGES];
    uint64_t bytes[ZERO_MAX_RANGES];
};
__global__ __launch_bounds__(256) void k_zero_many(ZeroRanges Z) {
    uint8_t *p = Z.p[blockIdx.y];
    const uint64_t bytes = Z.bytes[blockIdx.y];
    const uint64_t head = std::min<uint64_t>(bytes, (16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15);
    const uint64_t nv = (bytes - head) >> 4;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    uint4 *v = reinterpret_cast<uint4 *>(p + head);
    for (uint64_t i = t; i < nv; i += stride) v[i] = make_uint4(0, 0, 0, 0);
    if (t < head) p[t] = 0;
    const uint64_t tail = head + (nv << 4);
    if (t < bytes - tail) p[tail + t] = 0;
}
static void launch_zero_many(const ZeroRanges &Z, uint32_t nz, hipStream_t st) {
    if (!nz) return;
    uint64_t mx = 0;
    for (uint32_t i = 0; i < nz; ++i) mx = std::max(mx, Z.bytes[i]);
    const uint32_t bx = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ceil_div(mx, 16 * 256 * 4), 1), 1024);
    hipLaunchKernelGGL(k_zero_many, dim3(bx, nz), dim3(256), 0, st, Z);
    MKV_LAUNCH_CHECK();
}

// Scalar readback into the tree's pinned scratch (h_small), as a kernel store on stream st.
void small_d2h(mkv_tree *t, const void *h_dst, const void *src, uint64_t bytes, hipStream_t st) {
    const uint64_t off = static_cast<const uint8_t *>(h_dst) - reinterpret_cast<const uint8_t *>(t->h_small);
    copy_to_host(src, t->h_small_dev + off, bytes, st);
}

// Fringe entry i (48 B: level, valid, idx, digest) gets the digest of node nodes[idx[i]] at byte 16.
__global__ void k_fringe_digests(const uint8_t *__restrict__ nodes, const uint32_t *__restrict__ idx, uint32_t k,
                                 uint8_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * k) {  // two 16-B halves per entry
        const uint4 *src = reinterpret_cast<const uint4 *>(nodes + 32ull * idx[i >> 1]) + (i & 1);
        *reinterpret_cast<uint4 *>(out + 48ull * (i >> 1) + 16 + 16 * (i & 1)) = *src;
    }
}
void launch_fringe_digests(const uint8_t *nodes, const uint32_t *idx, uint32_t k, uint8_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_fringe_digests, dim3((2 * k + 255) / 256), dim3(256), 0, st, nodes, idx, k, out);
    MKV_LAUNCH_CHECK();
}
__global__ void k_widen_positions(const uint32_t *__restrict__ f, uint64_t m, uint64_t *__restrict__ k,
                                  uint32_t *__restrict__ v) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        k[i] = f[i];
        v[i] = (uint32_t)i;
    }
}
// Divergent leaf positions in ascending order without a sort (top-down diff): one bit per leaf in a
// bitmap that is all-zero between calls; per-block popcounts over POS_BLOCK_WORDS words; each emitting
// block finds its output base by summing the counts of the blocks before it (at most a few thousand
// u32, L2-resident), scans its own words and writes the positions, clearing the words it read.
// Round 6: 16 consecutive words per thread (4 uint4 loads in flight; 4x fewer blocks for the base sums):
// 100M value-only diff 0.151 -> 0.149 ms device (interleaved A/B)
constexpr uint32_t POS_TW = 16;                         // words per thread
constexpr uint32_t POS_BLOCK_WORDS = 256 * POS_TW;
constexpr uint64_t POS_MAX_BLOCKS = 8192;   // beyond this the O(blocks^2) base sums lose to the sort

__global__ void k_pos_setbits(const uint32_t *__restrict__ f, uint64_t m, uint32_t *__restrict__ bm) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        const uint32_t p = f[i];
        atomicOr(bm + (p >> 5), 1u << (p & 31));
    }
}

__global__ void k_pos_setbits_dev(const uint32_t *__restrict__ f, const uint32_t *__restrict__ mdev,
                                  uint32_t *__restrict__ bm) {
    const uint64_t m = *mdev;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = f[i];
        atomicOr(bm + (p >> 5), 1u << (p & 31));
    }
}

__device__ __forceinline__ uint4 pos_words(const uint32_t *bm, uint64_t w0, uint64_t words) {
    if (w0 + 3 < words) return *reinterpret_cast<const uint4 *>(bm + w0);
    uint4 x = make_uint4(0, 0, 0, 0);
    if (w0 < words) x.x = bm[w0];
    if (w0 + 1 < words) x.y = bm[w0 + 1];
    if (w0 + 2 < words) x.z = bm[w0 + 2];
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__device__ __forceinline__ uint32_t pos_load(const uint32_t *bm, uint64_t w0, uint64_t words, uint32_t x[POS_TW]) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < POS_TW / 4; ++j) {
        const uint4 v = pos_words(bm, w0 + 4 * j, words);
        x[4 * j] = v.x, x[4 * j + 1] = v.y, x[4 * j + 2] = v.z, x[4 * j + 3] = v.w;
        c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
    }
    return c;
}

__global__ __launch_bounds__(256) void k_pos_count(const uint32_t *__restrict__ bm, uint64_t words,
                                                   uint32_t *__restrict__ bc) {
    __shared__ uint32_t red[4];
    const uint64_t w0 = (uint64_t)blockIdx.x * POS_BLOCK_WORDS + POS_TW * threadIdx.x;
    uint32_t x[POS_TW];
    const uint32_t c = wave_sum(pos_load(bm, w0, words, x));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_pos_emit(uint32_t *__restrict__ bm, uint64_t words,
                                                  const uint32_t *__restrict__ bc, uint64_t *__restrict__ out) {
    __shared__ uint32_t base_w[4], tot_w[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += 256) s += bc[i];
    s = wave_sum(s);
    const uint64_t w0 = (uint64_t)blockIdx.x * POS_BLOCK_WORDS + POS_TW * threadIdx.x;
    uint32_t x[POS_TW];
    const uint32_t c = pos_load(bm, w0, words, x);
    uint32_t v = c;  // inclusive scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d);
        if (lane >= (uint32_t)d) v += y;
    }
    if (lane == 0) base_w[wave] = s;
    if (lane == 63) tot_w[wave] = v;
    __syncthreads();
    uint64_t o = (uint64_t)base_w[0] + base_w[1] + base_w[2] + base_w[3] + (v - c);
    for (uint32_t w = 0; w < wave; ++w) o += tot_w[w];
    if (!c) return;
#pragma unroll
    for (uint32_t q = 0; q < POS_TW; ++q) {
        uint32_t b = x[q];
        while (b) {
            out[o++] = (w0 + q) * 32 + (uint32_t)(__ffs(b) - 1);
            b &= b - 1;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < POS_TW / 4; ++j) {
        const uint64_t wj = w0 + 4 * j;
        if (wj + 3 < words) {
            *reinterpret_cast<uint4 *>(bm + wj) = make_uint4(0, 0, 0, 0);
        } else {
            for (int q = 0; q < 4; ++q)
                if (wj + q < words) bm[wj + q] = 0;
        }
    }
}

// m unique positions < n (u32 frontier) -> ascending u64 in `out`. bm: ceil(n/32) zero words
// (left zero); bc: one u32 per block. False when n is too large for this path (caller sorts).
bool positions_sorted_bitmap(const uint32_t *f, uint64_t m, uint64_t n, uint32_t *bm, uint32_t *bc, uint64_t *out,
                             hipStream_t st) {
    const uint64_t words = (n + 31) / 32, nb = ceil_div(words, POS_BLOCK_WORDS);
    if (nb > POS_MAX_BLOCKS) return false;
    if (!m) return true;
    hipLaunchKernelGGL(k_pos_setbits, dim3((uint32_t)ceil_div(m, 256)), dim3(256), 0, st, f, m, bm);
    hipLaunchKernelGGL(k_pos_count, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc);
    hipLaunchKernelGGL(k_pos_emit, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc, out);
    MKV_LAUNCH_CHECK();
    return true;
}

// The same from a device count (*mdev entries of f), positions into out (room for every position < n).
bool positions_sorted_bitmap_dev(const uint32_t *f, const uint32_t *mdev, uint64_t n, uint32_t *bm, uint32_t *bc,
                                 uint64_t *out, hipStream_t st, bool bits_set) {
    const uint64_t words = (n + 31) / 32, nb = ceil_div(words, POS_BLOCK_WORDS);
    if (nb > POS_MAX_BLOCKS) return false;
    if (!bits_set) hipLaunchKernelGGL(k_pos_setbits_dev, dim3(1024), dim3(256), 0, st, f, mdev, bm);
    hipLaunchKernelGGL(k_pos_count, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc);
    hipLaunchKernelGGL(k_pos_emit, dim3((uint32_t)nb), dim3(256), 0, st, bm, words, bc, out);
    MKV_LAUNCH_CHECK();
    return true;
}

__global__ void k_narrow_u64(const uint64_t *__restrict__ k, uint64_t m, uint32_t *__restrict__ f) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) f[i] = (uint32_t)k[i];
}
void launch_narrow_u64(const uint64_t *k, uint64_t m, uint32_t *f, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_narrow_u64, dim3((uint32_t)ceil_div(m, 256)), dim3(256), 0, st, k, m, f);
    MKV_LAUNCH_CHECK();
}
void launch_widen_positions(const uint32_t *f, uint64_t m, uint64_t *k, uint32_t *v, hipStream_t st) {
    if (!m) return;
    hipLaunchKernelGGL(k_widen_positions, dim3((uint32_t)ceil_div(m, 256)), dim3(256), 0, st, f, m, k, v);
    MKV_LAUNCH_CHECK();
}

void launch_clear_tomb(const uint8_t *tomb, const uint32_t *perm, uint64_t n, uint32_t *flags, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_clear_tomb, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, tomb, perm, n, flags);
    MKV_LAUNCH_CHECK();
}

size_t prof_begin(mkv_tree *t, const char *group, hipStream_t s = nullptr) {
    if (!t->prof) return SIZE_MAX;
    if (!s) s = t->st;
    if (t->evfree.empty()) {
        EvPair p;
        MKV_HIP(hipEventCreate(&p.a));
        MKV_HIP(hipEventCreate(&p.b));
        t->evpool.push_back(p);
        t->evfree.push_back(t->evpool.size() - 1);
    }
    size_t i = t->evfree.back();
    t->evfree.pop_back();
    t->evpool[i].group = group;
    t->evpool[i].closed = false;
    t->evpool[i].s = s;
    MKV_HIP(hipEventRecord(t->evpool[i].a, s));
    return i;
}
void prof_end(mkv_tree *t, size_t i) {
    if (i == SIZE_MAX) return;
    MKV_HIP(hipEventRecord(t->evpool[i].b, t->evpool[i].s));
    t->evpool[i].closed = true;
    t->evdone.push_back(i);
}
// after a stream sync: accumulate every closed pair (open ones stay pending)
void prof_collect(mkv_tree *t) {
    for (size_t i : t->evdone) {
        float ms = 0;
        MKV_HIP(hipEventElapsedTime(&ms, t->evpool[i].a, t->evpool[i].b));
        auto &g = t->pg[t->evpool[i].group];
        g.first += ms;
        g.second += 1;
        t->evfree.push_back(i);
    }
    t->evdone.clear();
}

// Low-latency wait: poll the stream instead of the runtime's blocking sync (tens of microseconds of
// wake-up latency per scalar readback otherwise). hipStreamQuery queues no marker, so an idle stream
// returns at once. The spin is bounded: after MKV_SPIN_US (default 200 µs) the thread yields, after
// 20 ms it sleeps in 50-µs steps (a long kernel does not pin a host core, nor a tokio blocking-pool
// thread), and after MKV_WAIT_TIMEOUT_S (default 120 s) the call fails with MKV_EHIP instead of
// waiting forever on a hung device.
static double wait_timeout_s() {
    static const double v = [] {
        const char *e = getenv("MKV_WAIT_TIMEOUT_S");
        const double x = e ? atof(e) : 120.0;
        return x > 0 ? x : 120.0;
    }();
    return v;
}
static double spin_us() {
    static const double v = [] {
        const char *e = getenv("MKV_SPIN_US");
        return e ? atof(e) : 200.0;
    }();
    return v;
}
void wait_idle(hipStream_t s) {
    hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    struct Mark {
        ~Mark() { HTRACE("wait-done"); }
    } mark_on_exit;
    if (e != hipErrorNotReady) MKV_HIP(e);
    const auto t0 = std::chrono::steady_clock::now();
    const double spin = spin_us(), limit = wait_timeout_s() * 1e6;
    for (uint64_t it = 0;; ++it) {
        e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) MKV_HIP(e);
        if ((it & 15) != 15) continue;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (us < spin) continue;
        if (us > limit)
            throw Error(ST_EHIP, "device wait timed out after " + std::to_string((int)(us / 1e6)) +
                                     " s (hung kernel?); raise MKV_WAIT_TIMEOUT_S for longer work");
        if (us < spin + 20000) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
void wait_stream(mkv_tree *t, hipStream_t s) {
    (void)t;
    wait_idle(s);
}

// Full completion point of an API call: both streams drained, profiling pairs collected.
void sync(mkv_tree *t) {
    wait_stream(t, t->st2);
    wait_stream(t, t->st);
    if (t->st3) wait_stream(t, t->st3);  // an asynchronous key-list copy (or the ragged key copy) of this tree
    prof_collect(t);
}

void swap_buf(DevBuf &a, DevBuf &b) {
    std::swap(a.p, b.p);
    std::swap(a.cap, b.cap);
}

template <class T> T *ens(DevBuf &b, uint64_t count) { return reinterpret_cast<T *>(b.ensure(count * sizeof(T))); }

// Scalar readback that waits only for the stream that produced it (the other stream keeps running).
uint64_t d2h_u64(mkv_tree *t, const void *dptr, hipStream_t s = nullptr) {
    if (!s) s = t->st;
    small_d2h(t, t->h_small, dptr, sizeof(uint64_t), s);
    wait_stream(t, s);
    return t->h_small[0];
}
uint32_t d2h_u32(mkv_tree *t, const void *dptr, hipStream_t s = nullptr) {
    if (!s) s = t->st;
    small_d2h(t, t->h_small, dptr, sizeof(uint32_t), s);
    wait_stream(t, s);
    return reinterpret_cast<uint32_t *>(t->h_small)[0];
}

// `words` u32 starting at dptr in one round trip (h_small holds 64); the walk reads its level counters
// and the key-set screen together this way instead of one wake-up per scalar.
const uint32_t *d2h_u32s(mkv_tree *t, const void *dptr, uint32_t words, hipStream_t s = nullptr) {
    if (!s) s = t->st;
    if (words > 64) throw std::runtime_error("d2h_u32s: more than 64 words");
    small_d2h(t, t->h_small, dptr, 4ull * words, s);
    wait_stream(t, s);
    return reinterpret_cast<const uint32_t *>(t->h_small);
}

int bits_for(uint64_t m) {
    int b = 0;
    while (b < 64 && (m >> b)) ++b;
    return b;
}

// ---------------------------------------------------------------------------------------------
// Level plan (R5 ownership): level k owns global nodes [a_k, a_k + c_k) of a level with S_k nodes.
// ---------------------------------------------------------------------------------------------
void plan_levels(mkv_tree *t, uint64_t o, uint64_t n, uint64_t N) {
    t->lev_cnt.clear();
    t->lev_off.clear();
    t->lev_base.clear();
    t->lev_S.clear();
    if (N == 0) return;
    uint64_t a = o, e = o + n, S = N, off = 0;
    while (true) {
        uint64_t c = e > a ? e - a : 0;
        t->lev_base.push_back(a);
        t->lev_cnt.push_back(c);
        t->lev_off.push_back(off);
        t->lev_S.push_back(S);
        off = (off + c + 3) & ~uint64_t(3);  // every level 128-B aligned: a 2- or 4-child group is whole lines
        if (S == 1) break;
        uint64_t a2 = (a + 1) / 2;
        uint64_t e2 = (e == S) ? (e + 1) / 2 : e / 2;
        a = a2;
        e = e2;
        S = (S + 1) / 2;
    }
}

// Node slots the level plan spans (levels start 128-B aligned, so a few pad slots between them).
uint64_t total_nodes(const mkv_tree *t) {
    return t->lev_off.empty() ? 0 : t->lev_off.back() + t->lev_cnt.back();
}
// Node slots to allocate for an unsharded tree of n leaves: 2n - 1 nodes + up to 3 pad slots per level.
static uint64_t node_slots(uint64_t n) { return 2 * n + 4 * MKV_MAXLEV + 66; }

// gperm/gdig: fuse the sorted-leaf gather (nodes[c] = dig[perm[c]]) into the first launch. Leaves whose
// parent is not owned (at most the first and the last of a shard) are gathered directly; a plan without
// an owned level-1 node (single leaf, or a one-leaf shard) gathers everything directly.
// l0 > 0: the levels above l0 only (level l0 is complete in nodes). ztab/nz: nz trees of t's level plan in
// one launch per step, tree z's node array at nodes + ztab[z] (device table; the dirty update's rehash
// above the climb).
void run_reduce(mkv_tree *t, uint8_t *nodes, const uint32_t *gperm = nullptr, const uint8_t *gdig = nullptr,
                size_t l0 = 0, const uint64_t *ztab = nullptr, uint32_t nz = 1, uint64_t top_tiles = RD_TOP_TILES) {
    const size_t L = t->lev_S.size();
    if (l0 > 0) gperm = nullptr;
    if (gperm) {
        if (L < 2 || t->lev_cnt[1] == 0) {
            launch_gather_digests(gperm, gdig, L ? t->lev_cnt[0] : 0, nodes, t->st);
            gperm = nullptr;
        } else {
            const uint64_t a0 = t->lev_base[0], c0 = t->lev_cnt[0], a1 = t->lev_base[1], c1 = t->lev_cnt[1];
            auto owned_parent = [&](uint64_t x) { return x / 2 >= a1 && x / 2 < a1 + c1; };
            if (!owned_parent(a0)) launch_gather_digests(gperm, gdig, 1, nodes, t->st);
            if (c0 > 1 && !owned_parent(a0 + c0 - 1))
                launch_gather_digests(gperm + (c0 - 1), gdig, 1, nodes + 32 * (c0 - 1), t->st);
        }
    }
    size_t l = l0;
    while (l + 1 < L && t->lev_cnt[l] > 0) {
        if (t->lev_cnt[l + 1] == 0) break;
        const uint64_t a1 = t->lev_base[l + 1], c1 = t->lev_cnt[l + 1];
        const uint64_t t0 = a1 / 512, t1 = (a1 + c1 - 1) / 512;
        const uint64_t ntiles = t1 - t0 + 1;
        const size_t remaining = L - 1 - l;
        // the latency-bound top: every remaining level in one launch (k_reduce_top). Only the levels
        // with owned nodes (a shard stops at its last owned level; the seam combine does the rest).
        size_t nown = 0;
        while (nown < remaining && t->lev_cnt[l + 1 + nown] > 0) ++nown;
        if (ntiles <= top_tiles && nown <= (size_t)TOP_MAX_LEVELS) {
            // one counter line per tree; every counter is 0 between launches, so zeroed on (re)allocation
            const bool fresh = t->rd_arrive.p == nullptr || t->rd_arrive.cap < 64ull * nz;
            uint32_t *arrive = ens<uint32_t>(t->rd_arrive, 16ull * nz);
            if (fresh) MKV_HIP(hipMemsetAsync(arrive, 0, t->rd_arrive.cap, t->st));
            TopPlan p{};
            p.ztab = ztab;
            p.nz = nz;
            p.in = nodes + 32 * t->lev_off[l];
            p.a[0] = t->lev_base[l];
            p.c[0] = t->lev_cnt[l];
            p.S[0] = t->lev_S[l];
            for (size_t k = 1; k <= nown; ++k) {
                p.out[k - 1] = nodes + 32 * t->lev_off[l + k];
                p.a[k] = t->lev_base[l + k];
                p.c[k] = t->lev_cnt[l + k];
                p.S[k] = t->lev_S[l + k];
            }
            p.nl = (int)nown;
            p.nf = (int)std::min<size_t>(nown, 10);
            p.tile0 = t0;
            p.ntiles = ntiles;
            if (l == 0 && gperm) {
                p.perm = gperm;
                p.dig = gdig;
            }
            p.arrive = arrive;
            launch_reduce_top(p, t->st);
            return;
        }
        const size_t nl = std::min<size_t>(remaining, ntiles == 1 ? MAX_FUSE : 4);
        FusePlan p{};
        p.ztab = ztab;
        p.nz = nz;
        p.in = nodes + 32 * t->lev_off[l];
        p.a[0] = t->lev_base[l];
        p.c[0] = t->lev_cnt[l];
        p.S[0] = t->lev_S[l];
        for (size_t k = 1; k <= nl; ++k) {
            p.out[k - 1] = nodes + 32 * t->lev_off[l + k];
            p.a[k] = t->lev_base[l + k];
            p.c[k] = t->lev_cnt[l + k];
            p.S[k] = t->lev_S[l + k];
        }
        p.nl = (int)nl;
        p.tile0 = t0;
        p.ntiles = ntiles;
        if (l == 0 && gperm) {
            p.perm = gperm;
            p.dig = gdig;
        }
        launch_reduce_fused(p, t->st);
        l += nl;
    }
}

// ---------------------------------------------------------------------------------------------
// Tie refinement (R3 on full keys): see k_sort.hip header. perm: sorted order (u32 input indices),
// tie[i] = position i equals position i-1 on everything compared so far.
// ---------------------------------------------------------------------------------------------
// start_depth 0: the sort covered only the top bits of chunk 0 (ties were marked on those bits), so
// chunk 0 is compared again and the re-ordered positions' prefixes are rewritten into pfx afterwards.
void refine_ties(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, uint64_t n, uint32_t *perm, uint8_t *tie,
                 uint32_t start_depth, uint64_t *pfx) {
    hipStream_t st = t->st2;
    uint32_t *flags = ens<uint32_t>(t->s_flags, n + 1);
    uint32_t *scan = ens<uint32_t>(t->s_scan, n + 1);
    uint32_t *pos = ens<uint32_t>(t->s_pos, n + 1);
    uint32_t *misc = ens<uint32_t>(t->s_misc, 64);
    void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n), scan_scratch_bytes(n)));

    auto active = [&]() -> uint64_t {
        launch_active_flags(tie, n, flags, st);
        exclusive_scan_u32(flags, scan, n, misc, radix, st);
        launch_compact_positions(flags, scan, n, pos, st);
        return d2h_u32(t, misc, st);
    };
    uint64_t m = active();
    if (m == 0) return;
    const uint64_t m0 = m;
    uint32_t *pos0 = nullptr;
    if (start_depth == 0 && pfx) {  // keep the initial tie-run positions for the prefix rewrite
        pos0 = ens<uint32_t>(t->s_pos0, m0 + 1);
        MKV_HIP(hipMemcpyAsync(pos0, pos, m0 * 4, hipMemcpyDeviceToDevice, st));
    }
    MKV_HIP(hipMemsetAsync(misc + 1, 0, 4, st));
    launch_max_keylen(pos, m, perm, koff, misc + 1, st);
    const uint32_t maxlen = d2h_u32(t, misc + 1, st);
    const uint32_t D = (maxlen + 7) / 8;  // chunks

    for (uint32_t depth = start_depth;; ++depth) {
        const int use_len = depth >= D;
        if (depth > start_depth) {
            m = active();
            if (m == 0) break;
        }
        uint64_t *chunk = ens<uint64_t>(t->r_chunk, 2 * m);
        uint64_t *chunk2 = ens<uint64_t>(t->r_chunk2, m);
        uint32_t *kidx = ens<uint32_t>(t->r_kidx, m);
        uint32_t *kidx2 = ens<uint32_t>(t->r_kidx2, m);
        uint32_t *permact = ens<uint32_t>(t->r_permact, m);
        uint32_t *head = ens<uint32_t>(t->r_head, m);
        uint32_t *gexcl = ens<uint32_t>(t->r_gexcl, m);
        uint64_t *key2 = ens<uint64_t>(t->r_key2, m);
        uint64_t *key22 = ens<uint64_t>(t->r_key22, m);
        launch_refine_keys(pos, m, perm, tie, kb, koff, depth, use_len, chunk, kidx, permact, head, st);
        exclusive_scan_u32(head, gexcl, m, nullptr, radix, st);
        // 1) stable sort by this round's chunk
        const int cbits = use_len ? 64 : 64;
        bool sw = radix_sort_pairs(chunk, kidx, chunk2, kidx2, m, 0, cbits, radix, st);
        uint32_t *kk = sw ? kidx2 : kidx;
        uint32_t *kk_alt = sw ? kidx : kidx2;
        // 2) stable sort by group id (restores group blocks in position order)
        launch_gid_keys(kk, gexcl, head, m, key2, st);
        bool sw2 = radix_sort_pairs(key2, kk, key22, kk_alt, m, 0, std::max(8, bits_for(m)), radix, st);
        uint32_t *kks = sw2 ? kk_alt : kk;
        MKV_HIP(hipMemsetAsync(misc + 2, 0, 4, st));
        launch_refine_apply(pos, m, kks, permact, chunk + m, perm, tie, misc + 2, st);
        const uint32_t left = d2h_u32(t, misc + 2, st);
        if (left == 0 || use_len) break;
    }
    if (pos0) launch_fix_pfx(pos0, m0, perm, kb, koff, pfx, st);
}

// Digits of the 8-byte prefix worth a radix pass, from the one-read histograms (counts[p*256+d],
// p = 0 least significant). Going down from the most significant byte, digits are added until the
// summed marginal entropies exceed log2(n) + 6 bits: below that, keys sharing every sorted digit are
// rare (~n/64 for independent bytes) and the tie refinement orders them on the full key. Constant
// digits carry no order and are skipped. (Round 2: with the block-aggregated tie marker a tie costs
// next to nothing, so 10M base64 keys take 5 passes and ~46K ties instead of 6 passes and ~730 ties:
// ordering stage 1.10 -> 1.00 ms beside the leaf hash.) Returns the digit mask; *lo_bit = lowest sorted bit.
uint32_t choose_prefix_digits(const uint32_t *counts, uint64_t n, int *lo_bit) {
    // margin bits beyond log2(n): fewer radix passes vs more prefix ties for the refinement (6: 5 passes
    // + ~46K ties at 10M base64 keys beat 6 passes + ~730 ties; 3 / 0 and 11 / 14 measured slower)
    constexpr double margin = 6.0;
    const double need = std::log2((double)(n > 1 ? n : 2)) + margin;
    double cum = 0;
    int p0 = 0;
    uint32_t mask = 0;
    for (int p = 7; p >= 0; --p) {
        double h = 0;
        uint32_t mx = 0;
        for (int d = 0; d < 256; ++d) {
            const uint32_t c = counts[p * 256 + d];
            mx = std::max(mx, c);
            if (c) {
                const double f = (double)c / (double)n;
                h -= f * std::log2(f);
            }
        }
        if (mx < n) mask |= 1u << p;
        cum += h;
        p0 = p;
        if (cum >= need) break;
    }
    *lo_bit = 8 * p0;
    return mask;
}

// ---------------------------------------------------------------------------------------------
// Core build over staged input records: keys (kb/koff, n_in), digests (s_dig, n_in), optional tombstones.
// Produces sorted unique keys (last write wins), leaf level, and the level plan for [o, o+n) of N
// (N == UINT64_MAX: unsharded, N = n).
// ---------------------------------------------------------------------------------------------
// Sorted unique view (R3 order, last write wins) of n_in records on the aux stream: returns the scratch
// buffers holding the sorted 8-byte prefixes and storage indices. drop_tomb: tombstoned records (after
// dedup) are dropped; otherwise they stay, flagged by tomb[storage index].
struct SortedSet {
    DevBuf *pk, *pm;
    uint64_t n;
    uint64_t fp[2];  // key-set fingerprint (sum, xor of the sort keys); valid when fp_ok
    bool fp_ok;
    uint64_t klen;   // every key has this length (0: lengths differ, or no keys)
};
// kbytes_out (optional): koff[n_in], read back with the sort's own counts (one host round trip).
SortedSet sort_unique(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, uint64_t n_in, const uint8_t *tomb,
                      bool drop_tomb, uint64_t *kbytes_out = nullptr) {
    hipStream_t st = t->st2;
    uint64_t *k1 = ens<uint64_t>(t->s_k1, n_in + 1);
    uint64_t *k2 = ens<uint64_t>(t->s_k2, n_in + 1);
    uint32_t *v1 = ens<uint32_t>(t->s_v1, n_in + 1);
    uint32_t *v2 = ens<uint32_t>(t->s_v2, n_in + 1);
    uint8_t *tie = ens<uint8_t>(t->s_tie, n_in + 2);
    uint32_t *misc = ens<uint32_t>(t->s_misc, 64);
    void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n_in), scan_scratch_bytes(n_in + 1)));
    // histogram / control words and look-back words of this sort: dedicated, so no zero-fill launches on
    // the ordering stream (each one queued behind the co-running leaf hash for tens of microseconds)
    const uint64_t lbw = radix_prefix_lookback_words(n_in);
    if (!t->s_lb.p || t->s_lb.cap < lbw * 8) {
        t->s_lb.ensure(lbw * 8);
        MKV_HIP(hipMemsetAsync(t->s_lb.p, 0, t->s_lb.cap, st));
        t->lb_epoch = 0;
    }
    if (!t->s_sortctl.p) t->s_sortctl.ensure(SORT_CTL_WORDS * 4);
    uint32_t *sctl = t->s_sortctl.as<uint32_t>();
    const bool ctl_zero = !t->sortctl_dirty;
    t->sortctl_dirty = true;

    size_t ps = prof_begin(t, "sort", st);
    // one read of the keys: 8-byte windows + all eight digit histograms (the indices come from pass 1),
    // plus the prefix every key shares. The window starts at the shared length the previous sort of this
    // handle found (sort_win_hint; repeated builds of one key space share it), so the second histogram
    // pass below only runs when the hint is off. The pass zeroes the tie marker's two counters; one small
    // kernel copies its words into mapped pinned memory.
    const uint64_t hint = n_in > 1 ? t->sort_win_hint : 0;
    launch_prefix_hist(kb, koff, n_in, k1, sctl, st, hint, true, ctl_zero, misc);
    if (n_in > 1) copy_to_host(sctl, reinterpret_cast<uint8_t *>(t->h_counts_dev), SORT_CTL_WORDS * 4, st);
    int lo_bit = 0;
    uint32_t digits = 0xFF;
    uint64_t win = hint;    // byte offset of the sort window
    uint64_t shared8 = 0;   // the first min(win, 8) bytes every key shares, big-endian at the top
    uint64_t klen_all = 0;  // every key has this length (from the histogram pass), else 0
    if (n_in > 1) {
        wait_stream(t, st);
        // Bytes every key shares carry no order: move the window past them ("tenant/0001/object/..."
        // keys would otherwise tie on the whole prefix and leave all n keys to the chunk-by-chunk
        // refinement). One more histogram pass when the shared length the first pass measured is not
        // the window it used.
        const uint64_t maxlen = t->h_counts[PH_MAXLEN_WORD];
        klen_all = n_in && (uint32_t)~t->h_counts[PH_NMINLEN_WORD] == maxlen ? maxlen : 0;
        const uint64_t lcp = (uint32_t)~t->h_counts[PH_NLCP_WORD];
        const uint64_t k0w = ((uint64_t)t->h_counts[PH_K0_WORD] << 32) | t->h_counts[PH_K0_WORD + 1];
        const uint64_t want = lcp > 0 && lcp < maxlen ? lcp : 0;
        if (want != hint) {
            win = want;
            launch_prefix_hist(kb, koff, n_in, k1, sctl, st, win, false, false);
            copy_to_host(sctl, reinterpret_cast<uint8_t *>(t->h_counts_dev), SORT_CTL_WORDS * 4, st);
            wait_stream(t, st);
        }
        shared8 = win == 0 ? 0 : win >= 8 ? k0w : k0w & (~0ull << (64 - 8 * win));
        t->sort_win_hint = win;
        digits = choose_prefix_digits(t->h_counts, n_in, &lo_bit);
    }
    const bool sw = radix_prefix_passes(k1, v1, k2, v2, n_in, digits, sctl, t->s_lb.as<uint64_t>(), &t->lb_epoch, st, true);
    DevBuf *pkbuf = sw ? &t->s_k2 : &t->s_k1, *pkalt = sw ? &t->s_k1 : &t->s_k2;
    DevBuf *pmbuf = sw ? &t->s_v2 : &t->s_v1, *pmalt = sw ? &t->s_v1 : &t->s_v2;
    uint64_t *pk = pkbuf->as<uint64_t>();
    uint32_t *perm = pmbuf->as<uint32_t>();
    // run heads into the dedup flag scratch (free until the dedup below), their count in misc[1]
    uint32_t *heads = ens<uint32_t>(t->s_flags, n_in + 1);
    launch_mark_ties(pk, n_in, tie, misc, heads, st, lo_bit, sctl, SORT_CTL_WORDS);  // clears sctl for the next sort
    t->sortctl_dirty = false;
    // Short tie runs are ordered in place right behind the tie marker (the kernel reads the head count on
    // the device, so no host round trip in between); ONE readback then brings the tie, duplicate and
    // long-run counts (misc[0], [4], [5]) and, for borrowed inputs, the key-byte total.
    if (n_in > 1) launch_refine_small(kb, koff, n_in, perm, pk, tie, misc + 4, heads, misc + 1, n_in / 2 + 1, st);
    prof_end(t, ps);
    small_d2h(t, t->h_small, misc, 48, st);
    if (kbytes_out && n_in) small_d2h(t, t->h_small + 6, koff + n_in, 8, st);
    wait_stream(t, st);
    const uint32_t *hm = reinterpret_cast<const uint32_t *>(t->h_small);
    const uint32_t nties = n_in ? hm[0] : 0, dups = hm[4], long_runs = hm[5];
    // key-set fingerprint of the sorted keys (k_mark_ties); meaningful only without duplicates (it counts
    // every input record) and with the key window the sort chose mixed in
    const uint64_t fp0 = t->h_small[4] ^ (win * 0x9E3779B97F4A7C15ull), fp1 = t->h_small[5];
    if (n_in > 1 && hm[7])  // a radix pass's look-back stalled past its spin limit: the order is not trustworthy
        throw Error(ST_EHIP, "sort: a radix pass's look-back exceeded its spin limit (device stalled)");
    if (kbytes_out) *kbytes_out = n_in ? t->h_small[6] : 0;
    static const bool dbg_sort = getenv("MKV_DEBUG_SORT") != nullptr;
    if (dbg_sort)
        fprintf(stderr, "[mkv sort] n=%llu win=%llu lo_bit=%d digits=0x%x ties=%u heads=%u\n", (unsigned long long)n_in,
                (unsigned long long)win, lo_bit, digits, nties, d2h_u32(t, misc + 1, st));
    bool dedup = false;
    if (nties) {
        size_t pr = prof_begin(t, "sort", st);
        // longer tie runs: the general chunk-by-chunk refinement, which reorders perm (and, when chunk 0
        // was sorted only in part, pk) inside tie runs only
        // chunks (8-byte aligned) fully ordered so far: bytes [0, win) are shared, window bytes above
        // lo_bit are sorted
        const uint32_t start_depth = (uint32_t)((win + 8 - lo_bit / 8) / 8);
        // with a moved window pk keeps window values (no prefix rewrite): they become key prefixes below
        if (long_runs) refine_ties(t, kb, koff, n_in, perm, tie, start_depth, win ? nullptr : pk);
        dedup = long_runs || dups;
        prof_end(t, pr);
    }
    uint64_t n = n_in;
    if (dedup || (tomb && drop_tomb)) {
        size_t pd = prof_begin(t, "sort", st);
        uint32_t *flags = ens<uint32_t>(t->s_flags, n_in + 1);
        uint32_t *scan = ens<uint32_t>(t->s_scan, n_in + 1);
        launch_keep_flags(tie, perm, n_in, UINT64_MAX, flags, st);  // dedup: keep the last write
        if (tomb && drop_tomb) launch_clear_tomb(tomb, perm, n_in, flags, st);  // removed keys never survive
        exclusive_scan_u32(flags, scan, n_in, misc + 3, radix, st);
        launch_compact_u32(perm, flags, scan, n_in, pmalt->as<uint32_t>(), st);
        launch_compact_u64(pk, flags, scan, n_in, pkalt->as<uint64_t>(), st);
        prof_end(t, pd);
        n = d2h_u32(t, misc + 3, st);
        std::swap(pkbuf, pkalt);
        std::swap(pmbuf, pmalt);
        perm = pmbuf->as<uint32_t>();
    }
    if (win) {  // the set's prefixes (diff, locate, merge) are the key prefixes, not the sort windows
        size_t pf = prof_begin(t, "sort", st);
        launch_pfx_from_window(pkbuf->as<uint64_t>(), n, shared8, (uint32_t)std::min<uint64_t>(win, 8), st);
        prof_end(t, pf);
    }
    return SortedSet{pkbuf, pmbuf, n, {fp0, fp1}, dups == 0 && n == n_in, n ? klen_all : 0};
}

// fused_kcap: the leaf kernels copied the borrowed keys into t->kb (capacity fused_kcap bytes; complete
// when the key bytes + 16 fit) and the offsets into t->koff (fused_koff); 0 / false: the copy is made here.
void sort_dedup_gather(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, uint64_t n_in, const uint8_t *tomb,
                       bool staged_inputs, uint64_t staged_kbytes, bool defer_gather, uint64_t fused_kcap = 0,
                       bool fused_koff = false) {
    // Ordering work runs on the aux stream and overlaps the VALU-bound leaf hashing already enqueued on
    // t->st (the caller made st2 wait for the staged inputs); the streams join before the digest gather.
    hipStream_t st = t->st2;
    const uint8_t *dig = t->s_dig.as<uint8_t>();
    uint64_t kb_total = 0;
    const SortedSet S = sort_unique(t, kb, koff, n_in, tomb, true, staged_inputs ? nullptr : &kb_total);
    DevBuf *pkbuf = S.pk, *pmbuf = S.pm;
    const uint64_t n = S.n;
    uint32_t *perm;
    t->n = n;
    // adopt the sorted prefixes and the permutation
    swap_buf(t->pfx, *pkbuf);
    ++t->pfx_gen;
    t->keyset = next_keyset();
    t->kfp[0] = S.fp[0];
    t->kfp[1] = S.fp[1];
    t->kfp_ok = S.fp_ok;
    t->klen_fixed = S.klen;
    swap_buf(t->perm, *pmbuf);
    perm = t->perm.as<uint32_t>();
    // key-byte count of borrowed inputs, read while st is still busy hashing (never after the join:
    // a readback there would hold the host until the gather finishes and delay the reduce launches)
    const uint64_t kbytes = staged_inputs ? staged_kbytes : kb_total;
    const bool keys_done = !staged_inputs && fused_kcap && kbytes + 16 <= fused_kcap;
    // The reduction on st needs only the sorted order: join here, before the key copy.
    MKV_HIP(hipEventRecord(t->ev_join, st));
    MKV_HIP(hipStreamWaitEvent(t->st, t->ev_join, 0));
    if (t->kc_pending) {  // the ragged key copy (st3) completes before st2 does: the call's sync covers it
        MKV_HIP(hipStreamWaitEvent(st, t->ev_kc, 0));
        t->kc_pending = false;
    }
    // Own the keys (storage order): adopt staged uploads, copy borrowed device inputs. The copy stays on
    // st2 after the join, so its ~0.8 GB of memory traffic (10M keys) overlaps the VALU-bound reduction
    // instead of lengthening the ordering stage that the reduction waits for; the call's final sync
    // drains st2 before anything reads t->kb.
    t->nstore = n_in;
    t->kbytes = kbytes;
    if (staged_inputs) {
        swap_buf(t->kb, t->s_kb);
        swap_buf(t->koff, t->s_koff);
    } else {
        uint8_t *dkb = ens<uint8_t>(t->kb, kbytes + 16);  // (a regrowth syncs the device first)
        uint64_t *dko = ens<uint64_t>(t->koff, n_in + 1);
        if (!keys_done || !fused_koff) {
            size_t pc = prof_begin(t, "keycopy", st);
            if (kbytes && !keys_done) MKV_HIP(hipMemcpyAsync(dkb, kb, kbytes, hipMemcpyDeviceToDevice, st));
            if (!fused_koff) MKV_HIP(hipMemcpyAsync(dko, koff, (n_in + 1) * 8, hipMemcpyDeviceToDevice, st));
            prof_end(t, pc);
        }
    }
    // leaf level = nodes[0 .. n). Every level is stored, promoted nodes included, so the tree holds
    // sum_l ceil(n/2^l) <= 2n + L nodes (L <= 64 levels).
    uint8_t *nodes = ens<uint8_t>(t->nodes, 32 * node_slots(n));
    t->gather_pending = defer_gather;
    if (!defer_gather) {
        size_t pg = prof_begin(t, "gather");
        launch_gather_digests(perm, dig, n, nodes, t->st);
        prof_end(t, pg);
    }
}

// Inputs staged on t->st become visible to the aux stream; call before enqueueing the leaf hash so the
// ordering work on st2 overlaps it.
void fork_streams(mkv_tree *t) {
    MKV_HIP(hipEventRecord(t->ev_in, t->st));
    MKV_HIP(hipStreamWaitEvent(t->st2, t->ev_in, 0));
}

// Sorted keys of the tree packed into (dst_kb, dst_koff[0..n]) starting at byte base; returns bytes.
uint64_t pack_sorted_keys(mkv_tree *t, DevBuf &dst_kb, DevBuf &dst_koff, uint64_t extra_bytes,
                          uint64_t extra_items) {
    const uint64_t n = t->n;
    uint64_t *lens = ens<uint64_t>(t->s_lens, n + 1);
    uint64_t *ko = ens<uint64_t>(dst_koff, n + extra_items + 1);
    void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n), scan_scratch_bytes(n + 1)));
    launch_gather_keylens(t->perm.as<uint32_t>(), t->koff.as<uint64_t>(), n, lens, t->st);
    exclusive_scan_u64(lens, ko, n, ko + n, radix, t->st);
    const uint64_t bytes = n ? d2h_u64(t, ko + n) : 0;
    if (!n) MKV_HIP(hipMemsetAsync(ko, 0, 8, t->st));
    uint8_t *kb = ens<uint8_t>(dst_kb, bytes + extra_bytes + 16);
    launch_gather_keys(t->perm.as<uint32_t>(), t->kb.as<uint8_t>(), t->koff.as<uint64_t>(), ko, n, kb, t->st);
    return bytes;
}

void finish_unsharded(mkv_tree *t) {
    t->sharded = false;
    t->combine_pending = false;
    t->goff = 0;
    t->gN = t->n;
    plan_levels(t, 0, t->n, t->n);
    size_t pr = prof_begin(t, "reduce");
    if (t->gather_pending)
        run_reduce(t, t->nodes.as<uint8_t>(), t->perm.as<uint32_t>(), t->s_dig.as<uint8_t>());
    else
        run_reduce(t, t->nodes.as<uint8_t>());
    t->gather_pending = false;
    prof_end(t, pr);
    t->has_root = t->n > 0;
    uint8_t *hroot = reinterpret_cast<uint8_t *>(t->h_small + 16);
    if (t->has_root) {
        const size_t L = t->lev_S.size();
        small_d2h(t, hroot, t->nodes.as<uint8_t>() + 32 * t->lev_off[L - 1], 32, t->st);
    }
    sync(t);
    if (t->has_root) std::memcpy(t->root, hroot, 32);
}

// Upload a host blob into (bytes, offsets) device buffers with offsets rebased to 0.
void upload_blob(mkv_tree *t, const mkv_blob &b, DevBuf &bytes, DevBuf &offs, uint64_t dst_first = 0,
                 uint64_t dst_index = 0, uint64_t byte_base = 0) {
    const uint64_t n = b.n;
    const uint64_t o0 = n ? b.offsets[0] : 0;
    const uint64_t nbytes = n ? b.offsets[n] - o0 : 0;
    (void)dst_first;
    if (nbytes) MKV_HIP(hipMemcpyAsync(bytes.as<uint8_t>() + byte_base, b.bytes + o0, nbytes, hipMemcpyHostToDevice, t->st));
    std::vector<uint64_t> tmp(n + 1);
    for (uint64_t i = 0; i <= n; ++i) tmp[i] = (n ? b.offsets[i] - o0 : 0) + byte_base;
    MKV_HIP(hipMemcpyAsync(offs.as<uint64_t>() + dst_index, tmp.data(), (n + 1) * sizeof(uint64_t),
                           hipMemcpyHostToDevice, t->st));
    MKV_HIP(hipStreamSynchronize(t->st));  // tmp goes out of scope
}

// A plain host pointer handed to a device-side argument would fault the GPU instead of failing the call:
// refuse anything the runtime does not know as device, managed or registered host memory.
void need_device_ptr(const void *p, const char *what) {
    if (!p) return;
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) (void)hipGetLastError();
    if (e != hipSuccess || a.type == hipMemoryTypeUnregistered)
        throw Error(ST_EINVAL, std::string(what) + ": not device-accessible memory (pass device buffers)");
}
void need_device_blob(const mkv_blob &b, const char *what) {
    need_device_ptr(b.bytes, what);
    need_device_ptr(b.offsets, what);
}

void check_blob(const mkv_blob &b, const char *what) {
    if (b.n && (!b.offsets)) throw Error(ST_EINVAL, std::string(what) + ": null offsets");
    if (b.n >= 0xFFFFFFF0ull) throw Error(ST_EINVAL, std::string(what) + ": too many records (max 2^32-16)");
    if (b.n && b.offsets[b.n] > b.offsets[0] && !b.bytes) throw Error(ST_EINVAL, std::string(what) + ": null bytes");
    for (uint64_t i = 0; i < b.n; ++i)
        if (b.offsets[i + 1] < b.offsets[i]) throw Error(ST_EINVAL, std::string(what) + ": offsets not monotone");
}

// Stage [existing leaves ++ batch] for upsert / remove / apply. Returns staged record count.
// Existing records carry their leaf digests; batch records are hashed on the device.
uint64_t stage_batch(mkv_tree *t, const mkv_blob &keys, const mkv_blob *values, const uint8_t *is_remove,
                     uint64_t *staged_kbytes) {
    if (t->sharded) throw Error(ST_ESTATE, "upsert/remove on a sharded tree is not supported");
    const uint64_t m = t->n, nb = keys.n, tot = m + nb;
    const uint64_t kb_new = nb ? keys.offsets[nb] - keys.offsets[0] : 0;
    // existing leaves first (sorted, unique, with their digests), then the batch in order
    const uint64_t old_bytes = pack_sorted_keys(t, t->s_kb, t->s_koff, kb_new, nb);
    uint8_t *sdig = ens<uint8_t>(t->s_dig, (tot ? tot : 1) * 32);
    if (m) MKV_HIP(hipMemcpyAsync(sdig, t->nodes.p, m * 32, hipMemcpyDeviceToDevice, t->st));
    upload_blob(t, keys, t->s_kb, t->s_koff, 0, m, old_bytes);
    *staged_kbytes = old_bytes + kb_new;
    if (values && nb) {
        const uint64_t vbytes = values->offsets[nb] - values->offsets[0];
        ens<uint8_t>(t->s_vb, vbytes + 16);
        ens<uint64_t>(t->s_voff, nb + 1);
        upload_blob(t, *values, t->s_vb, t->s_voff);
    }
    t->in_tomb = nullptr;
    if (is_remove) {
        uint8_t *tomb = ens<uint8_t>(t->s_tomb, tot + 1);
        MKV_HIP(hipMemsetAsync(tomb, 0, tot, t->st));
        if (nb) MKV_HIP(hipMemcpyAsync(tomb + m, is_remove, nb, hipMemcpyHostToDevice, t->st));
        MKV_HIP(hipStreamSynchronize(t->st));
        t->in_tomb = tomb;
    }
    return tot;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
#define MKV_TRY(...)                                                                                 \
    try {                                                                                            \
        __VA_ARGS__;                                                                                 \
        return MKV_OK;                                                                               \
    } catch (const Error &e) {                                                                       \
        g_err = e.what();                                                                            \
        return e.code;                                                                               \
    } catch (const std::bad_alloc &) {                                                               \
        g_err = "host allocation failed";                                                            \
        return MKV_ENOMEM;                                                                           \
    } catch (const std::exception &e) {                                                              \
        g_err = e.what();                                                                            \
        return MKV_EINVAL;                                                                           \
    }

#define NEED(cond, msg) \
    if (!(cond)) throw Error(ST_EINVAL, msg)

extern "C" {

const char *mkv_last_error(void) { return g_err.c_str(); }
const char *mkv_version(void) { return "merklekv_amd 0.1 (gfx950)"; }

mkv_status mkv_tree_create(int hip_device, mkv_tree **out) {
    MKV_TRY({
        NEED(out, "out is null");
        *out = nullptr;
        int ndev = 0;
        hipError_t e = hipGetDeviceCount(&ndev);
        if (e != hipSuccess || ndev == 0) throw Error(ST_EHIP, "no HIP device available (MI355X required)");
        NEED(hip_device >= 0 && hip_device < ndev, "bad device index");
        DevGuard g(hip_device);
        mkv_tree *t = new mkv_tree();
        t->dev = hip_device;
        hipError_t e2 = hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking);
        if (e2 != hipSuccess) {
            delete t;
            throw Error(ST_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(e2));
        }
        e2 = hipHostMalloc(reinterpret_cast<void **>(&t->h_small), 1024, hipHostMallocDefault);
        if (e2 == hipSuccess) {
            void *d = nullptr;
            e2 = hipHostGetDevicePointer(&d, t->h_small, 0);
            t->h_small_dev = static_cast<uint8_t *>(d);
        }
        if (e2 == hipSuccess)
            e2 = hipHostMalloc(reinterpret_cast<void **>(&t->h_counts), (8 * 256 + 64) * sizeof(uint32_t),
                               hipHostMallocDefault);
        if (e2 == hipSuccess) {
            void *d = nullptr;
            e2 = hipHostGetDevicePointer(&d, t->h_counts, 0);
            t->h_counts_dev = static_cast<uint32_t *>(d);
        }
        if (e2 == hipSuccess) {
            int lo = 0, hi = 0;  // aux (ordering) stream at the highest priority: its WGs dispatch first
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            e2 = hipStreamCreateWithPriority(&t->st2, hipStreamNonBlocking, hi);
        }
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_in, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_join, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_wait, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_fixed, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_kc, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_edge, hipEventDisableTiming);
        if (e2 == hipSuccess) e2 = hipEventCreateWithFlags(&t->ev_a, hipEventDisableTiming);
        if (e2 == hipSuccess) {
            // copy stream at the lowest priority: HIP keeps one pool of hardware queues per priority
            // (GPU_MAX_HW_QUEUES each) and multiplexes streams onto them, so this puts the asynchronous
            // key-list copies (and the ragged key copy) on queues no tree's st / st2 shares — work queued
            // behind a copy on a shared queue waited for it (configs[4]: the next update, 0.65 ms)
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            e2 = hipStreamCreateWithPriority(&t->st3, hipStreamNonBlocking, lo);
        }
        if (e2 != hipSuccess) {
            mkv_tree_destroy(t);
            throw Error(ST_EHIP, std::string("tree resources: ") + hipGetErrorString(e2));
        }
        ++g_live_trees;
        t->counted = true;
        *out = t;
    });
}

void mkv_tree_destroy(mkv_tree *t) {
    if (!t) return;
    (void)hipSetDevice(t->dev);
    if (t->st2) (void)hipStreamSynchronize(t->st2);
    if (t->st) (void)hipStreamSynchronize(t->st);
    if (t->st3) (void)hipStreamSynchronize(t->st3);
    if (t->ev_in) (void)hipEventDestroy(t->ev_in);
    if (t->ev_join) (void)hipEventDestroy(t->ev_join);
    if (t->ev_wait) (void)hipEventDestroy(t->ev_wait);
    if (t->ev_fixed) (void)hipEventDestroy(t->ev_fixed);
    if (t->ev_kc) (void)hipEventDestroy(t->ev_kc);
    if (t->ev_edge) (void)hipEventDestroy(t->ev_edge);
    if (t->ev_a) (void)hipEventDestroy(t->ev_a);
    t->a_ev.reset();
    if (t->st3) (void)hipStreamDestroy(t->st3);
    if (t->st2) (void)hipStreamDestroy(t->st2);
    for (auto &p : t->evpool) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    if (t->h_small) (void)hipHostFree(t->h_small);
    if (t->h_counts) (void)hipHostFree(t->h_counts);
    if (t->h_seam) (void)hipHostFree(t->h_seam);
    if (t->st) (void)hipStreamDestroy(t->st);
    const bool counted = t->counted;
    delete t;
    (void)hipGetLastError();
    if (counted && --g_live_trees <= 0) {  // last handle gone: unpin the pooled key-list blocks
        std::lock_guard<std::mutex> lk(g_pool_mu);
        pool_trim_locked();
    }
}

mkv_status mkv_debug_trace(char *buf, uint64_t cap, uint64_t *len) {
    MKV_TRY({
        NEED(len, "null argument");
        std::string s;
        for (int i = 0; i < g_trace.n; ++i) {
            if (i) s += ';';
            s += g_trace.label[i];
            s += '=';
            s += std::to_string((int64_t)g_trace.us[i]);
        }
        *len = s.size();
        if (buf && cap) {
            const size_t k = std::min<size_t>(cap - 1, s.size());
            std::memcpy(buf, s.data(), k);
            buf[k] = 0;
        }
    });
}

mkv_status mkv_pool_trim(void) {
    MKV_TRY({
        std::lock_guard<std::mutex> lk(g_pool_mu);
        pool_trim_locked();
    });
}

mkv_status mkv_pool_stats(uint64_t *out6) {
    MKV_TRY({
        NEED(out6, "null argument");
        std::lock_guard<std::mutex> lk(g_pool_mu);
        out6[0] = g_pin_allocs.load();
        out6[1] = g_pin_frees.load();
        out6[2] = g_pin_alloc_bytes.load();
        out6[3] = g_pin_ns.load();
        out6[4] = g_pool.size();
        out6[5] = g_pool_bytes;
    });
}

mkv_status mkv_tree_clone(const mkv_tree *src, mkv_tree *dst) {
    MKV_TRY({
        NEED(src && dst, "null argument");
        NEED(src->dev == dst->dev, "clone across devices");
        NEED(!src->prepared, "shard_reduce pending");
        if (src == dst) return MKV_OK;
        DevGuard g(src->dev);
        MKV_HIP(hipStreamSynchronize(src->st));
        const uint64_t nn = total_nodes(src);
        uint8_t *kb = ens<uint8_t>(dst->kb, src->kbytes + 16);
        uint64_t *ko = ens<uint64_t>(dst->koff, src->nstore + 1);
        uint32_t *pm = ens<uint32_t>(dst->perm, src->n + 1);
        uint64_t *pf = ens<uint64_t>(dst->pfx, src->n + 1);
        ++dst->pfx_gen;
        uint8_t *nd = ens<uint8_t>(dst->nodes, 32 * std::max(node_slots(src->n), total_nodes(src) + 2));
        if (src->kbytes) MKV_HIP(hipMemcpyAsync(kb, src->kb.p, src->kbytes, hipMemcpyDeviceToDevice, dst->st));
        if (src->koff.p)
            MKV_HIP(hipMemcpyAsync(ko, src->koff.p, (src->nstore + 1) * 8, hipMemcpyDeviceToDevice, dst->st));
        if (src->n) {
            MKV_HIP(hipMemcpyAsync(pm, src->perm.p, src->n * 4, hipMemcpyDeviceToDevice, dst->st));
            MKV_HIP(hipMemcpyAsync(pf, src->pfx.p, src->n * 8, hipMemcpyDeviceToDevice, dst->st));
            MKV_HIP(hipMemcpyAsync(nd, src->nodes.p, nn * 32, hipMemcpyDeviceToDevice, dst->st));
        }
        MKV_HIP(hipStreamSynchronize(dst->st));
        dst->n = src->n;
        dst->nstore = src->nstore;
        dst->keyset = src->keyset;
        dst->kfp[0] = src->kfp[0];
        dst->kfp[1] = src->kfp[1];
        dst->kfp_ok = src->kfp_ok;
        dst->klen_fixed = src->klen_fixed;
        dst->kbytes = src->kbytes;
        dst->lev_cnt = src->lev_cnt;
        dst->lev_off = src->lev_off;
        dst->lev_base = src->lev_base;
        dst->lev_S = src->lev_S;
        dst->has_root = src->has_root;
        std::memcpy(dst->root, src->root, 32);
        dst->goff = src->goff;
        dst->gN = src->gN;
        dst->sharded = src->sharded;
        dst->prepared = false;
        dst->combine_pending = src->combine_pending;
    });
}

// The leaf stage of a build: the fixed-shape kernel, then the ragged kernel for whatever it left. Borrowed
// device inputs (!staged): the tree must own a copy of the keys; the leaf kernels store the key words they
// load (and the offsets) into the tree's buffers when those from an earlier build are large enough (*kcap /
// *ko_fused), else sort_dedup_gather copies the keys afterwards.
static void leaf_hash_owning_keys(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                                  const uint64_t *voff, uint64_t n, uint8_t *dig, bool staged, uint64_t *kcap,
                                  bool *ko_fused) {
    *kcap = !staged && t->kb.p && (reinterpret_cast<uintptr_t>(kb) & 15) == 0 ? t->kb.cap : 0;
    *ko_fused = !staged && t->koff.p && t->koff.cap >= (n + 1) * 8;
    KeyOut KO{*kcap ? t->kb.as<uint8_t>() : nullptr, *ko_fused ? t->koff.as<uint64_t>() : nullptr, *kcap};
    if ((reinterpret_cast<uintptr_t>(kb) & 15) != 0) KO.kdst = nullptr;  // copies keep the source offsets
    uint32_t *ctr = ens<uint32_t>(t->leaf_ctr, leaf_ctr_words(n));
    launch_leaf_fixed(kb, koff, vb, voff, n, dig, ctr, t->st, KO);
    if (!n) return;
    // st3, beside the leaf kernels: the edge records from the start (inputs ready at the callers'
    // fork_streams event; joined into st before the reduction), then the ragged chunks' key bytes once
    // k_leaf_direct is done (joined into st2). The ragged kernel is queued right after k_leaf_direct: host
    // calls in between delayed its start by ~13 us.
    MKV_HIP(hipEventRecord(t->ev_fixed, t->st));
    launch_leaf_ragged(kb, koff, vb, voff, n, dig, ctr, t->st, KO);
    MKV_HIP(hipStreamWaitEvent(t->st3, t->ev_in, 0));
    launch_leaf_edges(kb, koff, vb, voff, n, dig, t->st3);
    MKV_HIP(hipEventRecord(t->ev_edge, t->st3));
    MKV_HIP(hipStreamWaitEvent(t->st, t->ev_edge, 0));  // the reduction reads the edge digests
    if (KO.kdst) {
        MKV_HIP(hipStreamWaitEvent(t->st3, t->ev_fixed, 0));
        launch_keycopy_ragged(kb, koff, n, ctr, KO.kdst, KO.kcap, t->st3);
        MKV_HIP(hipEventRecord(t->ev_kc, t->st3));
        t->kc_pending = true;
    }
}

static void build_from_staged(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                              const uint64_t *voff, uint64_t n, bool staged, uint64_t staged_kbytes) {
    size_t ptot = prof_begin(t, "total_build");
    uint8_t *dig = ens<uint8_t>(t->s_dig, (n ? n : 1) * 32);
    fork_streams(t);
    size_t pl = prof_begin(t, "leaf_hash");
    uint64_t kcap = 0;
    bool ko_fused = false;
    leaf_hash_owning_keys(t, kb, koff, vb, voff, n, dig, staged, &kcap, &ko_fused);
    HTRACE("leaf-queued");
    prof_end(t, pl);
    sort_dedup_gather(t, kb, koff, n, nullptr, staged, staged_kbytes, true, kcap, ko_fused);
    HTRACE("ordered");
    finish_unsharded(t);
    HTRACE("reduce-queued");
    prof_end(t, ptot);
    sync(t);
    HTRACE("synced");
}

mkv_status mkv_tree_build(mkv_tree *t, mkv_blob keys, mkv_blob values) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        check_blob(keys, "keys");
        check_blob(values, "values");
        DevGuard g(t->dev);
        const uint64_t n = keys.n;
        const uint64_t kbn = n ? keys.offsets[n] - keys.offsets[0] : 0;
        const uint64_t vbn = n ? values.offsets[n] - values.offsets[0] : 0;
        ens<uint8_t>(t->s_kb, kbn + 16);
        ens<uint64_t>(t->s_koff, n + 1);
        ens<uint8_t>(t->s_vb, vbn + 16);
        ens<uint64_t>(t->s_voff, n + 1);
        upload_blob(t, keys, t->s_kb, t->s_koff);
        upload_blob(t, values, t->s_vb, t->s_voff);
        build_from_staged(t, t->s_kb.as<uint8_t>(), t->s_koff.as<uint64_t>(), t->s_vb.as<uint8_t>(),
                          t->s_voff.as<uint64_t>(), n, true, kbn);
    });
}

mkv_status mkv_tree_build_digests(mkv_tree *t, mkv_blob keys, const uint8_t *digests) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(digests || keys.n == 0, "null digests");
        check_blob(keys, "keys");
        DevGuard g(t->dev);
        const uint64_t n = keys.n;
        const uint64_t kbn = n ? keys.offsets[n] - keys.offsets[0] : 0;
        ens<uint8_t>(t->s_kb, kbn + 16);
        ens<uint64_t>(t->s_koff, n + 1);
        uint8_t *dig = ens<uint8_t>(t->s_dig, (n ? n : 1) * 32);
        if (n) MKV_HIP(hipMemcpyAsync(dig, digests, 32 * n, hipMemcpyHostToDevice, t->st));
        upload_blob(t, keys, t->s_kb, t->s_koff);  // synchronises t->st: the digests have landed too
        // Kernel A is skipped: the leaf digests arrive ready-made (a peer's (key, leaf digest) pairs)
        size_t ptot = prof_begin(t, "total_build");
        fork_streams(t);
        sort_dedup_gather(t, t->s_kb.as<uint8_t>(), t->s_koff.as<uint64_t>(), n, nullptr, true, kbn, true);
        finish_unsharded(t);
        prof_end(t, ptot);
        sync(t);
    });
}

mkv_status mkv_tree_build_device(mkv_tree *t, mkv_blob keys, mkv_blob values) {
    g_trace.reset();
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        NEED(keys.n < 0xFFFFFFF0ull, "too many records");
        NEED(keys.n == 0 || (keys.offsets && values.offsets), "null offsets");
        DevGuard g(t->dev);
        need_device_blob(keys, "keys");
        need_device_blob(values, "values");
        HTRACE("validated");
        build_from_staged(t, keys.bytes, keys.offsets, values.bytes, values.offsets, keys.n, false, 0);
    });
}

static DiffSide side_of(const mkv_tree *t);

// Key-set-changing batch on a non-empty unsharded tree: only the batch is sorted (last
// write per key wins, tombstones kept as flags), then merged with the tree's sorted leaves (Kernel E
// merge: replaced / removed leaves drop out, existing digests are reused, never re-hashed), and the
// levels are reduced again. Batch key records are appended to the key storage; the storage is
// repacked in sorted order once dead records outnumber live ones.
static void merge_batch(mkv_tree *t, const mkv_blob &keys, const mkv_blob *values, const uint8_t *is_remove) {
    size_t ptot = prof_begin(t, "total_build");
    const uint64_t nb = keys.n;
    const uint64_t kbn = keys.offsets[nb] - keys.offsets[0];
    ens<uint8_t>(t->u_kb, kbn + 16);
    ens<uint64_t>(t->u_koff, nb + 1);
    upload_blob(t, keys, t->u_kb, t->u_koff);
    if (values) {
        ens<uint8_t>(t->u_vb, values->offsets[nb] - values->offsets[0] + 16);
        ens<uint64_t>(t->u_voff, nb + 1);
        upload_blob(t, *values, t->u_vb, t->u_voff);
    }
    const uint8_t *tomb = nullptr;
    if (is_remove) {
        uint8_t *tb = ens<uint8_t>(t->u_tomb, nb + 1);
        MKV_HIP(hipMemcpyAsync(tb, is_remove, nb, hipMemcpyHostToDevice, t->st));
        MKV_HIP(hipStreamSynchronize(t->st));
        tomb = tb;
    }
    fork_streams(t);
    uint8_t *bdig = nullptr;
    if (values) {
        bdig = ens<uint8_t>(t->u_dig, nb * 32);
        size_t pl = prof_begin(t, "leaf_hash");
        launch_leaf_hash(t->u_kb.as<uint8_t>(), t->u_koff.as<uint64_t>(), t->u_vb.as<uint8_t>(),
                         t->u_voff.as<uint64_t>(), nb, bdig, ens<uint32_t>(t->leaf_ctr, leaf_ctr_words(nb)), t->st);
        prof_end(t, pl);
    }
    const SortedSet B = sort_unique(t, t->u_kb.as<uint8_t>(), t->u_koff.as<uint64_t>(), nb, tomb, false);
    MKV_HIP(hipEventRecord(t->ev_join, t->st2));
    MKV_HIP(hipStreamWaitEvent(t->st, t->ev_join, 0));
    const DiffSide A = side_of(t);
    DiffSide Bs{};
    Bs.kb = t->u_kb.as<uint8_t>();
    Bs.koff = t->u_koff.as<uint64_t>();
    Bs.perm = B.pm->as<uint32_t>();
    Bs.pfx = B.pk->as<uint64_t>();
    Bs.dig = bdig;
    Bs.n = B.n;
    Bs.klen = B.klen;  // the batch's own key length when all its keys share one (its offsets are then arithmetic)
    const uint64_t M = A.n + Bs.n;
    if (t->nstore + nb >= 0xFFFFFFF0ull) throw Error(ST_EINVAL, "too many stored key records");
    uint64_t *npfx = ens<uint64_t>(t->m_pfx, M + 1);
    uint32_t *nperm = ens<uint32_t>(t->m_perm, M + 1);
    uint8_t *nnodes = ens<uint8_t>(t->m_nodes, 32 * node_slots(M));
    uint64_t *cnt = ens<uint64_t>(t->m_cnt, 4);
    void *scr = t->d_diffscr.ensure(umerge_scratch_bytes(M));
    size_t pm = prof_begin(t, "merge");
    launch_umerge(A, Bs, tomb, (uint32_t)t->nstore, scr, npfx, nperm, nnodes, cnt, t->st);
    prof_end(t, pm);
    // key storage: the tree's records, then the batch's (offsets shifted by the tree's byte count)
    const uint64_t nst = t->nstore, kbytes = t->kbytes;
    uint8_t *nkb = ens<uint8_t>(t->s_kb, kbytes + kbn + 16);
    uint64_t *nko = ens<uint64_t>(t->s_koff, nst + nb + 1);
    if (kbytes) MKV_HIP(hipMemcpyAsync(nkb, t->kb.p, kbytes, hipMemcpyDeviceToDevice, t->st));
    if (kbn) MKV_HIP(hipMemcpyAsync(nkb + kbytes, t->u_kb.p, kbn, hipMemcpyDeviceToDevice, t->st));
    MKV_HIP(hipMemcpyAsync(nko, t->koff.p, (nst + 1) * 8, hipMemcpyDeviceToDevice, t->st));
    launch_add_offset_u64(t->u_koff.as<uint64_t>() + 1, nb, kbytes, nko + nst + 1, t->st);
    const uint64_t n_new = d2h_u64(t, cnt);
    swap_buf(t->kb, t->s_kb);
    swap_buf(t->koff, t->s_koff);
    swap_buf(t->pfx, t->m_pfx);
    ++t->pfx_gen;
    t->keyset = next_keyset();
    t->kfp_ok = false;  // merged key set: no fingerprint
    t->klen_fixed = t->klen_fixed && B.klen == t->klen_fixed ? t->klen_fixed : 0;
    swap_buf(t->perm, t->m_perm);
    swap_buf(t->nodes, t->m_nodes);
    t->kbytes = kbytes + kbn;
    t->nstore = nst + nb;
    t->n = n_new;
    t->gather_pending = false;
    if (t->nstore > 2 * t->n + 4096) {  // repack live keys in sorted order: perm becomes the identity
        const uint64_t bytes = pack_sorted_keys(t, t->s_kb, t->s_koff, 0, 0);
        swap_buf(t->kb, t->s_kb);
        swap_buf(t->koff, t->s_koff);
        launch_iota_u32(t->perm.as<uint32_t>(), t->n, t->st);
        t->nstore = t->n;
        t->kbytes = bytes;
    }
    finish_unsharded(t);
    prof_end(t, ptot);
    sync(t);
}

static void apply_batch(mkv_tree *t, const mkv_blob &keys, const mkv_blob *values, const uint8_t *is_remove) {
    if (t->n > 0 && !t->sharded && !t->prepared) {
        merge_batch(t, keys, values, is_remove);
        return;
    }
    size_t ptot = prof_begin(t, "total_build");
    uint64_t kbytes = 0;
    const uint64_t tot = stage_batch(t, keys, values, is_remove, &kbytes);
    const uint64_t m = tot - keys.n;
    fork_streams(t);
    if (values && keys.n) {
        size_t pl = prof_begin(t, "leaf_hash");
        launch_leaf_hash(t->s_kb.as<uint8_t>(), t->s_koff.as<uint64_t>() + m, t->s_vb.as<uint8_t>(),
                         t->s_voff.as<uint64_t>(), keys.n, t->s_dig.as<uint8_t>() + 32 * m,
                         ens<uint32_t>(t->leaf_ctr, leaf_ctr_words(keys.n)), t->st);
        prof_end(t, pl);
    }
    sort_dedup_gather(t, t->s_kb.as<uint8_t>(), t->s_koff.as<uint64_t>(), tot, t->in_tomb, true, kbytes, true);
    finish_unsharded(t);
    prof_end(t, ptot);
    sync(t);
}

// Dirty-path update (k_update.hip) for a batch whose keys are all leaves already: same key order and
// level plan, so only changed leaves and their ancestors are rehashed. Batch records are device
// pointers. A batch with a key that is not a leaf changes nothing and reports false.
static bool same_plan(const mkv_tree *a, const mkv_tree *b);

struct DirtyBatch {
    const uint8_t *kb;
    const uint64_t *koff;
    const uint8_t *vb;
    const uint64_t *voff;
    uint64_t m;
};

// The tree's locate samples (every LOC_STRIDE-th sorted prefix), rebuilt on stream st when the prefixes
// changed since the last call (builds, merges, clones); value-only updates keep them.
// The hash index of t's sorted keys for the dirty path's locate (k_update.hip locate_hix), built on first
// use after every key-set change (pfx_gen): 2 x n slots of 8 B (2 GiB at 125M keys). Small trees keep the
// sample search.
constexpr uint64_t HIX_MIN_KEYS = 1ull << 20;
static const uint64_t *locate_index_of(mkv_tree *t, hipStream_t st, uint64_t *mask) {
    *mask = 0;
    if (t->n < HIX_MIN_KEYS || t->n >= (1ull << 32) - 2) return nullptr;
    uint64_t cap = 1;
    while (cap < 2 * t->n) cap <<= 1;
    const bool fresh = t->hix_gen != t->pfx_gen || t->hix_mask != cap - 1 || t->hix.cap < cap * 8;
    if (fresh && t->hix_skip_gen == t->pfx_gen + 1) return nullptr;  // no room for this key set's index
    uint64_t *tab = nullptr;
    if (fresh) {
        // The index is an accelerator (2n slots of 8 B: 2 GiB at 125M keys): when the device cannot hold it,
        // the locate keeps the sample search instead of failing the update, and the key set is
        // not retried until it changes.
        size_t free_b = 0, total_b = 0;
        const bool room = hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                          (uint64_t)free_b + t->hix.cap >= cap * 8 + (256ull << 20);
        try {
            if (!room) throw Error(ST_ENOMEM, "hash index does not fit");
            tab = ens<uint64_t>(t->hix, cap);
        } catch (const Error &) {
            (void)hipGetLastError();  // clear a failed hipMalloc
            t->hix.release();
            t->hix_gen = ~0ull;
            t->hix_skip_gen = t->pfx_gen + 1;
            return nullptr;
        }
    } else {
        tab = t->hix.as<uint64_t>();
    }
    if (fresh) {
        MKV_HIP(hipMemsetAsync(tab, 0, cap * 8, st));
        launch_hix_build(side_of(t), tab, cap - 1, st);
        t->hix_gen = t->pfx_gen;
        t->hix_mask = cap - 1;
    }
    *mask = cap - 1;
    return tab;
}

static const uint64_t *locate_samples_of(mkv_tree *t, hipStream_t st, uint64_t *ns) {
    *ns = locate_samples(t->n);
    uint64_t *ps = ens<uint64_t>(t->pfx_s, *ns + 1);
    if (t->pfx_s_gen != t->pfx_gen) {
        launch_locate_samples(t->pfx.as<uint64_t>(), t->n, ps, st);
        t->pfx_s_gen = t->pfx_gen;
    }
    return ps;
}

// k dirty-path updates at once (mkv_tree_upsert_device_many; k = 1 is mkv_tree_upsert_device). Trees
// sharing one level plan (replicas of one key set) form a group and run together on the first tree's
// stream: one locate (grid.y = tree) beside one hash of every batch on the aux stream, one radix sort of
// (tree << pbits | position) keys, then ONE k_dirty_climb launch for the whole climb of every tree (round 5;
// it replaced a level-0 scatter, one launch per level and a fused top launch) and one readback of every
// tree's missing-key count and root. ok[i] = false: tree i had a key that is not a leaf and is unchanged.
static void dirty_update_many(mkv_tree *const *ts, const DirtyBatch *bs, uint32_t k, bool *ok) {
    std::vector<uint32_t> act;
    for (uint32_t i = 0; i < k; ++i) {
        mkv_tree *t = ts[i];
        ok[i] = bs[i].m == 0 && t->n > 0;
        if (t->n > 0 && !t->prepared && bs[i].m > 0) act.push_back(i);
    }
    if (act.empty()) return;
    std::vector<std::vector<uint32_t>> groups;
    for (uint32_t i : act) {
        bool placed = false;
        for (auto &g : groups)
            if (g.size() < (size_t)DIRTY_MAX_TREES && ts[g[0]]->dev == ts[i]->dev && same_plan(ts[g[0]], ts[i])) {
                g.push_back(i);
                placed = true;
                break;
            }
        if (!placed) groups.push_back({i});
    }
    for (auto &g : groups) {
        mkv_tree *t0 = ts[g[0]];
        DevGuard dg(t0->dev);
        hipStream_t st = t0->st;
        const size_t L = t0->lev_S.size();
        if (L > (size_t)MKV_MAXLEV) throw Error(ST_EINVAL, "tree too deep for the dirty climb");
        std::vector<size_t> prof(g.size());
        std::vector<char> had_root(g.size()), had_pending(g.size());
        for (size_t q = 0; q < g.size(); ++q) {
            mkv_tree *t = ts[g[q]];
            prof[q] = prof_begin(t, "update", st);
            had_root[q] = t->has_root;
            had_pending[q] = t->combine_pending;
        }
        // any earlier work on the other trees' streams first. Only a busy stream gets the event: HIP
        // multiplexes every stream onto a few hardware queues (GPU_MAX_HW_QUEUES, 4), so a marker on an
        // idle tree's stream can sit behind unrelated work sharing its queue — e.g. another tree's
        // asynchronous key-list copy, which then held the whole update back (configs[4]: 0.65 ms).
        for (size_t q = 1; q < g.size(); ++q) {
            mkv_tree *t = ts[g[q]];
            const hipError_t e = hipStreamQuery(t->st);
            if (e == hipSuccess) continue;
            if (e != hipErrorNotReady) MKV_HIP(e);
            MKV_HIP(hipEventRecord(t->ev_in, t->st));
            MKV_HIP(hipStreamWaitEvent(st, t->ev_in, 0));
        }
        const uint32_t k2 = (uint32_t)g.size();
        LeafBatches B{};
        LocateMulti LM{};
        ClimbArgs CA{};
        static_assert(DIRTY_MAX_TREES + 1 <= ZERO_MAX_RANGES, "ZeroRanges: the counters of every tree + the boundary bits");
        ZeroRanges Z{};
        uint32_t nz = 0;
        uint64_t M = 0, mmax = 0;
        for (size_t q = 0; q < g.size(); ++q) {
            mkv_tree *t = ts[g[q]];
            const DirtyBatch &b = bs[g[q]];
            B.kb[q] = b.kb;
            B.koff[q] = b.koff;
            B.vb[q] = b.vb;
            B.voff[q] = b.voff;
            B.m[q] = b.m;
            B.base[q] = M;
            M += b.m;
            mmax = std::max(mmax, b.m);
            const void *old_cnt = t->u_cnt.p;
            uint32_t *cnt = ens<uint32_t>(t->u_cnt, L + 2);  // cnt[l] < L: dirty nodes per level; cnt[L+1]: missing
            if (cnt != old_cnt) t->ucnt_zero_words = 0;
            if (t->ucnt_zero_words < L + 2) {  // first update (or the last one did not finish): zero them here
                Z.p[nz] = reinterpret_cast<uint8_t *>(cnt);
                Z.bytes[nz++] = (L + 2) * 4;
            }
            t->ucnt_zero_words = 0;  // until the end-of-update readback has reset them
            // replicas sharing t0's key-set id hold the same sorted keys, so their batches are located
            // in t0: one tree's prefix / permutation / key arrays serve all lookups (a 1/k working set
            // for the caches and the TLB instead of k copies of the same data)
            mkv_tree *lt = same_keyset(t, t0) ? t0 : t;
            LM.T[q] = side_of(lt);
            LM.hix[q] = locate_index_of(lt, st, &LM.hmask[q]);
            LM.ps[q] = LM.hix[q] ? nullptr : locate_samples_of(lt, st, &LM.ns[q]);
            LM.missing[q] = cnt + L + 1;
            CA.nodes[q] = t->nodes.as<uint8_t>();
            CA.missing[q] = cnt + L + 1;
            CA.cnt[q] = cnt;
        }
        if (M >= (1ull << 32) - 2) throw Error(ST_EINVAL, "dirty path: too many batch entries");
        // entry-boundary bits of the climb's cross-workgroup rendezvous: all-zero after every climb, so
        // zeroed only when (re)allocated
        const uint64_t bfw = (M + 1) / 32 + 2;
        uint32_t *bflags = ens<uint32_t>(t0->u_bf, bfw);
        if (t0->bf_words < bfw) {
            Z.p[nz] = reinterpret_cast<uint8_t *>(bflags);
            Z.bytes[nz++] = t0->u_bf.cap;
            t0->bf_words = t0->u_bf.cap / 4;
        }
        launch_zero_many(Z, nz, st);
        HTRACE("setup-queued");
        const int pbits = bits_for(t0->n);
        uint64_t *pos = ens<uint64_t>(t0->u_pos, M + 1), *pos2 = ens<uint64_t>(t0->u_pos2, M + 1);
        uint32_t *idx = ens<uint32_t>(t0->u_idx, M + 1), *idx2 = ens<uint32_t>(t0->u_idx2, M + 1);
        uint8_t *bdig = ens<uint8_t>(t0->u_dig, M * 32);
        // the batch hash (VALU) runs beside the locate (random prefix / key reads) on the aux stream
        MKV_HIP(hipEventRecord(t0->ev_in, st));
        MKV_HIP(hipStreamWaitEvent(t0->st2, t0->ev_in, 0));
        launch_leaf_hash_multi(B, k2, mmax, bdig, t0->st2);
        MKV_HIP(hipEventRecord(t0->ev_join, t0->st2));
        launch_locate_multi(B, LM, k2, mmax, pbits, pos, idx, st);
        MKV_HIP(hipStreamWaitEvent(st, t0->ev_join, 0));
        void *radix = t0->s_radix.ensure(std::max(radix_scratch_bytes(M), scan_scratch_bytes(M + 1)));
        const bool sw = radix_sort_pairs(pos, idx, pos2, idx2, M, 0, std::max(8, pbits + bits_for(k2 - 1)), radix, st);
        HTRACE("phase1-queued");
        CA.pos = sw ? pos2 : pos;
        CA.bidx = sw ? idx2 : idx;
        CA.bdig = bdig;
        CA.M = (uint32_t)M;
        CA.pbits = pbits;
        CA.k = k2;
        CA.P.L = (int)L;
        for (size_t l = 0; l < L; ++l) {
            CA.P.base[l] = t0->lev_base[l];
            CA.P.cnt[l] = t0->lev_cnt[l];
            CA.P.off[l] = t0->lev_off[l];
            CA.P.S[l] = t0->lev_S[l];
        }
        // The climb (one wave per 64 entries) runs while the dirty nodes are spread, and stops at the level
        // whose nodes span the mean gap between dirty leaves (floor(log2(gap)) + 1: about half of its nodes
        // are dirty); the reduction then rehashes every level above it, all trees in one launch per step.
        const uint64_t gap = std::max<uint64_t>(1, t0->n / std::max<uint64_t>(1, mmax));
        const int lstop = std::max(1, bits_for(gap));
        const bool dense_top = lstop < (int)L - 1;
        CA.lstop = dense_top ? lstop : -1;
        CA.bflags = bflags;
        CA.mbox = reinterpret_cast<uint8_t *>(t0->u_mbox.ensure(climb_mbox_bytes(M)));
        CA.ztab = ens<uint64_t>(t0->u_ztab, DIRTY_MAX_TREES);
        const size_t pclimb = prof_begin(t0, "climb", st);
        launch_dirty_climb(CA, st);
        // (the top launch straight from configs[4]'s 7 x 120 tiles measured slower than a fused 4-level launch
        // + the top from 8 tiles: climb 0.97 vs 0.83 ms)
        if (dense_top) run_reduce(t0, t0->nodes.as<uint8_t>(), nullptr, nullptr, (size_t)lstop, CA.ztab, k2);
        for (size_t q = 0; q < g.size(); ++q) ts[g[q]]->upd_dense_from = dense_top ? lstop : -1;
        prof_end(t0, pclimb);
        // every tree's counters (dirty nodes per level, missing keys) and root, read back by one launch that
        // also zeroes the counters for the next update (mkv_tree_update_counts reads the host copy)
        SmallCopies SC{};
        uint32_t nc = 0;
        for (size_t q = 0; q < g.size(); ++q) {
            mkv_tree *t = ts[g[q]];
            SC.src[nc] = reinterpret_cast<const uint8_t *>(CA.cnt[q]);
            SC.dst[nc] = t->h_small_dev + UCNT_HOST;
            SC.zero |= 1u << nc;
            SC.bytes[nc++] = (uint32_t)((L + 2) * sizeof(uint32_t));
            if (!t->sharded) {
                SC.src[nc] = t->nodes.as<uint8_t>() + 32 * t->lev_off[L - 1];
                SC.dst[nc] = t->h_small_dev + 16 * sizeof(uint64_t);
                SC.bytes[nc++] = 32;
                t->has_root = true;
            } else {
                t->has_root = false;
                t->combine_pending = true;  // seam + global root: mkv_shard_fringe + all-gather + combine
            }
        }
        hipLaunchKernelGGL(k_copy_small_many, dim3(nc), dim3(64), 0, st, SC);
        MKV_LAUNCH_CHECK();
        for (size_t q = 0; q < g.size(); ++q) ts[g[q]]->ucnt_zero_words = L + 2;
        HTRACE("climb-queued");
        for (size_t q = 0; q < g.size(); ++q) prof_end(ts[g[q]], prof[q]);
        for (size_t q = 0; q < g.size(); ++q) {
            mkv_tree *t = ts[g[q]];
            // all of the group's work ran on t0's streams: one host wait orders it before anything later
            // queued on the other trees' streams (no event wait left on them: a pending one costs every
            // later query of that stream ~15 µs), and their profiling pairs were recorded on st
            if (q == 0) sync(t);
            else prof_collect(t);
            ok[g[q]] = reinterpret_cast<volatile uint32_t *>(reinterpret_cast<uint8_t *>(t->h_small) + UCNT_HOST)[L + 1] == 0;
            if (ok[g[q]] && !t->sharded) std::memcpy(t->root, t->h_small + 16, 32);
            if (!ok[g[q]]) {  // tree untouched (the rehash above the climb rewrote the same digests)
                t->upd_dense_from = -1;
                t->has_root = had_root[q];
                t->combine_pending = had_pending[q];
            }
        }
        HTRACE("synced");
    }
}

static bool dirty_update(mkv_tree *t, const uint8_t *kb, const uint64_t *koff, const uint8_t *vb,
                         const uint64_t *voff, uint64_t m) {
    const DirtyBatch b{kb, koff, vb, voff, m};
    bool ok = false;
    dirty_update_many(&t, &b, 1, &ok);
    return ok;
}

// Stage a host batch on the device for dirty_update.
static void upload_update_batch(mkv_tree *t, const mkv_blob &keys, const mkv_blob &values) {
    const uint64_t m = keys.n;
    ens<uint8_t>(t->u_kb, keys.offsets[m] - keys.offsets[0] + 16);
    ens<uint64_t>(t->u_koff, m + 1);
    ens<uint8_t>(t->u_vb, values.offsets[m] - values.offsets[0] + 16);
    ens<uint64_t>(t->u_voff, m + 1);
    upload_blob(t, keys, t->u_kb, t->u_koff);
    upload_blob(t, values, t->u_vb, t->u_voff);
}

// ---- snapshot ingestion from the SYNC wire format ----
// Rust str::split_whitespace / trim_end on the ASCII header line.
static bool parse_keys_header(const uint8_t *p, uint64_t len, uint64_t *n) {
    std::string h(reinterpret_cast<const char *>(p), len);
    size_t i = 0;
    auto ws = [](char c) { return c == ' ' || (c >= 0x09 && c <= 0x0D); };
    auto tok = [&](std::string *out) {
        while (i < h.size() && ws(h[i])) ++i;
        size_t j = i;
        while (j < h.size() && !ws(h[j])) ++j;
        *out = h.substr(i, j - i);
        i = j;
        return !out->empty();
    };
    std::string a, b;
    if (!tok(&a) || a != "KEYS" || !tok(&b)) return false;
    if (b.empty() || b.size() > 19) return false;
    for (char c : b)
        if (c < '0' || c > '9') return false;
    *n = std::stoull(b);
    return true;
}

// Line-break positions of a host response uploaded to `dst`: returns the line count.
static uint64_t wire_lines(mkv_tree *t, const uint8_t *host, uint64_t len, DevBuf &dst, DevBuf &nlbuf) {
    uint8_t *d = ens<uint8_t>(dst, len + 16);
    if (len) MKV_HIP(hipMemcpyAsync(d, host, len, hipMemcpyHostToDevice, t->st));
    void *scr = t->w_scr.ensure(wire_scratch_bytes(len));
    uint64_t *tot = ens<uint64_t>(t->m_cnt, 4);
    wire_count_lines(d, len, scr, tot, t->st);
    const uint64_t lines = d2h_u64(t, tot);
    uint64_t *nl = ens<uint64_t>(nlbuf, lines + 1);
    if (lines) wire_emit_lines(d, len, scr, nl, t->st);
    return lines;
}

mkv_status mkv_tree_build_wire(mkv_tree *t, const uint8_t *scan, uint64_t scan_len, const uint8_t *gets,
                               uint64_t gets_len) {
    MKV_TRY({
        NEED(t && (scan || !scan_len) && (gets || !gets_len), "null argument");
        DevGuard g(t->dev);
        const uint8_t *eol = scan_len ? static_cast<const uint8_t *>(std::memchr(scan, '\n', scan_len)) : nullptr;
        NEED(eol, "peer closed while reading SCAN header");
        uint64_t n = 0;
        if (!parse_keys_header(scan, (uint64_t)(eol - scan), &n))
            throw Error(ST_EINVAL, "unexpected SCAN response (want \"KEYS <n>\")");
        const uint64_t ls = wire_lines(t, scan, scan_len, t->w_scan, t->w_nl1);
        NEED(ls >= n + 1, "peer closed while reading key list");
        const uint64_t lg = wire_lines(t, gets, gets_len, t->w_gets, t->w_nl2);
        NEED(lg >= n, "peer closed on GET (fewer GET responses than keys)");
        NEED(n < 0xFFFFFFF0ull, "too many records");
        uint64_t *ks = ens<uint64_t>(t->w_ks, n + 1), *kl = ens<uint64_t>(t->w_kl, n + 1);
        uint64_t *vs = ens<uint64_t>(t->w_vs, n + 1), *vl = ens<uint64_t>(t->w_vl, n + 1);
        uint32_t *found = ens<uint32_t>(t->w_found, n + 1), *rank = ens<uint32_t>(t->w_rank, n + 1);
        uint32_t *misc = ens<uint32_t>(t->s_misc, 64);
        MKV_HIP(hipMemsetAsync(misc, 0, 8, t->st));
        const uint8_t *dscan = t->w_scan.as<uint8_t>(), *dgets = t->w_gets.as<uint8_t>();
        launch_scan_keys(dscan, t->w_nl1.as<uint64_t>(), n, ks, kl, t->st);
        launch_get_values(dgets, t->w_nl2.as<uint64_t>(), n, vs, vl, found, misc, t->st);
        void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n + 1), scan_scratch_bytes(n + 2)));
        exclusive_scan_u32(found, rank, n, misc + 1, radix, t->st);
        small_d2h(t, t->h_small, misc, 8, t->st);
        wait_stream(t, t->st);
        const uint32_t bad = reinterpret_cast<uint32_t *>(t->h_small)[0];
        const uint64_t m = reinterpret_cast<uint32_t *>(t->h_small)[1];
        NEED(bad == 0, "unexpected GET response (want \"VALUE <v>\" or \"NOT_FOUND\")");
        // packed keys / values of the found records (keys whose GET said NOT_FOUND are skipped, sync.rs:130-140)
        uint64_t *koff = ens<uint64_t>(t->s_koff, m + 1), *voff = ens<uint64_t>(t->s_voff, m + 1);
        uint64_t *lens = ens<uint64_t>(t->s_lens, m + 1);
        launch_found_lengths(kl, found, rank, n, lens, t->st);
        exclusive_scan_u64(lens, koff, m, koff + m, radix, t->st);
        const uint64_t kbytes = m ? d2h_u64(t, koff + m) : 0;
        if (!m) MKV_HIP(hipMemsetAsync(koff, 0, 8, t->st));
        uint8_t *kb = ens<uint8_t>(t->s_kb, kbytes + 16);
        launch_pack_records(dscan, ks, kl, found, rank, koff, n, kb, t->st);
        launch_found_lengths(vl, found, rank, n, lens, t->st);
        exclusive_scan_u64(lens, voff, m, voff + m, radix, t->st);
        const uint64_t vbytes = m ? d2h_u64(t, voff + m) : 0;
        if (!m) MKV_HIP(hipMemsetAsync(voff, 0, 8, t->st));
        uint8_t *vb = ens<uint8_t>(t->s_vb, vbytes + 16);
        launch_pack_records(dgets, vs, vl, found, rank, voff, n, vb, t->st);
        MKV_HIP(hipStreamSynchronize(t->st));
        build_from_staged(t, kb, koff, vb, voff, m, true, kbytes);
    });
}

mkv_status mkv_tree_upsert(mkv_tree *t, mkv_blob keys, mkv_blob values) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        check_blob(keys, "keys");
        check_blob(values, "values");
        DevGuard g(t->dev);
        if (keys.n == 0) return MKV_OK;
        NEED(!t->prepared, "shard_reduce pending");
        if (t->n) {
            upload_update_batch(t, keys, values);
            if (dirty_update(t, t->u_kb.as<uint8_t>(), t->u_koff.as<uint64_t>(), t->u_vb.as<uint8_t>(),
                             t->u_voff.as<uint64_t>(), keys.n))
                return MKV_OK;
        }
        if (t->sharded) throw Error(ST_ESTATE, "upsert of new keys on a sharded tree: rebuild the shard");
        apply_batch(t, keys, &values, nullptr);
    });
}

// Key-set change of a device batch: bring it to the host and take the general (merge/re-sort) path.
static void upsert_device_general(mkv_tree *t, const mkv_blob &keys, const mkv_blob &values) {
    if (t->sharded) throw Error(ST_ESTATE, "upsert of new keys on a sharded tree: rebuild the shard");
    std::vector<uint64_t> ko(keys.n + 1), vo(keys.n + 1);
    MKV_HIP(hipMemcpy(ko.data(), keys.offsets, ko.size() * 8, hipMemcpyDeviceToHost));
    MKV_HIP(hipMemcpy(vo.data(), values.offsets, vo.size() * 8, hipMemcpyDeviceToHost));
    std::vector<uint8_t> kbh(ko.back() - ko[0] + 1), vbh(vo.back() - vo[0] + 1);
    if (ko.back() > ko[0])
        MKV_HIP(hipMemcpy(kbh.data(), keys.bytes + ko[0], ko.back() - ko[0], hipMemcpyDeviceToHost));
    if (vo.back() > vo[0])
        MKV_HIP(hipMemcpy(vbh.data(), values.bytes + vo[0], vo.back() - vo[0], hipMemcpyDeviceToHost));
    const uint64_t k0 = ko[0], v0 = vo[0];
    for (auto &x : ko) x -= k0;
    for (auto &x : vo) x -= v0;
    mkv_blob hk{kbh.data(), ko.data(), keys.n}, hv{vbh.data(), vo.data(), values.n};
    check_blob(hk, "keys");
    check_blob(hv, "values");
    apply_batch(t, hk, &hv, nullptr);
}

mkv_status mkv_tree_upsert_device(mkv_tree *t, mkv_blob keys, mkv_blob values) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        NEED(keys.n < 0xFFFFFFF0ull, "too many records");
        NEED(keys.n == 0 || (keys.offsets && values.offsets), "null offsets");
        DevGuard g(t->dev);
        if (keys.n == 0) return MKV_OK;
        NEED(!t->prepared, "shard_reduce pending");
        need_device_blob(keys, "keys");
        need_device_blob(values, "values");
        if (dirty_update(t, keys.bytes, keys.offsets, values.bytes, values.offsets, keys.n)) return MKV_OK;
        upsert_device_general(t, keys, values);
    });
}

mkv_status mkv_tree_upsert_device_many(mkv_tree *const *trees, const mkv_blob *keys, const mkv_blob *values,
                                       uint32_t k) {
    g_trace.reset();
    MKV_TRY({
        NEED(trees || k == 0, "null trees");
        NEED((keys && values) || k == 0, "null batches");
        for (uint32_t i = 0; i < k; ++i) {
            NEED(trees[i], "tree is null");
            NEED(keys[i].n == values[i].n, "keys.n != values.n");
            NEED(keys[i].n < 0xFFFFFFF0ull, "too many records");
            NEED(keys[i].n == 0 || (keys[i].offsets && values[i].offsets), "null offsets");
            NEED(keys[i].n == 0 || !trees[i]->prepared, "shard_reduce pending");
            need_device_blob(keys[i], "keys");
            need_device_blob(values[i], "values");
            for (uint32_t j = 0; j < i; ++j) NEED(trees[j] != trees[i], "a tree appears twice");
        }
        if (k == 0) return MKV_OK;
        HTRACE("checked");
        std::vector<DirtyBatch> bs(k);
        for (uint32_t i = 0; i < k; ++i)
            bs[i] = DirtyBatch{keys[i].bytes, keys[i].offsets, values[i].bytes, values[i].offsets, keys[i].n};
        std::unique_ptr<bool[]> ok(new bool[k]);
        dirty_update_many(trees, bs.data(), k, ok.get());
        for (uint32_t i = 0; i < k; ++i) {
            if (ok[i] || keys[i].n == 0) continue;
            DevGuard g(trees[i]->dev);
            upsert_device_general(trees[i], keys[i], values[i]);
        }
    });
}

mkv_status mkv_tree_remove(mkv_tree *t, mkv_blob keys) {
    MKV_TRY({
        NEED(t, "tree is null");
        check_blob(keys, "keys");
        DevGuard g(t->dev);
        if (keys.n == 0 || t->n == 0) return MKV_OK;
        std::vector<uint8_t> rm(keys.n, 1);
        apply_batch(t, keys, nullptr, rm.data());
    });
}

mkv_status mkv_tree_apply(mkv_tree *t, mkv_blob keys, mkv_blob values, const uint8_t *is_remove) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        NEED(is_remove || keys.n == 0, "is_remove is null");
        check_blob(keys, "keys");
        check_blob(values, "values");
        DevGuard g(t->dev);
        if (keys.n == 0) return MKV_OK;
        bool any = false;
        for (uint64_t i = 0; i < keys.n; ++i) any |= is_remove[i] != 0;
        apply_batch(t, keys, &values, any ? is_remove : nullptr);
    });
}

mkv_status mkv_tree_root(const mkv_tree *t, uint8_t out32[32], int *has_root) {
    MKV_TRY({
        NEED(t && out32 && has_root, "null argument");
        NEED(!t->prepared, "shard_reduce pending");
        NEED(!t->combine_pending, "shard_combine pending (sharded tree updated in place)");
        *has_root = t->has_root ? 1 : 0;
        if (t->has_root) std::memcpy(out32, t->root, 32);
        else std::memset(out32, 0, 32);
    });
}

mkv_status mkv_tree_len(const mkv_tree *t, uint64_t *n) {
    MKV_TRY({
        NEED(t && n, "null argument");
        *n = t->n;
    });
}

mkv_status mkv_tree_node_count(const mkv_tree *t, uint64_t *count) {
    MKV_TRY({
        NEED(t && count, "null argument");
        *count = t->n ? 2 * t->n - 1 : 0;
    });
}

mkv_status mkv_tree_level_count(const mkv_tree *t, uint32_t *nlevels) {
    MKV_TRY({
        NEED(t && nlevels, "null argument");
        *nlevels = t->n ? (uint32_t)t->lev_S.size() : 0;
    });
}

mkv_status mkv_tree_level(const mkv_tree *t, uint32_t level, uint64_t *count, uint8_t *out) {
    MKV_TRY({
        NEED(t && count, "null argument");
        NEED(!t->prepared, "shard_reduce pending");
        if (!t->n || level >= t->lev_S.size()) {
            *count = 0;
            return MKV_OK;
        }
        *count = t->lev_cnt[level];
        if (out && t->lev_cnt[level]) {
            DevGuard g(t->dev);
            MKV_HIP(hipMemcpyAsync(out, t->nodes.as<uint8_t>() + 32 * t->lev_off[level], 32 * t->lev_cnt[level],
                                   hipMemcpyDeviceToHost, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
        }
    });
}

// Fill a key list from device offsets (m+1, starting at 0) and key bytes.
// klen != 0 (every key klen bytes): the host writes the offsets k x klen (PinnedBlock::fill_offsets) and
// only the key bytes are copied.
static void keylist_fill(mkv_tree *t, mkv_keylist *l, const uint64_t *d_off, const uint8_t *d_bytes, uint64_t m,
                         uint64_t bytes, uint64_t klen = 0) {
    l->n = m;
    if (!m) return;
    const uint64_t kpos = (8 * (m + 1) + 15) & ~uint64_t(15);  // key bytes 16-B aligned in the block
    l->blk = std::make_shared<PinnedBlock>(kpos + bytes + 16, klen != 0);
    uint64_t *ho = reinterpret_cast<uint64_t *>(l->blk->p);
    uint8_t *hb = l->blk->p + kpos;
    const size_t ph = prof_begin(t, "d2h", t->st);  // the PCIe part of a key list (profiling only)
    if (!klen) copy_to_host(d_off, l->blk->dp, (m + 1) * 8, t->st);
    copy_to_host(d_bytes, l->blk->dp + kpos, bytes, t->st);
    prof_end(t, ph);
    if (klen) l->blk->fill_offsets(klen, m + 1);
    l->offsets = ho;
    l->bytes = hb;
}

mkv_status mkv_tree_leaves(const mkv_tree *t, mkv_keylist **keys, uint8_t *digests_out) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(!t->prepared, "shard_reduce pending");
        DevGuard g(t->dev);
        if (keys) {
            mkv_tree *tm = const_cast<mkv_tree *>(t);
            const uint64_t bytes = pack_sorted_keys(tm, tm->d_out, tm->d_outoff, 0, 0);
            auto *l = new mkv_keylist();
            try {
                keylist_fill(tm, l, tm->d_outoff.as<uint64_t>(), tm->d_out.as<uint8_t>(), t->n, bytes);
                MKV_HIP(hipStreamSynchronize(t->st));
            } catch (...) {
                delete l;
                throw;
            }
            *keys = l;
        }
        if (digests_out && t->n) {
            MKV_HIP(hipMemcpyAsync(digests_out, t->nodes.p, 32 * t->n, hipMemcpyDeviceToHost, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
        }
    });
}

// Owned nodes of level l whose parent is not owned: the local roots of a shard's forest (the tree root
// at the top level of an unsharded tree). At most two per level: the first and the last owned node.
static void level_roots(const mkv_tree *t, size_t l, uint64_t r[2]) {
    r[0] = r[1] = UINT64_MAX;
    const size_t L = t->lev_S.size();
    const uint64_t a = t->lev_base[l], c = t->lev_cnt[l];
    if (!c) return;
    const uint64_t cand[2] = {a, a + c - 1};
    for (int q = 0; q < 2; ++q) {
        if (q == 1 && cand[1] == cand[0]) break;
        bool parent_owned = false;
        if (l + 1 < L) {
            const uint64_t p = cand[q] / 2, a2 = t->lev_base[l + 1], c2 = t->lev_cnt[l + 1];
            parent_owned = p >= a2 && p < a2 + c2;
        }
        if (!parent_owned) r[q] = cand[q] - a;
    }
}

static bool same_plan(const mkv_tree *a, const mkv_tree *b) {
    return a->n == b->n && a->lev_base == b->lev_base && a->lev_cnt == b->lev_cnt && a->lev_S == b->lev_S;
}

constexpr size_t TD_CHECK_LEVEL = 4;

// Seeds of a sharded jump from level l to lt: the shard's fringe roots (owned nodes whose parent is not
// owned, level_roots) of levels lt .. l - 1, and of l itself on the first jump (from the top, where the
// frontier starts empty), each as its span of level-lt descendants. No frontier entry covers them.
static TdSeeds fringe_seeds(const mkv_tree *a, size_t l, size_t lt, bool top) {
    TdSeeds S{};
    for (size_t j = lt; j < l || (top && j == l); ++j) {
        uint64_t r[2];
        level_roots(a, j, r);
        for (int z = 0; z < 2; ++z) {
            if (r[z] == UINT64_MAX) continue;
            if (S.n >= (uint32_t)TD_MAX_SEEDS) throw Error(ST_ESTATE, "too many fringe roots in one jump");
            S.first[S.n] = ((r[z] + a->lev_base[j]) << (j - lt)) - a->lev_base[lt];
            S.span[S.n] = 1u << (j - lt);
            S.total += S.span[S.n++];
        }
    }
    return S;
}

// Levels the jumping walk lands on: the top level, then every multiple of 4 below it down to 0.
// fine: below level 8 every multiple of 2 instead. A jump of k levels reads 2^k digests per frontier
// node; near the leaves of a dense diff the frontier holds about one node per divergent leaf, so
// two 2-level jumps read half the bytes of one 4-level jump (configs[4]: 7 replicas x 125K updates of
// 125M leaves, levels 8 -> 0: ~26M -> ~13.5M digest pairs, ~380 -> ~200 us).
// How many jumps of T the one-workgroup top (k_topdown_top) covers: targets of at most TD_TOP_MAX_NODES nodes,
// not below TD_CHECK_LEVEL (the abort test rides on the jump from that level), every frontier it keeps in
// LDS (k variants x the nodes of an intermediate target) within TD_TOP_MAX_FRONTIER, and at most
// TD_TOP_MAX_WORK descendants compared per jump. 0: none.
static size_t top_jumps(const mkv_tree *a, const std::vector<size_t> &T, uint32_t k, TdTop *P) {
    size_t nt = 0;
    for (size_t q = 1; q < T.size(); ++q) {
        if (T[q] < TD_CHECK_LEVEL || a->lev_cnt[T[q]] > TD_TOP_MAX_NODES) break;
        if (q >= 2 && (uint64_t)k * a->lev_cnt[T[q - 1]] > TD_TOP_MAX_FRONTIER) break;
        // one CU reads ~64 KB per pass of its 1,024 threads: a heavier jump is faster as its own launch
        // (configs[4]'s 20 -> 16 for 7 variants: 13K descendants, slower inside the top than launched)
        if ((uint64_t)k * (q >= 2 ? a->lev_cnt[T[q - 1]] : 1) << (T[q - 1] - T[q]) > TD_TOP_MAX_WORK) break;
        nt = q;
    }
    if (!nt) return 0;
    std::memset(P, 0, sizeof *P);
    for (size_t l = 0; l < a->lev_cnt.size() && l < (size_t)MKV_MAXLEV_TD; ++l) {
        P->off[l] = a->lev_off[l];
        P->cnt[l] = a->lev_cnt[l];
    }
    for (size_t q = 0; q <= nt; ++q) P->T[q] = (uint32_t)T[q];
    P->nt = (uint32_t)nt;
    return nt;
}

// Jumps whose target level is small for all variants together (k x nodes <= 2^19: <= ~34 MB of digest
// pairs even if every node were compared) are merged with the jump before them: the frontier above such a
// level is dense, so one deeper jump compares the same descendants and saves a launch (~6 us). Never
// across the level-4 gate, at most 12 levels per jump. Returns the index in T of the merged jump's target
// (the jump from T[q - 1]).
static size_t merge_small_jumps(const mkv_tree *a, const std::vector<size_t> &T, size_t q, uint64_t k) {
    const size_t l = T[q - 1];
    while (q + 1 < T.size() && T[q + 1] > TD_CHECK_LEVEL && l - T[q + 1] <= 12 && k * a->lev_cnt[T[q + 1]] <= (1ull << 19))
        ++q;
    return q;
}

static std::vector<size_t> jump_targets(size_t L, bool fine = false) {
    std::vector<size_t> T{L - 1};
    for (int64_t x = (int64_t)((L - 2) / 4) * 4; x >= 0; x -= (fine && x <= 8) ? 2 : 4) T.push_back((size_t)x);
    return T;
}

// Top-down diff of two trees with identical level plans (equal leaf counts, and for shards the same
// global offset and size): node (l, j) covers the same leaf positions in both. Equal digests prune
// whole subtrees; only the divergent frontier is expanded, up to 4 levels per launch, starting from the
// local roots (the root, or a shard's fringe roots seeded into the jumps). Returns false (caller falls back to the merge-join)
// when a divergent leaf position holds different keys, i.e. the key sets differ there.
static bool topdown_diff(mkv_tree *t, const mkv_tree *a, const mkv_tree *b, const DiffSide &A, const DiffSide &B,
                         uint64_t *refs, uint64_t *m_out, const uint32_t **nbad_out) {
    *m_out = 0;
    *nbad_out = nullptr;
    const bool roots_valid = !a->combine_pending && !b->combine_pending && a->has_root && b->has_root;
    if (roots_valid && std::memcmp(a->root, b->root, 32) == 0) return true;  // equal roots: identical leaves
    const size_t L = a->lev_S.size();
    const uint64_t n = a->n;
    uint32_t *f0 = ens<uint32_t>(t->td_f0, n + 2);
    uint32_t *f1 = ens<uint32_t>(t->td_f1, n + 2);
    uint32_t *cnt = ens<uint32_t>(t->td_cnt, L + 2);  // cnt[l]: frontier size at level l; cnt[L] = 0 (seed)
    MKV_HIP(hipMemsetAsync(cnt, 0, (L + 2) * 4, t->st));
    // Key-set screen: cnt[L + 1] counts sampled positions whose prefixes differ. It is read together
    // with the first frontier count the walk reads back (level 4, or the leaf count of a small tree),
    // so a clean screen costs no round trip of its own; a failed one aborts the walk there.
    launch_sample_pfx(A.pfx, B.pfx, n, 4096, cnt + L + 1, t->st);
    const uint8_t *na = a->nodes.as<uint8_t>(), *nb = b->nodes.as<uint8_t>();
    uint32_t *fin = f0, *fout = f1;
    t->walk_jumps.clear();  // mkv_tree_walk_stats describes this walk
    t->walk_L = (uint32_t)L;
    t->walk_k = 1;
    if (!a->sharded && !b->sharded && L > 1) {
        // Unsharded: seed with the root, then jump 4 levels per launch (landing on level 4 for the
        // key-shift check and on level 0).
        launch_topdown_level(na + 32 * a->lev_off[L - 1], nb + 32 * b->lev_off[L - 1], 1, 0, 0, 0, UINT64_MAX, fin,
                             cnt + L, fout, cnt + (L - 1), 0, t->st);
        std::swap(fin, fout);
        const std::vector<size_t> T = jump_targets(L);
        for (size_t q = 1; q < T.size(); ++q) {
            const size_t l = T[q - 1], lt = T[q];
            const int k = (int)(l - lt);
            t->walk_jumps.emplace_back((uint32_t)l, (uint32_t)lt);
            launch_topdown_jump(na + 32 * a->lev_off[lt], nb + 32 * b->lev_off[lt], a->lev_cnt[lt], k, fin, cnt + l, fout,
                                cnt + lt, std::min<uint64_t>(a->lev_cnt[l] << k, 1ull << 40), t->st);
            std::swap(fin, fout);
            if (lt == TD_CHECK_LEVEL && L > TD_CHECK_LEVEL + 2) {
                const uint32_t *h = d2h_u32s(t, cnt, (uint32_t)L + 2);
                if (h[L + 1] != 0 || 2 * (uint64_t)h[lt] > a->lev_cnt[lt]) return false;
            }
        }
    } else if (L > 1) {
        // Sharded: the same jumps from an empty top frontier, the shard's fringe roots seeded into the jump
        // whose levels they sit on (fringe_seeds). Inserted/deleted keys shift every later leaf position, so
        // nearly every node below the first shift diverges: one readback at level 4 (16-leaf nodes: a 0.1 %
        // value-only divergence marks ~1.6 % of them) stops such a walk before the expensive bottom levels;
        // the merge-join is exact for any key sets.
        const std::vector<size_t> T = jump_targets(L);
        for (size_t q = 1; q < T.size(); ++q) {
            const size_t l = T[q - 1], lt = T[q];
            const int k = (int)(l - lt);
            t->walk_jumps.emplace_back((uint32_t)l, (uint32_t)lt);
            launch_topdown_jump_sh(na + 32 * a->lev_off[lt], nb + 32 * b->lev_off[lt], a->lev_cnt[lt], k, a->lev_base[l],
                                   a->lev_base[lt], fringe_seeds(a, l, lt, q == 1), fin, cnt + l, fout, cnt + lt,
                                   std::min<uint64_t>(a->lev_cnt[l] << k, 1ull << 40), t->st);
            std::swap(fin, fout);
            if (lt == TD_CHECK_LEVEL && L > TD_CHECK_LEVEL + 2) {
                const uint32_t *h = d2h_u32s(t, cnt, (uint32_t)L + 2);
                if (h[L + 1] != 0 || 2 * (uint64_t)h[lt] > a->lev_cnt[lt]) return false;
            }
        }
    } else {  // a one-leaf plan: the leaf is the shard's only root
        launch_topdown_jump_sh(na, nb, a->lev_cnt[0], 0, 0, a->lev_base[0], fringe_seeds(a, 0, 0, true), fin, cnt + 1,
                               fout, cnt, 0, t->st);
        std::swap(fin, fout);
    }
    const uint32_t *h = d2h_u32s(t, cnt, (uint32_t)L + 2);
    if (h[L + 1] != 0) return false;  // key sets differ (screen): the merge-join is exact
    const uint64_t m = h[0];
    *nbad_out = cnt + L + 1;  // zero here; k_topdown_leaves counts key mismatches into it
    if (m) {
        // divergent leaf positions -> sorted u64 (they are appended in no particular order)
        uint64_t *k1 = ens<uint64_t>(t->td_k1, m + 1);
        const uint64_t *pos = k1;
        const uint64_t words = (n + 31) / 32;
        uint32_t *bm = ens<uint32_t>(t->td_bm, words + 4);
        uint32_t *bc = ens<uint32_t>(t->td_bc, ceil_div(words, 1024) + 1);
        if (t->td_bm_words < words) {
            MKV_HIP(hipMemsetAsync(bm, 0, (words + 4) * 4, t->st));
            t->td_bm_words = words;
        }
        t->td_bm_words = 0;  // until the emit pass has been queued (it leaves the bitmap zero)
        if (positions_sorted_bitmap(fin, m, n, bm, bc, k1, t->st)) {
            t->td_bm_words = words;
        } else {
            uint64_t *k2 = ens<uint64_t>(t->td_k2, m + 1);
            uint32_t *v1 = ens<uint32_t>(t->td_v1, m + 1), *v2 = ens<uint32_t>(t->td_v2, m + 1);
            void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(m), scan_scratch_bytes(m + 1)));
            launch_widen_positions(fin, m, k1, v1, t->st);
            const bool sw = radix_sort_pairs(k1, v1, k2, v2, m, 0, std::max(8, bits_for(n)), radix, t->st);
            pos = sw ? k2 : k1;
        }
        // mismatching keys (nbad != 0) are read back with the key list's byte count (keylist_from_refs)
        launch_topdown_leaves(pos, m, A, B, !same_keyset(a, b), refs, cnt + L + 1, t->st);
    }
    *m_out = m;
    return true;
}

// Top-down pair diff queued whole before ONE host wait (round 3; shards too since round 5, their fringe
// roots seeded into the jumps): the jumping walk, the level-4
// abort test on the device (k_td_gate), the divergent positions (bitmap, device count) written straight
// into refs, the leaf-key check, key lengths, scan, key gather and the copy into a mapped pinned block
// sized from earlier calls. Returns the key list, or nullptr with *fallback = 1 (key sets differ or the
// walk was abandoned: merge-join) or 2 (the list outgrew the pinned capacity: refs hold *m_out sorted
// positions; the caller copies them with keylist_from_refs). Round 2 waited four times: level-4 count,
// leaf count, key bytes, result.
constexpr uint64_t TAIL_MIN_KEYS = 4096;        // smallest staging capacity of the one-wait diff (keys)
constexpr uint64_t TAIL_COPY_MAX = 1ull << 20;  // results up to 1 MiB are copied out of the staging block

static mkv_keylist *topdown_pair_onewait(mkv_tree *t, const mkv_tree *a, const mkv_tree *b, const DiffSide &A,
                                         const DiffSide &B, uint64_t *refs, int *fallback, uint64_t *m_out) {
    *fallback = 0;
    *m_out = 0;
    const bool roots_valid = !a->combine_pending && !b->combine_pending && a->has_root && b->has_root;
    if (roots_valid && std::memcmp(a->root, b->root, 32) == 0) return new mkv_keylist();  // identical leaves
    const size_t L = a->lev_S.size();
    const uint64_t n = a->n;
    uint32_t *f0 = ens<uint32_t>(t->td_f0, n + 2);
    uint32_t *f1 = ens<uint32_t>(t->td_f1, n + 2);
    uint32_t *cnt = ens<uint32_t>(t->td_cnt, L + 2 + TD_SCREEN_SLOTS);  // + the screen's slots
    if (!t->tail_cap_m) {
        t->tail_cap_m = std::max<uint64_t>(TAIL_MIN_KEYS, n / 1024);
        t->tail_cap_b = 48 * t->tail_cap_m;
    }
    const uint64_t cap_m = t->tail_cap_m, cap_b = t->tail_cap_b;
    const uint64_t words = (n + 31) / 32;
    uint32_t *bm = ens<uint32_t>(t->td_bm, words + 4);
    uint32_t *bc = ens<uint32_t>(t->td_bc, ceil_div(words, 1024) + 1);
    uint64_t *lens = ens<uint64_t>(t->s_lens, cap_m + 1);
    uint64_t *off = ens<uint64_t>(t->d_outoff, cap_m + 1);
    void *scr = t->d_diffscr.ensure(scan_scratch_bytes(cap_m + 1));
    uint8_t *kout = ens<uint8_t>(t->d_out, cap_b + 16);
    const uint64_t kpos = (8 * (cap_m + 1) + 15) & ~uint64_t(15);
    // the staging block is the tree's own, reused call to call unless an earlier result still holds it
    if (!t->tail_blk || t->tail_blk.use_count() > 1 || t->tail_blk->cap < kpos + cap_b + 16)
        t->tail_blk = std::make_shared<PinnedBlock>(kpos + cap_b + 16, true);
    std::shared_ptr<PinnedBlock> blk = t->tail_blk;
    const uint64_t klen = pair_klen(a, b);
    // fixed-length keys: the list's offsets k x klen are written by the host into the staging block (once
    // per block: they stay there while it cycles through the pool), not copied over PCIe
    if (!klen) blk->fill_n = 0;  // the device writes the offsets region
    blk->fill_n = std::min<uint64_t>(blk->fill_n, cap_m + 1);  // the key bytes start at kpos
    const size_t pd = prof_begin(t, "diff");  // the queued device work (the wait excluded)
    const uint8_t *na = a->nodes.as<uint8_t>(), *nb = b->nodes.as<uint8_t>();
    uint32_t *fin = f0, *fout = f1;
    const bool sh = a->sharded;  // same plan: b is sharded the same way
    // below level 8 the jumps land on every second level: near the leaves the frontier holds about one node
    // per divergent leaf, and two 2-level jumps read half the bytes of one 4-level jump (100M value-only:
    // 0.170 -> 0.161 ms device)
    const std::vector<size_t> T = jump_targets(L, true);
    TdTop P;
    const size_t nt = sh ? 0 : top_jumps(a, T, 1, &P);
    const bool gated = L > TD_CHECK_LEVEL + 2;  // the walk has a jump from level 4 (the abort test rides on it)
    // Unsharded, with a one-workgroup top that ends above level 4: the top zeroes the counters itself and the
    // jump landing on level 4 (a full grid: 16 of its workgroups sample beside their walk work) takes the
    // key-set screen, into slots the gated jump reads. Round 6: the fill and the screen had been two launches
    // in front of the top (~12 us of the call); the screen on the aux stream beside the top measured slower
    // (0.164 vs 0.161 ms device: the cross-stream event pair), inside the first jump after the top (12
    // workgroups) it added ~3 us to that jump. (Also tried: the key tail's last workgroup writing the call's
    // scalars instead of k_copy_small_many — a device-scope fence + arrival atomic per workgroup, 0.177 vs
    // 0.153 ms; its first workgroup stores them instead, below.)
    const bool fast_head = !sh && nt && gated && T[nt] > TD_CHECK_LEVEL;
    if (!fast_head) {
        MKV_HIP(hipMemsetAsync(cnt, 0, (L + 2) * 4, t->st));
        // (one 1,024-thread workgroup zeroing and sampling in a single launch measured slower: 0.238 vs 0.231
        // ms; round 6: inside the one-workgroup top as well, 0.187-0.194 vs 0.172 ms — one CU's few thousand
        // random prefix reads are slower than 16 workgroups' — and the landing jump adding each divergent
        // leaf to its position block's count, so no count pass: 0.193 vs 0.187 ms)
        launch_sample_pfx(A.pfx, B.pfx, n, 4096, cnt + L + 1, t->st);
    }
    // the position bitmap is all-zero between calls; zeroed here (grown) before the jump that lands on the
    // leaves sets its bits
    if (t->td_bm_words < words) MKV_HIP(hipMemsetAsync(bm, 0, (words + 4) * 4, t->st));
    t->td_bm_words = 0;  // until the emit pass has been queued (it leaves the bitmap zero)
    t->walk_jumps.clear();  // mkv_tree_walk_stats describes this walk (one variant)
    t->walk_L = (uint32_t)L;
    t->walk_k = 1;
    t->walk_fused = 0;
    size_t q0 = 1;
    if (!sh) {
        if (nt) {  // the roots and the first nt jumps in one workgroup
            TdVariants V{};
            V.nodes[0] = nb;
            launch_topdown_top(na, V, 1, P, fout, false, cnt, t->st, fast_head ? (uint32_t)L + 2 : 0u);
            for (size_t q = 1; q <= nt; ++q) t->walk_jumps.emplace_back((uint32_t)T[q - 1], (uint32_t)T[q]);
            t->walk_fused = (uint32_t)nt;
            q0 = nt + 1;
        } else {
            launch_topdown_level(na + 32 * a->lev_off[L - 1], nb + 32 * b->lev_off[L - 1], 1, 0, 0, 0, UINT64_MAX, fin,
                                 cnt + L, fout, cnt + (L - 1), 0, t->st);
        }
        std::swap(fin, fout);
    }  // sharded: the frontier at the top level starts empty (cnt[L - 1] = 0); the roots come in as seeds
    for (size_t q = q0; q < T.size(); ++q) {
        const size_t l = T[q - 1];
        if (!sh) q = merge_small_jumps(a, T, q, 1);  // (100M: 16 -> 12 -> 8 becomes 16 -> 8)
        const size_t lt = T[q];
        const int k = (int)(l - lt);
        t->walk_jumps.emplace_back((uint32_t)l, (uint32_t)lt);
        const uint64_t maxd = std::min<uint64_t>(a->lev_cnt[l] << k, 1ull << 40);
        // the level-4 abort test rides on the jump from level 4 (no launch of its own)
        const bool gate = l == TD_CHECK_LEVEL && gated;
        if (!sh) {
            const TdScreen SC{A.pfx, B.pfx, n, fast_head && lt == TD_CHECK_LEVEL ? cnt + L + 2 : nullptr};
            launch_topdown_jump(na + 32 * a->lev_off[lt], nb + 32 * b->lev_off[lt], a->lev_cnt[lt], k, fin, cnt + l, fout,
                                cnt + lt, maxd, t->st, gate ? cnt : nullptr, (uint32_t)L + 1, a->lev_cnt[l],
                                lt == 0 ? bm : nullptr, gate && fast_head ? cnt + L + 2 : nullptr, SC);
        } else {
            if (gate) launch_td_gate(cnt, (uint32_t)L + 1, (uint32_t)l, a->lev_cnt[l], t->st);
            launch_topdown_jump_sh(na + 32 * a->lev_off[lt], nb + 32 * b->lev_off[lt], a->lev_cnt[lt], k, a->lev_base[l],
                                   a->lev_base[lt], fringe_seeds(a, l, lt, q == 1), fin, cnt + l, fout, cnt + lt, maxd,
                                   t->st);
        }
        std::swap(fin, fout);
    }
    positions_sorted_bitmap_dev(fin, cnt, n, bm, bc, refs, t->st, !sh);  // side-A refs = sorted positions
    t->td_bm_words = words;
    t->h_small[3] = 0;  // the key tail's mismatch flag (its kernels of earlier calls have completed)
    const bool scalars = launch_diff_tail_dev(refs, cnt, A, B, !same_keyset(a, b), cnt + L + 1, cap_m, cap_b, lens, off,
                                              scr, kout, blk->dp, blk->dp + kpos, t->st, klen, klen != 0,
                                              reinterpret_cast<uint64_t *>(t->h_small_dev));
    if (!scalars) {  // one launch: divergent positions, screen / abort / leaf-key mismatches, key bytes (when m <= cap_m)
        SmallCopies SC{};
        const uint8_t *srcs[3] = {reinterpret_cast<const uint8_t *>(cnt), reinterpret_cast<const uint8_t *>(cnt + L + 1),
                                  reinterpret_cast<const uint8_t *>(off + cap_m)};
        const uint32_t sizes[3] = {4, 4, 8};
        for (int q = 0; q < 3; ++q) {
            SC.src[q] = srcs[q];
            SC.dst[q] = t->h_small_dev + 8 * q;
            SC.bytes[q] = sizes[q];
        }
        hipLaunchKernelGGL(k_copy_small_many, dim3(3), dim3(64), 0, t->st, SC);
        MKV_LAUNCH_CHECK();
    }
    prof_end(t, pd);
    HTRACE("onewait-queued");
    if (klen) blk->fill_offsets(klen, cap_m + 1);  // while the device works
    sync(t);
    const uint64_t m = (uint32_t)t->h_small[0];
    const uint32_t word = (uint32_t)t->h_small[1] | (t->h_small[3] ? 1u : 0u);
    const uint64_t bytes = t->h_small[2];
    if (word != 0) {
        *fallback = 1;
        return nullptr;
    }
    if (m > cap_m || bytes > cap_b) {
        if (16 * m <= (256ull << 20)) {  // grow for the next call (bounded)
            t->tail_cap_m = std::max(cap_m, 2 * m);
            t->tail_cap_b = std::max(cap_b, m > cap_m ? 2 * m * 64 : 2 * bytes + 4096);
        }
        *fallback = 2;
        *m_out = m;
        return nullptr;
    }
    // capacity follows the results: halve towards twice this call's size (a burst of large diffs does not
    // keep every later staging block large)
    t->tail_cap_m = std::max<uint64_t>({TAIL_MIN_KEYS, 2 * m, cap_m / 2});
    t->tail_cap_b = std::max<uint64_t>({48 * TAIL_MIN_KEYS, 2 * bytes, cap_b / 2});
    auto *l = new mkv_keylist();
    l->n = m;
    if (m) {
        const uint64_t used = 8 * (m + 1) + bytes;
        if (used <= TAIL_COPY_MAX && 8 * used <= blk->cap) {
            // a small result in a large staging block: the list gets a block of its own size (a caller that
            // keeps many results alive must not pin a capacity-sized block for each), the tree keeps the
            // staging block for its next call
            auto own = std::make_shared<PinnedBlock>(used + 16);
            std::memcpy(own->p, blk->p, 8 * (m + 1));
            std::memcpy(own->p + 8 * (m + 1), blk->p + kpos, bytes);
            l->blk = own;
            l->offsets = reinterpret_cast<const uint64_t *>(own->p);
            l->bytes = own->p + 8 * (m + 1);
        } else {
            l->blk = blk;  // a large result: handed over whole; the next call stages into a fresh block
            t->tail_blk.reset();
            l->offsets = reinterpret_cast<const uint64_t *>(blk->p);
            l->bytes = blk->p + kpos;
        }
    }
    return l;
}

static DiffSide side_of(const mkv_tree *t) {
    DiffSide s{};
    s.kb = t->kb.as<uint8_t>();
    s.koff = t->koff.as<uint64_t>();
    s.perm = t->perm.as<uint32_t>();
    s.pfx = t->pfx.as<uint64_t>();
    s.dig = t->nodes.as<uint8_t>();
    s.n = t->n;
    s.klen = t->klen_fixed;
    return s;
}

// Key list of the refs (bit 63 = side B) gathered on the device and copied to the host. `reject`
// (optional device u32) is read back together with the byte count: nonzero -> nullptr, nothing copied.
static mkv_keylist *keylist_from_refs(mkv_tree *t, const uint64_t *refs, uint64_t m, const DiffSide &A,
                                      const DiffSide &B, const uint32_t *reject = nullptr, uint64_t klen = 0) {
    auto *l = new mkv_keylist();
    try {
        if (m && klen && !reject) {
            // every key of both trees has length klen: offsets k * klen, no length gather / scan / readback
            uint64_t *off = ens<uint64_t>(t->d_outoff, m + 1);
            uint8_t *ob = ens<uint8_t>(t->d_out, m * klen + 16);
            launch_fill_stride_u64(off, m, klen, t->st);
            launch_diff_keys(refs, m, A, B, off, ob, t->st);
            HTRACE("keys-queued");
            keylist_fill(t, l, off, ob, m, m * klen, klen);
            HTRACE("copies-queued");
        } else if (m) {
            size_t pk = prof_begin(t, "diff");
            uint64_t *lens = ens<uint64_t>(t->s_lens, m + 1);
            uint64_t *off = ens<uint64_t>(t->d_outoff, m + 1);
            void *scr = t->d_diffscr.ensure(scan_scratch_bytes(m + 1));
            launch_diff_keylens(refs, m, A, B, lens, t->st);
            exclusive_scan_u64(lens, off, m, off + m, scr, t->st);
            prof_end(t, pk);
            small_d2h(t, t->h_small, off + m, 8, t->st);
            if (reject) small_d2h(t, t->h_small + 1, reject, 4, t->st);
            HTRACE("keylens-queued");
            wait_stream(t, t->st);
            const uint64_t bytes = t->h_small[0];
            if (reject && reinterpret_cast<const uint32_t *>(t->h_small + 1)[0] != 0) {
                sync(t);
                delete l;
                return nullptr;
            }
            uint8_t *ob = ens<uint8_t>(t->d_out, bytes + 16);
            launch_diff_keys(refs, m, A, B, off, ob, t->st);
            HTRACE("keys-queued");
            keylist_fill(t, l, off, ob, m, bytes);
            HTRACE("copies-queued");
        }
        sync(t);
        HTRACE("synced");
    } catch (...) {
        delete l;
        throw;
    }
    return l;
}

// Device-resident form of keylist_from_refs (the sharded collectives, comm.cpp): the same gather into
// d_outoff / d_out, left on the device — offsets[0..m] (offsets[0] == 0) and the key bytes, valid until the
// tree's next diff / keys call. false when `reject` (optional device u32) is non-zero (nothing gathered).
static bool keys_from_refs_dev(mkv_tree *t, const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B,
                               const uint32_t *reject, DevKeys *out) {
    *out = DevKeys{};
    uint64_t *off = ens<uint64_t>(t->d_outoff, m + 1);
    if (!m) {
        MKV_HIP(hipMemsetAsync(off, 0, 8, t->st));
        out->off = off;
        out->kb = ens<uint8_t>(t->d_out, 16);
        if (reject) {
            small_d2h(t, t->h_small + 1, reject, 4, t->st);
            wait_stream(t, t->st);
            if (reinterpret_cast<const uint32_t *>(t->h_small + 1)[0] != 0) return false;
        }
        return true;
    }
    uint64_t *lens = ens<uint64_t>(t->s_lens, m + 1);
    void *scr = t->d_diffscr.ensure(scan_scratch_bytes(m + 1));
    launch_diff_keylens(refs, m, A, B, lens, t->st);
    exclusive_scan_u64(lens, off, m, off + m, scr, t->st);
    small_d2h(t, t->h_small, off + m, 8, t->st);
    if (reject) small_d2h(t, t->h_small + 1, reject, 4, t->st);
    wait_stream(t, t->st);
    const uint64_t bytes = t->h_small[0];
    if (reject && reinterpret_cast<const uint32_t *>(t->h_small + 1)[0] != 0) return false;
    uint8_t *ob = ens<uint8_t>(t->d_out, bytes + 16);
    launch_diff_keys(refs, m, A, B, off, ob, t->st);
    out->n = m;
    out->bytes = bytes;
    out->off = off;
    out->kb = ob;
    return true;
}

// The batched diff's key list (configs[4]: one list for every replica of the 1-vs-k walk): keys gathered
// on st as in keylist_from_refs, then the device -> pinned copy (PCIe-bound: ~28 MB for 7 x 125K keys)
// runs on st3 and the call returns without waiting for it; mkv_keylist_get waits when the bytes are
// first read. The caller's next work (the next step's updates) overlaps the copy.
static mkv_keylist *keylist_from_refs_async(mkv_tree *t, const uint64_t *refs, uint64_t m, const DiffSide &A,
                                            const DiffSide &B, uint64_t klen = 0, bool wait_st = true) {
    auto *l = new mkv_keylist();
    try {
        if (m) {
            if (t->a_ev) MKV_HIP(hipStreamWaitEvent(t->st, t->a_ev->e, 0));  // the last copy read a_out*
            size_t pk = prof_begin(t, "diff");
            uint64_t *off = ens<uint64_t>(t->a_outoff, m + 1);
            uint64_t bytes = m * klen;
            const bool g16 = klen && klen % 16 == 0 && klen < (1u << 20);  // granule gather, offsets implicit
            if (klen) {  // fixed-length keys: offsets k * klen, no length gather / scan / readback
                if (!g16) launch_fill_stride_u64(off, m, klen, t->st);
                prof_end(t, pk);
            } else {
                uint64_t *lens = ens<uint64_t>(t->a_lens, m + 1);
                void *scr = t->d_diffscr.ensure(scan_scratch_bytes(m + 1));
                launch_diff_keylens(refs, m, A, B, lens, t->st);
                exclusive_scan_u64(lens, off, m, off + m, scr, t->st);
                prof_end(t, pk);
                small_d2h(t, t->h_small, off + m, 8, t->st);
                wait_stream(t, t->st);
                bytes = t->h_small[0];
            }
            uint8_t *ob = ens<uint8_t>(t->a_out, bytes + 16);
            if (g16) launch_diff_keys_fixed(refs, m, A, B, klen, ob, t->st);
            else launch_diff_keys(refs, m, A, B, off, ob, t->st);
            l->n = m;
            const uint64_t kpos = (8 * (m + 1) + 15) & ~uint64_t(15);
            l->blk = std::make_shared<PinnedBlock>(kpos + bytes + 16, klen != 0);
            MKV_HIP(hipEventRecord(t->ev_a, t->st));
            MKV_HIP(hipStreamWaitEvent(t->st3, t->ev_a, 0));
            const size_t ph = prof_begin(t, "d2h", t->st3);
            // DMA engine, not a copy kernel: beside the next update, a kernel's PCIe writes into pinned
            // memory slowed the update's random-read locate 2x (configs[4] step 2.83 -> 2.37-2.43 ms).
            // Fixed-length keys: only the key bytes cross PCIe, the host writes the offsets k x klen (once
            // per pinned block: they stay there while it cycles through the pool; 7 MB of 35 at configs[4])
            if (!klen) MKV_HIP(hipMemcpyAsync(l->blk->p, off, (m + 1) * 8, hipMemcpyDeviceToHost, t->st3));
            MKV_HIP(hipMemcpyAsync(l->blk->p + kpos, ob, bytes, hipMemcpyDeviceToHost, t->st3));
            prof_end(t, ph);
            if (klen) l->blk->fill_offsets(klen, m + 1);
            auto ev = std::make_shared<KeyEvent>();
            MKV_HIP(hipEventRecord(ev->e, t->st3));
            l->ready = ev;
            t->a_ev = ev;
            l->offsets = reinterpret_cast<const uint64_t *>(l->blk->p);
            l->bytes = l->blk->p + kpos;
            // the caller reads counters its own work on st wrote into pinned memory (topdown_batch: the
            // per-variant check and segment words); the length path above waited already
            if (klen && wait_st) wait_stream(t, t->st);
        }
    } catch (...) {
        delete l;
        throw;
    }
    return l;
}

// dev != nullptr: the divergent keys stay in device memory (*dev; sharded collectives), returns nullptr.
static mkv_keylist *diff_pair(const mkv_tree *a, const mkv_tree *b, DevKeys *dev = nullptr) {
    mkv_tree *t = const_cast<mkv_tree *>(a);
    t->walk_L = 0;  // td_cnt is about to hold a pair walk's counters: no batched-walk stats any more
    // b's last work must be complete before a's stream reads it
    wait_idle(b->st);
    HTRACE("diff-start");
    DiffSide A = side_of(a), B = side_of(b);
    const uint64_t M = A.n + B.n;
    uint64_t *refs = ens<uint64_t>(t->d_refs, M + 1);
    uint64_t m = 0;
    bool done = false;
    const uint64_t nwords = (A.n + 31) / 32;
    if (!dev && A.n > 0 && same_plan(a, b) && !keysets_differ(a, b) && a->sharded == b->sharded && a->lev_S.size() > 1 &&
        ceil_div(nwords, POS_BLOCK_WORDS) <= POS_MAX_BLOCKS) {
        int fb = 0;
        mkv_keylist *l = topdown_pair_onewait(t, a, b, A, B, refs, &fb, &m);
        HTRACE("topdown-done");
        if (l) return l;
        if (fb == 2) return keylist_from_refs(t, refs, m, A, B, nullptr, pair_klen(a, b));
        m = 0;  // key sets differ (or the walk was abandoned): the merge-join below
    } else if (A.n > 0 && same_plan(a, b) && !keysets_differ(a, b)) {
        // Top-down: identical level plans, so node (l, j) covers the same leaf positions in both trees.
        size_t pd = prof_begin(t, "diff");
        const uint32_t *nbad = nullptr;
        done = topdown_diff(t, a, b, A, B, refs, &m, &nbad);
        prof_end(t, pd);
        HTRACE("topdown-done");
        if (done) {
            // the leaf-key check (nbad) comes back with the key list's byte count
            if (dev) {
                if (keys_from_refs_dev(t, refs, m, A, B, nbad, dev)) return nullptr;
            } else {
                mkv_keylist *l = keylist_from_refs(t, refs, m, A, B, nbad);
                if (l) return l;
            }
            m = 0;  // a divergent position holds different keys: the key sets differ
            done = false;
        }
    }
    if (!done) {
        size_t pd = prof_begin(t, "diff");
        uint64_t *cnt = ens<uint64_t>(t->s_misc, 64);
        void *scr = t->d_diffscr.ensure(diff_scratch_bytes(M));
        launch_diff(A, B, scr, refs, cnt, t->st, true);
        prof_end(t, pd);
        small_d2h(t, t->h_small, cnt, 16, t->st);  // count + deferred-check verdict
        wait_stream(t, t->st);
        m = t->h_small[0];
        if (t->h_small[1]) {  // equal prefixes with different keys (or too many checks): exact rerun
            pd = prof_begin(t, "diff");
            launch_diff(A, B, scr, refs, cnt, t->st, false);
            prof_end(t, pd);
            m = d2h_u64(t, cnt);
        }
    }
    if (dev) {
        keys_from_refs_dev(t, refs, m, A, B, nullptr, dev);
        return nullptr;
    }
    return keylist_from_refs(t, refs, m, A, B, nullptr, pair_klen(a, b));
}

// One top-down walk of base `a` against every variant in vs (same level plan, key sets screened
// equal): frontier entries carry the variant id, so each level is one launch for all of them.
// res[i] = keylist, or nullptr when variant i's key set turned out to differ (caller diffs it pairwise).
// Returns false (nothing decided) when the level-4 frontier says the walk is not worth finishing.
constexpr uint64_t VPOS_MAX_BITS = 1ull << 33;  // (variant, position) bitmap of the batched walk: <= 1 GiB
static bool topdown_batch(mkv_tree *t, const mkv_tree *a, const std::vector<const mkv_tree *> &vs,
                          std::vector<mkv_keylist *> &res) {
    const uint32_t k = (uint32_t)vs.size();
    const size_t L = a->lev_S.size();
    const uint64_t n = a->n;
    TdVariants V{};
    for (uint32_t i = 0; i < k; ++i) V.nodes[i] = vs[i]->nodes.as<uint8_t>();
    const uint64_t cap = (L > TD_CHECK_LEVEL + 2 ? k * n / 2 : k * n) + 2ull * k + 64;
    uint64_t *f0 = ens<uint64_t>(t->tb_f0, cap), *f1 = ens<uint64_t>(t->tb_f1, cap);
    uint32_t *cnt = ens<uint32_t>(t->td_cnt, L + 2 + 2 * k);  // per level; then nbad[k], count[k]
    const uint8_t *na = a->nodes.as<uint8_t>();
    uint64_t *fin = f0, *fout = f1;
    bool sharded = a->sharded;
    for (auto *v : vs) sharded |= v->sharded;
    const std::vector<size_t> T = jump_targets(L, true);
    TdTop P;
    const size_t nt = !sharded && L > 1 ? top_jumps(a, T, k, &P) : 0;
    // with a one-workgroup top the counters are zeroed by it (no fill launch in front of the walk)
    if (!nt) MKV_HIP(hipMemsetAsync(cnt, 0, (L + 2 + 2 * k) * 4, t->st));
    t->walk_jumps.clear();
    t->walk_L = (uint32_t)L;
    t->walk_k = k;
    // the (variant, position) bitmap that orders the level-0 entries (all-zero between calls; zeroed here
    // when grown): the jump that lands on the leaves sets its bits itself
    const uint64_t bits = (uint64_t)k * n, words = (bits + 31) / 32;
    const bool bitmap = bits <= VPOS_MAX_BITS;
    uint32_t *bm = nullptr;
    bool bits_set = false;
    if (bitmap) {
        bm = ens<uint32_t>(t->tb_bm, words + 4);
        if (t->tb_bm_words < words) MKV_HIP(hipMemsetAsync(bm, 0, (words + 4) * 4, t->st));
        t->tb_bm_words = 0;  // until the emit pass has been queued (it leaves the bitmap zero)
    }
    const size_t pwalk = prof_begin(t, "walk");
    t->walk_fused = 0;
    if (!sharded && L > 1) {  // seed with every variant's root, then jump 4 levels per launch
        size_t q0 = 1;
        if (nt) {  // the roots and the first nt jumps in one workgroup
            launch_topdown_top(na, V, k, P, fout, true, cnt, t->st, (uint32_t)(L + 2 + 2 * k), (uint32_t)(L + 2 + k));
            for (size_t q = 1; q <= nt; ++q) t->walk_jumps.emplace_back((uint32_t)T[q - 1], (uint32_t)T[q]);
            t->walk_fused = (uint32_t)nt;
            q0 = nt + 1;
        } else {
            launch_topdown_level_batch(na + 32 * a->lev_off[L - 1], V, 32 * a->lev_off[L - 1], 1, 0, 0, 0, UINT64_MAX,
                                       k, fin, cnt + L, fout, cnt + (L - 1), 0, t->st);
        }
        std::swap(fin, fout);
        for (size_t q = q0; q < T.size(); ++q) {
            const size_t l = T[q - 1];
            q = merge_small_jumps(a, T, q, k);  // (configs[4]: 20 -> 16 -> 12 becomes 20 -> 12)
            const size_t lt = T[q];
            const int kk = (int)(l - lt);
            t->walk_jumps.emplace_back((uint32_t)l, (uint32_t)lt);
            const bool land = bitmap && lt == 0;
            // the level-4 abort test rides on the jump from level 4 (frontier over half the level: nothing
            // compared, bit 31 in cnt[L + 1]), read back with the leaf count: no host round trip in the walk
            const bool gate = l == TD_CHECK_LEVEL && L > TD_CHECK_LEVEL + 2;
            launch_topdown_jump_batch(na + 32 * a->lev_off[lt], V, 32 * a->lev_off[lt], a->lev_cnt[lt], kk, fin, cnt + l,
                                      fout, cnt + lt, std::min<uint64_t>(k * (a->lev_cnt[l] << kk), 1ull << 40), t->st,
                                      land ? bm : nullptr, n, gate ? cnt : nullptr, (uint32_t)L + 1, k * a->lev_cnt[l]);
            bits_set |= land;
            std::swap(fin, fout);
        }
    } else
    for (size_t l = L; l >= 1; --l) {
        uint64_t r[2];
        level_roots(a, l - 1, r);
        if (l < L) t->walk_jumps.emplace_back((uint32_t)l, (uint32_t)(l - 1));
        const uint64_t a_par = l < L ? a->lev_base[l] : 0, max_par = l < L ? k * a->lev_cnt[l] : 0;
        launch_topdown_level_batch(na + 32 * a->lev_off[l - 1], V, 32 * a->lev_off[l - 1], a->lev_cnt[l - 1], a_par,
                                   a->lev_base[l - 1], r[0], r[1], k, fin, cnt + l, fout, cnt + (l - 1), max_par,
                                   t->st);
        std::swap(fin, fout);
        if (l - 1 == TD_CHECK_LEVEL && L > TD_CHECK_LEVEL + 2) {
            const uint64_t c = d2h_u32(t, cnt + (l - 1));
            if (2 * c > k * a->lev_cnt[l - 1]) {
                prof_end(t, pwalk);
                return false;
            }
        }
    }
    prof_end(t, pwalk);
    uint32_t *nbad = cnt + L + 2, *vcount = nbad + k;
    // per-variant key-check failures and segment starts come back through pinned memory
    static_assert(2 * TD_MAX_VARIANTS * 4 <= 512, "h_small holds the batched-walk counters");
    uint32_t *hb = reinterpret_cast<uint32_t *>(t->h_small + 64);
    for (uint32_t i = 0; i < k; ++i) hb[i] = 0;
    const DiffSide A = side_of(a);
    const int pb = std::max(1, bits_for(n));
    std::vector<DiffSide> hs(k);
    for (uint32_t i = 0; i < k; ++i) hs[i] = side_of(vs[i]);
    DiffSide *ds = reinterpret_cast<DiffSide *>(t->tb_sides.ensure(k * sizeof(DiffSide)));
    // the variants' sides on the device: uploaded only when they changed (a value-only update keeps every
    // array of a tree where it is; the upload is a staged copy of ~15 us on the walk's stream)
    const bool sides_fresh = t->tb_sides_dev != (void *)ds || t->tb_sides_host.size() != hs.size() ||
                             std::memcmp(t->tb_sides_host.data(), hs.data(), hs.size() * sizeof(DiffSide)) != 0;
    auto upload_sides = [&] {
        if (!sides_fresh) return;
        MKV_HIP(hipMemcpyAsync(ds, hs.data(), k * sizeof(DiffSide), hipMemcpyHostToDevice, t->st));
        t->tb_sides_host = hs;
        t->tb_sides_dev = ds;
    };
    // per-variant segment starts: 0xFFFFFFFF, set by the one-workgroup top when it ran
    const bool vcount_set = !sharded && L > 1 && nt;
    uint64_t check = 0;  // variants whose key set may differ from the base's
    for (uint32_t i = 0; i < k; ++i)
        if (!same_keyset(vs[i], a)) check |= 1ull << i;
    uint64_t m = 0;
    uint64_t *refs = nullptr;
    if (bitmap) {
        // the level-0 entries ordered on the device from the device count (k_vpos_*), the leaf checks
        // from the same count: one host wait for the count, the abort flag and the per-variant words
        const uint64_t sw = vpos_scratch_words(bits);
        uint32_t *bc = ens<uint32_t>(t->tb_bc, sw);
        void *scr = t->d_diffscr.ensure(scan_scratch_bytes(sw));
        launch_vpos_sorted_dev(fin, cnt, cap, n, k, pb, bm, bc, scr, fout, t->st, bits_set);
        t->tb_bm_words = words;
        upload_sides();
        if (!vcount_set) MKV_HIP(hipMemsetAsync(vcount, 0xFF, k * 4, t->st));
        refs = fin;  // the level-0 frontier is consumed: its buffer holds the refs
        launch_topdown_leaves_batch(fout, cap, pb, A, ds, check, refs, nbad, vcount, t->st, cnt);
        {  // the walk's counters and the per-variant words in one readback launch
            SmallCopies SC{};
            SC.src[0] = reinterpret_cast<const uint8_t *>(cnt);
            SC.dst[0] = t->h_small_dev;
            SC.bytes[0] = (uint32_t)(4 * (L + 2));
            SC.src[1] = reinterpret_cast<const uint8_t *>(nbad);
            SC.dst[1] = t->h_small_dev + (reinterpret_cast<uint8_t *>(hb) - reinterpret_cast<uint8_t *>(t->h_small));
            SC.bytes[1] = (uint32_t)(2 * k * 4);
            hipLaunchKernelGGL(k_copy_small_many, dim3(2), dim3(64), 0, t->st, SC);
            MKV_LAUNCH_CHECK();
        }
        wait_stream(t, t->st);
        const uint32_t *hc = reinterpret_cast<const uint32_t *>(t->h_small);
        if (hc[L + 1] != 0) return false;  // the gate stopped the walk: not worth finishing
        m = hc[0];
    } else {
        const uint32_t *hc = d2h_u32s(t, cnt, (uint32_t)L + 2);
        if (hc[L + 1] != 0) return false;  // the gate stopped the walk: not worth finishing
        m = hc[0];
        refs = ens<uint64_t>(t->d_refs, m + 1);
        if (m) {
            const int vb = std::max(1, bits_for(k - 1));
            uint64_t *k1 = ens<uint64_t>(t->td_k1, m + 1), *k2 = ens<uint64_t>(t->td_k2, m + 1);
            uint32_t *v1 = ens<uint32_t>(t->td_v1, m + 1), *v2 = ens<uint32_t>(t->td_v2, m + 1);
            void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(m), scan_scratch_bytes(m + 1)));
            launch_pack_entries(fin, m, pb, k1, v1, t->st);
            const bool swp = radix_sort_pairs(k1, v1, k2, v2, m, 0, pb + vb, radix, t->st);
            upload_sides();
            if (!vcount_set) MKV_HIP(hipMemsetAsync(vcount, 0xFF, k * 4, t->st));
            launch_topdown_leaves_batch(swp ? k2 : k1, m, pb, A, ds, check, refs, nbad, vcount, t->st);
            small_d2h(t, hb, nbad, 2 * k * 4, t->st);
        }
    }
    // waits for st (hb valid after) unless the bitmap path waited already
    mkv_keylist *all = keylist_from_refs_async(t, refs, m, A, A, a->klen_fixed, !bitmap);
    // segment starts -> per-variant counts (variants appear in ascending order)
    std::vector<uint64_t> cntv(k, 0);
    if (m) {
        uint64_t next = m;
        for (int64_t i = (int64_t)k - 1; i >= 0; --i) {
            if (hb[k + i] == 0xFFFFFFFFu) continue;
            cntv[i] = next - hb[k + i];
            next = hb[k + i];
        }
    }
    uint64_t at = 0;
    for (uint32_t i = 0; i < k; ++i) {
        const uint64_t c = cntv[i];
        if (hb[i] == 0) {
            auto *l = new mkv_keylist();  // a view into the shared block
            if (c) {
                l->blk = all->blk;
                l->ready = all->ready;
                l->bytes = all->bytes;
                l->offsets = all->offsets + at;
                l->n = c;
            }
            res[i] = l;
        }
        at += c;
    }
    all->ready.reset();  // the views wait for the copy; the shared block lives on in them
    delete all;
    return true;
}

mkv_status mkv_tree_diff(const mkv_tree *a, const mkv_tree *b, mkv_keylist **out) {
    g_trace.reset();
    MKV_TRY({
        NEED(a && b && out, "null argument");
        NEED(a->dev == b->dev, "trees on different devices");
        NEED(!a->prepared && !b->prepared, "shard_reduce pending");
        *out = nullptr;
        DevGuard g(a->dev);
        *out = diff_pair(a, b);
    });
}

mkv_status mkv_tree_diff_many(const mkv_tree *a, const mkv_tree *const *others, uint32_t k, mkv_keylist **outs) {
    g_trace.reset();
    MKV_TRY({
        NEED(a && (others || k == 0) && (outs || k == 0), "null argument");
        for (uint32_t i = 0; i < k; ++i) {
            NEED(others[i], "null tree");
            NEED(others[i]->dev == a->dev, "trees on different devices");
            NEED(!others[i]->prepared, "shard_reduce pending");
            outs[i] = nullptr;
        }
        NEED(!a->prepared, "shard_reduce pending");
        mkv_tree *t = const_cast<mkv_tree *>(a);
        DevGuard g(t->dev);
        std::vector<mkv_keylist *> res(k, nullptr);
        try {
            for (uint32_t i = 0; i < k; ++i) wait_idle(others[i]->st);
            // candidates for the shared walk: same level plan and a clean key-set screen
            std::vector<uint32_t> cand;
            if (a->n > 0) {
                for (uint32_t i = 0; i < k; ++i)
                    if (same_plan(a, others[i])) cand.push_back(i);
            }
            const bool roots_a = !a->combine_pending && a->has_root;
            std::vector<uint32_t> walk;
            // a variant with the base's key-set id holds the same key sequence: no sampled screen
            std::vector<uint32_t> same_ks, other_ks;
            for (uint32_t c : cand) (same_keyset(others[c], a) ? same_ks : other_ks).push_back(c);
            for (uint32_t c : same_ks) {
                const mkv_tree *o = others[c];
                if (roots_a && !o->combine_pending && o->has_root && std::memcmp(a->root, o->root, 32) == 0)
                    res[c] = new mkv_keylist();  // equal roots: identical leaves
                else
                    walk.push_back(c);
            }
            cand.swap(other_ks);
            if (!cand.empty()) {
                uint32_t *scr = ens<uint32_t>(t->tb_screen, cand.size() + 1);
                MKV_HIP(hipMemsetAsync(scr, 0, cand.size() * 4, t->st));
                for (size_t c = 0; c < cand.size(); ++c)
                    launch_sample_pfx(a->pfx.as<uint64_t>(), others[cand[c]]->pfx.as<uint64_t>(), a->n, 4096,
                                      scr + c, t->st);
                std::vector<uint32_t> hs(cand.size());
                MKV_HIP(hipMemcpyAsync(hs.data(), scr, cand.size() * 4, hipMemcpyDeviceToHost, t->st));
                sync(t);
                for (size_t c = 0; c < cand.size(); ++c) {
                    const mkv_tree *o = others[cand[c]];
                    if (hs[c]) continue;
                    if (roots_a && !o->combine_pending && o->has_root && std::memcmp(a->root, o->root, 32) == 0) {
                        res[cand[c]] = new mkv_keylist();  // equal roots: identical leaves
                    } else {
                        walk.push_back(cand[c]);
                    }
                }
            }
            for (size_t s0 = 0; s0 < walk.size(); s0 += TD_MAX_VARIANTS) {
                const size_t s1 = std::min(walk.size(), s0 + (size_t)TD_MAX_VARIANTS);
                std::vector<const mkv_tree *> vs;
                for (size_t i = s0; i < s1; ++i) vs.push_back(others[walk[i]]);
                std::vector<mkv_keylist *> part(vs.size(), nullptr);
                HTRACE("screened");
                size_t pd = prof_begin(t, "diff");
                const bool ok = topdown_batch(t, a, vs, part);
                prof_end(t, pd);
                if (ok)
                    for (size_t i = s0; i < s1; ++i) res[walk[i]] = part[i - s0];
            }
            for (uint32_t i = 0; i < k; ++i)
                if (!res[i]) res[i] = diff_pair(a, others[i]);
        } catch (...) {
            for (auto *l : res) delete l;
            throw;
        }
        for (uint32_t i = 0; i < k; ++i) outs[i] = res[i];
    });
}

// ---- anti-entropy exchange (README.md:310-347 protocol) ----
static const uint8_t *level_ptr(const mkv_tree *t, uint32_t level, uint64_t *count) {
    *count = level < t->lev_cnt.size() ? t->lev_cnt[level] : 0;
    return *count ? t->nodes.as<uint8_t>() + 32 * t->lev_off[level] : nullptr;
}

mkv_status mkv_tree_node_digests(const mkv_tree *tc, uint32_t level, const uint64_t *idx, uint64_t m, uint8_t *out) {
    MKV_TRY({
        NEED(tc && (m == 0 || (idx && out)), "null argument");
        NEED(!tc->prepared && !tc->sharded, "node exchange needs an unsharded tree");
        if (!m) return MKV_OK;
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        DevGuard g(t->dev);
        uint64_t cnt = 0;
        const uint8_t *lvl = level_ptr(t, level, &cnt);
        uint64_t *di = ens<uint64_t>(t->x_idx, m);
        uint8_t *dd = ens<uint8_t>(t->x_dig, 32 * m);
        MKV_HIP(hipMemcpyAsync(di, idx, m * 8, hipMemcpyHostToDevice, t->st));
        launch_node_digests(lvl ? lvl : dd, cnt, di, m, dd, t->st);
        MKV_HIP(hipMemcpyAsync(out, dd, 32 * m, hipMemcpyDeviceToHost, t->st));
        MKV_HIP(hipStreamSynchronize(t->st));
    });
}

mkv_status mkv_tree_compare_nodes(const mkv_tree *tc, uint32_t level, const uint64_t *idx, const uint8_t *peer,
                                  uint64_t m, uint64_t *out_idx, uint64_t *n_out) {
    MKV_TRY({
        NEED(tc && n_out && (m == 0 || (idx && peer && out_idx)), "null argument");
        NEED(!tc->prepared && !tc->sharded, "node exchange needs an unsharded tree");
        *n_out = 0;
        if (!m) return MKV_OK;
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        DevGuard g(t->dev);
        uint64_t cnt = 0;
        const uint8_t *lvl = level_ptr(t, level, &cnt);
        uint64_t *di = ens<uint64_t>(t->x_idx, m);
        uint8_t *dp = ens<uint8_t>(t->x_dig, 32 * m);
        uint8_t *df = ens<uint8_t>(t->x_flag, m);
        MKV_HIP(hipMemcpyAsync(di, idx, m * 8, hipMemcpyHostToDevice, t->st));
        MKV_HIP(hipMemcpyAsync(dp, peer, 32 * m, hipMemcpyHostToDevice, t->st));
        launch_compare_nodes(lvl ? lvl : dp, cnt, di, dp, m, df, t->st);
        std::vector<uint8_t> hf(m);
        MKV_HIP(hipMemcpyAsync(hf.data(), df, m, hipMemcpyDeviceToHost, t->st));
        MKV_HIP(hipStreamSynchronize(t->st));
        uint64_t k = 0;
        for (uint64_t i = 0; i < m; ++i)
            if (hf[i]) out_idx[k++] = idx[i];
        *n_out = k;
    });
}

mkv_status mkv_tree_keys_at(const mkv_tree *tc, const uint64_t *pos, uint64_t m, mkv_keylist **out) {
    MKV_TRY({
        NEED(tc && out && (m == 0 || pos), "null argument");
        *out = nullptr;  // valid right after mkv_shard_prepare too (sorted keys exist; shard range checks)
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        for (uint64_t i = 0; i < m; ++i) NEED(pos[i] < t->n, "leaf position out of range");
        DevGuard g(t->dev);
        uint64_t *refs = ens<uint64_t>(t->x_idx, m + 1);
        if (m) MKV_HIP(hipMemcpyAsync(refs, pos, m * 8, hipMemcpyHostToDevice, t->st));
        const DiffSide A = side_of(t);
        *out = keylist_from_refs(t, refs, m, A, A, nullptr, t->klen_fixed);
    });
}

mkv_status mkv_tree_prefix_root(const mkv_tree *tc, const uint8_t *prefix, uint64_t plen, uint8_t out32[32],
                                int *has_root) {
    MKV_TRY({
        NEED(tc && out32 && has_root, "null argument");
        NEED(plen == 0 || prefix, "null prefix");
        NEED(!tc->prepared && !tc->sharded, "prefix root needs an unsharded tree");
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        DevGuard g(t->dev);
        *has_root = 0;
        std::memset(out32, 0, 32);
        if (t->n == 0) return MKV_OK;
        uint64_t lo = 0, hi = t->n;
        if (plen) {
            uint8_t *dp = ens<uint8_t>(t->d_out, plen + 16);
            MKV_HIP(hipMemcpyAsync(dp, prefix, plen, hipMemcpyHostToDevice, t->st));
            uint64_t *lohi = ens<uint64_t>(t->s_misc, 64);
            launch_prefix_bounds(side_of(t), dp, (uint32_t)plen, lohi, t->st);
            small_d2h(t, t->h_small, lohi, 16, t->st);
            sync(t);
            lo = t->h_small[0];
            hi = t->h_small[1];
        }
        if (hi <= lo) return MKV_OK;
        const uint64_t c = hi - lo;
        // fresh reduction over leaves [lo, hi): a temporary plan on a scratch node buffer
        mkv_tree tmp;  // only its plan vectors are used
        plan_levels(&tmp, 0, c, c);
        uint64_t tn = total_nodes(&tmp);
        uint8_t *nodes = ens<uint8_t>(t->s_nodes2, tn * 32 + 64);
        MKV_HIP(hipMemcpyAsync(nodes, t->nodes.as<uint8_t>() + 32 * lo, 32 * c, hipMemcpyDeviceToDevice, t->st));
        tmp.st = t->st;
        run_reduce(&tmp, nodes);
        const size_t L = tmp.lev_S.size();
        MKV_HIP(hipMemcpyAsync(out32, nodes + 32 * tmp.lev_off[L - 1], 32, hipMemcpyDeviceToHost, t->st));
        MKV_HIP(hipStreamSynchronize(t->st));
        tmp.st = nullptr;
        *has_root = 1;
    });
}

mkv_status mkv_tree_hash_pattern(const mkv_tree *t, const uint8_t *pattern, uint64_t plen, uint8_t out32[32],
                                 int *has_root) {
    // server.rs:651-656: None, "" and "*" all mean scan("") (every key); anything else is a prefix
    if (plen == 0 || (plen == 1 && pattern && pattern[0] == '*')) return mkv_tree_prefix_root(t, nullptr, 0, out32, has_root);
    return mkv_tree_prefix_root(t, pattern, plen, out32, has_root);
}

mkv_status mkv_keylist_get(const mkv_keylist *l, uint64_t *n, const uint8_t **bytes, const uint64_t **offsets) {
    MKV_TRY({
        NEED(l && n, "null argument");
        *n = l->n;
        if (bytes || offsets) const_cast<mkv_keylist *>(l)->wait();  // a list still being copied out
        if (bytes) *bytes = l->bytes;
        if (offsets) *offsets = l->offsets;
    });
}

void mkv_keylist_free(mkv_keylist *l) { delete l; }

// ---------------- sharded ----------------
mkv_status mkv_shard_prepare(mkv_tree *t, mkv_blob keys, mkv_blob values, int on_device, uint64_t *n_local) {
    MKV_TRY({
        NEED(t && n_local, "null argument");
        NEED(keys.n == values.n, "keys.n != values.n");
        DevGuard g(t->dev);
        const uint64_t n = keys.n;
        const uint8_t *kb, *vb;
        const uint64_t *koff, *voff;
        uint64_t staged_kbytes = 0;
        if (on_device) {
            need_device_blob(keys, "keys");
            need_device_blob(values, "values");
            kb = keys.bytes;
            koff = keys.offsets;
            vb = values.bytes;
            voff = values.offsets;
        } else {
            check_blob(keys, "keys");
            check_blob(values, "values");
            const uint64_t kbn = n ? keys.offsets[n] - keys.offsets[0] : 0;
            const uint64_t vbn = n ? values.offsets[n] - values.offsets[0] : 0;
            ens<uint8_t>(t->s_kb, kbn + 16);
            ens<uint64_t>(t->s_koff, n + 1);
            ens<uint8_t>(t->s_vb, vbn + 16);
            ens<uint64_t>(t->s_voff, n + 1);
            upload_blob(t, keys, t->s_kb, t->s_koff);
            upload_blob(t, values, t->s_vb, t->s_voff);
            kb = t->s_kb.as<uint8_t>();
            koff = t->s_koff.as<uint64_t>();
            vb = t->s_vb.as<uint8_t>();
            voff = t->s_voff.as<uint64_t>();
            staged_kbytes = kbn;
        }
        size_t ptot = prof_begin(t, "total_build");
        uint8_t *dig = ens<uint8_t>(t->s_dig, (n ? n : 1) * 32);
        fork_streams(t);
        size_t pl = prof_begin(t, "leaf_hash");
        // device inputs: the key-ownership copy rides on the leaf hash as in the unsharded build (at 125M
        // keys per rank a separate copy is 4 GB of keys + 1 GB of offsets on the critical stream)
        uint64_t kcap = 0;
        bool ko_fused = false;
        leaf_hash_owning_keys(t, kb, koff, vb, voff, n, dig, !on_device, &kcap, &ko_fused);
        prof_end(t, pl);
        sort_dedup_gather(t, kb, koff, n, nullptr, !on_device, staged_kbytes, true, kcap, ko_fused);  // gather fused into reduce
        prof_end(t, ptot);
        sync(t);
        t->prepared = true;
        t->sharded = true;
        t->has_root = false;
        t->combine_pending = false;
        *n_local = t->n;
    });
}

mkv_status mkv_shard_reduce(mkv_tree *t, uint64_t global_offset, uint64_t global_n) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(t->prepared, "mkv_shard_prepare first");
        NEED(global_offset + t->n <= global_n, "shard outside the global range");
        DevGuard g(t->dev);
        t->goff = global_offset;
        t->gN = global_n;
        plan_levels(t, global_offset, t->n, global_n);
        const uint64_t need = total_nodes(t);
        if (need * 32 + 64 > t->nodes.cap) {
            // grow while keeping the leaf level
            DevBuf tmp;
            tmp.ensure(32 * (t->n ? t->n : 1));
            if (t->n) MKV_HIP(hipMemcpyAsync(tmp.p, t->nodes.p, 32 * t->n, hipMemcpyDeviceToDevice, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
            t->nodes.ensure(need * 32 + 64);
            if (t->n) MKV_HIP(hipMemcpyAsync(t->nodes.p, tmp.p, 32 * t->n, hipMemcpyDeviceToDevice, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
        }
        size_t ptot = prof_begin(t, "total_build");
        size_t pr = prof_begin(t, "reduce");
        if (t->gather_pending)
            run_reduce(t, t->nodes.as<uint8_t>(), t->perm.as<uint32_t>(), t->s_dig.as<uint8_t>());
        else
            run_reduce(t, t->nodes.as<uint8_t>());
        t->gather_pending = false;
        prof_end(t, pr);
        prof_end(t, ptot);
        sync(t);
        t->prepared = false;
        t->has_root = false;
    });
}

namespace {
struct FringeEntry {
    uint32_t level;
    uint32_t valid;
    uint64_t idx;
    uint8_t h[32];
};
static_assert(sizeof(FringeEntry) == MKV_FRINGE_ENTRY_BYTES, "fringe layout");
}  // namespace

// The fringe of a shard: owned nodes whose parent is not owned (<= 2 per level), as entries with their
// node-array index (digests filled by the caller).
static void fringe_entries(const mkv_tree *t, std::vector<FringeEntry> &fe, std::vector<uint32_t> &nodeidx) {
    const size_t L = t->lev_S.size();
    for (size_t l = 0; l < L; ++l) {
        const uint64_t a = t->lev_base[l], c = t->lev_cnt[l];
        if (!c) continue;
        uint64_t cand[2] = {a, a + c - 1};
        for (int q = 0; q < 2; ++q) {
            if (q == 1 && cand[1] == cand[0]) break;
            const uint64_t x = cand[q];
            bool parent_owned = false;
            if (l + 1 < L) {
                const uint64_t p = x / 2, a2 = t->lev_base[l + 1], c2 = t->lev_cnt[l + 1];
                parent_owned = p >= a2 && p < a2 + c2;
            }
            if (parent_owned) continue;
            FringeEntry e{};
            e.level = (uint32_t)l;
            e.valid = 1;
            e.idx = x;
            fe.push_back(e);
            nodeidx.push_back((uint32_t)(t->lev_off[l] + (x - a)));
        }
    }
    NEED(fe.size() <= MKV_FRINGE_MAX_ENTRIES, "fringe overflow");
}

mkv_status mkv_shard_fringe(const mkv_tree *tc, uint8_t *out) {
    MKV_TRY({
        NEED(tc && out, "null argument");
        NEED(!tc->prepared, "mkv_shard_reduce first");
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        DevGuard g(t->dev);
        std::memset(out, 0, MKV_FRINGE_BYTES);
        std::vector<FringeEntry> fe;
        std::vector<uint32_t> nodeidx;
        fringe_entries(t, fe, nodeidx);
        if (!fe.empty()) {
            uint32_t *didx = ens<uint32_t>(t->d_fr, fe.size() + 64);
            uint8_t *dh = ens<uint8_t>(t->d_seam, fe.size() * 32 + 64);
            MKV_HIP(hipMemcpyAsync(didx, nodeidx.data(), nodeidx.size() * 4, hipMemcpyHostToDevice, t->st));
            launch_gather_digests(didx, t->nodes.as<uint8_t>(), fe.size(), dh, t->st);
            std::vector<uint8_t> hh(fe.size() * 32);
            MKV_HIP(hipMemcpyAsync(hh.data(), dh, hh.size(), hipMemcpyDeviceToHost, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
            for (size_t i = 0; i < fe.size(); ++i) std::memcpy(fe[i].h, hh.data() + 32 * i, 32);
        }
        std::memcpy(out, fe.data(), fe.size() * sizeof(FringeEntry));
    });
}

// Pinned staging of at least `bytes` (seam inputs / fringe headers).
static uint8_t *seam_staging(mkv_tree *t, size_t bytes) {
    if (!t->h_seam || t->h_seam_cap < bytes) {
        if (t->h_seam) MKV_HIP(hipHostFree(t->h_seam));
        t->h_seam = nullptr;
        t->h_seam_cap = bytes + 4096;
        MKV_HIP(hipHostMalloc(reinterpret_cast<void **>(&t->h_seam), t->h_seam_cap, hipHostMallocDefault));
    }
    return t->h_seam;
}

mkv_status mkv_shard_fringe_device(const mkv_tree *tc, uint8_t *dout) {
    MKV_TRY({
        NEED(tc && dout, "null argument");
        NEED(!tc->prepared, "mkv_shard_reduce first");
        mkv_tree *t = const_cast<mkv_tree *>(tc);
        DevGuard g(t->dev);
        std::vector<FringeEntry> fe;
        std::vector<uint32_t> nodeidx;
        fringe_entries(t, fe, nodeidx);
        // headers (and zeroed slots) from pinned staging, digests gathered on the device in place
        uint8_t *h = seam_staging(t, MKV_FRINGE_BYTES + 4 * (nodeidx.size() + 1));
        std::memset(h, 0, MKV_FRINGE_BYTES);
        if (!fe.empty()) std::memcpy(h, fe.data(), fe.size() * sizeof(FringeEntry));
        if (!nodeidx.empty()) std::memcpy(h + MKV_FRINGE_BYTES, nodeidx.data(), 4 * nodeidx.size());
        uint32_t *didx = ens<uint32_t>(t->d_fr, nodeidx.size() + 64);
        MKV_HIP(hipMemcpyAsync(dout, h, MKV_FRINGE_BYTES, hipMemcpyHostToDevice, t->st));
        if (!nodeidx.empty()) {
            MKV_HIP(hipMemcpyAsync(didx, h + MKV_FRINGE_BYTES, 4 * nodeidx.size(), hipMemcpyHostToDevice, t->st));
            launch_fringe_digests(t->nodes.as<uint8_t>(), didx, (uint32_t)nodeidx.size(), dout, t->st);
        }
        wait_stream(t, t->st);  // dout is complete before the caller's collective reads it
    });
}

mkv_status mkv_shard_combine(mkv_tree *t, const uint8_t *fringes, uint32_t world, uint64_t global_n,
                             uint8_t out32[32], int *has_root) {
    MKV_TRY({
        NEED(t && fringes && out32 && has_root, "null argument");
        DevGuard g(t->dev);
        *has_root = 0;
        std::memset(out32, 0, 32);
        if (global_n == 0) return MKV_OK;
        std::vector<FringeEntry> all;
        for (uint32_t r = 0; r < world; ++r) {
            const FringeEntry *f = reinterpret_cast<const FringeEntry *>(fringes + (size_t)r * MKV_FRINGE_BYTES);
            for (int i = 0; i < MKV_FRINGE_MAX_ENTRIES && f[i].valid; ++i) all.push_back(f[i]);
        }
        std::sort(all.begin(), all.end(), [](const FringeEntry &x, const FringeEntry &y) {
            return x.level != y.level ? x.level < y.level : x.idx < y.idx;
        });
        std::vector<uint64_t> S;
        for (uint64_t s = global_n;; s = (s + 1) / 2) {
            S.push_back(s);
            if (s == 1) break;
        }
        // one pinned staging block: [S (64 x u64) | entries]; the root comes back through h_small
        const size_t sbytes = 64 * 8, ebytes = all.size() * sizeof(FringeEntry);
        seam_staging(t, sbytes + ebytes);
        NEED(S.size() <= 64, "too many levels");
        std::memcpy(t->h_seam, S.data(), S.size() * 8);
        if (ebytes) std::memcpy(t->h_seam + sbytes, all.data(), ebytes);
        uint8_t *dst = ens<uint8_t>(t->d_seam, sbytes + ebytes + 64);
        uint8_t *droot = ens<uint8_t>(t->d_fr, 64);
        MKV_HIP(hipMemcpyAsync(dst, t->h_seam, sbytes + ebytes, hipMemcpyHostToDevice, t->st));
        MKV_HIP(hipMemsetAsync(droot, 0, 32, t->st));
        launch_seam_combine(dst + sbytes, (uint32_t)all.size(), reinterpret_cast<const uint64_t *>(dst),
                            (uint32_t)S.size(), nullptr, droot, t->st);
        small_d2h(t, t->h_small, droot, 32, t->st);
        wait_stream(t, t->st);
        std::memcpy(out32, t->h_small, 32);
        *has_root = 1;
        std::memcpy(t->root, out32, 32);
        t->has_root = true;
        t->combine_pending = false;
    });
}

mkv_status mkv_shard_combine_device(mkv_tree *t, const uint8_t *dfringes, uint32_t world, uint64_t stride_bytes,
                                   uint64_t global_n, uint8_t out32[32], int *has_root) {
    MKV_TRY({
        NEED(t && dfringes && out32 && has_root, "null argument");
        NEED(world >= 1 && world <= 64, "world must be 1..64");
        NEED(stride_bytes >= MKV_FRINGE_BYTES && stride_bytes % 16 == 0, "bad fringe stride");
        DevGuard g(t->dev);
        *has_root = 0;
        std::memset(out32, 0, 32);
        if (global_n == 0) return MKV_OK;
        std::vector<uint64_t> S;
        for (uint64_t s = global_n;; s = (s + 1) / 2) {
            S.push_back(s);
            if (s == 1) break;
        }
        NEED(S.size() <= 64, "too many levels");
        uint8_t *h = seam_staging(t, 64 * 8);
        std::memcpy(h, S.data(), S.size() * 8);
        const size_t sbytes = 64 * 8, ebytes = (size_t)world * MKV_FRINGE_MAX_ENTRIES * sizeof(FringeEntry);
        uint8_t *dst = ens<uint8_t>(t->d_seam, sbytes + ebytes + 64);
        uint8_t *droot = ens<uint8_t>(t->d_fr, 64);
        MKV_HIP(hipMemcpyAsync(dst, h, sbytes, hipMemcpyHostToDevice, t->st));
        MKV_HIP(hipMemsetAsync(droot, 0, 32, t->st));
        launch_seam_prep_combine(dfringes, world, stride_bytes, MKV_FRINGE_MAX_ENTRIES,
                                 reinterpret_cast<const uint64_t *>(dst), (uint32_t)S.size(), dst + sbytes,
                                 reinterpret_cast<uint32_t *>(droot + 32), droot, t->st);
        small_d2h(t, t->h_small, droot, 32, t->st);
        wait_stream(t, t->st);
        std::memcpy(out32, t->h_small, 32);
        *has_root = 1;
        std::memcpy(t->root, out32, 32);
        t->has_root = true;
        t->combine_pending = false;
    });
}

// ---------------- redistribution of unpartitioned input ----------------
mkv_status mkv_route_sample(mkv_tree *t, mkv_blob keys, uint32_t m, uint64_t *samples_dev) {
    MKV_TRY({
        NEED(t && (samples_dev || m == 0), "null argument");
        NEED(keys.n == 0 || keys.offsets, "keys: null offsets");
        NEED(m <= keys.n, "more samples than records");
        DevGuard g(t->dev);
        need_device_blob(keys, "keys");
        need_device_ptr(samples_dev, "samples");
        launch_route_sample(keys.bytes, keys.offsets, keys.n, m, samples_dev, t->st);
        wait_stream(t, t->st);
    });
}

mkv_status mkv_route_splitters(const uint64_t *samples, uint64_t ns, uint32_t world, uint64_t *splitters) {
    MKV_TRY({
        NEED(world >= 1 && world <= MKV_ROUTE_MAX_WORLD, "world must be 1..256");
        NEED((samples || ns == 0) && (splitters || world == 1), "null argument");
        std::vector<uint64_t> s(samples, samples + ns);
        std::sort(s.begin(), s.end());
        // splitter r cuts at the sample of rank (r + 1) / world: each range gets ~1/world of the samples
        for (uint32_t r = 0; r + 1 < world; ++r)
            splitters[r] = ns ? s[std::min<uint64_t>(ns - 1, ((uint64_t)(r + 1) * ns) / world)] : ~0ull;
    });
}

mkv_status mkv_route_plan(mkv_tree *t, mkv_blob keys, mkv_blob values, uint32_t world, const uint64_t *splitters,
                          uint64_t *counts) {
    MKV_TRY({
        NEED(t && counts && (splitters || world == 1), "null argument");
        NEED(world >= 1 && world <= MKV_ROUTE_MAX_WORLD, "world must be 1..256");
        NEED(keys.n == values.n, "keys.n != values.n");
        NEED(keys.n == 0 || (keys.offsets && values.offsets), "null offsets");
        for (uint32_t r = 1; r + 1 < world; ++r) NEED(splitters[r - 1] <= splitters[r], "splitters not sorted");
        DevGuard g(t->dev);
        need_device_blob(keys, "keys");
        need_device_blob(values, "values");
        const uint64_t n = keys.n;
        t->rt_perm = nullptr;
        t->rt_n = 0;
        uint8_t *h = seam_staging(t, 3 * 8 * (size_t)MKV_ROUTE_MAX_WORLD + 8 * (size_t)MKV_ROUTE_MAX_WORLD);
        uint64_t *dspl = ens<uint64_t>(t->rt_spl, MKV_ROUTE_MAX_WORLD);
        uint64_t *dcnt = ens<uint64_t>(t->rt_cnt, 3 * MKV_ROUTE_MAX_WORLD);
        if (world > 1) {
            std::memcpy(h, splitters, 8 * (world - 1));
            MKV_HIP(hipMemcpyAsync(dspl, h, 8 * (world - 1), hipMemcpyHostToDevice, t->st));
        }
        MKV_HIP(hipMemsetAsync(dcnt, 0, 3 * 8 * world, t->st));
        uint64_t *k1 = ens<uint64_t>(t->s_k1, n + 1);
        uint64_t *k2 = ens<uint64_t>(t->s_k2, n + 1);
        uint32_t *v1 = ens<uint32_t>(t->s_v1, n + 1);
        uint32_t *v2 = ens<uint32_t>(t->s_v2, n + 1);
        void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n), scan_scratch_bytes(n + 1)));
        launch_route_dest(keys.bytes, keys.offsets, values.offsets, n, dspl, world, k1, dcnt, t->st);
        launch_iota_u32(v1, n, t->st);
        int bits = 0;
        while ((1u << bits) < world) ++bits;
        // one stable 8-bit pass (world <= 256): records grouped by destination, source order kept
        const bool sw = radix_sort_pairs(k1, v1, k2, v2, n, 0, bits, radix, t->st);
        MKV_HIP(hipMemcpyAsync(h + 8 * MKV_ROUTE_MAX_WORLD, dcnt, 3 * 8 * world, hipMemcpyDeviceToHost, t->st));
        wait_stream(t, t->st);
        const uint64_t *hc = reinterpret_cast<const uint64_t *>(h + 8 * MKV_ROUTE_MAX_WORLD);
        for (uint32_t r = 0; r < world; ++r) {  // counts is world x 3 (row per destination)
            counts[3 * r + 0] = hc[r];
            counts[3 * r + 1] = hc[world + r];
            counts[3 * r + 2] = hc[2 * world + r];
        }
        uint32_t *perm = ens<uint32_t>(t->rt_pbuf, n + 1);
        if (n) MKV_HIP(hipMemcpyAsync(perm, sw ? v2 : v1, 4 * n, hipMemcpyDeviceToDevice, t->st));
        wait_stream(t, t->st);
        t->rt_perm = perm;
        t->rt_n = n;
        t->rt_kb = keys.bytes;
        t->rt_koff = keys.offsets;
        t->rt_vb = values.bytes;
        t->rt_voff = values.offsets;
    });
}

mkv_status mkv_route_pack(mkv_tree *t, mkv_blob keys, mkv_blob values, uint8_t *kout, uint32_t *klen, uint8_t *vout,
                          uint32_t *vlen) {
    MKV_TRY({
        NEED(t, "tree is null");
        NEED(keys.n == values.n, "keys.n != values.n");
        NEED(t->rt_perm || keys.n == 0, "mkv_route_plan first");
        NEED(keys.n == t->rt_n && keys.bytes == t->rt_kb && keys.offsets == t->rt_koff &&
                 values.bytes == t->rt_vb && values.offsets == t->rt_voff,
             "mkv_route_pack: not the blobs of the last mkv_route_plan");
        const uint64_t n = keys.n;
        if (n == 0) return MKV_OK;
        NEED(kout && klen && vout && vlen, "null output");
        DevGuard g(t->dev);
        need_device_blob(values, "values");
        for (const void *p : {(const void *)kout, (const void *)klen, (const void *)vout, (const void *)vlen})
            need_device_ptr(p, "route_pack output");
        uint64_t *off = ens<uint64_t>(t->s_lens, n + 1);
        uint32_t *bad = ens<uint32_t>(t->s_misc, 64) + 8;
        void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n), scan_scratch_bytes(n + 1)));
        MKV_HIP(hipMemsetAsync(bad, 0, 4, t->st));
        for (int side = 0; side < 2; ++side) {
            const mkv_blob &b = side ? values : keys;
            launch_gather_keylens(t->rt_perm, b.offsets, n, off, t->st);
            exclusive_scan_u64(off, off, n, off + n, radix, t->st);
            launch_gather_keys(t->rt_perm, b.bytes, b.offsets, off, n, side ? vout : kout, t->st);
            launch_route_lens(t->rt_perm, b.offsets, n, side ? vlen : klen, bad, t->st);
        }
        small_d2h(t, t->h_small, bad, 4, t->st);
        wait_stream(t, t->st);
        NEED(reinterpret_cast<const uint32_t *>(t->h_small)[0] == 0, "a key or value of 4 GiB or more");
    });
}

mkv_status mkv_route_offsets(mkv_tree *t, const uint32_t *lens, uint64_t n, uint64_t *offs) {
    MKV_TRY({
        NEED(t && offs && (lens || n == 0), "null argument");
        DevGuard g(t->dev);
        need_device_ptr(lens, "lens");
        need_device_ptr(offs, "offs");
        if (n == 0) {
            MKV_HIP(hipMemsetAsync(offs, 0, 8, t->st));
        } else {
            void *radix = t->s_radix.ensure(std::max(radix_scratch_bytes(n), scan_scratch_bytes(n + 1)));
            launch_u32_to_u64(lens, n, offs, t->st);
            exclusive_scan_u64(offs, offs, n, offs + n, radix, t->st);
        }
        wait_stream(t, t->st);
    });
}

// ---------------- utilities ----------------
mkv_status mkv_prof_enable(mkv_tree *t, int on) {
    MKV_TRY({
        NEED(t, "tree is null");
        t->prof = on != 0;
    });
}
mkv_status mkv_prof_reset(mkv_tree *t) {
    MKV_TRY({
        NEED(t, "tree is null");
        t->pg.clear();
    });
}
mkv_status mkv_prof_read(const mkv_tree *t, const char *group, double *total_ms, uint64_t *count) {
    MKV_TRY({
        NEED(t && group && total_ms && count, "null argument");
        sync(const_cast<mkv_tree *>(t));  // collect event pairs of work still in flight (async copies)
        auto it = t->pg.find(group);
        *total_ms = it == t->pg.end() ? 0.0 : it->second.first;
        *count = it == t->pg.end() ? 0 : it->second.second;
    });
}

mkv_status mkv_tree_update_counts(const mkv_tree *t, uint64_t *out, uint32_t cap, uint32_t *nlevels) {
    MKV_TRY({
        NEED(t && nlevels && (out || cap == 0), "null argument");
        const uint32_t L = (uint32_t)t->lev_S.size();
        *nlevels = L;
        if (!t->u_cnt.p || L == 0) {
            *nlevels = 0;
            return MKV_OK;
        }
        DevGuard g(t->dev);
        MKV_HIP(hipStreamSynchronize(t->st));
        // the last update's counters, copied to the host (and reset on the device) when it ended
        const uint32_t *h = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t->h_small) + UCNT_HOST);
        for (uint32_t l = 0; l < L && l < cap; ++l)  // levels above the climb: rehashed whole
            out[l] = (t->upd_dense_from >= 0 && (int)l > t->upd_dense_from) ? t->lev_cnt[l] : h[l];
    });
}

mkv_status mkv_tree_walk_stats(const mkv_tree *t, uint64_t out[4]) {
    MKV_TRY({
        NEED(t && out, "null argument");
        out[0] = out[1] = out[2] = out[3] = 0;
        if (!t->td_cnt.p || t->walk_L == 0) return MKV_OK;
        DevGuard g(t->dev);
        const uint32_t L = t->walk_L;
        std::vector<uint32_t> h(L + 1);
        MKV_HIP(hipStreamSynchronize(t->st));
        MKV_HIP(hipMemcpy(h.data(), t->td_cnt.p, 4ull * (L + 1), hipMemcpyDeviceToHost));
        // a frontier entry at level l expanded to level lt compares its 2^(l-lt) descendants in the base
        // and in its variant (32 B each); the seed compares the k + 1 roots
        uint64_t entries = t->walk_k, bytes = 32ull * (t->walk_k + 1);
        for (auto &j : t->walk_jumps) {
            const uint64_t c = h[j.first];
            entries += c;
            bytes += c * 2ull * 32ull * (1ull << (j.first - j.second));
        }
        out[0] = entries;
        out[1] = bytes;
        out[2] = h[0];
        out[3] = t->walk_jumps.size() + 1 - t->walk_fused;  // launches (the one-workgroup top counts once)
    });
}

mkv_status mkv_gen_records_device(int hip_device, uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen,
                                  uint32_t vlen, uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb,
                                  uint64_t *koff, uint8_t *vb, uint64_t *voff) {
    MKV_TRY({
        NEED(kb && koff && vb && voff, "null buffer");
        NEED(nshards >= 1 && nshards <= 64 && shard < nshards, "bad shard spec");
        DevGuard g(hip_device);
        launch_gen_records(seed, idx0, n, klen, vlen, shard, nshards, vfield, kb, koff, vb, voff, nullptr);
        MKV_HIP(hipDeviceSynchronize());
    });
}

mkv_status mkv_gen_records_ragged_device(int hip_device, uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen,
                                         uint32_t vlen, uint32_t shard, uint32_t nshards, uint32_t vfield, uint8_t *kb,
                                         uint64_t *koff, uint8_t *vb, uint64_t *voff) {
    MKV_TRY({
        NEED(kb && koff && vb && voff, "null buffer");
        NEED(nshards >= 1 && nshards <= 64 && shard < nshards, "bad shard spec");
        NEED(klen >= 1, "klen must be >= 1");
        DevGuard g(hip_device);
        void *scratch = nullptr;
        MKV_HIP(hipMalloc(&scratch, scan_scratch_bytes(n + 1) + 256));
        try {
            launch_gen_records_ragged(seed, idx0, n, klen, vlen, shard, nshards, vfield, kb, koff, vb, voff, scratch,
                                      nullptr);
            MKV_HIP(hipDeviceSynchronize());
        } catch (...) {
            (void)hipFree(scratch);
            throw;
        }
        MKV_HIP(hipFree(scratch));
    });
}

mkv_status mkv_leaf_digests(int hip_device, mkv_blob keys, mkv_blob values, uint8_t *out) {
    MKV_TRY({
        NEED(out || keys.n == 0, "null out");
        NEED(keys.n == values.n, "keys.n != values.n");
        check_blob(keys, "keys");
        check_blob(values, "values");
        mkv_tree *t = nullptr;
        mkv_status s = mkv_tree_create(hip_device, &t);
        if (s != MKV_OK) throw Error(s, g_err);
        try {
            DevGuard g(t->dev);
            const uint64_t n = keys.n;
            ens<uint8_t>(t->s_kb, (n ? keys.offsets[n] - keys.offsets[0] : 0) + 16);
            ens<uint64_t>(t->s_koff, n + 1);
            ens<uint8_t>(t->s_vb, (n ? values.offsets[n] - values.offsets[0] : 0) + 16);
            ens<uint64_t>(t->s_voff, n + 1);
            upload_blob(t, keys, t->s_kb, t->s_koff);
            upload_blob(t, values, t->s_vb, t->s_voff);
            uint8_t *dig = ens<uint8_t>(t->s_dig, (n ? n : 1) * 32);
            // the build's leaf stage (k_leaf_direct, then k_leaf_ragged for other shapes)
            launch_leaf_hash(t->s_kb.as<uint8_t>(), t->s_koff.as<uint64_t>(), t->s_vb.as<uint8_t>(),
                             t->s_voff.as<uint64_t>(), n, dig, ens<uint32_t>(t->leaf_ctr, leaf_ctr_words(n)), t->st);
            if (n) MKV_HIP(hipMemcpyAsync(out, dig, 32 * n, hipMemcpyDeviceToHost, t->st));
            MKV_HIP(hipStreamSynchronize(t->st));
        } catch (...) {
            mkv_tree_destroy(t);
            throw;
        }
        mkv_tree_destroy(t);
    });
}

}  // extern "C"

// ---------------- internals shared with comm.cpp (device-resident sharded collectives) ----------------
namespace mkv {
DevKeys tree_diff_device(const mkv_tree *a, const mkv_tree *b) {
    if (!a || !b) throw Error(ST_EINVAL, "null argument");
    if (a->dev != b->dev) throw Error(ST_EINVAL, "trees on different devices");
    if (a->prepared || b->prepared) throw Error(ST_ESTATE, "shard_reduce pending");
    DevGuard g(a->dev);
    DevKeys d;
    diff_pair(a, b, &d);
    return d;
}
DevKeys tree_keys_at_device(const mkv_tree *tc, const uint64_t *pos, uint64_t m) {
    mkv_tree *t = const_cast<mkv_tree *>(tc);
    for (uint64_t i = 0; i < m; ++i)
        if (pos[i] >= t->n) throw Error(ST_EINVAL, "leaf position out of range");
    DevGuard g(t->dev);
    uint64_t *refs = ens<uint64_t>(t->x_idx, m + 1);
    if (m) MKV_HIP(hipMemcpyAsync(refs, pos, m * 8, hipMemcpyHostToDevice, t->st));
    const DiffSide A = side_of(t);
    DevKeys d;
    keys_from_refs_dev(t, refs, m, A, A, nullptr, &d);
    return d;
}
hipStream_t tree_stream(const mkv_tree *t) { return t->st; }
void wait_bounded(hipStream_t s) { wait_idle(s); }
int tree_device(const mkv_tree *t) { return t->dev; }
uint64_t tree_len(const mkv_tree *t) { return t->n; }
// One copy of a device key list (offsets[0..n], offsets[0] == 0, then the bytes) into a pinned block on
// stream st; complete on return.
mkv_keylist *keylist_from_device(const uint64_t *d_off, const uint8_t *d_kb, uint64_t n, uint64_t bytes, hipStream_t st) {
    auto *l = new mkv_keylist();
    if (!n) return l;
    try {
        const uint64_t kpos = (8 * (n + 1) + 15) & ~uint64_t(15);
        l->blk = std::make_shared<PinnedBlock>(kpos + bytes + 16);
        MKV_HIP(hipMemcpyAsync(l->blk->p, d_off, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        if (bytes) MKV_HIP(hipMemcpyAsync(l->blk->p + kpos, d_kb, bytes, hipMemcpyDeviceToHost, st));
        wait_idle(st);
        l->offsets = reinterpret_cast<const uint64_t *>(l->blk->p);
        l->bytes = l->blk->p + kpos;
        l->n = n;
    } catch (...) {
        delete l;
        throw;
    }
    return l;
}
}  // namespace mkv
