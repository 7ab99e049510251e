// comm.cpp — multi-GPU key-range shards behind the C ABI: a communicator (RCCL inside the
// library, or the caller's host all-gather) and the sharded build / root / diff that run the collectives
// themselves, so a host in any language (the reference's Rust SyncManager, sync.rs:56-87) gets the global
// root and the divergent-key list without a collective layer of its own.
//
// RCCL is loaded at run time: the already-resident copy when there is one (a PyTorch process has its own
// librccl loaded; two RCCL instances in one process would each bring up the devices), else
// librccl.so.1 from ROCm, with RTLD_LOCAL so its symbols never interpose on anyone else's.
//
// Every operation starts with a META all-gather: 32 bytes per rank = {status, three words} (leaf count and
// the shard's first / last key lengths; a diff's key count and byte count). A rank whose local step failed
// (bad blob, out of memory, ...) still joins it with its error code, so every rank returns the error
// together instead of waiting forever in a collective the failed rank never reaches; every later
// collective of the operation carries the same status word in its block header. The host reads these words
// back because it needs them for control flow (offsets, buffer sizes): counted as `meta` bytes.
// PAYLOADS never pass through the host in the RCCL form: the range check's boundary keys, the seam fringes
// and the diff's key lists are packed on the device, all-gathered device to device, checked and compacted
// by kernels; the only device -> host copy of a diff is its final result. mkv_comm_traffic reports the
// host-staged payload bytes per kind (0 for the RCCL form's sharded operations).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "mkv_merkle.h"

using namespace mkv;

namespace {

struct Rccl {
    void *h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char *name : {"librccl.so", "librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);  // a copy already in the process
            if (r.h) break;
        }
        if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) return;
        auto sym = [](const char *n) { return dlsym(r.h, n); };
        r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(sym("ncclGetUniqueId"));
        r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(sym("ncclCommInitRank"));
        r.AllGather = reinterpret_cast<decltype(r.AllGather)>(sym("ncclAllGather"));
        r.Send = reinterpret_cast<decltype(r.Send)>(sym("ncclSend"));
        r.Recv = reinterpret_cast<decltype(r.Recv)>(sym("ncclRecv"));
        r.GroupStart = reinterpret_cast<decltype(r.GroupStart)>(sym("ncclGroupStart"));
        r.GroupEnd = reinterpret_cast<decltype(r.GroupEnd)>(sym("ncclGroupEnd"));
        r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(sym("ncclCommDestroy"));
        r.CommAbort = reinterpret_cast<decltype(r.CommAbort)>(sym("ncclCommAbort"));
        r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(sym("ncclGetErrorString"));
    });
    if (!r.GetUniqueId || !r.CommInitRank || !r.AllGather || !r.Send || !r.Recv || !r.GroupStart || !r.GroupEnd ||
        !r.CommDestroy || !r.CommAbort)
        throw Error(ST_EHIP, "RCCL not available (librccl.so.1 could not be loaded)");
    return r;
}

void check_nccl(ncclResult_t e, const char *what) {
    if (e != ncclSuccess) {
        const Rccl &r = rccl();
        throw Error(ST_EHIP, std::string(what) + ": " + (r.GetErrorString ? r.GetErrorString(e) : "RCCL error"));
    }
}

constexpr uint64_t HDR = 32;  // block header: status, three words (u64 each)
__host__ __device__ inline uint64_t up16(uint64_t x) { return (x + 15) & ~uint64_t(15); }
// A diff block of the RCCL form: header {status, n, bytes, 0} | offsets[0..n] | key bytes, each part
// 16-B aligned. Sized by the rank's own list, so the all-gather-v moves no padding.
__host__ __device__ inline uint64_t list_block_bytes(uint64_t n, uint64_t nb) { return up16(HDR + 8 * (n + 1)) + up16(nb); }

// ---------------- device side of the RCCL form ----------------
// Header words of this rank's block (kernel arguments: no host -> device copy).
__global__ void k_put_header(uint64_t *dst, uint64_t status, uint64_t w1, uint64_t w2, uint64_t w3) {
    if (threadIdx.x == 0) {
        dst[0] = status;
        dst[1] = w1;
        dst[2] = w2;
        dst[3] = w3;
    }
}

// Range-check block: header {status, n, len_first, len_last}, then the first and the last key zero-padded
// to W bytes each (keys = offsets[0..2] + bytes of the two keys at sorted positions 0 and n-1).
__global__ void k_pack_ends(uint8_t *dst, uint64_t status, uint64_t n, const uint64_t *off, const uint8_t *kb,
                            uint64_t W) {
    uint64_t *h = reinterpret_cast<uint64_t *>(dst);
    const uint64_t lf = n ? off[1] - off[0] : 0, ll = n ? off[2] - off[1] : 0;
    if (threadIdx.x == 0) {
        h[0] = status;
        h[1] = n;
        h[2] = lf;
        h[3] = ll;
    }
    for (uint64_t i = threadIdx.x; i < 2 * W; i += blockDim.x) {
        const bool second = i >= W;
        const uint64_t j = second ? i - W : i, len = second ? ll : lf;
        dst[HDR + i] = (n && j < len) ? kb[(second ? off[1] : off[0]) + j] : 0;
    }
}

// Verdict over `world` gathered blocks (block r at recv + r * stride; stride 0: diff blocks back to back,
// each sized by its own header): v[0] = first rank whose header status is non-zero (or ~0), v[1] = its
// status; ranges: v[2] = first non-empty rank whose first key is not above the previous non-empty rank's
// last key (Rust String order: bytes, then length), or ~0. One thread: the headers are a few words per rank.
__global__ void k_check_blocks(const uint8_t *recv, uint64_t stride, uint32_t world, int ranges, uint64_t W,
                               uint64_t *v) {
    if (threadIdx.x != 0) return;
    v[0] = ~0ull;
    v[1] = 0;
    v[2] = ~0ull;
    uint64_t at = 0;
    for (uint32_t r = 0; r < world; ++r) {
        const uint64_t *h = reinterpret_cast<const uint64_t *>(recv + (stride ? r * stride : at));
        if (h[0]) {
            v[0] = r;
            v[1] = h[0];
            return;
        }
        at += list_block_bytes(h[1], h[2]);
    }
    if (!ranges) return;
    int64_t prev = -1;
    for (uint32_t r = 0; r < world; ++r) {
        const uint64_t *h = reinterpret_cast<const uint64_t *>(recv + r * stride);
        if (!h[1]) continue;
        if (prev >= 0) {
            const uint64_t *hp = reinterpret_cast<const uint64_t *>(recv + (uint64_t)prev * stride);
            const uint8_t *last = recv + (uint64_t)prev * stride + HDR + W, *first = recv + r * stride + HDR;
            const uint64_t la = hp[3], lb = h[2], m = la < lb ? la : lb;
            int c = 0;
            for (uint64_t j = 0; j < m && !c; ++j) c = (int)last[j] - (int)first[j];
            if (!c) c = la < lb ? -1 : (la > lb ? 1 : 0);
            if (c >= 0) {
                v[2] = r;
                return;
            }
        }
        prev = r;
    }
}

// This rank's diff block (list_block_bytes(n, nb)): header {status, n, nb, 0}, offsets[0..n] at +HDR; the key
// bytes follow at +up16(HDR + 8 (n + 1)) (copied separately).
__global__ void k_pack_list(uint8_t *dst, uint64_t status, uint64_t n, uint64_t nb, const uint64_t *off) {
    uint64_t *h = reinterpret_cast<uint64_t *>(dst);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    if (t == 0) {
        h[0] = status;
        h[1] = n;
        h[2] = nb;
        h[3] = 0;
    }
    uint64_t *o = reinterpret_cast<uint64_t *>(dst + HDR);
    for (uint64_t i = t; i <= n; i += stride) o[i] = off ? off[i] : 0;
}

// Global list from the gathered blocks (back to back, each sized by its header): rank r's keys go to the key
// range [K_r, K_r + n_r) and byte range [B_r, B_r + nb_r), K / B = the sums over the ranks before r (ranges
// are ordered by rank, so the concatenation is the sorted, unique global list, merkle.rs:171-196).
// grid.y = rank.
__global__ void k_compact_lists(const uint8_t *recv, uint64_t *out_off, uint8_t *out_kb, uint64_t total_n) {
    const uint32_t r = blockIdx.y;
    uint64_t K = 0, B = 0, at = 0;
    for (uint32_t q = 0; q < r; ++q) {
        const uint64_t *h = reinterpret_cast<const uint64_t *>(recv + at);
        K += h[1];
        B += h[2];
        at += list_block_bytes(h[1], h[2]);
    }
    const uint8_t *blk = recv + at;
    const uint64_t n = reinterpret_cast<const uint64_t *>(blk)[1], nb = reinterpret_cast<const uint64_t *>(blk)[2];
    const uint64_t *off = reinterpret_cast<const uint64_t *>(blk + HDR);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = t; i < n; i += step) out_off[K + i] = B + off[i];
    const uint8_t *kb = blk + up16(HDR + 8 * (n + 1));
    for (uint64_t i = t; i < nb; i += step) out_kb[B + i] = kb[i];
    if (r == gridDim.y - 1 && t == 0) out_off[total_n] = B + nb;
}

// Runs a local step of a collective operation; a failure is recorded (code + message), not thrown, so
// the rank still joins the operation's next collective with its status word set.
template <class F> void local_step(int &code, std::string &err, F f) {
    if (code) return;
    try {
        f();
    } catch (const Error &e) {
        code = e.code ? e.code : ST_EINVAL;
        err = e.what();
    } catch (const std::exception &e) {
        code = ST_ENOMEM;  // std::bad_alloc of a host staging buffer, in practice
        err = e.what();
    }
}

}  // namespace

struct mkv_comm {
    int rank = 0, world = 1, dev = -1;
    // RCCL form
    ncclComm_t nc = nullptr;
    hipStream_t st = nullptr;
    bool aborted = false;                           // a collective wait failed: ncclCommAbort was called
    DevBuf din, dout;                               // block staging (send, world x recv), sized by the plan
    DevBuf dsin, dsout, dverdict;                   // status / meta words: reserved at creation, never grow
    DevBuf dres_off, dres_kb;                       // the gathered global diff list (after the last collective)
    uint64_t *h_meta = nullptr;                     // pinned: meta words (world x 4) and verdicts, reserved
    uint64_t h_meta_cap = 0;
    // host form
    mkv_allgather_fn fn = nullptr;
    void *ctx = nullptr;
    std::vector<uint8_t> hin, hout;                 // block staging of the host form (same plan rule)
    // Capacities every rank is known to hold for block staging: identical on all ranks (the same requests
    // arrive in the same order) and back to 0 when an operation fails collectively (a failed rank may have
    // lost its buffers).
    uint64_t plan_in = 0, plan_out = 0;
    int fault = 0;  // mkv_comm_inject_fault (test hook)
    // per collective kind (MKV_COLL_*): host wall seconds around the collective and the wait for its
    // result, calls, payload bytes per rank; host <-> device bytes moved around it (payload / meta words)
    double secs[MKV_COLL_KINDS] = {};
    uint64_t calls[MKV_COLL_KINDS] = {}, nbytes[MKV_COLL_KINDS] = {}, staged[MKV_COLL_KINDS] = {},
             metab[MKV_COLL_KINDS] = {};
    int kind = MKV_COLL_COUNTS;  // kind of the collectives issued next
    bool device_form() const { return nc != nullptr; }

    void usable() const {
        if (aborted)
            throw Error(ST_ESTATE, "communicator aborted after a collective wait failed (MKV_WAIT_TIMEOUT_S); "
                                   "create a new one on every rank");
    }
    // Bounded wait for the communicator's stream (the library's wait: MKV_EHIP after MKV_WAIT_TIMEOUT_S).
    // A collective that does not complete — a peer that never joined, a dead link — aborts the RCCL
    // communicator (ncclCommAbort), so this rank returns instead of blocking forever; later calls on it
    // fail with MKV_ESTATE.
    void wait() {
        try {
            wait_bounded(st);
        } catch (const Error &e) {
            if (nc) {
                (void)rccl().CommAbort(nc);
                nc = nullptr;
                aborted = true;
            }
            throw Error(ST_EHIP, std::string("collective did not complete: ") + e.what() + "; communicator aborted");
        }
    }
    // Reserved at creation: the meta / status rounds never allocate, so they can always be joined.
    void reserve_status() {
        dsin.ensure(HDR);
        dsout.ensure(HDR * world);
        dverdict.ensure(64);
        MKV_HIP(hipHostMalloc(reinterpret_cast<void **>(&h_meta), (4ull * world + 8) * 8, hipHostMallocDefault));
        h_meta_cap = 4ull * world + 8;
    }
    // All-gather of `bytes` per rank: device pointers in the RCCL form, host pointers in the host form.
    void all_gather(const void *send, void *recv, uint64_t bytes) {
        const auto t0 = std::chrono::steady_clock::now();
        if (device_form()) {
            check_nccl(rccl().AllGather(send, recv, bytes, ncclUint8, nc, st), "ncclAllGather");
            wait();
        } else if (fn(ctx, send, recv, bytes) != 0) {
            throw Error(ST_EINVAL, "host all-gather callback failed");
        }
        secs[kind] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        calls[kind] += 1;
        nbytes[kind] += bytes;
    }
    // All-gather-v (RCCL form): rank r's `sizes[r]` bytes land at recv + offs[r]; point-to-point sends /
    // receives in one group, this rank's own block by a device copy. Every rank knows every size from the
    // operation's meta round.
    void all_gather_v(const uint8_t *send, uint8_t *recv, const std::vector<uint64_t> &sizes,
                      const std::vector<uint64_t> &offs) {
        const auto t0 = std::chrono::steady_clock::now();
        const Rccl &R = rccl();
        check_nccl(R.GroupStart(), "ncclGroupStart");
        ncclResult_t e = ncclSuccess;
        for (int q = 0; q < world && e == ncclSuccess; ++q) {
            if (q == rank) continue;
            e = R.Send(send, sizes[rank], ncclUint8, q, nc, st);
            if (e == ncclSuccess) e = R.Recv(recv + offs[q], sizes[q], ncclUint8, q, nc, st);
        }
        const ncclResult_t g = R.GroupEnd();
        check_nccl(e, "ncclSend / ncclRecv");
        check_nccl(g, "ncclGroupEnd");
        MKV_HIP(hipMemcpyAsync(recv + offs[rank], send, sizes[rank], hipMemcpyDeviceToDevice, st));
        wait();
        secs[kind] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        calls[kind] += 1;
        nbytes[kind] += sizes[rank];
    }
    // Any rank's status word non-zero -> every rank throws the same way (its own error when it failed
    // itself, else the first failing rank's code) and the staging plan drops to 0 on every rank.
    [[noreturn]] void fail_all(int r, uint64_t s, int my_code, const std::string &my_err, const char *op) {
        plan_in = plan_out = 0;
        if (my_code) throw Error(my_code, my_err);
        throw Error((int)s, std::string(op) + ": rank " + std::to_string(r) + " failed (status " + std::to_string(s) +
                                "); every rank returns the error");
    }
    void raise_if_failed(const uint64_t *statuses, uint64_t stride_words, int my_code, const std::string &my_err,
                         const char *op) {
        for (int r = 0; r < world; ++r)
            if (statuses[(uint64_t)r * stride_words]) fail_all(r, statuses[(uint64_t)r * stride_words], my_code, my_err, op);
    }
    // META all-gather: {status, w1, w2, w3} of every rank (host result, rank order), on the reserved
    // buffers.
    std::vector<uint64_t> gather_meta(uint64_t status, uint64_t w1, uint64_t w2, uint64_t w3) {
        std::vector<uint64_t> out(4ull * world);
        const uint64_t mine[4] = {status, w1, w2, w3};
        if (device_form()) {
            uint8_t *a = dsin.as<uint8_t>(), *b = dsout.as<uint8_t>();
            hipLaunchKernelGGL(k_put_header, dim3(1), dim3(64), 0, st, reinterpret_cast<uint64_t *>(a), status, w1, w2,
                               w3);
            MKV_LAUNCH_CHECK();
            all_gather(a, b, HDR);
            MKV_HIP(hipMemcpyAsync(h_meta, b, HDR * world, hipMemcpyDeviceToHost, st));
            wait();
            std::memcpy(out.data(), h_meta, HDR * world);
            metab[kind] += HDR * world;
        } else {
            all_gather(mine, out.data(), HDR);
        }
        return out;
    }
    // One status round: every rank learns whether any rank's local steps so far failed.
    void status_round(int code, const std::string &err, const char *op) {
        const std::vector<uint64_t> m = gather_meta((uint64_t)code, 0, 0, 0);
        raise_if_failed(m.data(), 4, code, err, op);
    }
    // Staging of a block collective: `send` bytes, `recv` bytes in all. Within the plan nothing is
    // allocated (a failure of a later local step rides on the block's header). Beyond it every rank
    // allocates inside a local step and ONE status round follows, so a rank whose allocation failed
    // reports it instead of missing the collective (an OOM between the meta gather and the
    // block gather used to throw on one rank while its peers entered ncclAllGather).
    void stage(uint64_t send, uint64_t recv, int &code, std::string &err, const char *op, bool may_fault = true) {
        const bool grow = send > plan_in || recv > plan_out;
        const bool inject = fault && may_fault && !code;
        if (inject) fault = 0;
        static const char *injected = "injected fault (mkv_comm_inject_fault) in a local step after the meta all-gather";
        if (!grow) {
            // within the plan: the buffers are only sized (the host form's block size is hin.size()), nothing
            // is allocated, and this runs whatever `code` says so every rank sends a block of the agreed size
            if (device_form()) {
                din.ensure(send);
                dout.ensure(recv);
            } else {
                hin.resize(send);
                hout.resize(recv);
            }
            if (inject) code = ST_ENOMEM, err = injected;
            return;
        }
        local_step(code, err, [&] {
            if (inject) {
                release_staging();  // as a failed hipMalloc leaves them (DevBuf::ensure)
                throw Error(ST_ENOMEM, injected);
            }
            if (device_form()) {
                din.ensure(send);
                dout.ensure(recv);
            } else {
                hin.resize(send);
                hout.resize(recv);
            }
        });
        status_round(code, err, op);  // raises on every rank when any rank failed so far
        plan_in = std::max(plan_in, send);
        plan_out = std::max(plan_out, recv);
    }
    void release_staging() {
        din.release();
        dout.release();
        std::vector<uint8_t>().swap(hin);
        std::vector<uint8_t>().swap(hout);
    }
    // Verdict of gathered device blocks (k_check_blocks), read back as meta; raises on every rank.
    void check_device_blocks(const uint8_t *recv, uint64_t stride, bool ranges, uint64_t W, int my_code,
                             const std::string &my_err, const char *op, uint64_t *order_bad) {
        uint64_t *v = dverdict.as<uint64_t>();
        hipLaunchKernelGGL(k_check_blocks, dim3(1), dim3(64), 0, st, recv, stride, (uint32_t)world, ranges ? 1 : 0, W, v);
        MKV_LAUNCH_CHECK();
        uint64_t *h = h_meta;
        MKV_HIP(hipMemcpyAsync(h, v, 24, hipMemcpyDeviceToHost, st));
        wait();
        metab[kind] += 24;
        if (h[0] != ~0ull) fail_all((int)h[0], h[1], my_code, my_err, op);
        if (order_bad) *order_bad = h[2];
    }
    // Host form: all-gather of the staged block hin (first u64 = the status word) into hout.
    const uint8_t *gather_host_blocks(int my_code, const std::string &my_err, const char *op) {
        const uint64_t st64 = (uint64_t)my_code, blk = hin.size();
        std::memcpy(hin.data(), &st64, 8);
        all_gather(hin.data(), hout.data(), blk);
        for (int r = 0; r < world; ++r) {
            uint64_t s;
            std::memcpy(&s, hout.data() + blk * r, 8);
            if (s) fail_all(r, s, my_code, my_err, op);
        }
        return hout.data();
    }
};

namespace {

#define COMM_TRY(...)                                                                                 \
    try {                                                                                             \
        __VA_ARGS__;                                                                                  \
        return MKV_OK;                                                                                \
    } catch (const Error &e) {                                                                        \
        set_last_error(e.what());                                                                     \
        return e.code;                                                                                \
    } catch (const std::exception &e) {                                                               \
        set_last_error(e.what());                                                                     \
        return MKV_EINVAL;                                                                            \
    }

// A failed tree call inside a sharded operation keeps the tree's own message.
void call(mkv_status s) {
    if (s != MKV_OK) throw Error(s, mkv_last_error());
}

struct Guard {
    int prev = -1;
    explicit Guard(int d) {
        (void)hipGetDevice(&prev);
        if (d >= 0) MKV_HIP(hipSetDevice(d));
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

struct ListFree {
    void operator()(mkv_keylist *l) const { mkv_keylist_free(l); }
};
using ListPtr = std::unique_ptr<mkv_keylist, ListFree>;

// Keys at sorted positions 0 and n-1 of a shard (host bytes), for the host form's range check.
std::pair<std::string, std::string> shard_ends(const mkv_tree *t, uint64_t n) {
    if (!n) return {};
    const uint64_t pos[2] = {0, n - 1};
    mkv_keylist *l = nullptr;
    call(mkv_tree_keys_at(t, pos, 2, &l));
    ListPtr own(l);
    uint64_t m = 0;
    const uint8_t *b = nullptr;
    const uint64_t *o = nullptr;
    mkv_keylist_get(l, &m, &b, &o);
    return {std::string(reinterpret_cast<const char *>(b + o[0]), o[1] - o[0]),
            std::string(reinterpret_cast<const char *>(b + o[1]), o[2] - o[1])};
}

[[noreturn]] void throw_range(int prev_rank, int r) {
    throw Error(ST_EINVAL, "shard key ranges overlap or are out of rank order (rank " + std::to_string(prev_rank) +
                               " vs rank " + std::to_string(r) +
                               "): the seam protocol needs contiguous key ranges ordered by rank");
}

// The seam protocol is exact only when rank r's keys all sort below rank r+1's (Rust String order = bytes
// order): every non-empty shard's last key < the next non-empty shard's first key. ONE collective: each
// rank's boundary keys padded to the widest rank's (the widths came with the counts' meta gather).
void check_ranges(mkv_comm *c, const mkv_tree *t, const std::vector<uint64_t> &meta, int &code, std::string &err) {
    c->kind = MKV_COLL_RANGE;
    static const char *op = "sharded build (range check)";
    uint64_t W = 1;
    for (int r = 0; r < c->world; ++r) W = std::max({W, meta[4 * r + 2], meta[4 * r + 3]});
    W = up16(W);
    const uint64_t n = meta[4 * c->rank + 1], blk = HDR + 2 * W;
    c->stage(blk, blk * c->world, code, err, op);
    if (c->device_form()) {
        uint8_t *src = c->din.as<uint8_t>(), *dst = c->dout.as<uint8_t>();
        DevKeys ends;
        local_step(code, err, [&] {
            if (n) {
                const uint64_t pos[2] = {0, n - 1};
                ends = tree_keys_at_device(t, pos, 2);
                wait_bounded(tree_stream(t));
            }
        });
        hipLaunchKernelGGL(k_pack_ends, dim3(1), dim3(256), 0, c->st, src, (uint64_t)code, code ? 0 : n, ends.off, ends.kb,
                           W);
        MKV_LAUNCH_CHECK();
        c->all_gather(src, dst, blk);
        uint64_t bad = ~0ull;
        c->check_device_blocks(dst, blk, true, W, code, err, op, &bad);
        if (bad != ~0ull) {
            int prev = -1;
            for (int r = 0; r < (int)bad; ++r)
                if (meta[4 * r + 1]) prev = r;
            throw_range(prev, (int)bad);
        }
        return;
    }
    local_step(code, err, [&] {
        std::fill(c->hin.begin(), c->hin.end(), 0);
        const auto ends = shard_ends(t, n);
        std::memcpy(c->hin.data() + HDR, ends.first.data(), ends.first.size());
        std::memcpy(c->hin.data() + HDR + W, ends.second.data(), ends.second.size());
    });
    const uint8_t *all = c->gather_host_blocks(code, err, op);
    std::string prev;
    int prev_rank = -1;
    for (int r = 0; r < c->world; ++r) {
        if (!meta[4 * r + 1]) continue;
        const uint8_t *p = all + blk * r;
        const std::string first(reinterpret_cast<const char *>(p + HDR), meta[4 * r + 2]);
        const std::string last(reinterpret_cast<const char *>(p + HDR + W), meta[4 * r + 3]);
        if (prev_rank >= 0 && !(prev < first)) throw_range(prev_rank, r);
        prev = last;
        prev_rank = r;
    }
}

// Fringe all-gather + device seam combine of k trees (replicas of one key range) in ONE collective: the
// global roots on every rank. Block per rank = [status header | k fringes]; a rank whose earlier step
// failed (code != 0) sends only its status.
void recombine(mkv_comm *c, mkv_tree *const *ts, uint32_t k, uint8_t *roots, int *has_root, int code,
               std::string err) {
    const uint64_t blk = HDR + (uint64_t)k * MKV_FRINGE_BYTES;
    static const char *op = "sharded root (fringe all-gather)";
    c->kind = MKV_COLL_FRINGE;
    c->stage(blk, blk * c->world, code, err, op);
    if (c->device_form()) {
        uint8_t *src = c->din.as<uint8_t>(), *dst = c->dout.as<uint8_t>();
        local_step(code, err, [&] {
            for (uint32_t i = 0; i < k; ++i)
                call(mkv_shard_fringe_device(ts[i], src + HDR + (uint64_t)i * MKV_FRINGE_BYTES));
        });
        hipLaunchKernelGGL(k_put_header, dim3(1), dim3(64), 0, c->st, reinterpret_cast<uint64_t *>(src), (uint64_t)code,
                           (uint64_t)k, 0ull, 0ull);
        MKV_LAUNCH_CHECK();
        c->all_gather(src, dst, blk);
        c->check_device_blocks(dst, blk, false, 0, code, err, op, nullptr);
        for (uint32_t i = 0; i < k; ++i)
            call(mkv_shard_combine_device(ts[i], dst + HDR + (uint64_t)i * MKV_FRINGE_BYTES, (uint32_t)c->world, blk,
                                          tree_global_n(ts[i]), roots + 32ull * i, has_root + i));
        return;
    }
    local_step(code, err, [&] {
        std::fill(c->hin.begin(), c->hin.end(), 0);
        for (uint32_t i = 0; i < k; ++i)
            call(mkv_shard_fringe(ts[i], c->hin.data() + HDR + (uint64_t)i * MKV_FRINGE_BYTES));
    });
    const uint8_t *all = c->gather_host_blocks(code, err, op);
    std::vector<uint8_t> mine((uint64_t)MKV_FRINGE_BYTES * c->world);
    for (uint32_t i = 0; i < k; ++i) {
        for (int r = 0; r < c->world; ++r)
            std::memcpy(mine.data() + (uint64_t)r * MKV_FRINGE_BYTES, all + r * blk + HDR + (uint64_t)i * MKV_FRINGE_BYTES,
                        MKV_FRINGE_BYTES);
        call(mkv_shard_combine(ts[i], mine.data(), (uint32_t)c->world, tree_global_n(ts[i]), roots + 32ull * i,
                               has_root + i));
    }
}

}  // namespace

extern "C" {

mkv_status mkv_comm_unique_id(uint8_t id[MKV_COMM_ID_BYTES]) {
    COMM_TRY({
        if (!id) throw Error(ST_EINVAL, "null id");
        static_assert(sizeof(ncclUniqueId) == MKV_COMM_ID_BYTES, "RCCL unique id size");
        ncclUniqueId u;
        check_nccl(rccl().GetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof u);
    });
}

mkv_status mkv_comm_init_rank(const uint8_t id[MKV_COMM_ID_BYTES], int rank, int world, int hip_device, mkv_comm **out) {
    COMM_TRY({
        if (!id || !out) throw Error(ST_EINVAL, "null argument");
        if (world < 1 || rank < 0 || rank >= world) throw Error(ST_EINVAL, "bad rank / world");
        *out = nullptr;
        Guard g(hip_device);
        auto *c = new mkv_comm();
        c->rank = rank;
        c->world = world;
        c->dev = hip_device;
        try {
            MKV_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
            c->reserve_status();
            ncclUniqueId u;
            std::memcpy(&u, id, sizeof u);
            check_nccl(rccl().CommInitRank(&c->nc, world, u, rank), "ncclCommInitRank");
        } catch (...) {
            mkv_comm_destroy(c);
            throw;
        }
        *out = c;
    });
}

mkv_status mkv_comm_create_host(int rank, int world, mkv_allgather_fn fn, void *ctx, mkv_comm **out) {
    COMM_TRY({
        if (!fn || !out) throw Error(ST_EINVAL, "null argument");
        if (world < 1 || rank < 0 || rank >= world) throw Error(ST_EINVAL, "bad rank / world");
        auto *c = new mkv_comm();
        c->rank = rank;
        c->world = world;
        c->fn = fn;
        c->ctx = ctx;
        *out = c;
    });
}

mkv_status mkv_comm_rank(const mkv_comm *c, int *rank, int *world) {
    COMM_TRY({
        if (!c || !rank || !world) throw Error(ST_EINVAL, "null argument");
        *rank = c->rank;
        *world = c->world;
    });
}

mkv_status mkv_comm_inject_fault(mkv_comm *c, int where) {
    COMM_TRY({
        if (!c) throw Error(ST_EINVAL, "null argument");
        if (where != 0 && where != MKV_FAULT_AFTER_META) throw Error(ST_EINVAL, "unknown fault point");
        c->fault = where;
    });
}

mkv_status mkv_comm_all_gather(mkv_comm *c, const void *send, void *recv, uint64_t bytes) {
    COMM_TRY({
        if (!c || (bytes && (!send || !recv))) throw Error(ST_EINVAL, "null argument");
        c->usable();
        if (!bytes) return MKV_OK;
        const int saved = c->kind;
        c->kind = MKV_COLL_USER;  // the caller's own bytes, counted apart from the sharded operations
        try {
            if (c->device_form()) {
                Guard g(c->dev);
                int code = 0;
                std::string err;
                // no header carries a status here: the test hook stays armed for the next sharded operation
                c->stage(bytes, bytes * c->world, code, err, "all-gather", false);
                uint8_t *a = c->din.as<uint8_t>(), *b = c->dout.as<uint8_t>();
                MKV_HIP(hipMemcpyAsync(a, send, bytes, hipMemcpyHostToDevice, c->st));
                c->all_gather(a, b, bytes);
                MKV_HIP(hipMemcpyAsync(recv, b, bytes * c->world, hipMemcpyDeviceToHost, c->st));
                c->wait();
                c->staged[MKV_COLL_USER] += bytes * (1 + c->world);  // host payloads by definition
            } else {
                c->all_gather(send, recv, bytes);
            }
        } catch (...) {
            c->kind = saved;
            throw;
        }
        c->kind = saved;
    });
}

mkv_status mkv_comm_stats(mkv_comm *c, double secs[MKV_COLL_KINDS], uint64_t calls[MKV_COLL_KINDS],
                          uint64_t bytes[MKV_COLL_KINDS], int reset) {
    COMM_TRY({
        if (!c) throw Error(ST_EINVAL, "null argument");
        for (int i = 0; i < MKV_COLL_KINDS; ++i) {
            if (secs) secs[i] = c->secs[i];
            if (calls) calls[i] = c->calls[i];
            if (bytes) bytes[i] = c->nbytes[i];
            if (reset) c->secs[i] = 0, c->calls[i] = 0, c->nbytes[i] = 0, c->staged[i] = 0, c->metab[i] = 0;
        }
    });
}

mkv_status mkv_comm_traffic(const mkv_comm *c, uint64_t staged[MKV_COLL_KINDS], uint64_t meta[MKV_COLL_KINDS]) {
    COMM_TRY({
        if (!c) throw Error(ST_EINVAL, "null argument");
        for (int i = 0; i < MKV_COLL_KINDS; ++i) {
            if (staged) staged[i] = c->staged[i];
            if (meta) meta[i] = c->metab[i];
        }
    });
}

void mkv_comm_destroy(mkv_comm *c) {
    if (!c) return;
    if (c->nc) {
        Guard g(c->dev);
        (void)rccl().CommDestroy(c->nc);
    }
    if (c->st) (void)hipStreamDestroy(c->st);
    if (c->h_meta) (void)hipHostFree(c->h_meta);
    c->din.release();
    c->dout.release();
    c->dsin.release();
    c->dsout.release();
    c->dres_off.release();
    c->dres_kb.release();
    c->dverdict.release();
    delete c;
}

mkv_status mkv_sharded_build(mkv_tree *t, mkv_comm *c, mkv_blob keys, mkv_blob values, int on_device,
                             int range_check, uint64_t *counts_out) {
    COMM_TRY({
        if (!t || !c) throw Error(ST_EINVAL, "null argument");
        c->usable();
        Guard g(c->dev);
        int code = 0;
        std::string err;
        uint64_t n_local = 0, lf = 0, ll = 0;
        local_step(code, err, [&] {
            call(mkv_shard_prepare(t, keys, values, on_device, &n_local));
            if (range_check && n_local) {  // the boundary keys' lengths ride on the count gather
                const uint64_t pos[2] = {0, n_local - 1};
                const DevKeys e = tree_keys_at_device(t, pos, 2);
                uint64_t o[3] = {0, 0, 0};
                MKV_HIP(hipMemcpyAsync(o, e.off, 24, hipMemcpyDeviceToHost, tree_stream(t)));
                wait_bounded(tree_stream(t));
                lf = o[1] - o[0];
                ll = o[2] - o[1];
                c->metab[MKV_COLL_RANGE] += 24;
            }
        });
        c->kind = MKV_COLL_COUNTS;
        const std::vector<uint64_t> meta = c->gather_meta((uint64_t)code, code ? 0 : n_local, lf, ll);
        c->raise_if_failed(meta.data(), 4, code, err, "sharded build");
        if (range_check) check_ranges(c, t, meta, code, err);
        uint64_t offset = 0, total = 0;
        for (int r = 0; r < c->world; ++r) {
            if (r < c->rank) offset += meta[4 * r + 1];
            total += meta[4 * r + 1];
        }
        local_step(code, err, [&] { call(mkv_shard_reduce(t, offset, total)); });
        uint8_t root[32];
        int has = 0;
        recombine(c, &t, 1, root, &has, code, err);
        if (counts_out)
            for (int r = 0; r < c->world; ++r) counts_out[r] = meta[4 * r + 1];
    });
}

mkv_status mkv_sharded_root(mkv_tree *t, mkv_comm *c, uint8_t out32[32], int *has_root) {
    COMM_TRY({
        if (!t || !c || !out32 || !has_root) throw Error(ST_EINVAL, "null argument");
        c->usable();
        Guard g(c->dev);
        recombine(c, &t, 1, out32, has_root, 0, std::string());
    });
}

mkv_status mkv_sharded_root_many(mkv_tree *const *ts, uint32_t k, mkv_comm *c, uint8_t *roots, int *has_root) {
    COMM_TRY({
        if (!c || (k && (!ts || !roots || !has_root))) throw Error(ST_EINVAL, "null argument");
        for (uint32_t i = 0; i < k; ++i)
            if (!ts[i]) throw Error(ST_EINVAL, "null tree");
        if (!k) return MKV_OK;
        c->usable();
        Guard g(c->dev);
        recombine(c, ts, k, roots, has_root, 0, std::string());
    });
}

mkv_status mkv_sharded_diff(const mkv_tree *a, const mkv_tree *b, mkv_comm *c, mkv_keylist **out) {
    COMM_TRY({
        if (!a || !b || !c || !out) throw Error(ST_EINVAL, "null argument");
        *out = nullptr;
        c->usable();
        Guard g(c->dev);
        int code = 0;
        std::string err;
        static const char *op = "sharded diff";
        c->kind = MKV_COLL_DIFF;
        if (c->device_form()) {
            // local diff left on the device -> (count, bytes) meta -> all-gather-v of device blocks
            // [header | offsets | key bytes], each sized by its own list -> status check + compaction kernels
            // -> ONE device -> host copy of the result
            DevKeys loc;
            local_step(code, err, [&] {
                loc = tree_diff_device(a, b);
                wait_bounded(tree_stream(a));
            });
            const std::vector<uint64_t> meta = c->gather_meta((uint64_t)code, loc.n, loc.bytes, 0);
            c->raise_if_failed(meta.data(), 4, code, err, op);
            std::vector<uint64_t> sizes(c->world), offs(c->world);
            uint64_t tn = 0, tb = 0, at = 0;
            for (int r = 0; r < c->world; ++r) {
                sizes[r] = list_block_bytes(meta[4 * r + 1], meta[4 * r + 2]);
                offs[r] = at;
                at += sizes[r];
                tn += meta[4 * r + 1];
                tb += meta[4 * r + 2];
            }
            c->stage(sizes[c->rank], at, code, err, op);
            uint8_t *src = c->din.as<uint8_t>(), *dst = c->dout.as<uint8_t>();
            local_step(code, err, [&] {
                hipLaunchKernelGGL(k_pack_list, dim3((uint32_t)std::min<uint64_t>(ceil_div(loc.n + 1, 256), 1024)), dim3(256),
                                   0, c->st, src, 0ull, loc.n, loc.bytes, loc.off);
                MKV_LAUNCH_CHECK();
                if (loc.bytes)
                    MKV_HIP(hipMemcpyAsync(src + up16(HDR + 8 * (loc.n + 1)), loc.kb, loc.bytes, hipMemcpyDeviceToDevice,
                                           c->st));
            });
            // the status word last, so a failed packing step still reaches every rank (sizes stay the meta's)
            hipLaunchKernelGGL(k_put_header, dim3(1), dim3(64), 0, c->st, reinterpret_cast<uint64_t *>(src), (uint64_t)code,
                               loc.n, loc.bytes, 0ull);
            MKV_LAUNCH_CHECK();
            c->all_gather_v(src, dst, sizes, offs);
            c->check_device_blocks(dst, 0, false, 0, code, err, op, nullptr);
            uint64_t *ro = reinterpret_cast<uint64_t *>(c->dres_off.ensure(8 * (tn + 1)));
            uint8_t *rk = reinterpret_cast<uint8_t *>(c->dres_kb.ensure(tb + 16));
            if (tn) {
                uint64_t mx = 0;
                for (int r = 0; r < c->world; ++r) mx = std::max({mx, meta[4 * r + 1], meta[4 * r + 2]});
                const uint32_t gx = (uint32_t)std::min<uint64_t>(ceil_div(mx + 1, 256 * 4), 1024);
                hipLaunchKernelGGL(k_compact_lists, dim3(gx, (uint32_t)c->world), dim3(256), 0, c->st, dst, ro, rk, tn);
                MKV_LAUNCH_CHECK();
            }
            *out = keylist_from_device(ro, rk, tn, tb, c->st);
            return MKV_OK;
        }
        // host form: local diff on the host, then (count, bytes) and one all-gather of blocks padded to the
        // largest rank's (the host callback moves equal sizes)
        ListPtr loc;
        local_step(code, err, [&] {
            mkv_keylist *l = nullptr;
            call(mkv_tree_diff(a, b, &l));
            loc.reset(l);
        });
        uint64_t n = 0;
        const uint8_t *kb = nullptr;
        const uint64_t *ko = nullptr;
        if (loc) mkv_keylist_get(loc.get(), &n, &kb, &ko);
        const uint64_t nb = n ? ko[n] - ko[0] : 0;
        const std::vector<uint64_t> meta = c->gather_meta((uint64_t)code, n, nb, 0);
        c->raise_if_failed(meta.data(), 4, code, err, op);
        uint64_t mn = 0, mb = 0, tn = 0, tb = 0;
        for (int r = 0; r < c->world; ++r) {
            mn = std::max(mn, meta[4 * r + 1]);
            mb = std::max(mb, meta[4 * r + 2]);
            tn += meta[4 * r + 1];
            tb += meta[4 * r + 2];
        }
        const uint64_t blk = HDR + 4 * mn + mb;
        c->stage(blk, blk * c->world, code, err, op);
        local_step(code, err, [&] {
            std::fill(c->hin.begin(), c->hin.end(), 0);
            for (uint64_t i = 0; i < n; ++i) {
                const uint32_t len = (uint32_t)(ko[i + 1] - ko[i]);
                std::memcpy(c->hin.data() + HDR + 4 * i, &len, 4);
            }
            if (nb) std::memcpy(c->hin.data() + HDR + 4 * mn, kb + ko[0], nb);
        });
        loc.reset();
        const uint8_t *all = c->gather_host_blocks(code, err, op);
        std::vector<uint64_t> offsv(tn + 1, 0);
        std::vector<uint8_t> bytes(tb);
        uint64_t k = 0, at = 0;
        for (int r = 0; r < c->world; ++r) {
            const uint8_t *p = all + blk * r;
            for (uint64_t i = 0; i < meta[4 * r + 1]; ++i, ++k) {
                uint32_t len;
                std::memcpy(&len, p + HDR + 4 * i, 4);
                offsv[k + 1] = offsv[k] + len;
            }
            if (meta[4 * r + 2]) std::memcpy(bytes.data() + at, p + HDR + 4 * mn, meta[4 * r + 2]);
            at += meta[4 * r + 2];
        }
        *out = keylist_from_host(bytes.data(), offsv.data(), tn);
    });
}

mkv_status mkv_sharded_diff_local(const mkv_tree *a, const mkv_tree *b, mkv_comm *c, mkv_keylist **out,
                                  uint64_t *global_offset, uint64_t *global_total) {
    COMM_TRY({
        if (!a || !b || !c || !out || !global_offset) throw Error(ST_EINVAL, "null argument");
        *out = nullptr;
        c->usable();
        Guard g(c->dev);
        int code = 0;
        std::string err;
        ListPtr loc;
        local_step(code, err, [&] {
            mkv_keylist *l = nullptr;
            call(mkv_tree_diff(a, b, &l));
            loc.reset(l);
        });
        uint64_t n = 0;
        if (loc) mkv_keylist_get(loc.get(), &n, nullptr, nullptr);
        c->kind = MKV_COLL_DIFF;
        const std::vector<uint64_t> meta = c->gather_meta((uint64_t)code, n, 0, 0);
        c->raise_if_failed(meta.data(), 4, code, err, "sharded diff (local slice)");
        uint64_t off = 0, tot = 0;
        for (int r = 0; r < c->world; ++r) {
            if (r < c->rank) off += meta[4 * r + 1];
            tot += meta[4 * r + 1];
        }
        *global_offset = off;
        if (global_total) *global_total = tot;
        *out = loc.release();
    });
}

}  // extern "C"
