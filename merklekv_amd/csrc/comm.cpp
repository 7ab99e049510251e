// comm.cpp — multi-GPU key-range shards behind the C ABI: a communicator (RCCL inside the
// library, or the caller's host all-gather) and the sharded build / root / diff that run the collectives
// themselves, so a host in any language (the reference's Rust SyncManager, sync.rs:56-87) gets the global
// root and the one sorted divergent-key list without a collective layer of its own.
//
// RCCL is loaded at run time: the already-resident copy when there is one (a PyTorch process has its own
// librccl loaded; two RCCL instances in one process would each bring up the devices), else
// librccl.so.1 from ROCm, with RTLD_LOCAL so its symbols never interpose on anyone else's.
//
// Per sharded build (every rank): hash + sort + dedup of the rank's key range (mkv_shard_prepare), ONE
// all-gather of the 8-B leaf counts, the shard's range check (one all-gather of its first and last key),
// the in-shard reduction (mkv_shard_reduce), ONE all-gather of the <= 6 KiB seam fringes and the seam
// combine on the device. With RCCL every payload stays in device memory; sizes are bytes, so the
// collectives are latency-bound and scaling is weak and near-linear by construction.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
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
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
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
        r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(dlsym(r.h, "ncclGetUniqueId"));
        r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(dlsym(r.h, "ncclCommInitRank"));
        r.AllGather = reinterpret_cast<decltype(r.AllGather)>(dlsym(r.h, "ncclAllGather"));
        r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(dlsym(r.h, "ncclCommDestroy"));
        r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(dlsym(r.h, "ncclGetErrorString"));
    });
    if (!r.GetUniqueId || !r.CommInitRank || !r.AllGather || !r.CommDestroy)
        throw Error(ST_EHIP, "RCCL not available (librccl.so.1 could not be loaded)");
    return r;
}

void check_nccl(ncclResult_t e, const char *what) {
    if (e != ncclSuccess) {
        const Rccl &r = rccl();
        throw Error(ST_EHIP, std::string(what) + ": " + (r.GetErrorString ? r.GetErrorString(e) : "RCCL error"));
    }
}

}  // namespace

struct mkv_comm {
    int rank = 0, world = 1, dev = -1;
    // RCCL form
    ncclComm_t nc = nullptr;
    hipStream_t st = nullptr;
    DevBuf din, dout;  // collective staging (device)
    // host form
    mkv_allgather_fn fn = nullptr;
    void *ctx = nullptr;
    // wall time / calls / bytes per rank of each collective kind (MKV_COLL_*), host clock around the
    // collective and the wait for its result
    double secs[MKV_COLL_KINDS] = {};
    uint64_t calls[MKV_COLL_KINDS] = {}, nbytes[MKV_COLL_KINDS] = {};
    int kind = MKV_COLL_COUNTS;  // kind of the collectives issued next
    bool device_form() const { return nc != nullptr; }

    // All-gather of `bytes` per rank: device pointers in the RCCL form, host pointers in the host form.
    void all_gather(const void *send, void *recv, uint64_t bytes) {
        const auto t0 = std::chrono::steady_clock::now();
        gather(send, recv, bytes);
        secs[kind] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        calls[kind] += 1;
        nbytes[kind] += bytes;
    }
    void gather(const void *send, void *recv, uint64_t bytes) {
        if (device_form()) {
            check_nccl(rccl().AllGather(send, recv, bytes, ncclUint8, nc, st), "ncclAllGather");
            MKV_HIP(hipStreamSynchronize(st));
        } else {
            if (fn(ctx, send, recv, bytes) != 0) throw Error(ST_EINVAL, "host all-gather callback failed");
        }
    }
    // All-gather of host bytes (any form); result on the host, rank order.
    std::vector<uint8_t> all_gather_host(const void *send, uint64_t bytes) {
        std::vector<uint8_t> out((size_t)bytes * world);
        if (!bytes) return out;
        if (device_form()) {
            uint8_t *a = reinterpret_cast<uint8_t *>(din.ensure(bytes));
            uint8_t *b = reinterpret_cast<uint8_t *>(dout.ensure(bytes * world));
            MKV_HIP(hipMemcpyAsync(a, send, bytes, hipMemcpyHostToDevice, st));
            all_gather(a, b, bytes);
            MKV_HIP(hipMemcpyAsync(out.data(), b, bytes * world, hipMemcpyDeviceToHost, st));
            MKV_HIP(hipStreamSynchronize(st));
        } else {
            all_gather(send, out.data(), bytes);
        }
        return out;
    }
    std::vector<uint64_t> all_gather_u64(uint64_t v) {
        const std::vector<uint8_t> raw = all_gather_host(&v, sizeof v);
        std::vector<uint64_t> out(world);
        std::memcpy(out.data(), raw.data(), 8ull * world);
        return out;
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

// Keys at sorted positions 0 and n-1 of a shard (host bytes), for the range check.
std::pair<std::string, std::string> shard_ends(const mkv_tree *t, uint64_t n) {
    if (!n) return {};
    const uint64_t pos[2] = {0, n - 1};
    mkv_keylist *l = nullptr;
    call(mkv_tree_keys_at(t, pos, 2, &l));
    uint64_t m = 0;
    const uint8_t *b = nullptr;
    const uint64_t *o = nullptr;
    mkv_keylist_get(l, &m, &b, &o);
    std::pair<std::string, std::string> r{std::string(reinterpret_cast<const char *>(b + o[0]), o[1] - o[0]),
                                          std::string(reinterpret_cast<const char *>(b + o[1]), o[2] - o[1])};
    mkv_keylist_free(l);
    return r;
}

// The seam protocol is exact only when rank r's keys all sort below rank r+1's (Rust String order =
// bytes order): every non-empty shard's last key < the next non-empty shard's first key.
void check_ranges(mkv_comm *c, const mkv_tree *t, const std::vector<uint64_t> &counts) {
    const auto ends = shard_ends(t, counts[c->rank]);
    const std::vector<uint64_t> lens0 = c->all_gather_u64(ends.first.size());
    const std::vector<uint64_t> lens1 = c->all_gather_u64(ends.second.size());
    uint64_t width = 1;
    for (int r = 0; r < c->world; ++r) width = std::max({width, lens0[r], lens1[r]});
    std::vector<uint8_t> pay(2 * width, 0);
    std::memcpy(pay.data(), ends.first.data(), ends.first.size());
    std::memcpy(pay.data() + width, ends.second.data(), ends.second.size());
    const std::vector<uint8_t> all = c->all_gather_host(pay.data(), pay.size());
    std::string prev;
    int prev_rank = -1;
    for (int r = 0; r < c->world; ++r) {
        if (!counts[r]) continue;
        const uint8_t *p = all.data() + 2 * width * r;
        const std::string first(reinterpret_cast<const char *>(p), lens0[r]);
        const std::string last(reinterpret_cast<const char *>(p + width), lens1[r]);
        if (prev_rank >= 0 && !(prev < first))
            throw Error(ST_EINVAL, "shard key ranges overlap or are out of rank order (rank " +
                                       std::to_string(prev_rank) + " vs rank " + std::to_string(r) +
                                       "): the seam protocol needs contiguous key ranges ordered by rank");
        prev = last;
        prev_rank = r;
    }
}

// Fringe all-gather + device seam combine of k trees (replicas of one key range) in ONE collective: the
// global roots on every rank.
void recombine(mkv_comm *c, mkv_tree *const *ts, uint32_t k, uint8_t *roots, int *has_root) {
    const uint64_t blk = (uint64_t)k * MKV_FRINGE_BYTES;
    c->kind = MKV_COLL_FRINGE;
    if (c->device_form()) {
        uint8_t *src = reinterpret_cast<uint8_t *>(c->din.ensure(blk));
        uint8_t *dst = reinterpret_cast<uint8_t *>(c->dout.ensure(blk * c->world));
        for (uint32_t i = 0; i < k; ++i) call(mkv_shard_fringe_device(ts[i], src + (uint64_t)i * MKV_FRINGE_BYTES));
        c->all_gather(src, dst, blk);
        for (uint32_t i = 0; i < k; ++i)
            call(mkv_shard_combine_device(ts[i], dst + (uint64_t)i * MKV_FRINGE_BYTES, (uint32_t)c->world, blk,
                                          tree_global_n(ts[i]), roots + 32ull * i, has_root + i));
    } else {
        std::vector<uint8_t> fr(blk);
        for (uint32_t i = 0; i < k; ++i) call(mkv_shard_fringe(ts[i], fr.data() + (uint64_t)i * MKV_FRINGE_BYTES));
        const std::vector<uint8_t> all = c->all_gather_host(fr.data(), fr.size());
        std::vector<uint8_t> mine((uint64_t)MKV_FRINGE_BYTES * c->world);
        for (uint32_t i = 0; i < k; ++i) {
            for (int r = 0; r < c->world; ++r)
                std::memcpy(mine.data() + (uint64_t)r * MKV_FRINGE_BYTES, all.data() + r * blk + (uint64_t)i * MKV_FRINGE_BYTES,
                            MKV_FRINGE_BYTES);
            call(mkv_shard_combine(ts[i], mine.data(), (uint32_t)c->world, tree_global_n(ts[i]), roots + 32ull * i,
                                   has_root + i));
        }
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

mkv_status mkv_comm_all_gather(mkv_comm *c, const void *send, void *recv, uint64_t bytes) {
    COMM_TRY({
        if (!c || (bytes && (!send || !recv))) throw Error(ST_EINVAL, "null argument");
        if (c->dev >= 0) {
            Guard g(c->dev);
            const std::vector<uint8_t> all = c->all_gather_host(send, bytes);
            if (bytes) std::memcpy(recv, all.data(), all.size());
        } else if (bytes) {
            c->all_gather(send, recv, bytes);
        }
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
            if (reset) c->secs[i] = 0, c->calls[i] = 0, c->nbytes[i] = 0;
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
    c->din.release();
    c->dout.release();
    delete c;
}

mkv_status mkv_sharded_build(mkv_tree *t, mkv_comm *c, mkv_blob keys, mkv_blob values, int on_device,
                             int range_check, uint64_t *counts_out) {
    COMM_TRY({
        if (!t || !c) throw Error(ST_EINVAL, "null argument");
        Guard g(c->dev);
        uint64_t n_local = 0;
        call(mkv_shard_prepare(t, keys, values, on_device, &n_local));
        c->kind = MKV_COLL_COUNTS;
        const std::vector<uint64_t> counts = c->all_gather_u64(n_local);
        c->kind = MKV_COLL_RANGE;
        if (range_check) check_ranges(c, t, counts);
        uint64_t offset = 0, total = 0;
        for (int r = 0; r < c->world; ++r) {
            if (r < c->rank) offset += counts[r];
            total += counts[r];
        }
        call(mkv_shard_reduce(t, offset, total));
        uint8_t root[32];
        int has = 0;
        recombine(c, &t, 1, root, &has);
        if (counts_out) std::memcpy(counts_out, counts.data(), 8ull * c->world);
    });
}

mkv_status mkv_sharded_root(mkv_tree *t, mkv_comm *c, uint8_t out32[32], int *has_root) {
    COMM_TRY({
        if (!t || !c || !out32 || !has_root) throw Error(ST_EINVAL, "null argument");
        Guard g(c->dev);
        recombine(c, &t, 1, out32, has_root);
    });
}

mkv_status mkv_sharded_root_many(mkv_tree *const *ts, uint32_t k, mkv_comm *c, uint8_t *roots, int *has_root) {
    COMM_TRY({
        if (!c || (k && (!ts || !roots || !has_root))) throw Error(ST_EINVAL, "null argument");
        for (uint32_t i = 0; i < k; ++i)
            if (!ts[i]) throw Error(ST_EINVAL, "null tree");
        if (!k) return MKV_OK;
        Guard g(c->dev);
        recombine(c, ts, k, roots, has_root);
    });
}

mkv_status mkv_sharded_diff(const mkv_tree *a, const mkv_tree *b, mkv_comm *c, mkv_keylist **out) {
    COMM_TRY({
        if (!a || !b || !c || !out) throw Error(ST_EINVAL, "null argument");
        *out = nullptr;
        Guard g(c->dev);
        mkv_keylist *loc = nullptr;
        call(mkv_tree_diff(a, b, &loc));
        uint64_t n = 0;
        const uint8_t *kb = nullptr;
        const uint64_t *ko = nullptr;
        mkv_keylist_get(loc, &n, &kb, &ko);
        const uint64_t nb = n ? ko[n] - ko[0] : 0;
        // (count, bytes) of every rank, then one block per rank: [u32 lengths (padded to the largest
        // count) | key bytes (padded to the largest byte count)]; rank order = key order (R7)
        c->kind = MKV_COLL_DIFF;
        const uint64_t meta[2] = {n, nb};
        const std::vector<uint8_t> mraw = c->all_gather_host(meta, sizeof meta);
        std::vector<uint64_t> cnt(c->world), byt(c->world);
        uint64_t mn = 0, mb = 0, tn = 0, tb = 0;
        for (int r = 0; r < c->world; ++r) {
            std::memcpy(&cnt[r], mraw.data() + 16 * r, 8);
            std::memcpy(&byt[r], mraw.data() + 16 * r + 8, 8);
            mn = std::max(mn, cnt[r]);
            mb = std::max(mb, byt[r]);
            tn += cnt[r];
            tb += byt[r];
        }
        std::vector<uint8_t> blk(4 * mn + mb, 0);
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t len = (uint32_t)(ko[i + 1] - ko[i]);
            std::memcpy(blk.data() + 4 * i, &len, 4);
        }
        if (nb) std::memcpy(blk.data() + 4 * mn, kb + ko[0], nb);
        mkv_keylist_free(loc);
        const std::vector<uint8_t> all = c->all_gather_host(blk.data(), blk.size());
        std::vector<uint64_t> offs(tn + 1, 0);
        std::vector<uint8_t> bytes(tb);
        uint64_t k = 0, at = 0;
        for (int r = 0; r < c->world; ++r) {
            const uint8_t *p = all.data() + blk.size() * r;
            for (uint64_t i = 0; i < cnt[r]; ++i, ++k) {
                uint32_t len;
                std::memcpy(&len, p + 4 * i, 4);
                offs[k + 1] = offs[k] + len;
            }
            if (byt[r]) std::memcpy(bytes.data() + at, p + 4 * mn, byt[r]);
            at += byt[r];
        }
        *out = keylist_from_host(bytes.data(), offs.data(), tn);
    });
}

}  // extern "C"
