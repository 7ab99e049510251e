// Sharded entry points of the C ABI (include/mkv_merkle.h mkv_comm_* / mkv_sharded_*), driven the way a
// non-Python host would drive them (the reference's SyncManager is Rust, sync.rs:56-87):
//   1. RCCL communicator at world 1 (unique id -> init_rank): sharded build, root, multi-replica root
//      and sharded diff equal the unsharded tree and an OpenSSL restatement of rebuild()/diff_keys();
//      mkv_sharded_diff_local gives the slice at its global offset; mkv_comm_traffic shows no host-staged
//      payload byte; a failing local step returns an error and the communicator stays usable;
//   2. host communicator at world 3 (three threads, one tree each, the host's own all-gather): every
//      rank's global root equals the unsharded root, the gathered divergent-key list is the whole sorted
//      diff on every rank, the local slices sit at their global offsets, in-range updates +
//      mkv_sharded_root_many track the new root, overlapping ranges are rejected (MKV_EINVAL) on every
//      rank, an invalid blob on ONE rank makes every rank's call fail (status words) without a hang, and so
//      does a failure injected on one rank AFTER the meta all-gather (mkv_comm_inject_fault: block header
//      and status-round paths).
// Built by __graft_entry__.build_cpp_tests(); run by tests/test_cpp_ports_gpu.py.
#include <openssl/evp.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mkv_merkle.h"

static int g_fail = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                  \
        }                                                              \
    } while (0)
#define OK(s)                                                                                          \
    do {                                                                                               \
        mkv_status st_ = (s);                                                                          \
        if (st_ != MKV_OK) {                                                                           \
            std::printf("  FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #s, st_, mkv_last_error()); \
            ++g_fail;                                                                                  \
        }                                                                                              \
    } while (0)

using Digest = std::string;  // 32 bytes
using Records = std::map<std::string, std::string>;

static Digest sha(const std::string &m) {
    unsigned char d[32];
    unsigned int len = 0;
    EVP_Digest(m.data(), m.size(), d, &len, EVP_sha256(), nullptr);
    return std::string(reinterpret_cast<char *>(d), 32);
}
static std::string u32be(size_t x) {
    std::string s(4, '\0');
    s[0] = (char)(x >> 24), s[1] = (char)(x >> 16), s[2] = (char)(x >> 8), s[3] = (char)x;
    return s;
}
// rebuild() (merkle.rs:73-121): leaves in key order, pairs hashed left to right, odd last promoted.
static Digest model_root(const Records &r) {
    std::vector<Digest> lv;
    for (const auto &kv : r) lv.push_back(sha(u32be(kv.first.size()) + kv.first + u32be(kv.second.size()) + kv.second));
    if (lv.empty()) return "";
    while (lv.size() > 1) {
        std::vector<Digest> up;
        for (size_t i = 0; i + 1 < lv.size(); i += 2) up.push_back(sha(lv[i] + lv[i + 1]));
        if (lv.size() & 1) up.push_back(lv.back());
        lv.swap(up);
    }
    return lv[0];
}
// diff_keys (merkle.rs:171-196): keys on one side only or with different values, sorted.
static std::vector<std::string> model_diff(const Records &a, const Records &b) {
    std::vector<std::string> out;
    auto i = a.begin();
    auto j = b.begin();
    while (i != a.end() || j != b.end()) {
        if (j == b.end() || (i != a.end() && i->first < j->first)) out.push_back((i++)->first);
        else if (i == a.end() || j->first < i->first) out.push_back((j++)->first);
        else {
            if (i->second != j->second) out.push_back(i->first);
            ++i, ++j;
        }
    }
    return out;
}

struct Packed {
    std::string bytes;
    std::vector<uint64_t> offs{0};
    void add(const std::string &s) {
        bytes += s;
        offs.push_back(bytes.size());
    }
    mkv_blob blob() const { return mkv_blob{reinterpret_cast<const uint8_t *>(bytes.data()), offs.data(), offs.size() - 1}; }
};
static void pack(const Records &r, Packed &k, Packed &v) {
    for (const auto &kv : r) k.add(kv.first), v.add(kv.second);
}
static std::vector<std::string> keylist(mkv_keylist *l) {
    uint64_t n = 0;
    const uint8_t *b = nullptr;
    const uint64_t *o = nullptr;
    mkv_keylist_get(l, &n, &b, &o);
    std::vector<std::string> out;
    for (uint64_t i = 0; i < n; ++i) out.emplace_back(reinterpret_cast<const char *>(b + o[i]), o[i + 1] - o[i]);
    mkv_keylist_free(l);
    return out;
}
static Digest root_of(mkv_tree *t) {
    uint8_t r[32];
    int has = 0;
    OK(mkv_tree_root(t, r, &has));
    return has ? std::string(reinterpret_cast<char *>(r), 32) : "";
}

// Key-range shards: rank r holds keys "s<r>-...", so ranges are ordered by rank.
static Records shard_records(int rank, int n, int salt) {
    Records r;
    for (int i = 0; i < n; ++i) {
        char k[64], v[64];
        std::snprintf(k, sizeof k, "s%d-key-%07d", rank, i * 7 + rank);
        std::snprintf(v, sizeof v, "value-%d-%d", i, (i % 53 == 0) ? salt : 0);
        if (salt && i % 97 == 5) continue;  // deleted on the second replica
        r[k] = v;
    }
    if (salt) r["s" + std::to_string(rank) + "-zz-new"] = "inserted";
    return r;
}

static void test_rccl_world1(int dev) {
    uint8_t id[MKV_COMM_ID_BYTES];
    mkv_status s = mkv_comm_unique_id(id);
    if (s != MKV_OK) {
        std::printf("  FAIL rccl unique id: %s\n", mkv_last_error());
        ++g_fail;
        return;
    }
    mkv_comm *c = nullptr;
    OK(mkv_comm_init_rank(id, 0, 1, dev, &c));
    if (!c) return;
    auto step = [](const char *what) {
        std::printf("  rccl world 1: %s\n", what);
        std::fflush(stdout);
    };
    int rank = -1, world = -1;
    OK(mkv_comm_rank(c, &rank, &world));
    CHECK(rank == 0 && world == 1);
    const Records ra = shard_records(0, 20011, 0), rb = shard_records(0, 20011, 9);
    Packed ka, va, kb, vb;
    pack(ra, ka, va);
    pack(rb, kb, vb);
    mkv_tree *a = nullptr, *b = nullptr, *a2 = nullptr, *u = nullptr;
    OK(mkv_tree_create(dev, &a));
    OK(mkv_tree_create(dev, &b));
    OK(mkv_tree_create(dev, &a2));
    OK(mkv_tree_create(dev, &u));
    uint64_t counts[1] = {0};
    OK(mkv_sharded_build(a, c, ka.blob(), va.blob(), 0, 1, counts));
    step("built a");
    CHECK(counts[0] == ra.size());
    OK(mkv_sharded_build(b, c, kb.blob(), vb.blob(), 0, 0, nullptr));
    OK(mkv_sharded_build(a2, c, ka.blob(), va.blob(), 0, 1, nullptr));
    OK(mkv_tree_build(u, ka.blob(), va.blob()));
    const Digest want = model_root(ra);
    CHECK(root_of(a) == want && root_of(u) == want);
    CHECK(root_of(b) == model_root(rb));
    uint8_t r1[32];
    int has = 0;
    OK(mkv_sharded_root(a, c, r1, &has));
    CHECK(has && std::string(reinterpret_cast<char *>(r1), 32) == want);
    mkv_tree *ts[3] = {a, b, a2};
    uint8_t roots[96];
    int hs[3] = {0, 0, 0};
    OK(mkv_sharded_root_many(ts, 3, c, roots, hs));
    CHECK(hs[0] && hs[1] && hs[2]);
    CHECK(std::string(reinterpret_cast<char *>(roots), 32) == want);
    CHECK(std::string(reinterpret_cast<char *>(roots + 32), 32) == model_root(rb));
    CHECK(std::string(reinterpret_cast<char *>(roots + 64), 32) == want);
    step("roots");
    mkv_keylist *l = nullptr;
    OK(mkv_sharded_diff(a, b, c, &l));
    if (l) CHECK(keylist(l) == model_diff(ra, rb));
    step("diff");
    // this rank's slice and its place in the global list (world 1: the whole list at offset 0)
    mkv_keylist *ls = nullptr;
    uint64_t goff = 99, gtot = 0;
    OK(mkv_sharded_diff_local(a, b, c, &ls, &goff, &gtot));
    const std::vector<std::string> want_d = model_diff(ra, rb);
    if (ls) CHECK(keylist(ls) == want_d);
    CHECK(goff == 0 && gtot == want_d.size());
    double secs[MKV_COLL_KINDS];
    uint64_t calls[MKV_COLL_KINDS], bytes[MKV_COLL_KINDS], staged[MKV_COLL_KINDS], meta[MKV_COLL_KINDS];
    OK(mkv_comm_traffic(c, staged, meta));
    OK(mkv_comm_stats(c, secs, calls, bytes, 1));
    // one meta gather per build (3); 5 fringe gathers + 2 status rounds (the fringe staging grew for 1 and
    // for 3 trees); the diff's meta + block gathers (+ a status round if its staging grew), the slice's meta
    CHECK(calls[MKV_COLL_COUNTS] == 3 && calls[MKV_COLL_FRINGE] == 7);
    CHECK(calls[MKV_COLL_DIFF] == 3 || calls[MKV_COLL_DIFF] == 4);
    CHECK(calls[MKV_COLL_RANGE] == 3);  // one boundary-key gather per range-checked build + the first's status round
    CHECK(bytes[MKV_COLL_FRINGE] == 7ull * MKV_FRINGE_BYTES + 7 * 32);  // 1 + 1 + 1 + 1 + 3 trees, 5 headers, 2 rounds
    // RCCL form: no payload byte crossed between host and device; only status / count words came back
    for (int k = 0; k < MKV_COLL_KINDS; ++k) CHECK(staged[k] == 0);
    CHECK(meta[MKV_COLL_COUNTS] == 3 * 32 && meta[MKV_COLL_DIFF] > 0);
    // a failing local step (keys.n != values.n) returns an error and leaves the communicator usable
    mkv_blob bad_v = va.blob();
    bad_v.n = bad_v.n - 1;
    CHECK(mkv_sharded_build(b, c, ka.blob(), bad_v, 0, 1, nullptr) == MKV_EINVAL);
    OK(mkv_sharded_build(b, c, kb.blob(), vb.blob(), 0, 1, nullptr));
    CHECK(root_of(b) == model_root(rb));
    // a local step failing AFTER the meta all-gather (test hook: as a failed staging allocation): within the
    // staging plan the status rides on the block header, beyond it on a status round; either way the call
    // returns the error and the communicator stays usable
    step("stats");
    OK(mkv_comm_inject_fault(c, MKV_FAULT_AFTER_META));
    l = nullptr;
    CHECK(mkv_sharded_diff(a, b, c, &l) == MKV_ENOMEM && l == nullptr);
    step("fault diff");
    OK(mkv_sharded_diff(a, b, c, &l));  // the plan was reset: the staging regrows behind a status round
    if (l) CHECK(keylist(l) == want_d);
    OK(mkv_comm_inject_fault(c, MKV_FAULT_AFTER_META));
    CHECK(mkv_sharded_build(b, c, kb.blob(), vb.blob(), 0, 1, nullptr) == MKV_ENOMEM);
    OK(mkv_sharded_build(b, c, kb.blob(), vb.blob(), 0, 1, nullptr));
    CHECK(root_of(b) == model_root(rb));
    for (mkv_tree *t : {a, b, a2, u}) mkv_tree_destroy(t);
    mkv_comm_destroy(c);
    std::printf("rccl world 1: %s\n", g_fail ? "FAILED" : "ok");
}

// The host's own all-gather among threads (one rank per thread): equal-size payloads, rank order.
struct ThreadGather {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::string> slots;
    int arrived = 0, departed = 0;
    uint64_t gen = 0;
    explicit ThreadGather(int w) : world(w), slots(w) {}
};
struct RankCtx {
    ThreadGather *g;
    int rank;
};
static int thread_all_gather(void *ctx, const void *send, void *recv, uint64_t bytes) {
    RankCtx *rc = static_cast<RankCtx *>(ctx);
    ThreadGather &g = *rc->g;
    std::unique_lock<std::mutex> lk(g.mu);
    // bounded waits: a protocol bug (ranks in different collectives) fails the test instead of hanging it
    const auto limit = std::chrono::seconds(60);
    if (!g.cv.wait_for(lk, limit, [&] { return g.departed == 0; })) {  // the previous round has drained
        std::printf("  FAIL rank %d: all-gather of %llu B: previous round never drained\n", rc->rank,
                    (unsigned long long)bytes);
        std::fflush(stdout);
        std::_Exit(3);
    }
    const uint64_t my = g.gen;
    g.slots[rc->rank].assign(static_cast<const char *>(send), bytes);
    if (++g.arrived == g.world) {
        ++g.gen;
        g.cv.notify_all();
    } else if (!g.cv.wait_for(lk, limit, [&] { return g.gen != my; })) {
        std::printf("  FAIL rank %d: all-gather of %llu B: peers never arrived\n", rc->rank, (unsigned long long)bytes);
        std::fflush(stdout);
        std::_Exit(3);
    }
    bool same = true;
    for (int r = 0; r < g.world; ++r) {
        if (g.slots[r].size() != bytes) same = false;
        else std::memcpy(static_cast<char *>(recv) + bytes * r, g.slots[r].data(), bytes);
    }
    if (!same) {
        std::printf("  FAIL rank %d: all-gather sizes differ across ranks (%llu B here)\n", rc->rank,
                    (unsigned long long)bytes);
        std::fflush(stdout);
    }
    if (++g.departed == g.world) {
        g.arrived = g.departed = 0;
        g.cv.notify_all();
    }
    return same ? 0 : 1;
}

static void test_host_world3(int dev) {
    const int world = 3;
    ThreadGather g(world);
    std::vector<Records> sa(world), sb(world);
    Records all_a, all_b;
    for (int r = 0; r < world; ++r) {
        sa[r] = shard_records(r, r == 1 ? 9001 : 15000 + 1000 * r, 0);
        sb[r] = shard_records(r, r == 1 ? 9001 : 15000 + 1000 * r, 3 + r);
        all_a.insert(sa[r].begin(), sa[r].end());
        all_b.insert(sb[r].begin(), sb[r].end());
    }
    const Digest want_a = model_root(all_a), want_b = model_root(all_b);
    const std::vector<std::string> want_diff = model_diff(all_a, all_b);
    // the update: rank r changes one value in its own range
    Records upd = all_a;
    for (int r = 0; r < world; ++r) upd[sa[r].begin()->first] = "updated-" + std::to_string(r);
    const Digest want_upd = model_root(upd);
    std::vector<std::string> got_a(world), got_b(world), got_upd(world);
    std::vector<std::vector<std::string>> got_diff(world);
    std::vector<int> bad_status(world, -1), fail_status(world, -1), fault_diff(world, -1), fault_build(world, -1),
        fault_root(world, -1);
    std::vector<std::vector<std::string>> got_diff2(world);
    std::vector<std::vector<std::string>> got_slice(world);
    std::vector<uint64_t> got_off(world), got_tot(world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            RankCtx rc{&g, r};
            mkv_comm *c = nullptr;
            OK(mkv_comm_create_host(r, world, thread_all_gather, &rc, &c));
            mkv_tree *a = nullptr, *b = nullptr;
            OK(mkv_tree_create(dev, &a));
            OK(mkv_tree_create(dev, &b));
            Packed ka, va, kb, vb;
            pack(sa[r], ka, va);
            pack(sb[r], kb, vb);
            std::vector<uint64_t> counts(world);
            OK(mkv_sharded_build(a, c, ka.blob(), va.blob(), 0, 1, counts.data()));
            OK(mkv_sharded_build(b, c, kb.blob(), vb.blob(), 0, 1, nullptr));
            got_a[r] = root_of(a);
            got_b[r] = root_of(b);
            mkv_keylist *l = nullptr;
            OK(mkv_sharded_diff(a, b, c, &l));
            if (l) got_diff[r] = keylist(l);
            mkv_keylist *ls = nullptr;
            uint64_t goff = 0, gtot = 0;
            OK(mkv_sharded_diff_local(a, b, c, &ls, &goff, &gtot));
            if (ls) got_slice[r] = keylist(ls);
            got_off[r] = goff;
            got_tot[r] = gtot;
            // rank 1's blob is invalid (keys.n != values.n): EVERY rank gets an error from this call (rank 1
            // its own EINVAL, the others rank 1's code through the status word), nobody waits forever
            {
                Packed bk, bv;
                pack(sb[r], bk, bv);
                mkv_blob vbl = bv.blob();
                if (r == 1) vbl.n -= 1;
                fail_status[r] = mkv_sharded_build(b, c, bk.blob(), vbl, 0, 1, nullptr);
                OK(mkv_sharded_build(b, c, bk.blob(), bv.blob(), 0, 1, nullptr));  // back in step
            }
            // rank 1 fails AFTER the meta all-gather (test hook): (1) a diff whose staging fits the plan (the
            // status rides on the block header), (2) the same diff again succeeds (the staging regrows behind a
            // status round), (3) a range-checked build right after another failure (plan reset: the failure
            // is reported by the status round before the boundary-key gather), (4) a root recombine; every
            // rank returns MKV_ENOMEM from each failing call, nobody hangs
            if (r == 1) OK(mkv_comm_inject_fault(c, MKV_FAULT_AFTER_META));
            mkv_keylist *lf = nullptr;
            fault_diff[r] = mkv_sharded_diff(a, b, c, &lf);
            if (lf) mkv_keylist_free(lf);
            lf = nullptr;
            OK(mkv_sharded_diff(a, b, c, &lf));
            if (lf) got_diff2[r] = keylist(lf);
            {
                Packed bk, bv;
                pack(sb[r], bk, bv);
                if (r == 1) OK(mkv_comm_inject_fault(c, MKV_FAULT_AFTER_META));
                fault_build[r] = mkv_sharded_build(b, c, bk.blob(), bv.blob(), 0, 1, nullptr);
                OK(mkv_sharded_build(b, c, bk.blob(), bv.blob(), 0, 1, nullptr));
                uint8_t rr[32];
                int hh = 0;
                if (r == 1) OK(mkv_comm_inject_fault(c, MKV_FAULT_AFTER_META));
                fault_root[r] = mkv_sharded_root(b, c, rr, &hh);
            }
            // in-range update of this shard, then the global root of both replicas in one all-gather
            Packed uk, uv;
            uk.add(sa[r].begin()->first);
            uv.add("updated-" + std::to_string(r));
            OK(mkv_tree_upsert(a, uk.blob(), uv.blob()));
            mkv_tree *ts[2] = {a, b};
            uint8_t roots[64];
            int hs[2] = {0, 0};
            OK(mkv_sharded_root_many(ts, 2, c, roots, hs));
            got_upd[r] = hs[0] ? std::string(reinterpret_cast<char *>(roots), 32) : "";
            CHECK(hs[1] && std::string(reinterpret_cast<char *>(roots + 32), 32) == want_b);
            // overlapping ranges: every rank builds rank 0's records -> MKV_EINVAL everywhere
            Packed ok_, ov_;
            pack(sa[0], ok_, ov_);
            bad_status[r] = mkv_sharded_build(b, c, ok_.blob(), ov_.blob(), 0, 1, nullptr);
            mkv_tree_destroy(a);
            mkv_tree_destroy(b);
            mkv_comm_destroy(c);
        });
    for (auto &t : th) t.join();
    for (int r = 0; r < world; ++r) {
        CHECK(got_a[r] == want_a);
        CHECK(got_b[r] == want_b);
        CHECK(got_diff[r] == want_diff);
        CHECK(got_upd[r] == want_upd);
        CHECK(bad_status[r] == MKV_EINVAL);
        CHECK(fail_status[r] == MKV_EINVAL);
        CHECK(fault_diff[r] == MKV_ENOMEM && fault_build[r] == MKV_ENOMEM && fault_root[r] == MKV_ENOMEM);
        CHECK(got_diff2[r] == want_diff);
        // the slices are the global list cut at the global offsets (ranges ordered by rank)
        CHECK(got_tot[r] == want_diff.size());
        CHECK(got_off[r] + got_slice[r].size() <= want_diff.size());
        CHECK(std::vector<std::string>(want_diff.begin() + got_off[r], want_diff.begin() + got_off[r] + got_slice[r].size()) ==
              got_slice[r]);
    }
    CHECK(got_off[0] == 0 && got_off[1] == got_slice[0].size() && got_off[2] == got_off[1] + got_slice[1].size());
    CHECK(got_off[2] + got_slice[2].size() == want_diff.size());
    std::printf("host world 3: %s (diff %zu keys)\n", g_fail ? "FAILED" : "ok", want_diff.size());
}

int main(int argc, char **argv) {
    const int dev = 0;
    const bool rccl = !(argc > 1 && std::string(argv[1]) == "--no-rccl");
    if (rccl) test_rccl_world1(dev);
    test_host_world3(dev);
    std::printf("sharded: %s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}
