// mkv_merkle.hpp — header-only C++ mirror of MerkleKV's `crate::store::merkle::MerkleTree`
// (/root/reference/src/store/merkle.rs) over the C ABI in mkv_merkle.h.
//
// The reference is Rust; no Rust toolchain exists in this image, so the host side above the C ABI is
// provided in C++ with the reference's method names, argument meaning and None/empty behaviour.
// The reference API is infallible (no Result); this facade throws mkv::MerkleError on a non-OK status
// (the Rust facade in INTEGRATION.md panics instead). There is no CPU fallback.
//
// Semantics note: insert()/remove() are queued and applied as one ordered device batch before the
// next observation. The reference rebuilds after every insert (merkle.rs:52-56), and a rebuild is a
// function of the final leaf map only, so every observable result is identical.
//
// Const contract: the observers keep the reference's receivers — get_root_hash(&self),
// diff_keys(&self, &MerkleTree), leaves(&self), ... are const here — so call sites written against
// immutable bindings (sync.rs:61-67, server.rs:661-675) compile unchanged. Applying the queued
// operations from a const observer is interior mutability (the queue is `mutable`; the device tree is
// behind the handle): the observable value is the same as the reference's eager rebuild. Like the
// reference (Send, not shared across threads without a lock), one object must not be used from two
// threads at once.
#pragma once
#include <array>
#include <cstdint>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "mkv_merkle.h"

namespace mkv {

struct MerkleError : std::runtime_error {
    int status;
    MerkleError(int s, const std::string &m) : std::runtime_error(m), status(s) {}
};

inline void check(mkv_status s) {
    if (s != MKV_OK) throw MerkleError(s, std::string("mkv status ") + std::to_string(s) + ": " + mkv_last_error());
}

using Digest = std::array<uint8_t, 32>;

// Packs byte strings into an mkv_blob (owns the storage while alive).
struct PackedBlob {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offsets{0};
    void push(std::string_view s) {
        bytes.insert(bytes.end(), s.begin(), s.end());
        offsets.push_back(bytes.size());
    }
    mkv_blob blob() const { return mkv_blob{bytes.data(), offsets.data(), offsets.size() - 1}; }
    size_t size() const { return offsets.size() - 1; }
};

class MerkleTree {
   public:
    // MerkleTree::new() — merkle.rs:36-41
    explicit MerkleTree(int device = 0) : dev_(device) { check(mkv_tree_create(device, &h_)); }
    ~MerkleTree() {
        if (h_) mkv_tree_destroy(h_);
    }
    MerkleTree(const MerkleTree &o) : dev_(o.dev_) {  // #[derive(Clone)] — merkle.rs:27
        o.flush();
        check(mkv_tree_create(dev_, &h_));
        check(mkv_tree_clone(o.h_, h_));
    }
    MerkleTree &operator=(const MerkleTree &) = delete;
    MerkleTree(MerkleTree &&o) noexcept : dev_(o.dev_), h_(o.h_), pending_(std::move(o.pending_)) { o.h_ = nullptr; }

    // insert(&mut self, key, value) — merkle.rs:52-56
    void insert(std::string_view key, std::string_view value) { pending_.push_back({false, std::string(key), std::string(value)}); }
    // remove(&mut self, key) — merkle.rs:59-62
    void remove(std::string_view key) { pending_.push_back({true, std::string(key), {}}); }

    // Bulk new() + n x insert() as one device build (sync.rs:104-143, server.rs:661-669).
    void build(const std::vector<std::pair<std::string, std::string>> &kv) {
        pending_.clear();
        PackedBlob k, v;
        for (auto &p : kv) {
            k.push(p.first);
            v.push(p.second);
        }
        check(mkv_tree_build(h_, k.blob(), v.blob()));
    }

    // get_root_hash() — merkle.rs:65-67
    std::optional<Digest> get_root_hash() const {
        flush();
        Digest d{};
        int has = 0;
        check(mkv_tree_root(h_, d.data(), &has));
        if (!has) return std::nullopt;
        return d;
    }

    size_t len() const {
        flush();
        uint64_t n = 0;
        check(mkv_tree_len(h_, &n));
        return n;
    }

    // inorder_keys() — merkle.rs:126-130
    std::vector<std::string> inorder_keys() const {
        std::vector<std::string> out;
        for (auto &kv : leaves()) out.push_back(kv.first);
        return out;
    }

    // leaves() — merkle.rs:133-138
    std::vector<std::pair<std::string, Digest>> leaves() const {
        flush();
        uint64_t n = 0;
        check(mkv_tree_len(h_, &n));
        std::vector<uint8_t> dg(32 * (n ? n : 1));
        mkv_keylist *kl = nullptr;
        check(mkv_tree_leaves(h_, &kl, dg.data()));
        auto keys = take(kl);
        std::vector<std::pair<std::string, Digest>> out;
        for (size_t i = 0; i < keys.size(); ++i) {
            Digest d;
            std::memcpy(d.data(), dg.data() + 32 * i, 32);
            out.emplace_back(std::move(keys[i]), d);
        }
        return out;
    }

    // Level l of the implicit tree (0 = leaf digests in key order).
    std::vector<Digest> level(uint32_t l) const {
        flush();
        uint64_t c = 0;
        check(mkv_tree_level(h_, l, &c, nullptr));
        std::vector<Digest> out(c);
        if (c) check(mkv_tree_level(h_, l, &c, out.data()->data()));
        return out;
    }
    uint32_t level_count() const {
        flush();
        uint32_t L = 0;
        check(mkv_tree_level_count(h_, &L));
        return L;
    }

    // preorder_hashes() — merkle.rs:142-153 (a promoted node is the same node as its child: visited once)
    std::vector<Digest> preorder_hashes() const {
        uint32_t L = level_count();
        std::vector<std::vector<Digest>> lv;
        for (uint32_t l = 0; l < L; ++l) lv.push_back(level(l));
        std::vector<Digest> out;
        if (!L) return out;
        struct Item {
            uint32_t l;
            uint64_t j;
            bool emit;
        };
        std::vector<Item> st{{L - 1, 0, true}};
        while (!st.empty()) {
            Item it = st.back();
            st.pop_back();
            if (it.emit) out.push_back(lv[it.l][it.j]);
            if (it.l == 0) continue;
            if (2 * it.j + 1 < lv[it.l - 1].size()) {
                st.push_back({it.l - 1, 2 * it.j + 1, true});
                st.push_back({it.l - 1, 2 * it.j, true});
            } else {
                st.push_back({it.l - 1, 2 * it.j, false});
            }
        }
        return out;
    }

    // node_count() — merkle.rs:156-163
    size_t node_count() const {
        flush();
        uint64_t c = 0;
        check(mkv_tree_node_count(h_, &c));
        return c;
    }

    // Shape of the root's children (merkle.rs:343-358 tests): is child `right` (or left) a leaf?
    // A promoted node is the same node as its only child (R5), exactly as in the reference.
    bool root_child_is_leaf(bool right) const {
        uint32_t L = level_count();
        if (L < 2) return false;
        std::vector<uint64_t> sizes;
        for (uint32_t l = 0; l < L; ++l) {
            uint64_t c = 0;
            check(mkv_tree_level(h_, l, &c, nullptr));
            sizes.push_back(c);
        }
        uint32_t l = L - 2;
        uint64_t j = right ? 1 : 0;
        while (l > 0 && 2 * j + 1 >= sizes[l - 1]) {
            --l;
            j *= 2;
        }
        return l == 0;
    }

    // diff_keys(&other) — merkle.rs:171-196
    std::vector<std::string> diff_keys(const MerkleTree &other) const {
        flush();
        other.flush();
        mkv_keylist *kl = nullptr;
        check(mkv_tree_diff(h_, other.h_, &kl));
        return take(kl);
    }
    // diff_first_key(&other) — merkle.rs:199-204
    std::optional<std::string> diff_first_key(const MerkleTree &other) const {
        auto d = diff_keys(other);
        if (d.empty()) return std::nullopt;
        return d.front();
    }

    // Root of a fresh tree over the keys starting with the byte prefix (range reduction; '*' is a byte).
    std::optional<Digest> prefix_root(std::string_view prefix) const {
        flush();
        Digest d{};
        int has = 0;
        check(mkv_tree_prefix_root(h_, reinterpret_cast<const uint8_t *>(prefix.data()), prefix.size(), d.data(), &has));
        if (!has) return std::nullopt;
        return d;
    }
    // HASH [pattern] — server.rs:647-685 with its convention (:651-656): "" or "*" = every key.
    std::optional<Digest> hash_pattern(std::string_view pattern) const {
        flush();
        Digest d{};
        int has = 0;
        check(mkv_tree_hash_pattern(h_, reinterpret_cast<const uint8_t *>(pattern.data()), pattern.size(), d.data(), &has));
        if (!has) return std::nullopt;
        return d;
    }

    mkv_tree *handle() const {
        flush();
        return h_;
    }

   private:
    struct Op {
        bool rm;
        std::string k, v;
    };
    int dev_;
    mkv_tree *h_ = nullptr;
    mutable std::vector<Op> pending_;  // interior mutability: applied by the first observer

    static std::vector<std::string> take(mkv_keylist *kl) {
        uint64_t n = 0;
        const uint8_t *b = nullptr;
        const uint64_t *o = nullptr;
        mkv_status s = mkv_keylist_get(kl, &n, &b, &o);
        std::vector<std::string> out;
        if (s == MKV_OK)
            for (uint64_t i = 0; i < n; ++i) out.emplace_back(reinterpret_cast<const char *>(b + o[i]), o[i + 1] - o[i]);
        mkv_keylist_free(kl);
        check(s);
        return out;
    }

    void flush() const {
        if (pending_.empty()) return;
        PackedBlob k, v;
        std::vector<uint8_t> rm;
        bool any = false, all = true;
        for (auto &op : pending_) {
            k.push(op.k);
            v.push(op.v);
            rm.push_back(op.rm ? 1 : 0);
            any |= op.rm;
            all &= op.rm;
        }
        pending_.clear();
        if (all) check(mkv_tree_remove(h_, k.blob()));
        else if (!any) check(mkv_tree_upsert(h_, k.blob(), v.blob()));
        else check(mkv_tree_apply(h_, k.blob(), v.blob(), rm.data()));
    }
};

}  // namespace mkv
