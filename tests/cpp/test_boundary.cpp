// Boundary contract test: the reference's callers hold MerkleTree through immutable bindings and call
// get_root_hash(&self) / diff_keys(&self, &MerkleTree) on them (sync.rs:61-67, server.rs:661-675).
// These functions are written exactly that way against include/mkv_merkle.hpp — const references
// only, inserts queued before — so this file compiling is the "call sites compile unchanged" check, and
// running it checks the results through the C ABI (HIP path). Built by __graft_entry__.build().
#include <openssl/evp.h>

#include <algorithm>
#include <cstdio>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "mkv_merkle.hpp"

using mkv::MerkleTree;

static int g_fail = 0;
#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

static std::string hexs(const mkv::Digest &d) {
    static const char *x = "0123456789abcdef";
    std::string s;
    for (uint8_t b : d) {
        s += x[b >> 4];
        s += x[b & 15];
    }
    return s;
}

// sync.rs:61-67 — `let diffs = local_tree.diff_keys(&remote_tree);` with both trees immutable.
static std::vector<std::string> sync_diff(const MerkleTree &local_tree, const MerkleTree &remote_tree) {
    return local_tree.diff_keys(remote_tree);
}

// server.rs:672-682 — `match tree.get_root_hash() { Some(h) => hex::encode(h), None => "0".repeat(64) }`
static std::string hash_line(const MerkleTree &tree, const std::string &pat) {
    auto r = tree.get_root_hash();
    const std::string hex_root = r ? hexs(*r) : std::string(64, '0');
    return pat.empty() ? "HASH " + hex_root + "\r\n" : "HASH " + pat + " " + hex_root + "\r\n";
}

static mkv::Digest sha(const std::string &m) {
    mkv::Digest d{};
    unsigned int len = 0;
    EVP_Digest(m.data(), m.size(), d.data(), &len, EVP_sha256(), nullptr);
    return d;
}
static std::string u32be(size_t x) {
    std::string s(4, '\0');
    s[0] = (char)(x >> 24); s[1] = (char)(x >> 16); s[2] = (char)(x >> 8); s[3] = (char)x;
    return s;
}
static mkv::Digest leaf(const std::string &k, const std::string &v) { return sha(u32be(k.size()) + k + u32be(v.size()) + v); }

int main() {
    MerkleTree local, remote;
    for (int i = 0; i < 1000; ++i) {
        const std::string k = "key" + std::to_string(i), v = "v" + std::to_string(i);
        local.insert(k, v);
        remote.insert(k, i % 100 == 7 ? v + "-changed" : v);
    }
    remote.remove("key500");
    remote.insert("zz-remote-only", "x");
    // observers only through const references; the queued inserts are applied by the first of them
    const std::vector<std::string> d = sync_diff(local, remote);
    std::vector<std::string> want;
    for (int i = 0; i < 1000; ++i)
        if (i % 100 == 7 || i == 500) want.push_back("key" + std::to_string(i));
    want.push_back("zz-remote-only");
    std::sort(want.begin(), want.end());
    CHECK(d == want);
    const MerkleTree &cl = local;
    CHECK(cl.get_root_hash().has_value());
    CHECK(cl.get_root_hash() == local.get_root_hash());
    CHECK(cl.diff_first_key(remote) == std::optional<std::string>(want.front()));
    // HASH on an empty tree prints 64 zeros (server.rs:674); single leaf root = its leaf digest
    MerkleTree empty;
    CHECK(hash_line(empty, "") == "HASH " + std::string(64, '0') + "\r\n");
    MerkleTree one;
    one.insert("k", "v");
    CHECK(hash_line(one, "") == "HASH " + hexs(leaf("k", "v")) + "\r\n");
    CHECK(hexs(*one.get_root_hash()) == "5e4df0632cddbef333f4e40c3250f9ddaade5073bc56f239e52c1ecac1c2bca0");
    // HASH "*" = every key (server.rs:654); a real prefix narrows
    const MerkleTree &cr = remote;
    CHECK(cr.hash_pattern("*") == cr.get_root_hash());
    CHECK(cr.hash_pattern("") == cr.get_root_hash());
    CHECK(cr.hash_pattern("zz") == std::optional<mkv::Digest>(leaf("zz-remote-only", "x")));
    CHECK(!cr.hash_pattern("nope").has_value());
    // a const copy (Clone) observes the same state
    const MerkleTree copy(remote);
    CHECK(sync_diff(copy, remote).empty());
    std::printf("boundary: %s\n", g_fail ? "FAILED" : "ok");
    return g_fail ? 1 : 0;
}
