// C++ ports of the 56 unit tests in /root/reference/src/store/merkle.rs:207-1184, against the HIP path
// through the C ABI (include/mkv_merkle.hpp). Expected digests are computed like the reference's own
// tests (its leaf_hash helper, merkle.rs:222-226, and manual SHA-256 of concatenated children), here
// with OpenSSL. Seeded StdRng tests (rand 0.8.5 ChaCha12) use std::mt19937_64 with the same seeds:
// the asserted property (diff == changed/removed/extra set) does not depend on the stream.
// Built by __graft_entry__.build() (g++); run by tests/test_cpp_ports_gpu.py on a GPU box.
#include <openssl/evp.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "mkv_merkle.hpp"

using mkv::Digest;
using mkv::MerkleTree;

static Digest sha(const std::string &m) {
    Digest d{};
    unsigned int len = 0;
    EVP_Digest(m.data(), m.size(), d.data(), &len, EVP_sha256(), nullptr);
    return d;
}
static std::string u32be(size_t x) {
    std::string s(4, '\0');
    s[0] = (char)(x >> 24); s[1] = (char)(x >> 16); s[2] = (char)(x >> 8); s[3] = (char)x;
    return s;
}
static Digest leaf_hash(const std::string &k, const std::string &v) { return sha(u32be(k.size()) + k + u32be(v.size()) + v); }
static std::string raw(const Digest &d) { return std::string(reinterpret_cast<const char *>(d.data()), 32); }
static Digest H2(const Digest &a, const Digest &b) { return sha(raw(a) + raw(b)); }

using KV = std::vector<std::pair<std::string, std::string>>;
static void ins(MerkleTree &t, const KV &kv) {
    for (auto &p : kv) t.insert(p.first, p.second);
}
static std::set<std::string> S(const std::vector<std::string> &v) { return {v.begin(), v.end()}; }
static std::string NUL(const char *s, size_t n) { return std::string(s, n); }

static int g_fail = 0;
#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);           \
            ++g_fail;                                                            \
            return;                                                              \
        }                                                                        \
    } while (0)

static std::vector<std::pair<const char *, std::function<void()>>> g_tests;
#define TEST(name)                                                          \
    static void name();                                                     \
    static struct name##_reg {                                              \
        name##_reg() { g_tests.push_back({#name, name}); }                  \
    } name##_inst;                                                          \
    static void name()

static KV kn(size_t n, const char *kp = "k", const char *vp = "v") {
    KV kv;
    for (size_t i = 0; i < n; ++i) kv.push_back({kp + std::to_string(i), vp + std::to_string(i)});
    return kv;
}

TEST(test_single_leaf_root_equals_leaf_hash) {
    MerkleTree t0;
    CHECK(!t0.get_root_hash());
    MerkleTree t1;
    t1.insert("k", "v");
    CHECK(t1.get_root_hash() == leaf_hash("k", "v"));
    MerkleTree t2;
    t2.insert("key1", "value1");
    t2.insert("key2", "value2");
    auto rb = t2.get_root_hash();
    t2.insert("key2", "new_value");
    CHECK(t2.get_root_hash() != rb);
    t2.remove("key1");
    CHECK(t2.get_root_hash().has_value());
    t2.remove("key2");
    CHECK(!t2.get_root_hash());
}
TEST(test_root_hash_is_32_bytes) {
    MerkleTree t;
    t.insert("a", "1");
    CHECK(t.get_root_hash()->size() == 32);
}
TEST(test_insert_same_value_idempotent) {
    MerkleTree t;
    t.insert("k1", "v1");
    auto r1 = t.get_root_hash();
    t.insert("k1", "v1");
    CHECK(t.get_root_hash() == r1);
}
TEST(test_update_value_changes_root) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}});
    auto r = t.get_root_hash();
    t.insert("k2", "v2'");
    CHECK(t.get_root_hash() != r);
}
TEST(test_remove_nonexistent_keeps_root) {
    MerkleTree t;
    ins(t, {{"a", "1"}, {"b", "2"}});
    auto r = t.get_root_hash();
    t.remove("c");
    CHECK(t.get_root_hash() == r);
}
TEST(test_odd_number_of_leaves_promotes_one_leaf) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    CHECK(t.root_child_is_leaf(false) != t.root_child_is_leaf(true));
}
TEST(test_many_items_and_unicode_stability) {
    KV d{{"α", "1"}, {"β", "2"}, {"γ", "3"}, {"中文", "值"}, {"emoji🙂", "ok"}, {"key6", "v6"}, {"key7", "v7"},
         {"key8", "v8"}, {"key9", "v9"}, {"key10", "v10"}};
    MerkleTree t;
    ins(t, d);
    auto r1 = t.get_root_hash();
    ins(t, d);
    CHECK(t.get_root_hash() == r1);
}
TEST(hard_determinism_even_count_different_insert_orders) {
    KV p{{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}, {"k4", "v4"}};
    MerkleTree a, b;
    ins(a, p);
    KV r(p.rbegin(), p.rend());
    ins(b, r);
    CHECK(a.get_root_hash() == b.get_root_hash());
}
TEST(hard_determinism_odd_count_different_insert_orders) {
    MerkleTree a, b;
    ins(a, {{"a", "1"}, {"b", "2"}, {"c", "3"}});
    ins(b, {{"b", "2"}, {"c", "3"}, {"a", "1"}});
    CHECK(a.get_root_hash() == b.get_root_hash());
}
TEST(hard_serialization_ambiguity_colon_separator) {
    MerkleTree a, b;
    ins(a, {{"x", "y"}, {"a:", "b"}});
    ins(b, {{"x", "y"}, {"a", ":b"}});
    CHECK(a.get_root_hash() != b.get_root_hash());
}
TEST(hard_two_independent_trees_same_set_same_root) {
    KV s{{"u", "1"}, {"v", "2"}, {"w", "3"}, {"z", "4"}, {"q", "5"}};
    MerkleTree a, b;
    ins(a, {s[2], s[0], s[4], s[1], s[3]});
    ins(b, {s[4], s[3], s[2], s[1], s[0]});
    CHECK(a.get_root_hash() == b.get_root_hash());
}
TEST(hard_manual_root_two_leaves) {
    MerkleTree t;
    ins(t, {{"a", "A"}, {"b", "B"}});
    CHECK(t.get_root_hash() == H2(leaf_hash("a", "A"), leaf_hash("b", "B")));
}
TEST(hard_empty_and_nul_bytes) {
    KV c{{"", ""}, {"", "nonempty"}, {"nonempty", ""}, {NUL("has\0nul", 7), "v"}, {"k", NUL("va\0lue", 6)},
         {NUL("a\0b", 3), NUL("\0\0\0", 3)}};
    MerkleTree t;
    ins(t, c);
    auto r1 = t.get_root_hash();
    ins(t, c);
    CHECK(t.get_root_hash() == r1);
}
TEST(hard_remove_then_reinsert_restores_root) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    auto r0 = t.get_root_hash();
    t.remove("k2");
    CHECK(t.get_root_hash() != r0);
    t.insert("k2", "v2");
    CHECK(t.get_root_hash() == r0);
}
TEST(hard_update_vs_new_key_diff) {
    MerkleTree base;
    ins(base, {{"k1", "v1"}, {"k2", "v2"}});
    auto rb = base.get_root_hash();
    MerkleTree a(base), b(base);
    a.insert("k2", "v2_updated");
    b.insert("k3", "v3");
    CHECK(rb != a.get_root_hash());
    CHECK(rb != b.get_root_hash());
    CHECK(a.get_root_hash() != b.get_root_hash());
}
TEST(hard_multiple_idempotent_updates) {
    MerkleTree t;
    t.insert("k", "v");
    auto r1 = t.get_root_hash();
    for (int i = 0; i < 10; ++i) {
        t.insert("k", "v");
        CHECK(t.get_root_hash() == r1);
    }
    t.insert("k", "v2");
    CHECK(t.get_root_hash() != r1);
}
TEST(hard_shape_three_leaves) {
    MerkleTree t;
    ins(t, {{"a", "1"}, {"b", "2"}, {"c", "3"}});
    CHECK(t.root_child_is_leaf(false) != t.root_child_is_leaf(true));
}
TEST(hard_clone_then_mutate_diverges) {
    MerkleTree t1;
    ins(t1, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    MerkleTree t2(t1);
    CHECK(t1.get_root_hash() == t2.get_root_hash());
    MerkleTree t2m(t2);
    t2m.insert("k2", "v2_new");
    CHECK(t1.get_root_hash() != t2m.get_root_hash());
}
TEST(hard_stress_delete_half_then_restore) {
    MerkleTree t;
    ins(t, kn(200));
    auto r0 = t.get_root_hash();
    for (int i = 0; i < 100; ++i) t.remove("k" + std::to_string(i));
    CHECK(t.get_root_hash() != r0);
    for (int i = 0; i < 100; ++i) t.insert("k" + std::to_string(i), "v" + std::to_string(i));
    CHECK(t.get_root_hash() == r0);
}
TEST(hard_manual_root_four_leaves) {
    KV it{{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}, {"k4", "v4"}};
    MerkleTree t;
    ins(t, it);
    std::vector<Digest> h;
    for (auto &p : it) h.push_back(leaf_hash(p.first, p.second));
    CHECK(t.get_root_hash() == H2(H2(h[0], h[1]), H2(h[2], h[3])));
}
TEST(diff_no_difference_returns_empty) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    CHECK(a.get_root_hash() == b.get_root_hash());
    CHECK(a.diff_keys(b).empty());
    CHECK(!a.diff_first_key(b));
}
TEST(diff_single_value_change_returns_that_key) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}});
    ins(b, {{"k1", "v1"}, {"k2", "DIFF"}});
    CHECK(S(a.diff_keys(b)) == std::set<std::string>{"k2"});
    CHECK(a.diff_first_key(b) == std::string("k2"));
}
TEST(diff_missing_key_is_detected) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}});
    CHECK(S(a.diff_keys(b)) == std::set<std::string>{"k3"});
    CHECK(a.diff_first_key(b) == std::string("k3"));
}
TEST(diff_extra_key_is_detected) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}, {"kX", "vX"}});
    CHECK(S(a.diff_keys(b)) == std::set<std::string>{"kX"});
    CHECK(a.diff_first_key(b) == std::string("kX"));
}
TEST(diff_multiple_keys_detected_unordered) {
    MerkleTree a, b;
    KV base{{"a", "1"}, {"b", "2"}, {"c", "3"}, {"d", "4"}};
    ins(a, base);
    ins(b, base);
    b.insert("b", "2'");
    b.insert("d", "4'");
    std::set<std::string> e{"b", "d"};
    CHECK(S(a.diff_keys(b)) == e);
    CHECK(e.count(*a.diff_first_key(b)));
}
TEST(diff_empty_vs_nonempty_returns_all_keys) {
    MerkleTree a, b;
    ins(a, {{"x", "1"}, {"y", "2"}, {"z", "3"}});
    CHECK(S(a.diff_keys(b)) == (std::set<std::string>{"x", "y", "z"}));
    CHECK(a.diff_first_key(b).has_value());
}
TEST(diff_unicode_and_nul_bytes) {
    KV c{{"α", "1"}, {"中文", "值"}, {"emoji🙂", "ok"}, {NUL("nu\0l", 4), "v"}, {"k", NUL("va\0lue", 6)}};
    MerkleTree a, b;
    ins(a, c);
    ins(b, c);
    b.insert("中文", "变");
    CHECK(S(a.diff_keys(b)) == std::set<std::string>{"中文"});
    CHECK(a.diff_first_key(b) == std::string("中文"));
}
TEST(diff_structure_mismatch_due_to_odd_promotion) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}, {"k4", "v4"}});
    CHECK(S(a.diff_keys(b)) == std::set<std::string>{"k4"});
    CHECK(a.diff_first_key(b) == std::string("k4"));
}
TEST(diff_collects_all_keys_when_both_sides_have_unique_extras) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}});
    a.insert("kA", "vA");
    b.insert("kB", "vB");
    std::set<std::string> e{"kA", "kB"};
    CHECK(S(a.diff_keys(b)) == e);
    CHECK(e.count(*a.diff_first_key(b)));
}
TEST(diff_when_both_changed_same_key) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "A"}});
    ins(b, {{"k1", "v1"}, {"k2", "B"}});
    CHECK(S(a.diff_keys(b)).count("k2"));
    CHECK(a.diff_first_key(b) == std::string("k2"));
}
TEST(diff_remove_then_reinsert_restores_no_diff) {
    MerkleTree a, b;
    KV base{{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}};
    ins(a, base);
    ins(b, base);
    b.remove("k2");
    CHECK(S(a.diff_keys(b)).count("k2"));
    b.insert("k2", "v2");
    CHECK(a.diff_keys(b).empty());
}
TEST(diff_random_value_changes_detected_correctly) {
    MerkleTree a, b;
    ins(a, kn(120));
    ins(b, kn(120));
    std::mt19937_64 rng(2024);
    std::set<std::string> changed;
    for (int i = 0; i < 15; ++i) {
        size_t idx = rng() % 120;
        b.insert("k" + std::to_string(idx), "DIFF" + std::to_string(idx));
        changed.insert("k" + std::to_string(idx));
    }
    CHECK(S(a.diff_keys(b)) == changed);
}
TEST(diff_random_removals_detected_correctly) {
    MerkleTree a, b;
    ins(a, kn(150));
    ins(b, kn(150));
    std::mt19937_64 rng(99);
    std::set<std::string> removed;
    for (int i = 0; i < 25; ++i) {
        std::string k = "k" + std::to_string(rng() % 150);
        if (!removed.count(k)) {
            b.remove(k);
            removed.insert(k);
        }
    }
    CHECK(S(a.diff_keys(b)) == removed);
}
TEST(diff_structure_mismatch_large_random_subset) {
    MerkleTree a, b;
    ins(a, kn(300));
    ins(b, kn(300));
    std::set<std::string> e;
    for (int j = 0; j < 40; ++j) {
        b.insert("extra" + std::to_string(j), "val" + std::to_string(j));
        e.insert("extra" + std::to_string(j));
    }
    CHECK(S(a.diff_keys(b)) == e);
}
TEST(t01_empty_tree_root_none) {
    MerkleTree t;
    CHECK(!t.get_root_hash());
    CHECK(t.node_count() == 0);
}
TEST(t02_single_leaf_root_equals_leaf) {
    MerkleTree t;
    t.insert("a", "A");
    CHECK(t.get_root_hash() == leaf_hash("a", "A"));
    CHECK(t.node_count() == 1);
}
TEST(t03_root_len_32) {
    MerkleTree t;
    t.insert("x", "1");
    CHECK(t.get_root_hash()->size() == 32);
}
TEST(t04_inorder_keys_sorted) {
    MerkleTree t;
    ins(t, {{"k2", "v2"}, {"k1", "v1"}, {"k10", "v10"}});
    CHECK(t.inorder_keys() == (std::vector<std::string>{"k1", "k10", "k2"}));
}
TEST(t05_deterministic_root_order_independent) {
    KV it{{"a", "1"}, {"b", "2"}, {"c", "3"}, {"d", "4"}, {"e", "5"}};
    MerkleTree a, b;
    ins(a, it);
    KV r(it.rbegin(), it.rend());
    ins(b, r);
    CHECK(a.get_root_hash() == b.get_root_hash());
}
TEST(t06_manual_internal_hash_two_leaves) {
    MerkleTree t;
    ins(t, {{"a", "A"}, {"b", "B"}});
    CHECK(t.get_root_hash() == H2(leaf_hash("a", "A"), leaf_hash("b", "B")));
}
TEST(t07_manual_root_four_leaves) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}, {"k4", "v4"}});
    auto h = [](int i) { return leaf_hash("k" + std::to_string(i), "v" + std::to_string(i)); };
    CHECK(t.get_root_hash() == H2(H2(h(1), h(2)), H2(h(3), h(4))));
}
TEST(t08_odd_count_promotes_one) {
    MerkleTree t;
    ins(t, {{"a", "1"}, {"b", "2"}, {"c", "3"}});
    CHECK(t.root_child_is_leaf(false) != t.root_child_is_leaf(true));
}
TEST(t09_idempotent_insert) {
    MerkleTree t;
    t.insert("k", "v");
    auto r = t.get_root_hash();
    t.insert("k", "v");
    CHECK(t.get_root_hash() == r);
}
TEST(t10_update_changes_root) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}});
    auto r = t.get_root_hash();
    t.insert("k2", "v2_new");
    CHECK(t.get_root_hash() != r);
}
TEST(t11_remove_nonexistent_keeps_root) {
    MerkleTree t;
    ins(t, {{"a", "1"}, {"b", "2"}});
    auto r = t.get_root_hash();
    t.remove("zzz");
    CHECK(t.get_root_hash() == r);
}
TEST(t12_leaves_view_sorted_and_hashed) {
    MerkleTree t;
    ins(t, {{"b", "2"}, {"a", "1"}, {"c", "3"}});
    auto lv = t.leaves();
    CHECK(lv.size() == 3 && lv[0].first == "a" && lv[1].first == "b" && lv[2].first == "c");
    CHECK(lv[0].second == leaf_hash("a", "1") && lv[1].second == leaf_hash("b", "2") && lv[2].second == leaf_hash("c", "3"));
}
TEST(t13_preorder_non_empty) {
    MerkleTree t;
    ins(t, {{"a", "1"}, {"b", "2"}});
    auto pre = t.preorder_hashes();
    CHECK(!pre.empty() && pre[0] == *t.get_root_hash());
}
TEST(t14_node_count_two_pow) {
    MerkleTree t;
    ins(t, kn(4));
    CHECK(t.node_count() == 7);
}
TEST(t15_diff_no_change_empty_vec) {
    MerkleTree a, b;
    KV base{{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}};
    ins(a, base);
    ins(b, base);
    CHECK(a.diff_keys(b).empty() && b.diff_keys(a).empty());
    CHECK(!a.diff_first_key(b));
}
TEST(t16_diff_single_value_change) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}});
    ins(b, {{"k1", "v1"}, {"k2", "DIFF"}});
    CHECK(a.diff_keys(b) == std::vector<std::string>{"k2"});
    CHECK(a.diff_first_key(b) == std::string("k2"));
}
TEST(t17_diff_missing_key) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}});
    CHECK(a.diff_keys(b) == std::vector<std::string>{"k3"});
}
TEST(t18_diff_extra_key) {
    MerkleTree a, b;
    ins(a, {{"k1", "v1"}, {"k2", "v2"}});
    ins(b, {{"k1", "v1"}, {"k2", "v2"}, {"kX", "vX"}});
    CHECK(a.diff_keys(b) == std::vector<std::string>{"kX"});
}
TEST(t19_unicode_and_nul) {
    KV c{{"中文", "值"}, {NUL("nu\0l", 4), "v"}, {"k", NUL("va\0lue", 6)}};
    MerkleTree t;
    ins(t, c);
    auto r1 = t.get_root_hash();
    ins(t, c);
    CHECK(t.get_root_hash() == r1);
}
TEST(t20_remove_then_reinsert_restores) {
    MerkleTree t;
    ins(t, {{"k1", "v1"}, {"k2", "v2"}, {"k3", "v3"}});
    auto r0 = t.get_root_hash();
    t.remove("k2");
    CHECK(t.get_root_hash() != r0);
    t.insert("k2", "v2");
    CHECK(t.get_root_hash() == r0);
}
TEST(t21_many_items_stability) {
    MerkleTree t;
    ins(t, kn(50));
    auto r1 = t.get_root_hash();
    ins(t, kn(50));
    CHECK(t.get_root_hash() == r1);
}
TEST(t22_preorder_len_equals_node_count) {
    MerkleTree t;
    ins(t, kn(5));
    CHECK(t.preorder_hashes().size() == t.node_count());
}

int main() {
    int n = 0;
    for (auto &[name, fn] : g_tests) {
        int before = g_fail;
        try {
            fn();
        } catch (const std::exception &e) {
            std::printf("  EXCEPTION %s\n", e.what());
            ++g_fail;
        }
        std::printf("%s %s\n", g_fail == before ? "PASS" : "FAIL", name);
        ++n;
    }
    std::printf("%d tests, %d failed\n", n, g_fail);
    return g_fail ? 1 : 0;
}
