// kernels.hpp — internal launcher API between the C-ABI runtime (tree.cpp) and the HIP kernels.
// All launchers are asynchronous on `st`; none allocates or synchronises.
#pragma once
#include "common.hpp"
#include "leaf.hpp"

namespace mkv {

// ---- Kernel A: leaf hashing (k_leaf.hip) ----
// Up to 16 record batches hashed in one launch (dirty-path updates of several replicas).
constexpr int LEAF_MULTI_MAX = 16;
struct LeafBatches {
    const uint8_t *kb[LEAF_MULTI_MAX];
    const uint64_t *koff[LEAF_MULTI_MAX];
    const uint8_t *vb[LEAF_MULTI_MAX];
    const uint64_t *voff[LEAF_MULTI_MAX];
    uint64_t m[LEAF_MULTI_MAX];
    uint64_t base[LEAF_MULTI_MAX];  // batch b's digests at out + 32 x base[b]
};
void launch_leaf_hash_multi(const LeafBatches &B, uint32_t k, uint64_t mmax, uint8_t *out, hipStream_t st);
// Words of the leaf stage's device counter block (ctr, leaf.hpp): chunk hand-out counters and the list of
// chunks the fixed-shape kernel leaves to the ragged one.
size_t leaf_ctr_words(uint64_t n);
// Waves of the fixed-shape kernel's grid for n records (its hand-off slots; the ragged stage reads them).
uint32_t leaf_fixed_waves(uint64_t n);
// The fixed-shape kernel (k_leaf_direct): zeroes the counter head and the hand-off slots, hashes every
// chunk of the configs' 32/100-B shape and hands every other chunk to the ragged stage.
void launch_leaf_fixed(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t *out_digests, uint32_t *ctr, hipStream_t st, const KeyOut &KO);
// Every chunk launch_leaf_fixed left (k_ragged.hip: any key / value lengths and alignments) except the
// records near the blobs' ends. Same stream, after launch_leaf_fixed.
void launch_leaf_ragged(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                        uint8_t *out_digests, uint32_t *ctr, hipStream_t st, const KeyOut &KO);
// The records near the blobs' ends (a prefix and a suffix it finds itself; k_ragged.hip rg_inner): needs
// nothing from the other leaf kernels, so it may run on another stream beside them (it may rehash a record
// k_leaf_direct also hashes: the same 32 bytes).
void launch_leaf_edges(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                       uint8_t *out_digests, hipStream_t st);
// Key bytes of the chunks the ragged stage hashes (k_leaf_ragged stores only their offsets), 16-B
// granules at the source offsets into kdst (<= kcap). Needs only launch_leaf_fixed's hand-off words: may
// run on another stream once launch_leaf_fixed is done.
void launch_keycopy_ragged(const uint8_t *kb, const uint64_t *koff, uint64_t n, const uint32_t *ctr, uint8_t *kdst,
                           uint64_t kcap, hipStream_t st);
// Both (the whole leaf stage; the ragged key copy queued after it). KO: optional key-ownership copy
// (leaf.hpp; used only when kb is 16-B aligned).
void launch_leaf_hash(const uint8_t *kb, const uint64_t *koff, const uint8_t *vb, const uint64_t *voff, uint64_t n,
                      uint8_t *out_digests, uint32_t *ctr, hipStream_t st, const KeyOut &KO = KeyOut{});

// ---- Kernel C: ordering (k_sort.hip) ----
// pfx[i] = big-endian first 8 key bytes, zero padded (key i of kb/koff); idx[i] = i
void launch_prefix64(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint64_t *pfx, uint32_t *idx,
                     hipStream_t st);
// Scratch bytes needed by radix_sort_pairs / scans for n elements.
size_t radix_scratch_bytes(uint64_t n);
size_t scan_scratch_bytes(uint64_t n);
// Stable LSD radix sort of (key, val) pairs on key bits [bit0, bit1). Ping-pongs between (k, v) and
// (k2, v2); returns true if the result ended in (k2, v2).
bool radix_sort_pairs(uint64_t *k, uint32_t *v, uint64_t *k2, uint32_t *v2, uint64_t n, int bit0, int bit1,
                      void *scratch, hipStream_t st);
// Exclusive scans (out may alias in). total (device, may be null) receives the sum.
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total, void *scratch,
                        hipStream_t st);
void exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, void *scratch,
                        hipStream_t st);

// tie[i] = (pfx[i] == pfx[i-1]) for i>0, tie[0] = 0; count[0] += number of ties. tie has n+1 entries
// (tie[n] = 0 sentinel). Tie-run heads (tie[i] == 0, tie[i+1] == 1) go to heads[] (capacity n / 2 + 1,
// any order), count[1] += their number.
// zero / nzero (optional): words the first workgroup zeroes (a sort's histogram and control words, for the
// next sort; the passes that read them are done).
void launch_mark_ties(const uint64_t *pfx, uint64_t n, uint8_t *tie, uint32_t *count, uint32_t *heads,
                      hipStream_t st, int shift = 0, uint32_t *zero = nullptr, uint32_t nzero = 0);
// Adaptive prefix sort (tree builds): one histogram read gives all eight byte-digit histograms
// (counts[p*256+d], p = 0 the least significant byte) in `scratch`; the host then picks the digits
// worth a pass (radix_prefix_passes: bit p of digit_mask = sort on byte p). Digits below the chosen
// ones are left to the tie refinement; constant digits are skipped outright.
void radix_prefix_hist(const uint64_t *k, uint64_t n, void *scratch, hipStream_t st);
// Fused form for builds: pfx[i] = the 8 key bytes at byte offset `off` (0 = the prefix) AND all eight
// digit histograms, one read of the keys. Control words the onesweep passes never touch (they use
// 8 * 256 + 0..31): PH_MAXLEN_WORD = longest key length; with lcp = true (whatever `off` is) also
// PH_NLCP_WORD = ~(shortest zero-padded common prefix of any key with key 0, measured from byte 0) and
// PH_K0_WORD/+1 = key 0's first 8 bytes (hi, lo).
constexpr uint32_t PH_MAXLEN_WORD = 8 * 256 + 63;
constexpr uint32_t PH_NLCP_WORD = 8 * 256 + 62;
constexpr uint32_t PH_K0_WORD = 8 * 256 + 60;
constexpr uint32_t PH_NMINLEN_WORD = 8 * 256 + 58;  // ~(shortest key length)
constexpr uint32_t SORT_CTL_WORDS = 8 * 256 + 64;
void launch_pfx_from_window(uint64_t *pk, uint64_t n, uint64_t shared, uint32_t win, hipStream_t st);
// lcp: also measure the shared prefix with key 0 (PH_NLCP_WORD) and key 0's first bytes (PH_K0_WORD),
// for any window offset.
// zeroed: the SORT_CTL_WORDS words at scratch are already zero (else they are zeroed here). zero2: eight
// words zeroed on the way (the tie marker's and the short-run refinement's counters).
void launch_prefix_hist(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint64_t *pfx, void *scratch,
                        hipStream_t st, uint64_t off = 0, bool lcp = true, bool zeroed = false,
                        uint32_t *zero2 = nullptr);
// v_identity: the values are the input indices 0..n-1 and are not read (the first pass generates them;
// with no pass at all v is filled with them). The result is in (k, v) or, when true is returned, (k2, v2).
// scratch: the SORT_CTL_WORDS histogram / control words of launch_prefix_hist. lookback: ceil(n / 6144) x
// 256 u64 words that hold nothing but look-back words (zeroed once when allocated); *epoch: the caller's
// epoch counter, advanced once per pass.
bool radix_prefix_passes(uint64_t *k, uint32_t *v, uint64_t *k2, uint32_t *v2, uint64_t n, uint32_t digit_mask,
                         void *scratch, uint64_t *lookback, uint32_t *epoch, hipStream_t st, bool v_identity = false);
uint64_t radix_prefix_lookback_words(uint64_t n);
// Orders every tie run of <= 16 positions on the full key in place (one thread per run); tie[] becomes
// full-key equality there. count[0] += duplicate positions, count[1] += longer runs (left as they are).
// Visits only the *nheads run heads of launch_mark_ties (max_heads: a host-side upper bound on *nheads).
void launch_refine_small(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint32_t *perm, uint64_t *pfx,
                         uint8_t *tie, uint32_t *count, const uint32_t *heads, const uint32_t *nheads,
                         uint64_t max_heads, hipStream_t st);
// pfx[pos[k]] = 8-byte prefix of sorted key pos[k] (after a refinement that re-ordered tie runs).
// pfx[pos[k]] = prefix of key perm[pos[k]] (pos null: every position k < m)
void launch_fix_pfx(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint8_t *kb, const uint64_t *koff,
                    uint64_t *pfx, hipStream_t st);
// Refinement helpers (see tree.cpp refine_ties for the algorithm).
void launch_active_flags(const uint8_t *tie, uint64_t n, uint32_t *flags, hipStream_t st);
void launch_compact_positions(const uint32_t *flags, const uint32_t *scan, uint64_t n, uint32_t *out, hipStream_t st);
void launch_max_keylen(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint64_t *koff, uint32_t *out,
                       hipStream_t st);
void launch_refine_keys(const uint32_t *pos, uint64_t m, const uint32_t *perm, const uint8_t *tie, const uint8_t *kb,
                        const uint64_t *koff, uint32_t depth, int use_len, uint64_t *chunk, uint32_t *kidx,
                        uint32_t *perm_act, uint32_t *headflag, hipStream_t st);
void launch_gid_keys(const uint32_t *kidx, const uint32_t *excl, const uint32_t *head, uint64_t m, uint64_t *key2,
                     hipStream_t st);
void launch_gather_u64_by_u32(const uint64_t *src, const uint32_t *idx, uint64_t m, uint64_t *dst, hipStream_t st);
void launch_gather_u32_to_u64(const uint32_t *src, const uint32_t *idx, uint64_t m, uint64_t *dst, hipStream_t st);
void launch_refine_apply(const uint32_t *pos, uint64_t m, const uint32_t *sorted_k, const uint32_t *perm_act,
                         const uint64_t *chunk, uint32_t *perm, uint8_t *tie, uint32_t *count, hipStream_t st);
// keep[i] = !tie[i+1] && perm[i] < n_live
void launch_keep_flags(const uint8_t *tie, const uint32_t *perm, uint64_t n, uint64_t n_live, uint32_t *flags,
                       hipStream_t st);
void launch_compact_u64(const uint64_t *src, const uint32_t *flags, const uint32_t *scan, uint64_t n, uint64_t *dst,
                        hipStream_t st);
void launch_compact_u32(const uint32_t *src, const uint32_t *flags, const uint32_t *scan, uint64_t n, uint32_t *dst,
                        hipStream_t st);

// ---- gathers into sorted order ----
void launch_gather_digests(const uint32_t *perm, const uint8_t *dig_in, uint64_t n, uint8_t *out, hipStream_t st);
void launch_gather_keylens(const uint32_t *perm, const uint64_t *koff, uint64_t n, uint64_t *lens, hipStream_t st);
void launch_gather_keys(const uint32_t *perm, const uint8_t *kb, const uint64_t *koff, const uint64_t *koff_out,
                        uint64_t n, uint8_t *kb_out, hipStream_t st);
void launch_gather_u64(const uint32_t *perm, const uint64_t *src, uint64_t n, uint64_t *dst, hipStream_t st);
void launch_add_offset_u64(const uint64_t *src, uint64_t n, uint64_t add, uint64_t *dst, hipStream_t st);
void launch_iota_u32(uint32_t *dst, uint64_t n, hipStream_t st);

// ---- Kernel B: level reduction (k_reduce.hip) ----
// One fused launch produces up to MAX_FUSE levels. Level k (1-based within the launch) owns global
// node indices [a[k], a[k]+c[k]); S[k-1] is the global size of its child level.
constexpr int MAX_FUSE = 10;
struct FusePlan {
    const uint8_t *in;       // child level (local array; global index of in[0] is a[0])
    uint8_t *out[MAX_FUSE];  // out[k-1] = level k's local array
    uint64_t a[MAX_FUSE + 1];
    uint64_t c[MAX_FUSE + 1];
    uint64_t S[MAX_FUSE + 1];
    int nl;
    uint64_t tile0;  // first tile index (global, in units of 512 first-level parents)
    uint64_t ntiles;
    // Fused leaf gather (unsharded first launch only): level-0 child c is read from dig[perm[c]] and
    // also written to in[c], so the sorted leaf level is produced by the reduction itself.
    const uint32_t *perm;
    const uint8_t *dig;
    // Several trees of one level plan in one launch (grid.y = nz, the dirty update's rehash above the
    // climb): tree z's arrays sit ztab[z] bytes (two's complement) from the ones named above. null: one.
    const uint64_t *ztab;
    uint32_t nz;
};
void launch_reduce_fused(const FusePlan &p, hipStream_t st);
// Every remaining level in one launch (k_reduce_top): ntiles <= RD_TOP_TILES tiles of 512 parents fuse
// nf (<= 10) levels each, then the last tile to arrive climbs levels nf+1 .. nl (level nf holds <= ntiles
// nodes). arrive: a device counter that is 0 before the launch (the kernel leaves it 0 again). 64 tiles:
// starting the top at 1,024 tiles (a 10M tree from level 4 instead of one more fused launch + the top
// from level 8) measured slower in round 4 (229 vs 63 + 105 us).
constexpr int TOP_MAX_LEVELS = 40;
constexpr uint64_t RD_TOP_TILES = 64;
struct TopPlan {
    const uint8_t *in;
    uint8_t *out[TOP_MAX_LEVELS];
    uint64_t a[TOP_MAX_LEVELS + 1];
    uint64_t c[TOP_MAX_LEVELS + 1];
    uint64_t S[TOP_MAX_LEVELS + 1];
    int nl, nf;
    uint64_t tile0, ntiles;
    const uint32_t *perm;
    const uint8_t *dig;
    uint32_t *arrive;        // tree z: arrive[16 z] (one 64-B line per tree)
    const uint64_t *ztab;    // as FusePlan
    uint32_t nz;
};
void launch_reduce_top(const TopPlan &p, hipStream_t st);

// Seam combine for sharded trees (k_reduce.hip). entries: (level, index, digest) records sorted by
// (level, index); see tree.cpp. Writes the root.
void launch_seam_combine(const uint8_t *entries, uint32_t nent, const uint64_t *level_sizes, uint32_t nlevels,
                         uint8_t *scratch, uint8_t *root_out, hipStream_t st);
// Same from `world` raw fringe blocks in device memory (block r at blocks + r * stride, max_entries
// slots each): ordered on the device (scratch >= world * max_entries * 48 B, *count = entries), then
// combined. No host round trip.
void launch_seam_prep_combine(const uint8_t *blocks, uint32_t world, uint64_t stride, uint32_t max_entries,
                              const uint64_t *level_sizes, uint32_t nlevels, uint8_t *scratch, uint32_t *count,
                              uint8_t *root_out, hipStream_t st);

// ---- Kernel D: diff (k_diff.hip) ----
struct DiffSide {
    const uint8_t *kb;      // keys in storage order
    const uint64_t *koff;
    const uint32_t *perm;   // sorted position -> storage index
    const uint64_t *pfx;
    const uint8_t *dig;
    uint64_t n;
    // every key of the tree is klen bytes (tree klen_fixed): key s sits at kb + koff[0] + s * klen, one
    // dependent random read (perm) instead of two (perm, koff); 0 = variable lengths
    uint64_t klen;
};
constexpr int DIFF_ITEMS = 8;     // merged outputs per thread
constexpr int DIFF_THREADS = 256;
size_t diff_scratch_bytes(uint64_t nmerged);
// Pass 1 + scan + pass 2: writes refs (bit 63 = side B, low bits = sorted index) of the divergent keys
// in sorted order; count[0] (device) receives the number. defer: the aligned tiles' key checks run in a
// separate kernel after pass 2; count[1] = 1 when one failed (or their list overflowed): the refs are
// then not valid and the caller runs launch_diff again with defer = false (exact for any key sets).
void launch_diff(const DiffSide &A, const DiffSide &B, void *scratch, uint64_t *refs, uint64_t *count,
                 hipStream_t st, bool defer = true);
// Top-down diff for trees with equal leaf counts (identical level shapes).
// fin/fout: local indices; a_par/a_child: global index of local 0 at the parent/child level; r0/r1:
// extra child-level candidates (owned nodes with an unowned parent; UINT64_MAX = none).
void launch_topdown_level(const uint8_t *ca, const uint8_t *cb, uint64_t child_count, uint64_t a_par, uint64_t a_child,
                          uint64_t r0, uint64_t r1, const uint32_t *fin, const uint32_t *nin, uint32_t *fout,
                          uint32_t *nout, uint64_t max_frontier, hipStream_t st);
// *count += sampled positions whose sorted key prefixes differ (key-set screen for the top-down walk).
void launch_sample_pfx(const uint64_t *pa, const uint64_t *pb, uint64_t n, uint32_t samples, uint32_t *count,
                       hipStream_t st);
// The screen inside a jump (launch_topdown_jump SC): min(n, 256 x TD_SCREEN_SLOTS) samples into
// TD_SCREEN_SLOTS words (plain stores, so no zeroing), read by a later gated jump (scr).
constexpr int TD_SCREEN_SLOTS = 16;
struct TdScreen {
    const uint64_t *pa, *pb;
    uint64_t n;
    uint32_t *slots;  // nullptr: no screen in this jump
};
// check == false: the caller knows both key sequences are equal (same key-set id): refs only.
void launch_topdown_leaves(const uint64_t *pos, uint64_t m, const DiffSide &A, const DiffSide &B, bool check, uint64_t *refs,
                           uint32_t *nbad, hipStream_t st);
void launch_diff_keylens(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, uint64_t *lens,
                         hipStream_t st);
// off[k] = k * stride, k <= m (key-list offsets of keys of one fixed length).
void launch_fill_stride_u64(uint64_t *off, uint64_t m, uint64_t stride, hipStream_t st);
void launch_diff_keys(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, const uint64_t *off,
                      uint8_t *out, hipStream_t st);
// Fixed-length keys (klen % 16 == 0, klen < 2^20): key k at out + k x klen, one 16-B granule per thread.
void launch_diff_keys_fixed(const uint64_t *refs, uint64_t m, const DiffSide &A, const DiffSide &B, uint64_t klen,
                            uint8_t *out, hipStream_t st);
// One-wait tail of the unsharded top-down pair diff: k_td_gate after the landing on level 4 (screen word
// cnt[word] != 0 or a frontier over half the level: bit 31 set there, frontier emptied); then from the
// sorted side-A refs (count *mdev on the device): leaf-key check (nbad), key lengths padded to cap_m,
// scan (total at off[cap_m]), key bytes (cap_b) and their copy into the mapped pinned views doff / dkeys
// -- skipped when the list outgrows the capacity (the host then copies it from the refs). host_offsets
// (fixed-length keys): the host writes the offsets k x klen into doff's block itself; only the key bytes
// cross PCIe.
void launch_td_gate(uint32_t *cnt, uint32_t word, uint32_t level, uint64_t level_count, hipStream_t st);
// hsmall (optional, mapped pinned): the fixed-length form into host memory also stores the call's scalars —
// hsmall[0] = count, [1] = *nbad as it stands before the key check, [2] = key bytes, [3] = 1 on a leaf-key
// mismatch (the caller zeroes [3] first). Returns whether it did.
bool launch_diff_tail_dev(const uint64_t *refs, const uint32_t *mdev, const DiffSide &A, const DiffSide &B, bool check,
                          uint32_t *nbad, uint64_t cap_m, uint64_t cap_b, uint64_t *lens, uint64_t *off, void *scan_scr,
                          uint8_t *kout, uint8_t *doff, uint8_t *dkeys, hipStream_t st, uint64_t klen = 0,
                          bool host_offsets = false, uint64_t *hsmall = nullptr);
// Batched top-down walk (one base vs up to TD_MAX_VARIANTS trees with the same level plan).
constexpr int TD_MAX_VARIANTS = 64;
constexpr int MKV_MAXLEV_TD = 48;  // = MKV_MAXLEV (levels of a tree)
struct TdVariants {
    const uint8_t *nodes[TD_MAX_VARIANTS];  // each variant's node array (levels at the base's offsets)
};
void launch_topdown_level_batch(const uint8_t *ca, const TdVariants &V, uint64_t child_off, uint64_t child_count,
                                uint64_t a_par, uint64_t a_child, uint64_t r0, uint64_t r1, uint32_t k,
                                const uint64_t *fin, const uint32_t *nin, uint64_t *fout, uint32_t *nout,
                                uint64_t max_frontier, hipStream_t st);
// The top of an unsharded walk in ONE workgroup (round 6): the roots, then the jumps T[0] -> T[1] -> ...
// -> T[nt] (every target level holding <= TD_TOP_MAX_NODES nodes) with the frontier in LDS between them;
// the last level's divergent nodes go to fout (pair: u32 node; batch: variant << 32 | node) and its count to
// cnt[T[nt]], every target level's count to cnt[T[q]] (walk statistics). k = variants (pair: 1, V.nodes[0] =
// the other tree). Node (l, j) of any tree sits at 32 x (off[l] + j).
constexpr uint64_t TD_TOP_MAX_NODES = 2048;
constexpr uint64_t TD_TOP_MAX_FRONTIER = 8192;  // LDS frontier entries between the top's jumps
constexpr uint64_t TD_TOP_MAX_WORK = 4096;      // descendants one jump of the top may compare (4 passes of the workgroup)
struct TdTop {
    uint64_t off[MKV_MAXLEV_TD], cnt[MKV_MAXLEV_TD];
    uint32_t T[MKV_MAXLEV_TD];
    uint32_t nt;  // jumps T[0] -> ... -> T[nt]
};
// zero_n: cnt[0 .. zero_n) initialised by the kernel first (no fill launch before it): 0 below ff_from,
// 0xFFFFFFFF from ff_from on.
void launch_topdown_top(const uint8_t *na, const TdVariants &V, uint32_t k, const TdTop &P, void *fout, bool wide,
                        uint32_t *cnt, hipStream_t st, uint32_t zero_n = 0, uint32_t ff_from = ~0u);
// Jump k levels down from divergent parents (unsharded plans): fout gets every divergent descendant
// at the target level (desc_count nodes there). max_desc: upper bound on parents << k (grid sizing).
// gate: the one-wait pair diff's level-4 abort test folded into the jump from level 4 (k_td_gate's rule on
// gate[word] and *nin against level_count); nullptr = none. bm: a jump landing on the leaves also sets each
// divergent position's bit there (zeroed bitmap; positions_sorted_bitmap_dev then skips its set pass).
void launch_topdown_jump(const uint8_t *ca, const uint8_t *cb, uint64_t desc_count, int k, const uint32_t *fin,
                         const uint32_t *nin, uint32_t *fout, uint32_t *nout, uint64_t max_desc, hipStream_t st,
                         uint32_t *gate = nullptr, uint32_t word = 0, uint64_t level_count = 0, uint32_t *bm = nullptr,
                         const uint32_t *scr = nullptr, const TdScreen &SC = TdScreen{});
// Sharded plans: the frontier holds local indices of level l (global = local + a_par), descendants are
// addressed at level l - k as global - a_desc; seeds = a shard's fringe roots at levels lt..l (owned nodes
// whose parent is not owned), each compared through its span of level-lt descendants starting at first[i].
constexpr int TD_MAX_SEEDS = 12;
struct TdSeeds {
    uint32_t n, total;
    uint32_t span[TD_MAX_SEEDS];
    uint64_t first[TD_MAX_SEEDS];
};
void launch_topdown_jump_sh(const uint8_t *ca, const uint8_t *cb, uint64_t desc_count, int k, uint64_t a_par,
                            uint64_t a_desc, const TdSeeds &S, const uint32_t *fin, const uint32_t *nin, uint32_t *fout,
                            uint32_t *nout, uint64_t max_desc, hipStream_t st);
void launch_topdown_jump_batch(const uint8_t *ca, const TdVariants &V, uint64_t desc_off, uint64_t desc_count, int k,
                               const uint64_t *fin, const uint32_t *nin, uint64_t *fout, uint32_t *nout,
                               uint64_t max_desc, hipStream_t st, uint32_t *bm = nullptr,
                               uint64_t bn = 0, uint32_t *gate = nullptr, uint32_t word = 0, uint64_t level_count = 0);
// ent: sorted (variant << pb) | position.
// check: bit v set = variant v's keys at its divergent positions are compared with the base's.
void launch_topdown_leaves_batch(const uint64_t *ent, uint64_t m, int pb, const DiffSide &A, const DiffSide *Bs, uint64_t check,
                                 uint64_t *refs, uint32_t *nbad, uint32_t *count, hipStream_t st,
                                 const uint32_t *mdev = nullptr);
// Level-0 entries (variant << 32 | position; *mdev of them in f, at most cap) -> (variant << pb | position)
// in ascending order in out, through a k x n-bit bitmap bm (all-zero before and after) and bc
// (vpos_scratch_words(k x n) words).
uint64_t vpos_scratch_words(uint64_t bits);
void launch_vpos_sorted_dev(const uint64_t *f, const uint32_t *mdev, uint64_t cap, uint64_t n, uint32_t k, int pb,
                            uint32_t *bm, uint32_t *bc, void *scan_scr, uint64_t *out, hipStream_t st, bool bits_set = false);
// key[k] = (variant << pb) | position of frontier entry (variant << 32) | position; val[k] = k.
void launch_pack_entries(const uint64_t *ent, uint64_t m, int pb, uint64_t *key, uint32_t *val, hipStream_t st);
// Anti-entropy exchange: digests of level nodes by index (absent -> zeros); flags of indices whose local
// digest differs from the peer's (absent -> divergent).
void launch_node_digests(const uint8_t *lvl, uint64_t count, const uint64_t *idx, uint64_t m, uint8_t *out,
                         hipStream_t st);
void launch_compare_nodes(const uint8_t *lvl, uint64_t count, const uint64_t *idx, const uint8_t *peer, uint64_t m,
                          uint8_t *flag, hipStream_t st);
// Prefix range [lo, hi) of sorted keys starting with prefix (single-thread binary search).
void launch_prefix_bounds(const DiffSide &A, const uint8_t *prefix, uint32_t plen, uint64_t *lohi, hipStream_t st);

// ---- incremental dirty-path update (k_update.hip) ----
// pos[i] = sorted leaf position of batch key i (UINT64_MAX if it is not a leaf), idx[i] = i;
// *missing += keys that are not leaves.
// ps / ns: the locate samples of T's prefixes (launch_locate_samples).
void launch_locate(const uint8_t *kb, const uint64_t *koff, uint64_t m, const DiffSide &T, const uint64_t *ps,
                   uint64_t ns, uint64_t *pos, uint32_t *idx, uint32_t *missing, hipStream_t st);
// Every LOC_STRIDE-th sorted prefix (ps[j] = pfx[LOC_STRIDE x j], locate_samples(n) entries): the upper
// part of the locate binary search runs on this 1/64 copy.
constexpr uint64_t LOC_STRIDE = 64;
inline uint64_t locate_samples(uint64_t n) { return (n + LOC_STRIDE - 1) / LOC_STRIDE; }
void launch_locate_samples(const uint64_t *pfx, uint64_t n, uint64_t *ps, hipStream_t st);
// k trees at once (grid.y = tree): batch b of tree b (keys B.kb/B.koff, B.m records) located in T[b];
// pos[base_b + i] = (b << pbits) | position (position (1 << pbits) - 1 when the key is not a leaf: then
// *missing[b] += 1), idx[base_b + i] = base_b + i.
struct LocateMulti {
    DiffSide T[LEAF_MULTI_MAX];
    const uint64_t *ps[LEAF_MULTI_MAX];  // locate samples of T[b] (launch_locate_samples)
    uint64_t ns[LEAF_MULTI_MAX];
    uint32_t *missing[LEAF_MULTI_MAX];
    const uint64_t *hix[LEAF_MULTI_MAX];  // hash index of T[b] (launch_hix_build) or null: the sample search
    uint64_t hmask[LEAF_MULTI_MAX];
};
// Hash index of a tree's sorted keys: open addressing (linear probing) over cap = 2^k >= 2n slots, entry =
// (tag << 32 | sorted position), 0 = empty; tab zeroed by the caller.
void launch_hix_build(const DiffSide &T, uint64_t *tab, uint64_t mask, hipStream_t st);
void launch_locate_multi(const LeafBatches &B, const LocateMulti &L, uint32_t k, uint64_t mmax, int pbits,
                         uint64_t *pos, uint32_t *idx, hipStream_t st);
constexpr int DIRTY_MAX_TREES = 16;
// Level plan of a tree handle (owned global range [base, base + cnt) of a level of S nodes, stored at
// node offset off), shared by the replicas of one batched update.
constexpr int MKV_MAXLEV = 48;
struct LevelPlan {
    uint64_t base[MKV_MAXLEV], cnt[MKV_MAXLEV], off[MKV_MAXLEV], S[MKV_MAXLEV];
    int L;
};
// The dirty climb of k replicas sharing a level plan (k_update.hip k_dirty_climb): pos / bidx = the batch
// entries sorted by (tree << pbits | leaf position) with their batch indices, bdig = the batch digests;
// cnt[q][l]: tree q's dirty nodes per level (added to; zeroed by the caller). The climb stops at level
// lstop (-1: the top), where the dirty nodes are dense; the levels above are rehashed whole by the
// reduction (run_reduce from lstop, every tree in one launch: ztab = the trees' node-array offsets from
// tree 0's, written by the climb). bflags: one bit per entry boundary, all-zero before and after; mbox:
// climb_mbox_bytes(M) of scratch.
struct ClimbArgs {
    const uint64_t *pos;
    const uint32_t *bidx;
    const uint8_t *bdig;
    uint32_t M;
    int pbits;
    uint32_t k;
    uint8_t *nodes[DIRTY_MAX_TREES];
    const uint32_t *missing[DIRTY_MAX_TREES];  // non-zero: a batch key of that tree is not a leaf, tree untouched
    uint32_t *cnt[DIRTY_MAX_TREES];
    LevelPlan P;
    int lstop;
    uint32_t *bflags;
    uint8_t *mbox;
    uint64_t *ztab;
};
uint32_t climb_grid(uint64_t m);
size_t climb_mbox_bytes(uint64_t m);
void launch_dirty_climb(const ClimbArgs &A, hipStream_t st);

// Batch merge (k_update.hip): A = the tree's sorted leaves (dig = leaf level, indexed by position),
// B = sorted unique batch (perm = batch storage index, dig = batch digests in storage order, tomb =
// remove flags in batch storage order or null). Writes the surviving leaves' prefixes, storage indices
// (batch records at nstore_a + index) and digests; *count (device) = new leaf count.
size_t umerge_scratch_bytes(uint64_t M);
void launch_umerge(const DiffSide &A, const DiffSide &B, const uint8_t *tomb, uint32_t nstore_a, void *scratch,
                   uint64_t *pfx_out, uint32_t *perm_out, uint8_t *dig_out, uint64_t *count, hipStream_t st);

// ---- wire-format snapshot ingestion (k_wire.hip) ----
size_t wire_scratch_bytes(uint64_t len);
// Counts '\n' bytes (tile counts + exclusive scan in scratch; *d_total = line count); returns #tiles.
uint64_t wire_count_lines(const uint8_t *buf, uint64_t len, void *scratch, uint64_t *d_total, hipStream_t st);
// nl[j] = position of the j-th '\n' (needs the scratch of wire_count_lines).
void wire_emit_lines(const uint8_t *buf, uint64_t len, const void *scratch, uint64_t *nl, hipStream_t st);
// SCAN key i = line i+1 trimmed (str::trim_end); GET line i -> value / NOT_FOUND / malformed (*bad).
void launch_scan_keys(const uint8_t *buf, const uint64_t *nl, uint64_t n, uint64_t *kstart, uint64_t *klen,
                      hipStream_t st);
void launch_get_values(const uint8_t *buf, const uint64_t *nl, uint64_t n, uint64_t *vstart, uint64_t *vlen,
                       uint32_t *found, uint32_t *bad, hipStream_t st);
void launch_found_lengths(const uint64_t *len, const uint32_t *found, const uint32_t *rank, uint64_t n, uint64_t *out,
                          hipStream_t st);
void launch_pack_records(const uint8_t *src, const uint64_t *start, const uint64_t *len, const uint32_t *found,
                         const uint32_t *rank, const uint64_t *off_out, uint64_t n, uint8_t *dst, hipStream_t st);

// ---- redistribution into key-range shards (k_route.hip) ----
constexpr uint32_t ROUTE_MAX_WORLD = 256;
void launch_route_sample(const uint8_t *kb, const uint64_t *koff, uint64_t n, uint32_t m, uint64_t *out,
                         hipStream_t st);
// dkey[i] = destination rank of record i; counts (3 x world u64, zeroed): records, key bytes, value bytes.
void launch_route_dest(const uint8_t *kb, const uint64_t *koff, const uint64_t *voff, uint64_t n, const uint64_t *spl,
                       uint32_t world, uint64_t *dkey, uint64_t *counts, hipStream_t st);
void launch_route_lens(const uint32_t *perm, const uint64_t *off, uint64_t n, uint32_t *out, uint32_t *bad,
                       hipStream_t st);
void launch_u32_to_u64(const uint32_t *in, uint64_t n, uint64_t *out, hipStream_t st);

// ---- synthetic generator (k_gen.hip) — bench/test utility, not part of the reference API ----
// Ragged mode 2 of orc_gen_records (keys [klen/8, klen], values [vlen/16, vlen], packed); scan_scratch =
// scan_scratch_bytes(n) bytes.
void launch_gen_records_ragged(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, uint32_t shard,
                               uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb,
                               uint64_t *voff, void *scan_scratch, hipStream_t st);
void launch_gen_records(uint64_t seed, uint64_t idx0, uint64_t n, uint32_t klen, uint32_t vlen, uint32_t shard,
                        uint32_t nshards, uint32_t vfield, uint8_t *kb, uint64_t *koff, uint8_t *vb, uint64_t *voff,
                        hipStream_t st);

}  // namespace mkv
