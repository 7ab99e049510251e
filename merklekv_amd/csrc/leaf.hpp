// leaf.hpp — shared layout of Kernel A's two leaf-hash kernels (k_leaf.hip: fixed-shape k_leaf_direct;
// k_ragged.hip: store-shaped k_leaf_ragged) and of the counter block that hands chunks between them.
#pragma once
#include <stdint.h>

namespace mkv {

// A chunk is 64 consecutive records (one wave's worth).
constexpr uint32_t LEAF_CHUNK = 64;

// Counter block (leaf_ctr_words(n) u32; head + one slot per fixed-kernel wave zeroed before every stage):
//   [CTR_FIXED]  k_leaf_direct's hand-out counter: wave w of NW starts with chunk w, later grabs take
//                LEAF_GRAIN chunks from NW + counter. B = min(NW + final counter, nch) is the first chunk
//                it never handed out.
//   [CTR_STOP]   set by any wave that met a chunk of another shape (that wave stops there and leaves the
//                chunk and the rest of its range in its slot); other waves go on.
//   [CTR_RAGGED] k_leaf_ragged's hand-out counter over its virtual chunk space: the slots' chunks first
//                (NW x LEAF_GRAIN ids, empty ones skipped), then chunks [B, nch).
//   [CTR_LIST + w] wave w's slot: (first chunk << 5) | count (0: nothing left to the ragged stage).
// No same-address atomics when every chunk is ragged: the waves' first chunks are static.
constexpr uint32_t CTR_FIXED = 0, CTR_STOP = 1, CTR_RAGGED = 2, CTR_HEAD = 4, CTR_LIST = 8;
constexpr uint32_t LEAF_GRAIN = 4;     // k_leaf_direct: chunks per hand-out atomic
constexpr uint32_t LEAF_MAX_WAVES = 16384;  // slots: fixed-kernel waves (persistent grid, <= 16 per CU)

// Key ownership of a build from borrowed device blobs: the leaf kernels store the key bytes they load at
// their source byte offsets into kdst (the tree's key buffer; kb 16-B aligned, so offsets coincide), and
// every record's key offset into odst. kcap: kdst's capacity in bytes (a store past it is skipped; the
// host then copies instead). Null pointers: no copy.
struct KeyOut {
    uint8_t *kdst;
    uint64_t *odst;
    uint64_t kcap;
};

}  // namespace mkv
