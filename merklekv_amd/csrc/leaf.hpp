// leaf.hpp — shared layout of Kernel A's two leaf-hash kernels (k_leaf.hip: fixed-shape k_leaf_direct;
// k_ragged.hip: store-shaped k_leaf_ragged) and of the counter block that hands chunks between them.
#pragma once
#include <stdint.h>

namespace mkv {

// A chunk is 64 consecutive records (one wave's worth).
constexpr uint32_t LEAF_CHUNK = 64;

// Counter block (leaf_ctr_words(n) u32, head zeroed before every leaf stage):
//   [CTR_FIXED]  k_leaf_direct's chunk hand-out counter. The first wave that meets a chunk of another
//                shape pushes it to CTR_ABORT with one atomicMax, so every later grab ends its wave.
//   [CTR_BP1]    1 + the first chunk k_leaf_direct never handed out (0: it handed out all of them).
//   [CTR_NLIST]  chunks k_leaf_direct handed out but left unhashed (the rest of an aborting wave's grab);
//                their ids follow at [CTR_LIST, CTR_LIST + nlist).
//   [CTR_RAGGED] k_leaf_ragged's hand-out counter over its virtual chunk space: the listed chunks
//                first, then chunks [B, nchunks).
constexpr uint32_t CTR_FIXED = 0, CTR_BP1 = 1, CTR_NLIST = 2, CTR_RAGGED = 3, CTR_HEAD = 4, CTR_LIST = 8;
constexpr uint32_t CTR_ABORT = 0x40000000u;

// Optional key-ownership copy fused into the fixed-shape kernel (builds from borrowed device inputs: the
// caller may reuse its buffers, so the tree keeps the key bytes and offsets): keys are stored to kdst at
// their source byte offsets (at most kcap bytes), offsets to odst. The chunks left to the ragged stage
// are copied by k_keycopy_rest.
struct KeyOut {
    uint8_t *kdst;   // null: no copy
    uint64_t *odst;  // null: offsets not copied
    uint64_t kcap;
};

}  // namespace mkv
