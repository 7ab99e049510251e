// common.hpp — shared host/device definitions for the MI355X (gfx950) Merkle hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <stdexcept>
#include <string>

namespace mkv {

// Error type carried from the runtime to the C ABI (mkv_status + thread-local message).
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

enum : int { ST_OK = 0, ST_EINVAL = 1, ST_EHIP = 2, ST_ENOMEM = 3, ST_ESTATE = 4 };

#define MKV_HIP(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            throw ::mkv::Error(e_ == hipErrorOutOfMemory ? ::mkv::ST_ENOMEM : ::mkv::ST_EHIP,          \
                               std::string(#expr " failed: ") + hipGetErrorString(e_));               \
    } while (0)

#define MKV_LAUNCH_CHECK()                                                                             \
    do {                                                                                               \
        hipError_t e_ = hipGetLastError();                                                             \
        if (e_ != hipSuccess)                                                                          \
            throw ::mkv::Error(::mkv::ST_EHIP, std::string("kernel launch in ") + __func__ + ": " +     \
                                                   hipGetErrorString(e_));                             \
    } while (0)

// Growable device buffer. Grows only; steady-state builds of the same size never re-allocate.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) {
            (void)hipDeviceSynchronize();  // growth is rare; never free under in-flight work
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    // Contents are NOT preserved on growth. 256 B of tail padding keeps wide over-reads in bounds.
    // Growth leaves 1/16 headroom (64 KiB granules) so sizes that fluctuate call to call (diff and
    // update outputs) do not reallocate — each reallocation is a device-wide sync + free + malloc.
    void *ensure(size_t bytes) {
        if (bytes <= cap && p) return p;
        release();
        size_t c = bytes + bytes / 16;
        c = (c + 65535) & ~size_t(65535);
        MKV_HIP(hipMalloc(&p, c + 256));
        cap = c;
        return p;
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

}  // namespace mkv

struct mkv_keylist;
struct mkv_tree;
namespace mkv {
// tree.cpp internals shared with comm.cpp: a library-owned key list (pinned host block) over host bytes
// (offsets[0] == 0); the thread's mkv_last_error message; a tree's global leaf count (its shard plan's N,
// or n when unsharded).
mkv_keylist *keylist_from_host(const uint8_t *bytes, const uint64_t *offsets, uint64_t n);
void set_last_error(const char *msg);
uint64_t tree_global_n(const mkv_tree *t);
// A key list in device memory: offsets[0..n] (offsets[0] == 0) and the key bytes (`bytes` of them).
struct DevKeys {
    uint64_t n = 0, bytes = 0;
    const uint64_t *off = nullptr;
    const uint8_t *kb = nullptr;
};
// diff_keys of a pair / the keys at sorted positions, left in the tree's device scratch (valid until the
// tree's next diff or keys call); the tree's stream, device and local leaf count; one device -> pinned
// copy of a device key list on stream st (complete on return).
DevKeys tree_diff_device(const mkv_tree *a, const mkv_tree *b);
DevKeys tree_keys_at_device(const mkv_tree *t, const uint64_t *pos, uint64_t m);
hipStream_t tree_stream(const mkv_tree *t);
// The library's bounded wait for a stream (poll, then yield, then sleep; MKV_EHIP after
// MKV_WAIT_TIMEOUT_S instead of blocking forever).
void wait_bounded(hipStream_t s);
int tree_device(const mkv_tree *t);
uint64_t tree_len(const mkv_tree *t);
mkv_keylist *keylist_from_device(const uint64_t *d_off, const uint8_t *d_kb, uint64_t n, uint64_t bytes, hipStream_t st);

}  // namespace mkv
