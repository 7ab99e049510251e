// k_wire.hip — snapshot ingestion from the SYNC wire format on the device.
//
// SyncManager::build_remote_merkle_snapshot (src/sync.rs:122-143) reads "SCAN" ("KEYS <n>\r\n" + one
// key per line, src/server.rs:580-587) and then one "GET <key>" per key ("VALUE <v>\r\n" or
// "NOT_FOUND\r\n", server.rs:551-552), one TCP round trip each, and inserts every pair into a tree.
// Here the response bytes are parsed in HBM instead: line breaks are found by a tiled count + scan +
// emit over the byte stream, every line is trimmed like Rust's str::trim_end (the client's
// read_line + trim_end, sync.rs:160-214), GET lines are classified (VALUE / NOT_FOUND / malformed),
// and the surviving (key, value) records are packed into the blob layout Kernel A reads.
#include "common.hpp"
#include "dev_util.hpp"
#include "kernels.hpp"

namespace mkv {

namespace {

constexpr int WT_THREADS = 256;
constexpr int WT_BYTES = 64;                       // bytes per thread
constexpr int WT_TILE = WT_THREADS * WT_BYTES;     // bytes per workgroup

__global__ __launch_bounds__(WT_THREADS) void k_count_newlines(const uint8_t *__restrict__ buf, uint64_t len,
                                                              uint64_t *__restrict__ tilecnt) {
    __shared__ uint64_t lds[17];
    const uint64_t b0 = (uint64_t)blockIdx.x * WT_TILE + (uint64_t)threadIdx.x * WT_BYTES;
    uint64_t c = 0;
    for (int i = 0; i < WT_BYTES; ++i)
        if (b0 + i < len && buf[b0 + i] == '\n') ++c;
    uint64_t tot;
    (void)block_excl_scan<uint64_t>(c, lds, &tot);
    if (threadIdx.x == 0) tilecnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(WT_THREADS) void k_emit_newlines(const uint8_t *__restrict__ buf, uint64_t len,
                                                             const uint64_t *__restrict__ tileoff,
                                                             uint64_t *__restrict__ nl) {
    __shared__ uint64_t lds[17];
    const uint64_t b0 = (uint64_t)blockIdx.x * WT_TILE + (uint64_t)threadIdx.x * WT_BYTES;
    uint64_t c = 0;
    for (int i = 0; i < WT_BYTES; ++i)
        if (b0 + i < len && buf[b0 + i] == '\n') ++c;
    uint64_t o = block_excl_scan<uint64_t>(c, lds, nullptr) + tileoff[blockIdx.x];
    for (int i = 0; i < WT_BYTES && c; ++i)
        if (b0 + i < len && buf[b0 + i] == '\n') {
            nl[o++] = b0 + i;
            --c;
        }
}

// Length of s[0..len) after Rust's str::trim_end (Unicode White_Space, UTF-8 encoded).
__device__ uint64_t trim_end_len(const uint8_t *s, uint64_t len) {
    while (len > 0) {
        const uint8_t c = s[len - 1];
        if (c == ' ' || (c >= 0x09 && c <= 0x0D)) {
            --len;
            continue;
        }
        if (len >= 2 && s[len - 2] == 0xC2 && (c == 0x85 || c == 0xA0)) {  // U+0085, U+00A0
            len -= 2;
            continue;
        }
        if (len >= 3) {
            const uint8_t a = s[len - 3], b = s[len - 2];
            const bool ws = (a == 0xE1 && b == 0x9A && c == 0x80) ||                      // U+1680
                            (a == 0xE2 && b == 0x80 && ((c >= 0x80 && c <= 0x8A) ||      // U+2000..200A
                                                        c == 0xA8 || c == 0xA9 ||        // U+2028, 2029
                                                        c == 0xAF)) ||                    // U+202F
                            (a == 0xE2 && b == 0x81 && c == 0x9F) ||                      // U+205F
                            (a == 0xE3 && b == 0x80 && c == 0x80);                        // U+3000
            if (ws) {
                len -= 3;
                continue;
            }
        }
        break;
    }
    return len;
}

// SCAN key lines 1..n of the response: key i = trimmed line i+1.
__global__ void k_scan_keys(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ nl, uint64_t n,
                            uint64_t *__restrict__ kstart, uint64_t *__restrict__ klen) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = nl[i] + 1, e = nl[i + 1];  // line i+1 spans (nl[i], nl[i+1])
    kstart[i] = s;
    klen[i] = trim_end_len(buf + s, e - s);
}

// GET response lines: "VALUE <v>" -> value, "NOT_FOUND" -> skipped, anything else -> *bad += 1.
__global__ void k_get_values(const uint8_t *__restrict__ buf, const uint64_t *__restrict__ nl, uint64_t n,
                             uint64_t *__restrict__ vstart, uint64_t *__restrict__ vlen, uint32_t *__restrict__ found,
                             uint32_t *__restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0, e = nl[i];
    const uint64_t L = trim_end_len(buf + s, e - s);
    const uint8_t *p = buf + s;
    const char nf[] = "NOT_FOUND";
    const char vp[] = "VALUE ";
    bool is_nf = L == 9, is_v = L >= 6;
    for (int k = 0; k < 9 && is_nf; ++k) is_nf = p[k] == (uint8_t)nf[k];
    for (int k = 0; k < 6 && is_v; ++k) is_v = p[k] == (uint8_t)vp[k];
    found[i] = is_v ? 1u : 0u;
    vstart[i] = s + 6;
    vlen[i] = is_v ? L - 6 : 0;
    if (!is_v && !is_nf) atomicAdd(bad, 1u);
}

// Packed copy of the found records: dst[off_out[r] ..] = src[start[i] .. +len[i]) for found i.
__global__ void k_pack_records(const uint8_t *__restrict__ src, const uint64_t *__restrict__ start,
                               const uint64_t *__restrict__ len, const uint32_t *__restrict__ found,
                               const uint32_t *__restrict__ rank, const uint64_t *__restrict__ off_out, uint64_t n,
                               uint8_t *__restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !found[i]) return;
    const uint64_t o = off_out[rank[i]];
    for (uint64_t b = 0; b < len[i]; ++b) dst[o + b] = src[start[i] + b];
}

__global__ void k_found_lengths(const uint64_t *__restrict__ len, const uint32_t *__restrict__ found,
                                const uint32_t *__restrict__ rank, uint64_t n, uint64_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && found[i]) out[rank[i]] = len[i];
}

inline dim3 grid1d(uint64_t n, uint32_t bs = 256) { return dim3((uint32_t)ceil_div(n ? n : 1, bs)); }

}  // namespace

size_t wire_scratch_bytes(uint64_t len) {
    const uint64_t nt = ceil_div(len ? len : 1, WT_TILE);
    return (nt + 2) * sizeof(uint64_t) + scan_scratch_bytes(nt + 1) + 1024;
}

uint64_t wire_count_lines(const uint8_t *buf, uint64_t len, void *scratch, uint64_t *d_total, hipStream_t st) {
    const uint64_t nt = ceil_div(len ? len : 1, WT_TILE);
    uint64_t *tc = reinterpret_cast<uint64_t *>(scratch);
    void *sc = tc + (nt + 2);
    hipLaunchKernelGGL(k_count_newlines, dim3((uint32_t)nt), dim3(WT_THREADS), 0, st, buf, len, tc);
    MKV_LAUNCH_CHECK();
    exclusive_scan_u64(tc, tc, nt, d_total, sc, st);
    return nt;
}

void wire_emit_lines(const uint8_t *buf, uint64_t len, const void *scratch, uint64_t *nl, hipStream_t st) {
    const uint64_t nt = ceil_div(len ? len : 1, WT_TILE);
    hipLaunchKernelGGL(k_emit_newlines, dim3((uint32_t)nt), dim3(WT_THREADS), 0, st, buf, len,
                       reinterpret_cast<const uint64_t *>(scratch), nl);
    MKV_LAUNCH_CHECK();
}

void launch_scan_keys(const uint8_t *buf, const uint64_t *nl, uint64_t n, uint64_t *kstart, uint64_t *klen,
                      hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_scan_keys, grid1d(n), dim3(256), 0, st, buf, nl, n, kstart, klen);
    MKV_LAUNCH_CHECK();
}

void launch_get_values(const uint8_t *buf, const uint64_t *nl, uint64_t n, uint64_t *vstart, uint64_t *vlen,
                       uint32_t *found, uint32_t *bad, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_get_values, grid1d(n), dim3(256), 0, st, buf, nl, n, vstart, vlen, found, bad);
    MKV_LAUNCH_CHECK();
}

void launch_found_lengths(const uint64_t *len, const uint32_t *found, const uint32_t *rank, uint64_t n, uint64_t *out,
                          hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_found_lengths, grid1d(n), dim3(256), 0, st, len, found, rank, n, out);
    MKV_LAUNCH_CHECK();
}

void launch_pack_records(const uint8_t *src, const uint64_t *start, const uint64_t *len, const uint32_t *found,
                         const uint32_t *rank, const uint64_t *off_out, uint64_t n, uint8_t *dst, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_pack_records, grid1d(n), dim3(256), 0, st, src, start, len, found, rank, off_out, n, dst);
    MKV_LAUNCH_CHECK();
}

}  // namespace mkv
