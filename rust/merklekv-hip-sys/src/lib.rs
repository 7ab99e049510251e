//! Raw FFI to `include/mkv_merkle.h` — the C ABI of the MI355X (gfx950) Merkle anti-entropy hot path
//! that replaces `crate::store::merkle::MerkleTree` of MerkleKV (`src/store/merkle.rs`) as consumed by
//! `src/sync.rs` (anti-entropy SYNC) and `src/server.rs:647-685` (HASH). Every declaration mirrors one
//! header prototype, in header order; `tests/test_rust_ffi.py` checks the two against each other (names,
//! arity, parameter and return types). The safe drop-in wrapper with the reference's receivers is
//! [`merkle`]. No CPU fallback: without a HIP device every compute call returns `MKV_EHIP`.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub mod merkle;

pub type mkv_status = i32;
pub const MKV_OK: mkv_status = 0;
pub const MKV_EINVAL: mkv_status = 1;
pub const MKV_EHIP: mkv_status = 2;
pub const MKV_ENOMEM: mkv_status = 3;
pub const MKV_ESTATE: mkv_status = 4;

pub const MKV_FRINGE_ENTRY_BYTES: usize = 48;
pub const MKV_FRINGE_MAX_ENTRIES: usize = 130;
pub const MKV_FRINGE_BYTES: usize = MKV_FRINGE_ENTRY_BYTES * MKV_FRINGE_MAX_ENTRIES;
pub const MKV_COMM_ID_BYTES: usize = 128;
pub const MKV_FAULT_AFTER_META: c_int = 1;
pub const MKV_COLL_COUNTS: usize = 0;
pub const MKV_COLL_RANGE: usize = 1;
pub const MKV_COLL_FRINGE: usize = 2;
pub const MKV_COLL_DIFF: usize = 3;
pub const MKV_COLL_USER: usize = 4;
pub const MKV_COLL_KINDS: usize = 5;
pub const MKV_ROUTE_MAX_WORLD: u32 = 256;

/// Opaque tree handle: device-resident sorted keys, leaf digests, every level.
#[repr(C)]
pub struct mkv_tree {
    _p: [u8; 0],
}
/// Opaque packed key list (diff / leaves results), freed with `mkv_keylist_free`.
#[repr(C)]
pub struct mkv_keylist {
    _p: [u8; 0],
}
/// Opaque communicator of the sharded entry points (RCCL inside the library, or the host's all-gather).
#[repr(C)]
pub struct mkv_comm {
    _p: [u8; 0],
}
/// Packed byte strings: item i is bytes[offsets[i] .. offsets[i + 1]), offsets has n + 1 entries.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct mkv_blob {
    pub bytes: *const u8,
    pub offsets: *const u64,
    pub n: u64,
}
/// The host form's all-gather: `bytes` from every rank into recv in rank order; 0 on success.
pub type mkv_allgather_fn =
    Option<unsafe extern "C" fn(ctx: *mut c_void, send: *const c_void, recv: *mut c_void, bytes: u64) -> c_int>;

#[link(name = "merklekv_hip")]
extern "C" {
    // ---- MerkleTree API (merkle.rs) ----
    pub fn mkv_tree_create(hip_device: c_int, out: *mut *mut mkv_tree) -> mkv_status; // new() :36-41
    pub fn mkv_tree_destroy(t: *mut mkv_tree);
    pub fn mkv_tree_clone(src: *const mkv_tree, dst: *mut mkv_tree) -> mkv_status; // #[derive(Clone)] :27
    pub fn mkv_tree_build(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob) -> mkv_status; // new() + n x insert
    pub fn mkv_tree_build_device(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob) -> mkv_status;
    pub fn mkv_tree_build_digests(t: *mut mkv_tree, keys: mkv_blob, digests: *const u8) -> mkv_status;
    pub fn mkv_tree_build_wire(t: *mut mkv_tree, scan: *const u8, scan_len: u64, gets: *const u8, gets_len: u64)
        -> mkv_status; // sync.rs:122-214 responses, parsed on the device
    pub fn mkv_tree_upsert(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob) -> mkv_status; // insert :52-56
    pub fn mkv_tree_upsert_device(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob) -> mkv_status;
    pub fn mkv_tree_upsert_device_many(trees: *const *mut mkv_tree, keys: *const mkv_blob, values: *const mkv_blob,
                                       k: u32) -> mkv_status;
    pub fn mkv_tree_remove(t: *mut mkv_tree, keys: mkv_blob) -> mkv_status; // remove :59-62
    pub fn mkv_tree_apply(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob, is_remove: *const u8) -> mkv_status;
    pub fn mkv_tree_root(t: *const mkv_tree, out32: *mut u8, has_root: *mut c_int) -> mkv_status; // get_root_hash :65-67
    pub fn mkv_tree_len(t: *const mkv_tree, n: *mut u64) -> mkv_status;
    pub fn mkv_tree_node_count(t: *const mkv_tree, count: *mut u64) -> mkv_status; // node_count :156-163
    pub fn mkv_tree_level_count(t: *const mkv_tree, nlevels: *mut u32) -> mkv_status;
    pub fn mkv_tree_level(t: *const mkv_tree, level: u32, count: *mut u64, out: *mut u8) -> mkv_status;
    pub fn mkv_tree_leaves(t: *const mkv_tree, keys: *mut *mut mkv_keylist, digests_out: *mut u8) -> mkv_status; // :126-138
    pub fn mkv_tree_diff(a: *const mkv_tree, b: *const mkv_tree, out: *mut *mut mkv_keylist) -> mkv_status; // diff_keys :171-196
    pub fn mkv_tree_diff_many(a: *const mkv_tree, others: *const *const mkv_tree, k: u32, outs: *mut *mut mkv_keylist)
        -> mkv_status;
    pub fn mkv_tree_node_digests(t: *const mkv_tree, level: u32, idx: *const u64, m: u64, out: *mut u8) -> mkv_status;
    pub fn mkv_tree_compare_nodes(t: *const mkv_tree, level: u32, idx: *const u64, peer: *const u8, m: u64,
                                  out_idx: *mut u64, n_out: *mut u64) -> mkv_status;
    pub fn mkv_tree_keys_at(t: *const mkv_tree, pos: *const u64, m: u64, out: *mut *mut mkv_keylist) -> mkv_status;
    pub fn mkv_tree_prefix_root(t: *const mkv_tree, prefix: *const u8, plen: u64, out32: *mut u8, has_root: *mut c_int)
        -> mkv_status;
    pub fn mkv_tree_hash_pattern(t: *const mkv_tree, pattern: *const u8, plen: u64, out32: *mut u8,
                                 has_root: *mut c_int) -> mkv_status; // HASH server.rs:647-685
    pub fn mkv_keylist_get(l: *const mkv_keylist, n: *mut u64, bytes: *mut *const u8, offsets: *mut *const u64)
        -> mkv_status;
    pub fn mkv_keylist_free(l: *mut mkv_keylist);
    pub fn mkv_last_error() -> *const c_char;

    // ---- key-range shards ----
    pub fn mkv_shard_prepare(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob, on_device: c_int, n_local: *mut u64)
        -> mkv_status;
    pub fn mkv_shard_reduce(t: *mut mkv_tree, global_offset: u64, global_n: u64) -> mkv_status;
    pub fn mkv_shard_fringe(t: *const mkv_tree, out: *mut u8) -> mkv_status;
    pub fn mkv_shard_combine(t: *mut mkv_tree, fringes: *const u8, world: u32, global_n: u64, out32: *mut u8,
                             has_root: *mut c_int) -> mkv_status;
    pub fn mkv_shard_fringe_device(t: *const mkv_tree, dout: *mut u8) -> mkv_status;
    pub fn mkv_shard_combine_device(t: *mut mkv_tree, dfringes: *const u8, world: u32, stride_bytes: u64,
                                    global_n: u64, out32: *mut u8, has_root: *mut c_int) -> mkv_status;

    // ---- communicator + sharded entry points (the collectives run inside the library) ----
    pub fn mkv_comm_unique_id(id: *mut u8) -> mkv_status;
    pub fn mkv_comm_init_rank(id: *const u8, rank: c_int, world: c_int, hip_device: c_int, out: *mut *mut mkv_comm)
        -> mkv_status;
    pub fn mkv_comm_create_host(rank: c_int, world: c_int, fn_: mkv_allgather_fn, ctx: *mut c_void,
                                out: *mut *mut mkv_comm) -> mkv_status;
    pub fn mkv_comm_rank(c: *const mkv_comm, rank: *mut c_int, world: *mut c_int) -> mkv_status;
    pub fn mkv_comm_inject_fault(c: *mut mkv_comm, where_: c_int) -> mkv_status;
    pub fn mkv_comm_all_gather(c: *mut mkv_comm, send: *const c_void, recv: *mut c_void, bytes: u64) -> mkv_status;
    pub fn mkv_comm_stats(c: *mut mkv_comm, secs: *mut f64, calls: *mut u64, bytes: *mut u64, reset: c_int)
        -> mkv_status;
    pub fn mkv_comm_traffic(c: *const mkv_comm, staged: *mut u64, meta: *mut u64) -> mkv_status;
    pub fn mkv_comm_destroy(c: *mut mkv_comm);
    pub fn mkv_sharded_build(t: *mut mkv_tree, c: *mut mkv_comm, keys: mkv_blob, values: mkv_blob, on_device: c_int,
                             range_check: c_int, counts_out: *mut u64) -> mkv_status;
    pub fn mkv_sharded_root(t: *mut mkv_tree, c: *mut mkv_comm, out32: *mut u8, has_root: *mut c_int) -> mkv_status;
    pub fn mkv_sharded_root_many(ts: *const *mut mkv_tree, k: u32, c: *mut mkv_comm, roots: *mut u8,
                                 has_root: *mut c_int) -> mkv_status;
    pub fn mkv_sharded_diff(a: *const mkv_tree, b: *const mkv_tree, c: *mut mkv_comm, out: *mut *mut mkv_keylist)
        -> mkv_status; // diff_keys over every rank's range, sync.rs:67
    pub fn mkv_sharded_diff_local(a: *const mkv_tree, b: *const mkv_tree, c: *mut mkv_comm,
                                  out: *mut *mut mkv_keylist, global_offset: *mut u64, global_total: *mut u64)
        -> mkv_status;

    // ---- redistribution of unpartitioned input ----
    pub fn mkv_route_sample(t: *mut mkv_tree, keys: mkv_blob, m: u32, samples_dev: *mut u64) -> mkv_status;
    pub fn mkv_route_splitters(samples: *const u64, ns: u64, world: u32, splitters: *mut u64) -> mkv_status;
    pub fn mkv_route_plan(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob, world: u32, splitters: *const u64,
                          counts: *mut u64) -> mkv_status;
    pub fn mkv_route_pack(t: *mut mkv_tree, keys: mkv_blob, values: mkv_blob, kout: *mut u8, klen: *mut u32,
                          vout: *mut u8, vlen: *mut u32) -> mkv_status;
    pub fn mkv_route_offsets(t: *mut mkv_tree, lens: *const u32, n: u64, offs: *mut u64) -> mkv_status;

    // ---- profiling / diagnostics / generators ----
    pub fn mkv_prof_enable(t: *mut mkv_tree, on: c_int) -> mkv_status;
    pub fn mkv_prof_reset(t: *mut mkv_tree) -> mkv_status;
    pub fn mkv_prof_read(t: *const mkv_tree, group: *const c_char, total_ms: *mut f64, count: *mut u64) -> mkv_status;
    pub fn mkv_tree_update_counts(t: *const mkv_tree, out: *mut u64, cap: u32, nlevels: *mut u32) -> mkv_status;
    pub fn mkv_tree_walk_stats(t: *const mkv_tree, out: *mut u64) -> mkv_status;
    pub fn mkv_gen_records_device(hip_device: c_int, seed: u64, idx0: u64, n: u64, klen: u32, vlen: u32, shard: u32,
                                  nshards: u32, vfield: u32, kb: *mut u8, koff: *mut u64, vb: *mut u8,
                                  voff: *mut u64) -> mkv_status;
    pub fn mkv_gen_records_ragged_device(hip_device: c_int, seed: u64, idx0: u64, n: u64, klen: u32, vlen: u32,
                                         shard: u32, nshards: u32, vfield: u32, kb: *mut u8, koff: *mut u64,
                                         vb: *mut u8, voff: *mut u64) -> mkv_status;
    pub fn mkv_leaf_digests(hip_device: c_int, keys: mkv_blob, values: mkv_blob, out: *mut u8) -> mkv_status;
    pub fn mkv_pool_trim() -> mkv_status;
    pub fn mkv_pool_stats(out6: *mut u64) -> mkv_status;
    pub fn mkv_debug_trace(buf: *mut c_char, cap: u64, len: *mut u64) -> mkv_status;
    pub fn mkv_version() -> *const c_char;
}
