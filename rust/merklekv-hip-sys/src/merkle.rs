//! The drop-in for MerkleKV's `src/store/merkle.rs`: `crate::store::merkle::MerkleTree` with the
//! reference's public surface AND receivers (`new`, `insert(&mut self)`, `remove(&mut self)`,
//! `get_root_hash(&self) -> Option<&Vec<u8>>`, `diff_keys(&self, &MerkleTree)`, `diff_first_key`,
//! `inorder_keys`, `leaves`, `node_count`, `Clone`, `Debug`), so `src/sync.rs:61-67` and
//! `src/server.rs:661-675` compile unchanged: the module body becomes `pub use merklekv_hip_sys::merkle::*;`.
//!
//! Queued inserts / removes are applied by the first observer through interior mutability (`RefCell`
//! for the queue, `OnceCell` for the cached root) — that is what lets `get_root_hash(&self)` hand out a
//! `&Vec<u8>` like `self.root.as_ref().map(|n| &n.hash)` does (merkle.rs:65-67). A batch equals the
//! reference's rebuild-after-every-insert because a rebuild depends only on the final leaf map. The type
//! is `Send` (held across `.await` in `sync_once`, sync.rs:61-64) and `!Sync` (RefCell), like the
//! reference, whose callers serialise access behind tokio `Mutex`es (server.rs:386-390). Every call
//! blocks until its results are host-visible; inside the tokio server wrap snapshot builds and diffs in
//! `spawn_blocking`. The reference API is infallible, so a device failure panics (no CPU fallback).
//!
//! [`ShardComm`] and the `*_sharded` methods are the multi-GPU form (one process per GPU, key-range
//! shards, the collectives inside the library: INTEGRATION.md section 4).
use std::cell::{OnceCell, RefCell};
use std::ffi::CStr;

use crate::*;

fn ok(s: mkv_status) {
    if s != MKV_OK {
        let msg = unsafe { CStr::from_ptr(mkv_last_error()) }.to_string_lossy().into_owned();
        panic!("merklekv_hip: status {}: {}", s, msg);
    }
}

fn pack<'a>(items: impl Iterator<Item = &'a [u8]>) -> (Vec<u8>, Vec<u64>) {
    let (mut b, mut o) = (Vec::new(), vec![0u64]);
    for it in items {
        b.extend_from_slice(it);
        o.push(b.len() as u64);
    }
    (b, o)
}

fn blob(b: &[u8], o: &[u64]) -> mkv_blob {
    mkv_blob { bytes: b.as_ptr(), offsets: o.as_ptr(), n: (o.len() - 1) as u64 }
}

fn take_keys(l: *mut mkv_keylist) -> Vec<String> {
    let (mut n, mut b, mut o) = (0u64, std::ptr::null(), std::ptr::null());
    ok(unsafe { mkv_keylist_get(l, &mut n, &mut b, &mut o) });
    let out = (0..n as usize)
        .map(|i| unsafe {
            let (s, e) = (*o.add(i) as usize, *o.add(i + 1) as usize);
            // keys went in as &str, so they come back as valid UTF-8
            String::from_utf8_unchecked(std::slice::from_raw_parts(b.add(s), e - s).to_vec())
        })
        .collect();
    unsafe { mkv_keylist_free(l) };
    out
}

enum Op {
    Insert(String, String),
    Remove(String),
}

pub struct MerkleTree {
    h: *mut mkv_tree,
    pending: RefCell<Vec<Op>>,       // insert / remove queue, applied by the first observer
    root: OnceCell<Option<Vec<u8>>>, // get_root_hash(&self) hands out &Vec<u8> from here
}
unsafe impl Send for MerkleTree {} // the handle moves between threads; RefCell keeps it !Sync

impl Default for MerkleTree {
    fn default() -> Self {
        Self::new()
    }
}

impl MerkleTree {
    /// MerkleTree::new() — merkle.rs:36-41 (HIP device 0).
    pub fn new() -> Self {
        let mut h = std::ptr::null_mut();
        ok(unsafe { mkv_tree_create(0, &mut h) });
        Self { h, pending: RefCell::new(Vec::new()), root: OnceCell::new() }
    }
    /// insert — merkle.rs:52-56 (queued; last write wins).
    pub fn insert(&mut self, key: &str, value: &str) {
        self.pending.get_mut().push(Op::Insert(key.to_owned(), value.to_owned()));
        self.root = OnceCell::new();
    }
    /// remove — merkle.rs:59-62 (queued).
    pub fn remove(&mut self, key: &str) {
        self.pending.get_mut().push(Op::Remove(key.to_owned()));
        self.root = OnceCell::new();
    }
    // Runs of inserts -> one mkv_tree_upsert, runs of removes -> one mkv_tree_remove, order preserved.
    fn flush(&self) {
        let ops = std::mem::take(&mut *self.pending.borrow_mut());
        let mut i = 0;
        while i < ops.len() {
            let rm = matches!(ops[i], Op::Remove(_));
            let mut j = i;
            while j < ops.len() && matches!(ops[j], Op::Remove(_)) == rm {
                j += 1;
            }
            let (kb, ko) = pack(ops[i..j].iter().map(|o| match o {
                Op::Insert(k, _) | Op::Remove(k) => k.as_bytes(),
            }));
            if rm {
                ok(unsafe { mkv_tree_remove(self.h, blob(&kb, &ko)) });
            } else {
                let (vb, vo) = pack(ops[i..j].iter().map(|o| match o {
                    Op::Insert(_, v) => v.as_bytes(),
                    Op::Remove(_) => unreachable!(),
                }));
                ok(unsafe { mkv_tree_upsert(self.h, blob(&kb, &ko), blob(&vb, &vo)) });
            }
            i = j;
        }
    }
    /// get_root_hash — merkle.rs:65-67, same receiver and return type.
    pub fn get_root_hash(&self) -> Option<&Vec<u8>> {
        self.root
            .get_or_init(|| {
                self.flush();
                let (mut out, mut has) = (vec![0u8; 32], 0);
                ok(unsafe { mkv_tree_root(self.h, out.as_mut_ptr(), &mut has) });
                if has != 0 {
                    Some(out)
                } else {
                    None
                }
            })
            .as_ref()
    }
    /// diff_keys — merkle.rs:171-196: sorted, unique (BTreeSet order).
    pub fn diff_keys(&self, other: &MerkleTree) -> Vec<String> {
        self.flush();
        other.flush();
        let mut l = std::ptr::null_mut();
        ok(unsafe { mkv_tree_diff(self.h, other.h, &mut l) });
        take_keys(l)
    }
    /// diff_first_key — merkle.rs:199-204.
    pub fn diff_first_key(&self, other: &MerkleTree) -> Option<String> {
        self.diff_keys(other).into_iter().next()
    }
    /// inorder_keys — merkle.rs:126-130.
    pub fn inorder_keys(&self) -> Vec<String> {
        self.flush();
        let mut l = std::ptr::null_mut();
        ok(unsafe { mkv_tree_leaves(self.h, &mut l, std::ptr::null_mut()) });
        take_keys(l)
    }
    /// leaves — merkle.rs:133-138: (key, leaf digest) in key order.
    pub fn leaves(&self) -> Vec<(String, Vec<u8>)> {
        self.flush();
        let mut n = 0u64;
        ok(unsafe { mkv_tree_len(self.h, &mut n) });
        let mut dig = vec![0u8; 32 * n as usize];
        let mut l = std::ptr::null_mut();
        ok(unsafe { mkv_tree_leaves(self.h, &mut l, dig.as_mut_ptr()) });
        take_keys(l).into_iter().zip(dig.chunks(32).map(|c| c.to_vec())).collect()
    }
    /// node_count — merkle.rs:156-163.
    pub fn node_count(&self) -> usize {
        self.flush();
        let mut c = 0u64;
        ok(unsafe { mkv_tree_node_count(self.h, &mut c) });
        c as usize
    }
    /// HASH [pattern] (server.rs:647-685) in one call: "" / "*" = every key, else a prefix.
    pub fn hash_pattern(&self, pattern: &str) -> Option<Vec<u8>> {
        self.flush();
        let (mut out, mut has) = (vec![0u8; 32], 0);
        ok(unsafe { mkv_tree_hash_pattern(self.h, pattern.as_ptr(), pattern.len() as u64, out.as_mut_ptr(), &mut has) });
        if has != 0 {
            Some(out)
        } else {
            None
        }
    }
    /// sync.rs:104-119 / :122-143 in one call: a snapshot's (key, value) pairs, last write wins.
    pub fn build_from(&mut self, pairs: &[(String, String)]) {
        let (kb, ko) = pack(pairs.iter().map(|(k, _)| k.as_bytes()));
        let (vb, vo) = pack(pairs.iter().map(|(_, v)| v.as_bytes()));
        self.pending.get_mut().clear();
        self.root = OnceCell::new();
        ok(unsafe { mkv_tree_build(self.h, blob(&kb, &ko), blob(&vb, &vo)) });
    }
}

impl Clone for MerkleTree {
    /// #[derive(Clone)] — merkle.rs:27.
    fn clone(&self) -> Self {
        self.flush();
        let t = MerkleTree::new();
        ok(unsafe { mkv_tree_clone(self.h, t.h) });
        t
    }
}

impl std::fmt::Debug for MerkleTree {
    /// #[derive(Debug)] — merkle.rs:27.
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        f.debug_struct("MerkleTree").field("root", &self.get_root_hash()).finish()
    }
}

impl Drop for MerkleTree {
    fn drop(&mut self) {
        unsafe { mkv_tree_destroy(self.h) }
    }
}

/// A communicator of the sharded entry points: RCCL over xGMI (one process per GPU) or the host's own
/// all-gather. Every sharded call is collective; when one rank's local step fails every rank gets the
/// error, and a rank whose peers never join returns `MKV_EHIP` after `MKV_WAIT_TIMEOUT_S`.
pub struct ShardComm {
    c: *mut mkv_comm,
    world: usize,
}
unsafe impl Send for ShardComm {}

impl ShardComm {
    /// RCCL: rank 0 calls `unique_id()` and sends the bytes to every peer (e.g. over the sync
    /// connection), then every rank calls `rccl(&id, ..)` on its GPU.
    pub fn unique_id() -> [u8; MKV_COMM_ID_BYTES] {
        let mut id = [0u8; MKV_COMM_ID_BYTES];
        ok(unsafe { mkv_comm_unique_id(id.as_mut_ptr()) });
        id
    }
    pub fn rccl(id: &[u8; MKV_COMM_ID_BYTES], rank: usize, world: usize, gpu: i32) -> Self {
        let mut c = std::ptr::null_mut();
        ok(unsafe { mkv_comm_init_rank(id.as_ptr(), rank as i32, world as i32, gpu, &mut c) });
        Self { c, world }
    }
}

impl Drop for ShardComm {
    fn drop(&mut self) {
        unsafe { mkv_comm_destroy(self.c) }
    }
}

impl MerkleTree {
    /// This node's key range of a sharded snapshot (sync.rs:104-119 with keys in [lo, hi)); afterwards
    /// get_root_hash() is the root of the union over every rank, identical to one unsharded tree.
    /// Returns every rank's leaf count.
    pub fn build_sharded(&mut self, comm: &ShardComm, pairs: &[(String, String)]) -> Vec<u64> {
        let (kb, ko) = pack(pairs.iter().map(|(k, _)| k.as_bytes()));
        let (vb, vo) = pack(pairs.iter().map(|(_, v)| v.as_bytes()));
        let mut counts = vec![0u64; comm.world];
        self.pending.get_mut().clear();
        self.root = OnceCell::new();
        ok(unsafe { mkv_sharded_build(self.h, comm.c, blob(&kb, &ko), blob(&vb, &vo), 0, 1, counts.as_mut_ptr()) });
        counts
    }
    /// Global root again after in-range inserts on this shard (merkle.rs:52-56 then :65-67).
    pub fn root_sharded(&mut self, comm: &ShardComm) -> Option<Vec<u8>> {
        self.flush();
        self.root = OnceCell::new();
        let (mut out, mut has) = (vec![0u8; 32], 0);
        ok(unsafe { mkv_sharded_root(self.h, comm.c, out.as_mut_ptr(), &mut has) });
        if has != 0 {
            Some(out)
        } else {
            None
        }
    }
    /// diff_keys over the whole sharded key space (merkle.rs:171-196), the same list on every rank.
    pub fn diff_keys_sharded(&self, other: &MerkleTree, comm: &ShardComm) -> Vec<String> {
        self.flush();
        other.flush();
        let mut l = std::ptr::null_mut();
        ok(unsafe { mkv_sharded_diff(self.h, other.h, comm.c, &mut l) });
        take_keys(l)
    }
    /// This rank's slice of diff_keys_sharded() and its offset in the global list (plus the global
    /// length): a sharded sync_once applies only its own keys (sync.rs:74-83).
    pub fn diff_keys_sharded_local(&self, other: &MerkleTree, comm: &ShardComm) -> (Vec<String>, u64, u64) {
        self.flush();
        other.flush();
        let (mut l, mut off, mut tot) = (std::ptr::null_mut(), 0u64, 0u64);
        ok(unsafe { mkv_sharded_diff_local(self.h, other.h, comm.c, &mut l, &mut off, &mut tot) });
        (take_keys(l), off, tot)
    }
}
