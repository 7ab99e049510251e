"""Snapshot ingestion from SYNC wire bytes (mkv_tree_build_wire) vs host blobs (mkv_tree_build), 10M keys."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from merklekv_amd import MerkleTree
from oracle import coracle
from oracle.merkle_oracle import DEFAULT_SEED

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
kb, ko, vb, vo = coracle.gen_records(DEFAULT_SEED, 0, n)
K = kb.reshape(n, 32)
V = vb.reshape(n, 100)
crlf = np.frombuffer(b"\r\n", np.uint8)
scan = np.concatenate([np.frombuffer(b"KEYS %d\r\n" % n, np.uint8),
                       np.hstack([K, np.broadcast_to(crlf, (n, 2))]).reshape(-1)]).tobytes()
gets = np.hstack([np.broadcast_to(np.frombuffer(b"VALUE ", np.uint8), (n, 6)), V,
                  np.broadcast_to(crlf, (n, 2))]).reshape(-1).tobytes()
t = MerkleTree()
for rep in range(3):
    t0 = time.perf_counter(); t.build_wire(scan, gets); t1 = time.perf_counter()
    r1 = t.get_root_hash()
    t2 = time.perf_counter(); t.build((kb, ko), (vb, vo)); t3 = time.perf_counter()
    assert t.get_root_hash() == r1
    print(f"rep {rep}: wire {1e3*(t1-t0):.1f} ms ({len(scan)+len(gets)} B)  blobs {1e3*(t3-t2):.1f} ms", flush=True)
