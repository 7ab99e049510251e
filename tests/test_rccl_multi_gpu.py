"""RCCL with more than one rank: one process per visible GPU (torch.cuda.device_count() ranks; skipped on
a one-GPU box), each driving the library's RCCL communicator through the C ABI the way a non-Python host
would (mkv_comm_unique_id in the parent, shared out of band, mkv_comm_init_rank per rank):
mkv_sharded_build / _root_many / _diff / _diff_local over key-range shards, checked against the C oracle
(coracle) of the union — rebuild() and diff_keys(), /root/reference/src/store/merkle.rs:73-121 and :171-196,
as SyncManager consumes them, /root/reference/src/sync.rs:56-87. Then the failure paths: a local step that
fails on rank 1 after the meta all-gather (mkv_comm_inject_fault) returns MKV_ENOMEM on every rank, and a
rank that never joins a collective makes the others' bounded wait fail (MKV_EHIP, the communicator
aborted) instead of hanging.

Every rank process runs under a deadline (join timeout, then kill), so a protocol bug fails the test
instead of holding the box."""
import os

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x4D65726B6C654B56
N_PER_RANK = 60_001


def _ndev() -> int:
    import torch
    return torch.cuda.device_count()


def _replica_b(keys, vals, rank):
    """Replica b of one key range: every 97th value changed, every 101st key deleted, and keys inserted
    right after existing ones (key + b"~" sorts between a key and its successor, so it stays in range)."""
    kb, vb = [], []
    for i, (k, v) in enumerate(zip(keys, vals)):
        if i % 101 == 3:
            continue
        kb.append(k)
        vb.append(v + b"!" if i % 97 == 5 else v)
        if i % 211 == 7:
            kb.append(k + b"~")
            vb.append(b"new-%d" % rank)
    return kb, vb


def _records(rank, world):
    from oracle.merkle_oracle import gen_records, split_blob
    kb, ko, vb, vo = gen_records(SEED, 0, N_PER_RANK, shard=rank, nshards=world)
    keys, vals = split_blob(kb, ko), split_blob(vb, vo)
    order = sorted(range(len(keys)), key=lambda i: keys[i])
    keys, vals = [keys[i] for i in order], [vals[i] for i in order]
    return (keys, vals), _replica_b(keys, vals, rank)


def _kl(kl) -> list:
    raw, offs = kl.raw.tobytes(), kl.offs.tolist()
    return [raw[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def _rank_main(rank, world, uid, mode, q):
    try:
        os.environ.setdefault("MKV_WAIT_TIMEOUT_S", "20")
        from merklekv_amd import MerkleTree
        from merklekv_amd._lib import lib
        from merklekv_amd.comm import Comm
        comm = Comm.rccl(uid, rank, world, rank)
        (ka, va), (kb, vb) = _records(rank, world)
        a, b = MerkleTree(rank), MerkleTree(rank)
        out = {"rank": rank}
        out["counts"] = a.sharded_build(comm, ka, va)
        b.sharded_build(comm, kb, vb)
        out["roots"] = (a.get_root_hash(), b.get_root_hash())
        out["roots_many"] = MerkleTree.sharded_root_many([a, b], comm)
        out["diff"] = _kl(a.sharded_diff(b, comm))
        kl, off, tot = a.sharded_diff_local(b, comm)
        out["slice"] = (_kl(kl), off, tot)
        out["staged"] = {k: v[0] for k, v in comm.traffic().items()}
        if mode == "faults":
            # rank 1 fails after the meta all-gather: every rank's call returns MKV_ENOMEM (3)
            if rank == 1:
                assert lib().mkv_comm_inject_fault(comm.handle, 1) == 0
            try:
                a.sharded_diff(b, comm)
                out["fault_diff"] = 0
            except Exception as e:  # MerkleError
                out["fault_diff"] = getattr(e, "status", -1)
            out["diff_again"] = _kl(a.sharded_diff(b, comm))
            # rank 1 never joins the next root recombine: the others' bounded wait fails (EHIP) and aborts
            if rank != 1:
                try:
                    a.sharded_root(comm)
                    out["timeout"] = 0
                except Exception as e:
                    out["timeout"] = getattr(e, "status", -1)
        q.put(out)
        if mode != "faults":
            comm.close()
    except BaseException as e:  # the parent asserts on it
        q.put({"rank": rank, "error": repr(e)})


def _run(world, mode, deadline):
    import torch.multiprocessing as mp

    from merklekv_amd.comm import Comm
    uid = Comm.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, world, uid, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = {}
    try:
        for _ in range(world):
            o = q.get(timeout=deadline)
            outs[o["rank"]] = o
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return outs


def _want(world):
    from oracle import coracle
    from oracle.merkle_oracle import pack
    A, B = ([], []), ([], [])
    for r in range(world):
        (ka, va), (kb, vb) = _records(r, world)
        A[0].extend(ka), A[1].extend(va), B[0].extend(kb), B[1].extend(vb)
    oa = coracle.OracleTree.build(*pack(A[0]), *pack(A[1]))
    ob = coracle.OracleTree.build(*pack(B[0]), *pack(B[1]))
    return oa.root(), ob.root(), oa.diff(ob), [len(_records(r, world)[0][0]) for r in range(world)]


@pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs (one RCCL rank per device)")
def test_rccl_world_n_sharded_build_root_diff_vs_oracle():
    world = _ndev()
    outs = _run(world, "plain", deadline=300)
    ra, rb, diff, counts = _want(world)
    for r in range(world):
        o = outs[r]
        assert "error" not in o, o
        assert o["counts"] == counts
        assert o["roots"] == (ra, rb)
        assert o["roots_many"] == [ra, rb]
        assert o["diff"] == diff  # the whole sorted list on every rank
        keys, off, tot = o["slice"]
        assert tot == len(diff) and diff[off:off + len(keys)] == keys
        assert all(v == 0 for v in o["staged"].values() if v is not None)
    offs = [outs[r]["slice"][1] for r in range(world)]
    assert offs == sorted(offs) and offs[0] == 0


@pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs (one RCCL rank per device)")
def test_rccl_world_n_failure_after_meta_and_missing_rank():
    world = _ndev()
    outs = _run(world, "faults", deadline=300)
    _, _, diff, _ = _want(world)
    for r in range(world):
        o = outs[r]
        assert "error" not in o, o
        assert o["fault_diff"] == 3  # MKV_ENOMEM everywhere: rank 1's own, the others through the status word
        assert o["diff_again"] == diff
        if r != 1:
            assert o["timeout"] == 2  # MKV_EHIP: bounded wait, communicator aborted
