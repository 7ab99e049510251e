"""CPU tests of the library's communicator (csrc/comm.cpp, include/mkv_merkle.h mkv_comm_*): the host form
over torch.distributed gloo at world 2 and 3 — the C library calls back into the caller's all-gather, the
payloads come back in rank order, per-kind timings are counted, and a failing callback surfaces as a
MerkleError carrying the callback's own exception on every rank. No GPU: the host form needs none (the
sharded build / root / diff through the same communicator run on the GPU tests and
tests/cpp/test_sharded.cpp)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from merklekv_amd import MerkleError
    from merklekv_amd.comm import Comm, clear_cache
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = Comm.from_dist(dist, "cpu")
        assert c.form == "host" and Comm.from_dist(dist, "cpu") is c  # cached per group / device
        got = [c.all_gather(bytes([rank]) * 5 + b"%03d" % rank) for _ in range(3)]
        empty = c.all_gather(b"")
        st = c.stats(reset=True)
        after = c.stats()

        def bad(p):
            raise RuntimeError(f"rank {rank} transport down")

        failing = Comm.host(rank, world, bad)
        try:
            failing.all_gather(b"abc")
            err = None
        except MerkleError as e:
            err = (str(e), type(e.__cause__).__name__)
        short = Comm.host(rank, world, lambda p: [p])  # wrong part count for world > 1
        try:
            short.all_gather(b"xy")
            err2 = None
        except MerkleError as e:
            err2 = str(e)
        q.put((rank, got, empty, st, after, err, err2))
        clear_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_comm_all_gather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [bytes([r]) * 5 + b"%03d" % r for r in range(world)]
    for rank, got, empty, st, after, err, err2 in res:
        assert got == [want] * 3
        assert empty == [b""] * world
        assert sum(v[1] for v in st.values()) == 3 and sum(v[2] for v in st.values()) == 3 * 8
        assert all(v == (0.0, 0, 0) for v in after.values())
        assert err is not None and "transport down" in err[0] and err[1] == "RuntimeError"
        assert err2 is not None and "parts" in err2


def test_comm_rejects_bad_rank():
    from merklekv_amd import MerkleError
    from merklekv_amd.comm import Comm
    with pytest.raises(MerkleError):
        Comm.host(2, 2, lambda p: [p, p])
    with pytest.raises(MerkleError):
        Comm.host(0, 0, lambda p: [p])
