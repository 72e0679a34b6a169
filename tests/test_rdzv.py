"""The stdlib TCP rendezvous of the multi-process bench (kalibr_amd/rdzv.py): id broadcast, barrier and max over
ranks, world sizes 1 and 3, rank processes started out of order (CPU)."""
import multiprocessing as mp
import socket
import struct

from kalibr_amd import rdzv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    g = rdzv.TcpGroup(rank, world, addr="127.0.0.1", port=port, timeout=60.0)
    uid = g.broadcast(bytes(range(128)) if rank == 0 else b"")
    g.barrier()
    m = g.max(float(rank) * 1.5 + 0.25)
    g.barrier()
    g.close()
    q.put((rank, uid, m))


def test_three_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 3, port, q)) for r in (2, 1, 0)]  # clients before the server
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, uid, m in res:
        assert uid == bytes(range(128))
        assert m == 3.25


def test_world_one_is_local():
    g = rdzv.TcpGroup(0, 1)
    assert g.broadcast(b"abc") == b"abc"
    g.barrier()
    assert g.max(2.0) == 2.0


def test_foreign_service_is_rejected():
    """a client that reaches a non-rendezvous server does not take its reply for rank 0's handshake"""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    import threading

    def serve():
        c, _ = srv.accept()
        c.recv(64)
        c.sendall(struct.pack("<Q", 5) + b"hello")
        c.close()

    t = threading.Thread(target=serve)
    t.start()
    try:
        rdzv.TcpGroup(1, 2, addr="127.0.0.1", port=port, timeout=1.5)
        raise AssertionError("expected a timeout")
    except TimeoutError:
        pass
    t.join()
    srv.close()
