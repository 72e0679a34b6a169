"""The stdlib TCP rendezvous of the multi-process bench (kalibr_amd/rdzv.py): id broadcast, barrier and max over
ranks, world sizes 1 and 3, rank processes started out of order (CPU)."""
import multiprocessing as mp
import socket
import struct
import time

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


def _raw_client(port, payload, q, tag, framed=True):
    """a client that sends one hello (framed with its length, or the raw bytes of a foreign protocol) and reports
    whether rank 0 answered with the handshake"""
    import time as _t
    deadline = _t.monotonic() + 30.0
    while True:
        try:
            s = socket.create_connection(("127.0.0.1", port), timeout=2.0)
            break
        except OSError:
            if _t.monotonic() > deadline:
                q.put((tag, "no server"))
                return
            _t.sleep(0.1)
    s.settimeout(10.0)
    try:
        s.sendall((struct.pack("<Q", len(payload)) if framed else b"") + payload)
        r = s.recv(64)
        q.put((tag, "reply" if r else "closed"))
    except OSError:
        q.put((tag, "closed"))
    finally:
        s.close()


def test_bad_hello_and_duplicate_rank_are_refused():
    """rank 0 survives a malformed hello, an out-of-range rank and a duplicate rank id: each is closed without the
    handshake reply, and the real ranks still form the group"""
    import threading
    import queue
    port = _free_port()
    q = queue.Queue()
    res = {}

    def server():
        g = rdzv.TcpGroup(0, 3, addr="127.0.0.1", port=port, timeout=30.0)
        res["server"] = g.max(1.0)
        g.close()

    t0 = threading.Thread(target=server)
    t0.start()
    bad = [(rdzv._MAGIC + b"x1", "malformed"), (rdzv._MAGIC + b"7", "out of range"), (b"GET / HTTP/1.0", "foreign")]
    for payload, tag in bad:
        _raw_client(port, payload, q, tag)
    # unframed: 'GET / HT' reads as a ~6e18-byte length, which must be refused at once (no allocation, no wait)
    t_raw = time.monotonic()
    _raw_client(port, b"GET / HTTP/1.1\r\nHost: x\r\n\r\n", q, "unframed", framed=False)
    got = dict(q.get(timeout=30) for _ in range(len(bad) + 1))
    assert time.monotonic() - t_raw < 5.0
    assert all(v == "closed" for v in got.values()), got

    out = {}

    def client(r):
        g = rdzv.TcpGroup(r, 3, addr="127.0.0.1", port=port, timeout=30.0)
        out[r] = g.max(float(r))
        g.close()

    t1 = threading.Thread(target=client, args=(1,))
    t1.start()
    # wait until rank 1 is registered, then a second "rank 1" must be refused
    import time as _t
    _t.sleep(1.0)
    _raw_client(port, rdzv._MAGIC + b"1", q, "duplicate")
    assert q.get(timeout=30) == ("duplicate", "closed")
    t2 = threading.Thread(target=client, args=(2,))
    t2.start()
    for t in (t0, t1, t2):
        t.join(timeout=60)
    assert res["server"] == 2.0 and out == {1: 2.0, 2: 2.0}


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
