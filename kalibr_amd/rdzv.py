"""Host-side rendezvous for the one-process-per-GPU runs, stdlib only (no torch in the product processes).

`torch.distributed.run` (or any launcher that sets RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT) starts one
process per GPU.  The processes need three host-side services and nothing else: broadcast the 128-byte RCCL
unique id from rank 0, barriers around the timed region, and the max over ranks of the wall time.  All data-path
traffic goes over RCCL inside the captured pass graphs (kb_comm_init).  Importing torch here would load torch's
bundled HIP runtime and RCCL into the process next to the library's /opt/rocm ones, so this is a small star of TCP
connections to rank 0 instead.

Port: MASTER_PORT belongs to the launcher's own store, so rank 0 listens on MASTER_PORT + 1 (KB_RDZV_PORT overrides);
clients retry until rank 0 is up and check a handshake, so a foreign service on that port is never mistaken for
it.
"""
import os
import socket
import struct
import time

_MAGIC = b"KBRDZV01"
_MAX_HELLO = len(_MAGIC) + 16  # magic + a decimal rank id


def _send(sock, data: bytes):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class TcpGroup:
    """rank 0 holds one connection per other rank; every collective is a gather to rank 0 and a reply."""

    def __init__(self, rank, world, addr=None, port=None, timeout=300.0):
        self.rank, self.world = int(rank), int(world)
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("KB_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        self.peers = []
        self.sock = None
        if self.world == 1:
            return
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            by_rank = {}
            try:
                while len(by_rank) < self.world - 1:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        raise TimeoutError(f"rank 0: {len(by_rank)} of {self.world - 1} ranks reached {addr}:{port}")
                    srv.settimeout(left)  # recomputed per connection: foreign connects cannot extend the deadline
                    try:
                        c, _ = srv.accept()
                    except socket.timeout:
                        continue
                    # a peer gets at most the remaining time (and 10 s) to say hello
                    c.settimeout(max(0.1, min(10.0, deadline - time.monotonic())))
                    peer = self._hello_rank(c)
                    if peer is None or peer in by_rank:
                        # not a rendezvous client, a rank id outside 1..world-1, or a duplicate rank: refused before
                        # the handshake reply, so the refused client never takes this server for rank 0
                        c.close()
                        continue
                    c.settimeout(timeout)
                    by_rank[peer] = c
                    _send(c, _MAGIC)
            except BaseException:
                for c in by_rank.values():
                    c.close()
                raise
            finally:
                srv.close()
            self.peers = [by_rank[r] for r in range(1, self.world)]
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    s.settimeout(timeout)
                    _send(s, _MAGIC + str(self.rank).encode())
                    if _recv(s) == _MAGIC:
                        self.sock = s
                        break
                    s.close()
                except (OSError, ConnectionError):
                    pass
                if time.monotonic() > deadline:
                    raise TimeoutError(f"rank {self.rank}: no rendezvous with rank 0 at {addr}:{port}")
                time.sleep(0.2)

    def _hello_rank(self, c):
        """the rank id of a client's hello, or None for anything else (a foreign service, a malformed or truncated
        hello, a rank outside 1..world-1)"""
        try:
            (n,) = struct.unpack("<Q", _recv_exact(c, 8))
            # a hello is the magic and a rank id: an unframed foreign client's first bytes read as a huge length,
            # which is refused before anything is allocated for it
            if n > _MAX_HELLO:
                return None
            hello = _recv_exact(c, n)
        except (OSError, ConnectionError, struct.error):
            return None
        if not hello.startswith(_MAGIC):
            return None
        try:
            peer = int(hello[len(_MAGIC):].decode("ascii"))
        except (UnicodeDecodeError, ValueError):
            return None
        return peer if 1 <= peer < self.world else None

    def _gather_reply(self, payload: bytes, reply_fn):
        """every rank sends payload to rank 0; rank 0 computes reply_fn([payload of rank 0..world-1]) and sends it
        back to all; returns the reply on every rank"""
        if self.world == 1:
            return reply_fn([payload])
        if self.rank == 0:
            parts = [payload] + [_recv(p) for p in self.peers]
            rep = reply_fn(parts)
            for p in self.peers:
                _send(p, rep)
            return rep
        _send(self.sock, payload)
        return _recv(self.sock)

    def broadcast(self, data: bytes = b"") -> bytes:
        return self._gather_reply(data if self.rank == 0 else b"", lambda parts: parts[0])

    def barrier(self):
        self._gather_reply(b"", lambda parts: b"")

    def max(self, x: float) -> float:
        rep = self._gather_reply(struct.pack("<d", float(x)),
                                 lambda parts: struct.pack("<d", max(struct.unpack("<d", p)[0] for p in parts)))
        return struct.unpack("<d", rep)[0]

    def close(self):
        for s in self.peers + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = [], None
