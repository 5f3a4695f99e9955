"""Node-to-node object transfer (reference: src/ray/object_manager/ —
object_manager.cc pull/push over gRPC chunks).

Every node (the head node and each node agent) runs one ``ObjectServer``
thread next to its shared-memory store. A worker that needs an object whose
primary copy lives on another node pulls it directly from that node's server
(no hop through the head): request = 24-byte object id, response = 8-byte
length + the sealed object bytes, sent straight from the pinned shm buffer
(``sendall`` on a memoryview, no intermediate copy)."""
from __future__ import annotations

import socket
import struct
import threading
from typing import Optional

_LEN = struct.Struct("<q")
OID_BYTES = 24


def _recv_exact(s: socket.socket, n: int, into: Optional[memoryview] = None):
    buf = into if into is not None else memoryview(bytearray(n))
    got = 0
    while got < n:
        k = s.recv_into(buf[got:], n - got)
        if k == 0:
            raise ConnectionError("object server closed the connection")
        got += k
    return buf


class ObjectServer:
    def __init__(self, store, host: str = "0.0.0.0", port: int = 0):
        self.store = store
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(256)
        self.port = self.sock.getsockname()[1]
        self.alive = True
        self.bytes_served = 0
        self.thread = threading.Thread(target=self._accept, name="caamd-objsrv", daemon=True)
        self.thread.start()

    def address(self, host: str = "127.0.0.1") -> str:
        return f"{host}:{self.port}"

    def _accept(self):
        while self.alive:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c: socket.socket):
        try:
            while True:
                try:
                    oid = bytes(_recv_exact(c, OID_BYTES))
                except ConnectionError:
                    return
                pb = self.store.get_pinned(oid)
                if pb is None:
                    c.sendall(_LEN.pack(-1))
                    continue
                mv = memoryview(pb)
                c.sendall(_LEN.pack(mv.nbytes))
                c.sendall(mv)
                self.bytes_served += mv.nbytes
                del mv, pb
        finally:
            c.close()

    def close(self):
        self.alive = False
        try:
            self.sock.close()
        except OSError:
            pass


_conns = threading.local()


def pull(address: str, oid: bytes) -> Optional[bytearray]:
    """Fetch the bytes of ``oid`` from the object server at ``address``."""
    pool = getattr(_conns, "pool", None)
    if pool is None:
        pool = _conns.pool = {}
    s = pool.get(address)
    for attempt in range(2):
        if s is None:
            host, port = address.rsplit(":", 1)
            s = socket.create_connection((host, int(port)))
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            pool[address] = s
        try:
            s.sendall(oid)
            (n,) = _LEN.unpack(bytes(_recv_exact(s, 8)))
            if n < 0:
                return None
            buf = bytearray(n)
            _recv_exact(s, n, memoryview(buf))
            return buf
        except (ConnectionError, OSError):
            pool.pop(address, None)
            try:
                s.close()
            except OSError:
                pass
            s = None
            if attempt == 1:
                raise
    return None
