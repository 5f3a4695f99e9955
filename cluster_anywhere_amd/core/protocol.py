"""Length-prefixed pickle messages over stream sockets (unix or TCP).

The control plane (reference: the gRPC services in src/ray/protobuf/*.proto)
is a set of tuples ``(msg_type, ...)`` pickled with protocol 5. Framing is an
8-byte little-endian length. Sends are serialised by a per-connection lock so
several threads of one process can share a connection.
"""
from __future__ import annotations

import pickle
import socket
import struct
import threading

_LEN = struct.Struct("<Q")


class ConnectionClosed(Exception):
    pass


class Conn:
    __slots__ = ("sock", "_send_lock", "_rbuf", "closed", "peer")

    def __init__(self, sock: socket.socket, peer=None):
        self.sock = sock
        self._send_lock = threading.Lock()
        self._rbuf = bytearray()
        self.closed = False
        self.peer = peer
        if sock.family in (socket.AF_INET, socket.AF_INET6):
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def send(self, msg) -> None:
        data = pickle.dumps(msg, protocol=5)
        with self._send_lock:
            try:
                self.sock.sendall(_LEN.pack(len(data)) + data if len(data) < 65536 else _LEN.pack(len(data)))
                if len(data) >= 65536:
                    self.sock.sendall(data)
            except OSError as e:
                self.closed = True
                raise ConnectionClosed(str(e)) from e

    def send_many(self, msgs) -> None:
        parts = []
        for m in msgs:
            d = pickle.dumps(m, protocol=5)
            parts.append(_LEN.pack(len(d)))
            parts.append(d)
        with self._send_lock:
            try:
                self.sock.sendall(b"".join(parts))
            except OSError as e:
                self.closed = True
                raise ConnectionClosed(str(e)) from e

    def _read_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(max(n - len(buf), 1 << 16))
            if not chunk:
                self.closed = True
                raise ConnectionClosed("peer closed")
            buf += chunk
        return bytes(buf)

    def recv(self):
        """Blocking receive of one message."""
        while len(self._rbuf) < 8:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                self.closed = True
                raise ConnectionClosed("peer closed")
            self._rbuf += chunk
        (n,) = _LEN.unpack_from(self._rbuf, 0)
        while len(self._rbuf) < 8 + n:
            chunk = self.sock.recv(max(8 + n - len(self._rbuf), 1 << 16))
            if not chunk:
                self.closed = True
                raise ConnectionClosed("peer closed")
            self._rbuf += chunk
        data = bytes(self._rbuf[8 : 8 + n])
        del self._rbuf[: 8 + n]
        return pickle.loads(data)

    def feed(self, data: bytes):
        """Non-blocking path (selector loop): append bytes, yield complete messages."""
        self._rbuf += data
        out = []
        while len(self._rbuf) >= 8:
            (n,) = _LEN.unpack_from(self._rbuf, 0)
            if len(self._rbuf) < 8 + n:
                break
            out.append(pickle.loads(bytes(self._rbuf[8 : 8 + n])))
            del self._rbuf[: 8 + n]
        return out

    def close(self):
        self.closed = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass


class BatchSender:
    """Coalescing sender for one Conn. ``put`` pickles in the calling thread; when
    nothing is queued or being sent it also SENDS in the calling thread (a lone
    message — a sync actor call, its reply — costs no thread hand-off); otherwise
    it queues, and a daemon thread sends everything queued in ONE sendall, so a
    burst of small messages costs one syscall and one GIL hand-off instead of one
    per message. FIFO order holds: at most one send is in progress at a time."""

    def __init__(self, conn: Conn, name: str = "caamd-sender"):
        self.conn = conn
        self._q = []
        self._cv = threading.Condition()
        self._busy = False
        self.closed = False
        self._thread = threading.Thread(target=self._run, name=name, daemon=True)
        self._thread.start()

    def put(self, msg) -> None:
        d = pickle.dumps(msg, protocol=5)
        with self._cv:
            if self.closed:
                raise ConnectionClosed("sender closed")
            if self._q or self._busy:
                self._q.append(_LEN.pack(len(d)))
                self._q.append(d)
                self._cv.notify()
                return
            self._busy = True
        try:
            with self.conn._send_lock:
                self.conn.sock.sendall(_LEN.pack(len(d)) + d)
        except OSError:
            self.conn.closed = True
            with self._cv:
                self.closed = True
        finally:
            with self._cv:
                self._busy = False
                self._cv.notify()

    def _run(self):
        while True:
            with self._cv:
                while (not self._q and not self.closed) or self._busy:
                    self._cv.wait()
                if not self._q:
                    return  # closed and drained
                parts, self._q = self._q, []
                self._busy = True
            try:
                with self.conn._send_lock:
                    self.conn.sock.sendall(b"".join(parts))
            except OSError:
                self.conn.closed = True
                with self._cv:
                    self.closed = True
                    self._busy = False
                    self._cv.notify_all()
                return
            with self._cv:
                self._busy = False
                self._cv.notify_all()

    def close(self):
        with self._cv:
            self.closed = True
            self._cv.notify_all()

    def drain(self, timeout: float = 2.0):
        """Close, then wait until everything queued so far has been sent."""
        self.close()
        if self._thread is not threading.current_thread():
            self._thread.join(timeout)


def connect(address: str) -> Conn:
    """``address`` is a unix socket path or ``host:port``."""
    if address.startswith("unix:") or address.startswith("/"):
        path = address[5:] if address.startswith("unix:") else address
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect(path)
    else:
        host, port = address.rsplit(":", 1)
        s = socket.create_connection((host, int(port)))
    return Conn(s, address)
