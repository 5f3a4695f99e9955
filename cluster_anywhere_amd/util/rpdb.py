"""Remote debugger for tasks/actors (reference: util/rpdb.py, ``ray.util.pdb``):
``set_trace()`` inside a worker opens a pdb session on a TCP port (printed to
the worker log, which streams to the driver) — connect with ``nc host port``
or ``python -m cluster_anywhere_amd debug``. In an interactive driver it is
plain pdb."""
from __future__ import annotations

import os
import pdb
import socket
import sys


class RemotePdb(pdb.Pdb):
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self._listen = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._listen.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._listen.bind((host, port))
        self._listen.listen(1)
        self.address = "%s:%d" % self._listen.getsockname()
        print(f"RemotePdb session open at {self.address} (pid={os.getpid()}); connect with `nc {host} "
              f"{self._listen.getsockname()[1]}`", file=sys.stderr, flush=True)
        conn, _ = self._listen.accept()
        self._conn = conn
        fh = conn.makefile("rw")
        super().__init__(stdin=fh, stdout=fh)
        self.use_rawinput = False
        self.prompt = "(caamd-pdb) "

    def do_continue(self, arg):
        r = super().do_continue(arg)
        self._close()
        return r

    do_c = do_cont = do_continue

    def _close(self):
        try:
            self._conn.close()
            self._listen.close()
        except OSError:
            pass


def set_trace(breakpoint_uuid=None):
    from ..core import context

    w = context.worker
    if w is None or getattr(w, "kind", "driver") == "driver":
        pdb.Pdb().set_trace(sys._getframe().f_back)
        return
    RemotePdb(os.environ.get("CAAMD_DEBUG_HOST", "127.0.0.1")).set_trace(sys._getframe().f_back)


def post_mortem():
    pdb.post_mortem()
