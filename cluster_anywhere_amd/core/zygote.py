"""Pre-initialised fork server for worker processes (a "zygote").

Starting a worker that uses PyTorch costs ~1.6 s of ``import torch`` before it
can run anything — that is most of a GPU actor's start-up (Data GPU map
actors, Train workers, learner actors, Serve replicas). The head starts ONE
zygote process per node that imports numpy, torch and the worker runtime
(never touching HIP: no GPU is initialised) and then forks a worker per request
in a few milliseconds. The fork happens in a single-threaded process, so no
lock is inherited mid-held; the child:

* takes the environment the head computed for the worker (``ROCR_VISIBLE_DEVICES``
  etc. are read when HIP first initialises, which is after the fork),
* redirects stdout/stderr to the worker log, changes to the requested cwd,
* reseeds Python / numpy / torch RNGs (forked children would otherwise share
  the zygote's random state),
* and runs ``worker_main.main()``.

Workers are children of the zygote (which reaps them); the head tracks them by
pid through ``ForkedProc`` (``poll`` / ``wait`` / ``kill``, like ``Popen``). If
the zygote is not ready yet or a request fails, the head falls back to a plain
``subprocess.Popen``.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import struct
import subprocess
import sys
import threading
import time
from typing import Dict, Optional


# ------------------------------------------------------------------ zygote process
def _reap(*_):
    while True:
        try:
            pid, _ = os.waitpid(-1, os.WNOHANG)
        except ChildProcessError:
            return
        if pid == 0:
            return


def _recv_exact(c, n):
    buf = b""
    while len(buf) < n:
        part = c.recv(n - len(buf))
        if not part:
            raise ConnectionError("closed")
        buf += part
    return buf


def _child(req: Dict, srv: socket.socket):
    try:
        srv.close()
        signal.signal(signal.SIGCHLD, signal.SIG_DFL)
        fd = os.open(req["log"], os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(fd, 1)
        os.dup2(fd, 2)
        os.close(fd)
        nul = os.open(os.devnull, os.O_RDONLY)
        os.dup2(nul, 0)
        os.close(nul)
        os.environ.clear()
        os.environ.update(req["env"])
        if req.get("cwd") and os.path.isdir(req["cwd"]):
            os.chdir(req["cwd"])
        import random

        random.seed()
        try:
            import numpy as np

            np.random.seed(None)
        except ImportError:
            pass
        try:
            import torch

            torch.seed()
        except ImportError:
            pass
        sys.argv = [sys.executable, "-m", "cluster_anywhere_amd.core.worker_main"]
        from . import worker_main

        worker_main.main()
    except BaseException:  # noqa: BLE001
        import traceback

        traceback.print_exc()
    finally:
        os._exit(1)


def zygote_main(sock_path: str):
    from .worker_main import _die_with_parent

    _die_with_parent()
    import numpy  # noqa: F401
    try:
        import torch  # noqa: F401  (host-side import only: no HIP call)
    except ImportError:
        pass
    from . import worker  # noqa: F401  (the worker runtime, pre-imported)

    # Warm the RNG seeding paths the children run: numpy's first seed-from-entropy
    # imports and initialises its entropy machinery (secrets / hashlib), ~140 ms that
    # every forked worker otherwise paid again between fork and main() (measured on
    # the CPU container: actor .remote() -> __init__ 125-170 ms, 140 of it here)
    import random

    random.seed()
    numpy.random.seed(None)
    try:
        torch.seed()  # (lazy: queues the device seeding, no HIP initialisation)
    except Exception:
        pass

    signal.signal(signal.SIGCHLD, _reap)
    try:
        os.unlink(sock_path)
    except OSError:
        pass
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(sock_path + ".tmp")
    srv.listen(64)
    os.rename(sock_path + ".tmp", sock_path)  # appears only once everything is imported
    while True:
        try:
            c, _ = srv.accept()
        except InterruptedError:
            continue
        try:
            n = struct.unpack("!I", _recv_exact(c, 4))[0]
            req = json.loads(_recv_exact(c, n))
            if threading.active_count() != 1:  # never fork a multi-threaded process
                c.sendall(struct.pack("!i", -1))
                continue
            pid = os.fork()
            if pid == 0:
                c.close()
                _child(req, srv)
            c.sendall(struct.pack("!i", pid))
        except (ConnectionError, OSError, ValueError):
            pass
        finally:
            c.close()


# ------------------------------------------------------------------ head side
class ForkedProc:
    """Popen-like view of a worker forked by the zygote (not our child: liveness
    comes from /proc)."""

    def __init__(self, pid: int):
        self.pid = pid
        self.returncode: Optional[int] = None

    def poll(self) -> Optional[int]:
        if self.returncode is not None:
            return self.returncode
        try:
            with open(f"/proc/{self.pid}/stat") as f:
                state = f.read().rsplit(")", 1)[1].split()[0]
            if state in ("Z", "X"):
                self.returncode = -1
        except (FileNotFoundError, ProcessLookupError, IndexError):
            self.returncode = -1
        return self.returncode

    def wait(self, timeout: Optional[float] = None) -> int:
        deadline = None if timeout is None else time.time() + timeout
        while self.poll() is None:
            if deadline is not None and time.time() > deadline:
                raise subprocess.TimeoutExpired(f"pid {self.pid}", timeout)
            time.sleep(0.01)
        return self.returncode

    def send_signal(self, sig):
        try:
            os.kill(self.pid, sig)
        except ProcessLookupError:
            pass

    def kill(self):
        self.send_signal(signal.SIGKILL)

    def terminate(self):
        self.send_signal(signal.SIGTERM)


class Zygote:
    def __init__(self, session_dir: str):
        self.sock = os.path.join(session_dir, f"zygote-{os.getpid()}.sock")
        log = open(os.path.join(session_dir, "zygote.log"), "ab")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self.proc = subprocess.Popen([sys.executable, "-c",
                                      "import sys; from cluster_anywhere_amd.core.zygote import zygote_main; "
                                      "zygote_main(sys.argv[1])", self.sock],
                                     env=env, stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL)
        log.close()
        self.failures = 0

    def ready(self) -> bool:
        return self.proc.poll() is None and os.path.exists(self.sock) and self.failures < 3

    def spawn(self, env: Dict[str, str], log_path: str, cwd: str) -> Optional[ForkedProc]:
        if not self.ready():
            return None
        try:
            c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            c.settimeout(5.0)
            c.connect(self.sock)
            body = json.dumps({"env": env, "log": log_path, "cwd": cwd}).encode()
            c.sendall(struct.pack("!I", len(body)) + body)
            pid = struct.unpack("!i", _recv_exact(c, 4))[0]
            c.close()
        except (OSError, ConnectionError, struct.error):
            self.failures += 1
            return None
        if pid <= 0:
            self.failures += 1
            return None
        return ForkedProc(pid)

    def stop(self):
        try:
            self.proc.kill()
            self.proc.wait(timeout=5)
        except Exception:
            pass
        try:
            os.unlink(self.sock)
        except OSError:
            pass


def enabled() -> bool:
    if os.environ.get("CAAMD_ZYGOTE", "1") != "1":
        return False
    import importlib.util

    return importlib.util.find_spec("torch") is not None
