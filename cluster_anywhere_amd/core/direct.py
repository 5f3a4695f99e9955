"""Direct actor-call transport: callers send actor tasks straight to the actor's
worker process and get the results straight back; the head is off the call path.

Reference roles: ``src/ray/core_worker/transport/actor_task_submitter.cc:158``
(direct actor task submission) and the owner-side bookkeeping of
``reference_count.h:66``. MI355X-node design:

* every worker process serves a Unix-socket ``DirectServer`` (same-node callers;
  cross-node calls keep the head path);
* a caller switches an actor to direct mode only when it has NO head-routed call to
  that actor still running (owner notifications tell it when they finish), so the
  per-caller FIFO order of actor calls is preserved across the switch; all direct
  calls of one caller share one connection and one reader on the actor side;
* results come back in the reply and land in the caller's owner-side store (get /
  wait are local); the caller then registers the return objects with the head in
  one ``dseal`` message on its own ordered control connection — so the head learns
  them before any later decref from the same caller, and refs that escaped to other
  processes resolve normally. Decrefs of refs dropped while the call is in flight
  are held back until that seal;
* nested refs inside results are pinned by the actor (``dpin``) before it replies
  and released by the head when the caller's seal arrives;
* if the actor's connection breaks, pending calls are resubmitted through the head
  (which restarts the actor and applies ``max_task_retries``) when retries are
  allowed, otherwise they fail locally with ``ActorDiedError`` and are sealed as
  errors at the head.
"""
from __future__ import annotations

import os
import socket
import tempfile
import threading
import time
from typing import Dict, Optional

from .head import NORMAL
from .protocol import BatchSender, Conn, ConnectionClosed, connect


class DirectServer:
    """Worker side: accept direct connections, feed ``dexec`` into the worker."""

    def __init__(self, worker):
        self.worker = worker
        self.path = os.path.join(tempfile.gettempdir(), f"caamd-d-{worker.worker_id.hex()[:12]}.sock")
        try:
            os.unlink(self.path)
        except OSError:
            pass
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.bind(self.path)
        self.sock.listen(256)
        self.senders = []
        threading.Thread(target=self._accept, name="caamd-direct-accept", daemon=True).start()

    def _accept(self):
        while True:
            try:
                s, _ = self.sock.accept()
            except OSError:
                return
            c = Conn(s)
            threading.Thread(target=self._serve, args=(c,), name="caamd-direct", daemon=True).start()

    def _serve(self, c: Conn):
        w = self.worker
        out = BatchSender(c, "caamd-direct-reply")  # replies coalesce into few sends
        self.senders.append(out)
        while True:
            try:
                msg = c.recv()
            except (ConnectionClosed, OSError):
                out.close()
                return
            if msg[0] == "dexec":
                # (spec, resolved args the caller already had, function blob on first use)
                spec = msg[1]
                resolved = msg[2] if len(msg) > 2 else None
                fn_blob = msg[3] if len(msg) > 3 else None
                if fn_blob is not None and spec.fn_id not in w.fn_cache:
                    from . import serialization

                    w.fn_cache[spec.fn_id] = serialization.loads_function(fn_blob)
                if w.actor_id is None and w._n_blocked > 0 and spec.kind == NORMAL:
                    # our running task is blocked in get(): a queued task could be what
                    # it waits for, so the owner re-dispatches it to another lease
                    try:
                        out.put(("dreturn", spec.task_id))
                    except (ConnectionClosed, OSError):
                        pass
                    continue
                w.direct_origin[spec.task_id] = out
                w._on_execute((spec, fn_blob, resolved if resolved is not None else {}))
            elif msg[0] == "dcancel":
                _, task_id, force = msg
                if force and w.actor_id is None and task_id in w.running_tasks:
                    # force-cancel of a running leased task ends the worker; the tasks
                    # queued behind it go back to their owners first (no attempt spent)
                    w._return_unstarted_leased(exclude=task_id)
                    for o in list(self.senders):
                        o.drain(1.0)
                    os._exit(1)
                w._on_cancel(task_id)

    def close(self):
        try:
            self.sock.close()
            os.unlink(self.path)
        except OSError:
            pass
        for out in list(self.senders):  # replies already produced still reach their callers
            out.drain(2.0)


class DirectClient:
    """Caller side: one connection to one worker (an actor, or a leased task
    worker when ``sink`` is a lease manager — core/lease.py)."""

    def __init__(self, worker, actor_id: bytes, addr: str, sink=None):
        self.worker = worker
        self.actor_id = actor_id
        self.sink = sink
        self.conn = connect(addr)
        self.out = BatchSender(self.conn, "caamd-direct-send")
        self.alive = True
        self.lock = threading.Lock()
        self.idle = threading.Condition(self.lock)
        self.pending: Dict[bytes, tuple] = {}  # task_id -> (spec, keep-alive refs, t_submit)
        self.sent_fns = set()
        threading.Thread(target=self._read, name="caamd-direct-client", daemon=True).start()

    def submit(self, spec, keep, resolved=None, fn_blob=None):
        with self.lock:
            if not self.alive:
                return False
            self.pending[spec.task_id] = (spec, keep, time.time())
        try:
            self.out.put(("dexec", spec, resolved, fn_blob))
        except ConnectionClosed:
            return True  # the reader's failure path resubmits / fails it
        return True

    def cancel(self, task_id: bytes, force: bool = False):
        try:
            self.out.put(("dcancel", task_id, force))
        except ConnectionClosed:
            pass

    def _read(self):
        while True:
            try:
                msg = self.conn.recv()
            except (ConnectionClosed, OSError):
                break
            if msg[0] == "ddone":
                task_id, results, error_kind, t0, t1, pid = msg[1:7]
                retryable = msg[7] if len(msg) > 7 else False
                with self.lock:
                    rec = self.pending.pop(task_id, None)
                    drained = not self.pending
                    if drained:
                        self.idle.notify_all()
                if rec is None:
                    continue
                if self.sink is not None:
                    self.sink._done(self, rec[0], results, error_kind, retryable, (t0, t1, pid))
                else:
                    self.worker._on_direct_done(rec[0], results, (t0, t1, pid))
                    if drained:
                        self.worker._direct_drained(self.actor_id)
        with self.lock:
            self.alive = False
            recs = sorted(self.pending.values(), key=lambda r: r[2])
            self.pending.clear()
            self.idle.notify_all()
        if self.sink is not None:
            self.sink._lost(self, [r[0] for r in recs])
        else:
            self.worker._on_direct_lost(self.actor_id, [r[0] for r in recs])
            self.worker._direct_drained(self.actor_id)  # after the resubmits, on the same connection

    def wait_idle(self, timeout: float) -> bool:
        """Block until every call sent on this connection has been answered (or the
        connection died). False on timeout."""
        deadline = time.time() + timeout
        with self.lock:
            while self.pending and self.alive:
                left = deadline - time.time()
                if left <= 0:
                    return False
                self.idle.wait(min(left, 1.0))
        return True

    def close(self):
        self.alive = False
        self.out.close()
        self.conn.close()


def result_kinds(results, my_node: str):
    """(oid, kind, payload) for the owner-side store from packaged task results."""
    out = []
    for (oid, inline, size, node_hex, _contained, is_err) in results:
        if inline is not None:
            out.append((oid, "err" if is_err else "inline", inline))
        elif node_hex == my_node:
            out.append((oid, "err_store" if is_err else "store", size))
        else:
            out.append((oid, None, None))  # not local: resolve through the head
    return out


def addr_usable(addr: Optional[str]) -> bool:
    return bool(addr) and os.path.exists(addr)
