"""CoreWorker: the per-process client of the head (reference role:
src/ray/core_worker/core_worker.cc + python/ray/_private/worker.py).

Owns the control connection, the ordered reference-count stream, object
put/get/wait against the shared-memory store, task submission, and (in worker
processes) task execution: normal tasks, actor construction and actor methods
(sequential, threaded via ``max_concurrency`` or asyncio for ``async def``
methods), streaming / dynamic generators, cancellation and error propagation.
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import ctypes
import hashlib
import inspect
import itertools
import operator
import os
import queue
import sys
import threading
import time
import traceback
from typing import Any, Callable, Dict, List, Optional

from . import context, serialization
from .head import ACTOR_CREATE, ACTOR_METHOD, INLINE_MAX, NORMAL, TaskSpec
from .ids import ObjectID
from .object_ref import DynamicObjectRefGenerator, ObjectRef, ObjectRefGenerator
from .protocol import ConnectionClosed, connect


_COPY_THREADS = max(1, min(8, (os.cpu_count() or 1) // 2))


class RefCounter:
    """Process-local counts; 0->1 borrow announcements and 1->0 releases are
    queued IN ORDER and flushed ahead of the next control message."""

    def __init__(self):
        self.counts: Dict[bytes, int] = {}
        self.lock = threading.Lock()
        self.ops: List[tuple] = []
        # owner-side results of tasks this process submitted, pushed by the head as
        # they finish: oid -> (kind, payload); ``owned`` = submitted, not yet pushed
        self.ready: Dict[bytes, tuple] = {}
        self.owned = set()
        self.cv = threading.Condition(self.lock)
        # return oids of direct actor calls not yet sealed at the head; decrefs of
        # those dropped meanwhile are held back until the seal (see core/direct.py)
        self.direct_pending = set()
        self.direct_dropped = set()
        self.dseal_buf: List[tuple] = []
        # resolved (kind, payload) of immutable objects this process holds refs
        # to: ray.get of them needs no round trip to the head (the reference's
        # in-process memory store for owned/inlined objects)
        self.cache: Dict[bytes, tuple] = {}
        # releases queued by finalizers that found the lock busy (see remove())
        self.deferred: collections.deque = collections.deque()
        # inline results of direct calls / leased tasks the head has not been told
        # about: oid -> (inline, size, is_err). Sealed at the head (``lseal``) only
        # when the ref escapes this process; dropping it needs no message at all.
        self.local_only: Dict[bytes, tuple] = {}
        # direct results still in flight whose refs already escaped: sealed normally
        self.must_seal = set()
        # actor handle refs whose last local handle went away while direct calls to
        # the actor were still unanswered: their decref (which lets the head append
        # __ray_terminate__ to the actor's queue) waits until those calls are done,
        # since the head's terminate would otherwise overtake them (Pool race, r3)
        self.handle_busy: Optional[Callable[[bytes], bool]] = None
        self.held_handles = set()

    def release_held_handle(self, oid: bytes):
        """The direct calls that held back ``oid``'s decref are all answered."""
        with self.lock:
            if oid in self.held_handles and oid not in self.counts:
                self.held_handles.discard(oid)
                self.ops.append(("d", oid))

    def add(self, oid: bytes, announce: bool):
        with self.lock:
            if self.deferred:
                self._run_deferred()
            c = self.counts.get(oid, 0)
            self.counts[oid] = c + 1
            if c == 0 and announce:
                self.ops.append(("a", oid))

    def remove(self, oid: bytes, blocking: bool = True):
        """``blocking=False`` (ObjectRef finalizers): a finalizer may run from the
        garbage collector INSIDE one of this thread's own critical sections (e.g.
        popping a cached payload that holds nested refs), so it must never wait
        for the lock; when the lock is busy the release is queued and applied by
        the next lock holder (the flush loop drains within 50 ms)."""
        if not self.lock.acquire(blocking):
            self.deferred.append(oid)
            return
        try:
            if self.deferred:
                self._run_deferred()
            self._remove_locked(oid)
        finally:
            self.lock.release()

    def _run_deferred(self):
        while self.deferred:
            try:
                oid = self.deferred.popleft()
            except IndexError:
                return
            self._remove_locked(oid)

    def _remove_locked(self, oid: bytes):
        c = self.counts.get(oid)
        if c is None:
            return
        if c <= 1:
            del self.counts[oid]
            # nested refs inside a dropped payload finalize right here, inside the lock:
            # their (non-blocking) releases are queued in ``deferred``
            self.cache.pop(oid, None)
            self.ready.pop(oid, None)
            self.owned.discard(oid)
            if oid in self.local_only:
                del self.local_only[oid]
            elif oid in self.direct_pending:
                self.direct_dropped.add(oid)
            elif self.handle_busy is not None and self.handle_busy(oid):
                self.held_handles.add(oid)
            else:
                self.ops.append(("d", oid))
        else:
            self.counts[oid] = c - 1

    def escape(self, oids) -> List[tuple]:
        """Owner-local results among ``oids`` that must now be sealed at the head."""
        out = []
        with self.lock:
            lo, dp = self.local_only, self.direct_pending
            for o in oids:
                ent = lo.pop(o, None)
                if ent is not None:
                    out.append((o, *ent))
                elif o in dp:
                    self.must_seal.add(o)
        return out

    def drain(self):
        with self.lock:
            return self.drain_locked()

    def drain_locked(self):
        if self.deferred:
            self._run_deferred()
        ops, self.ops = self.ops, []
        msgs = []
        for kind, group in itertools.groupby(ops, key=lambda x: x[0]):
            ids = [o for _, o in group]
            msgs.append(("addref" if kind == "a" else "decref", ids))
        return msgs


class _Cancelled(BaseException):
    pass


class CoreWorker:
    def __init__(self, address: str, kind: str, worker_id: bytes, node_hex: str = "",
                 job_id: bytes = b"\x00\x00\x00\x01", extra: Optional[dict] = None):
        self.address = address
        self.kind = kind
        self.worker_id = worker_id
        self.job_id = job_id
        self.conn = connect(address)
        self.refs = RefCounter()
        self.refs.handle_busy = self._handle_busy
        # re-entrant: pickling a message may seal an escaping owner-local ref first
        self.send_lock = threading.RLock()
        self._req = itertools.count(1)
        self.pending: Dict[int, concurrent.futures.Future] = {}
        self.task_queue: "queue.Queue" = queue.Queue()
        self.fn_cache: Dict[bytes, Any] = {}
        self.sent_fns = set()
        self.fn_blobs: Dict[bytes, bytes] = {}
        self._ready_cbs: Dict[bytes, list] = {}  # oid -> callbacks when it completes here
        self.running_tasks: Dict[bytes, threading.Thread] = {}
        self.cancelled_tasks = set()
        self.actor_instance = None
        self.actor_id = None
        self.actor_opts = {}
        self.async_loop = None
        self.thread_pool = None
        self.alive = True
        # direct actor-call transport (core/direct.py)
        self.direct_origin: Dict[bytes, Any] = {}
        self._n_blocked = 0  # running normal tasks currently blocked in get()/wait()
        self.actor_direct: Dict[bytes, Any] = {}
        self.actor_head_inflight: Dict[bytes, set] = {}
        self.head_inflight_actor: Dict[bytes, bytes] = {}
        self.actor_head_only = set()
        self._direct_lock = threading.Lock()
        self.direct_server = None
        # head restart (core/gcs_persist.py): with reconnect_s > 0 this process keeps
        # running when the head goes away, reconnects, re-registers and replays its
        # outstanding requests and head-path task submissions
        self.reconnect_s = float(os.environ.get("CAAMD_HEAD_RECONNECT_S", "0") or 0)
        self._conn_cv = threading.Condition()
        self._req_builds: Dict[int, Any] = {}
        self._head_specs: Dict[bytes, Any] = {}  # head-path tasks in flight (replayed on re-attach)
        self._ret_task: Dict[bytes, bytes] = {}
        self._running_res: Dict[bytes, dict] = {}
        self._unsent_done = set()
        self.reattaches = 0
        self._subs: Dict[str, List[Any]] = {}  # pubsub channel -> callbacks (run in the reader thread)
        self.gen_drops: collections.deque = collections.deque()  # dropped generators (finalizers)
        from . import lease

        self.leases = lease.LeaseManager(self) if lease.enabled() and kind in ("driver", "worker") else None
        if kind == "worker" and os.environ.get("CAAMD_DIRECT_CALLS", "1") == "1":
            from .direct import DirectServer

            self.direct_server = DirectServer(self)
            extra = dict(extra or {}, direct=self.direct_server.path)
        self.conn.send(("register", kind, worker_id, os.getpid(), node_hex, dict(extra or {}, job_id=job_id)))
        msg = self.conn.recv()
        assert msg[0] == "registered", msg
        info = msg[1]
        self.reconnect_s = max(self.reconnect_s, float(info.get("reconnect_s") or 0))
        self.node_hex = info["node_id"]
        self.namespace = info["namespace"]
        self.session_dir = info["session_dir"]
        self.store = self._attach_store(info["store_name"])
        self._reader = threading.Thread(target=self._read_loop, name="caamd-reader", daemon=True)
        self._reader.start()
        self._flush_evt = threading.Event()
        self._flusher = threading.Thread(target=self._flush_loop, name="caamd-flush", daemon=True)
        self._flusher.start()

    def _attach_store(self, store_name):
        from .. import _native

        return _native.ObjectStore(store_name, 0, 0, False)

    # ------------------------------------------------------------- transport
    def send(self, msg):
        # borrow announcements go BEFORE the message, releases AFTER it: a message
        # may pin objects (task_done with nested refs, submit args) whose last
        # local reference died while it was being built.
        while True:
            conn = self.conn
            try:
                with self.send_lock:
                    ops = self.refs.drain()
                    if ops:
                        adds = [m for m in ops if m[0] == "addref"]
                        decs = [m for m in ops if m[0] == "decref"]
                        conn.send_many(adds + [msg] + decs)
                    else:
                        conn.send(msg)
                return
            except (ConnectionClosed, OSError):
                if not self._await_reconnect(conn):
                    raise

    def _await_reconnect(self, old) -> bool:
        """Block a sender until the reader thread has re-attached to a restarted head
        (True) or given up (False)."""
        if self.reconnect_s <= 0 or threading.current_thread() is getattr(self, "_reader", None):
            return False
        deadline = time.time() + self.reconnect_s + 5
        with self._conn_cv:
            while self.conn is old and self.alive and time.time() < deadline:
                self._conn_cv.wait(0.5)
        return self.conn is not old

    def request(self, build, timeout=None):
        req = next(self._req)
        fut = concurrent.futures.Future()
        self.pending[req] = fut
        if self.reconnect_s > 0:
            self._req_builds[req] = build
        try:
            self.send(build(req))
            return fut.result(timeout)
        finally:
            self.pending.pop(req, None)
            self._req_builds.pop(req, None)

    def request_cb(self, build, cb):
        """Send a request; ``cb(value)`` runs in the reader thread (None on failure)."""
        req = next(self._req)
        fut = concurrent.futures.Future()

        def done(f, r=req):
            self.pending.pop(r, None)
            self._req_builds.pop(r, None)
            cb(None if f.exception() is not None else f.result())

        fut.add_done_callback(done)
        self.pending[req] = fut
        if self.reconnect_s > 0:
            self._req_builds[req] = build
        self.send(build(req))

    def _escape(self, oids):
        """Seal owner-local results at the head before their refs leave this
        process (ordered ahead of whatever message carries them)."""
        items = self.refs.escape(oids)
        if items:
            self.send(("lseal", items))

    def request_async(self, build) -> concurrent.futures.Future:
        req = next(self._req)
        fut = concurrent.futures.Future()
        self.pending[req] = fut
        if self.reconnect_s > 0:
            self._req_builds[req] = build
        fut.add_done_callback(lambda f, r=req: (self.pending.pop(r, None), self._req_builds.pop(r, None)))
        self.send(build(req))
        return fut

    def _flush_dseals(self):
        """Register finished direct calls with the head: ONE message per batch. The
        held-back decrefs of their return refs are released atomically with it."""
        r = self.refs
        with self.send_lock:
            with r.cv:
                buf, r.dseal_buf = r.dseal_buf, []
                if not buf:
                    return
                items = []
                for (tid, name, results, rids, timing) in buf:
                    dropped = []
                    for oid in rids:
                        r.direct_pending.discard(oid)
                        r.must_seal.discard(oid)
                        if oid in r.direct_dropped:
                            r.direct_dropped.discard(oid)
                            dropped.append(oid)
                    items.append((tid, name, results, dropped, *timing))
                ops = r.drain_locked()
            msgs = [m for m in ops if m[0] == "addref"] + [("dseal_batch", items)] + \
                   [m for m in ops if m[0] == "decref"]
        while True:
            conn = self.conn
            try:
                with self.send_lock:
                    conn.send_many(msgs)
                return
            except (ConnectionClosed, OSError):
                if not self._await_reconnect(conn):
                    raise

    def _flush_loop(self):
        while self.alive:
            self._flush_evt.wait(0.005 if self.refs.dseal_buf else 0.05)
            self._flush_evt.clear()
            while self.gen_drops:
                try:
                    self.send(("gen_drop", self.gen_drops.popleft()))
                except (ConnectionClosed, OSError, IndexError):
                    break
            if self.refs.dseal_buf:
                try:
                    self._flush_dseals()
                except (ConnectionClosed, OSError):
                    return
            if self.refs.ops or self.refs.deferred:
                conn = self.conn
                try:
                    with self.send_lock:
                        ops = self.refs.drain()
                        if ops:
                            conn.send_many(ops)
                except (ConnectionClosed, OSError):
                    # released refs are re-counted from scratch on re-attach
                    if not self._await_reconnect(conn):
                        return

    def _read_loop(self):
        while self.alive:
            try:
                msg = self.conn.recv()
            except (ConnectionClosed, OSError):
                if self.reconnect_s > 0 and self.alive and self._reconnect():
                    continue
                self.alive = False
                with self._conn_cv:
                    self._conn_cv.notify_all()
                with self.refs.cv:
                    self.refs.cv.notify_all()
                for f in list(self.pending.values()):
                    if not f.done():
                        f.set_exception(ConnectionError("connection to the head was lost"))
                self.task_queue.put(None)
                return
            t = msg[0]
            if t == "reply":
                f = self.pending.get(msg[1])
                if f is not None and not f.done():
                    f.set_result(msg[2])
            elif t == "ready":
                self._on_ready(msg[1])
            elif t == "execute":
                self._on_execute(msg[1])
            elif t == "cancel":
                self._on_cancel(msg[1])
            elif t == "pub":
                for cb in list(self._subs.get(msg[1], ())):
                    try:
                        cb(msg[2], msg[3])
                    except Exception:
                        traceback.print_exc()
            elif t == "exit":
                self.task_queue.put(None)

    # ------------------------------------------------------------------ pubsub
    def subscribe(self, channel: str, callback):
        """``callback(key, info)`` for every state change the head publishes on
        ``channel`` ("actor": actor id -> state/name/pid/death cause; "node": node id
        -> ALIVE / DEAD). Runs in the reader thread: keep it short."""
        first = channel not in self._subs
        self._subs.setdefault(channel, []).append(callback)
        if first:
            self.send(("subscribe", channel))

    def unsubscribe(self, channel: str, callback):
        cbs = self._subs.get(channel, [])
        if callback in cbs:
            cbs.remove(callback)
        if not cbs and channel in self._subs:
            del self._subs[channel]
            self.send(("unsubscribe", channel))

    # ------------------------------------------------ head restart: re-attach
    def _reconnect(self) -> bool:
        """The head connection broke: reconnect to the (restarted) head at the same
        address, re-register with this process's live state and replay what was in
        flight. False if no head came back within ``reconnect_s``."""
        old = self.conn
        deadline = time.time() + self.reconnect_s
        while self.alive and time.time() < deadline:
            try:
                conn = connect(self.address)
            except OSError:
                time.sleep(0.2)
                continue
            try:
                conn.send(("reregister", self.kind, self.worker_id, os.getpid(), self.node_hex,
                           self._reattach_state()))
                msg = conn.recv()
            except (ConnectionClosed, OSError):
                conn.close()
                time.sleep(0.2)
                continue
            if msg[0] != "registered":
                conn.close()
                return False
            with self._conn_cv:
                self.conn = conn
                self.reattaches += 1
                self._conn_cv.notify_all()
            try:
                old.close()
            except Exception:
                pass
            try:
                for ch in list(self._subs):
                    self.send(("subscribe", ch))
                for req, build in sorted(self._req_builds.items()):
                    if req in self.pending:
                        self.send(build(req))
                for spec in list(self._head_specs.values()):
                    self.send(("submit", spec))
            except (ConnectionClosed, OSError):
                continue
            return True
        return False

    def _reattach_state(self) -> dict:
        gpus = [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]
        st = {"job_id": self.job_id, "gpu_ids": gpus, "actor_id": self.actor_id,
              "direct": self.direct_server.path if self.direct_server is not None else None}
        renv = os.environ.get("CAAMD_RUNTIME_ENV")
        if renv:  # the head keys its idle pools by runtime env: keep this worker in its own
            import json

            st["runtime_env"] = json.loads(renv)
        st["running"] = [(tid, self._running_res.get(tid) or {}) for tid in list(self._running_res)
                         if tid in self.running_tasks]
        st["finishing"] = list(self._unsent_done)
        r = self.refs
        refs, inline = {}, {}
        with r.lock:
            for oid, n in r.counts.items():
                if n <= 0:
                    continue
                refs[oid] = 1  # the head counts holders, not local references
                ent = r.ready.get(oid) or r.cache.get(oid)
                if ent is not None and ent[0] in ("inline", "err") and ent[1] is not None:
                    inline[oid] = (ent[1], ent[0] == "err")
                elif oid in r.local_only:
                    blob, _size, is_err = r.local_only[oid]
                    inline[oid] = (blob, is_err)
        st["refs"], st["inline"] = refs, inline
        if self.leases is not None:
            st["leases"] = [(lc.worker_id, dict(k.resources), {"strategy": k.strategy, "env": k.env})
                            for k in list(self.leases.keys.values()) for lc in list(k.leases) if lc.alive]
        return st

    def _track_head_spec(self, spec):
        if self.reconnect_s <= 0 or spec.generator is not None or spec.kind == ACTOR_CREATE:
            return
        self._head_specs[spec.task_id] = spec
        for o in spec.return_ids or ():
            self._ret_task[o] = spec.task_id

    def _on_ready(self, items):
        if self._ret_task:
            for (oid, _k, _p) in items:
                tid = self._ret_task.pop(oid, None)
                if tid is not None:
                    spec = self._head_specs.pop(tid, None)
                    for o in (spec.return_ids if spec is not None else ()) or ():
                        self._ret_task.pop(o, None)
        r = self.refs
        with r.cv:
            for (oid, kind, payload) in items:
                r.owned.discard(oid)
                if oid in r.counts:
                    r.ready[oid] = (kind, payload)
            r.cv.notify_all()
        if self._ready_cbs:
            for (oid, _k, _p) in items:
                for f in self._ready_cbs.pop(oid, None) or ():
                    f()
        if self.head_inflight_actor:
            with self._direct_lock:
                for (oid, _k, _p) in items:
                    aid = self.head_inflight_actor.pop(oid, None)
                    if aid is not None:
                        s_ = self.actor_head_inflight.get(aid)
                        if s_ is not None:
                            s_.discard(oid)

    # ------------------------------------------------------ direct actor calls
    def _direct_for(self, actor_id):
        """The actor's DirectClient, or None to use the head path (see core/direct.py)."""
        from .direct import DirectClient, addr_usable

        if actor_id in self.actor_head_only:
            return None  # killed, or a streaming call went through the head: stay there
        st = self.actor_direct.get(actor_id)
        if st is not None and not isinstance(st, tuple):
            if st.alive:
                return st
            st = None
        if self.actor_head_inflight.get(actor_id):
            return None
        now = time.monotonic()
        if st is not None and now - st[1] < 0.05:
            return None
        try:
            state, addr, node = self.request(lambda r: ("actor_addr", r, actor_id), timeout=30)
        except Exception:
            return None
        if state == "ALIVE" and node == self.node_hex and addr_usable(addr):
            try:
                dc = DirectClient(self, actor_id, addr)
            except OSError:
                dc = None
            if dc is not None:
                self.actor_direct[actor_id] = dc
                return dc
        self.actor_direct[actor_id] = ("head", now)
        return None

    def _handle_busy(self, oid: bytes) -> bool:
        """RefCounter hook (called under its lock): is ``oid`` an actor-handle ref
        whose actor still owes this process answers to direct calls?"""
        from .actor import HANDLE_SUFFIX

        if len(oid) <= len(HANDLE_SUFFIX) or not oid.endswith(HANDLE_SUFFIX):
            return False
        dc = self.actor_direct.get(oid[: -len(HANDLE_SUFFIX)])
        return dc is not None and not isinstance(dc, tuple) and bool(dc.pending)

    def _direct_drained(self, actor_id: bytes):
        """Every direct call to ``actor_id`` is answered (or resubmitted through the
        head): a handle decref held back for them may go now."""
        from .actor import handle_ref_id

        # no unlocked `if held_handles` shortcut: a remover that saw this actor busy may
        # be adding the handle right now, under the RefCounter lock; release_held_handle
        # takes that lock, so it runs after the add and finds the handle
        self.refs.release_held_handle(handle_ref_id(actor_id))

    def _to_head_path(self, actor_id, drop: bool = False):
        """Route this caller's later calls to ``actor_id`` through the head. Calls
        already sent on the direct connection finish first, so the caller's FIFO
        order holds across the switch (the head path cannot overtake them); with
        ``drop`` (ray.kill) the connection is closed instead of drained."""
        self.actor_head_only.add(actor_id)
        dc = self.actor_direct.get(actor_id)
        if dc is None or isinstance(dc, tuple):
            return
        if drop:
            self.actor_direct[actor_id] = ("head", 0.0)
            dc.close()
            return
        dc.wait_idle(timeout=float(os.environ.get("CAAMD_DIRECT_DRAIN_S", "600")))

    def _on_direct_done(self, spec, results, timing):
        from .direct import result_kinds

        r = self.refs
        lazy = bool(results) and all(res[1] is not None and not res[4] for res in results)
        if lazy:
            # all inline, nothing nested: the results stay owner-local until a ref
            # escapes (RefCounter.local_only); the head only gets the task events
            with r.cv:
                if r.must_seal and any(res[0] in r.must_seal for res in results):
                    lazy = False  # a ref already left this process: seal at the head
                else:
                    for (oid, inline, size, _n, _c, is_err) in results:
                        r.owned.discard(oid)
                        r.direct_pending.discard(oid)
                        if oid in r.direct_dropped:
                            r.direct_dropped.discard(oid)
                            continue
                        if oid in r.counts:
                            r.ready[oid] = ("err" if is_err else "inline", inline)
                            r.local_only[oid] = (inline, size, is_err)
                    r.cv.notify_all()
                    r.dseal_buf.append((spec.task_id, spec.fn_name, [], (), timing))
                    if len(r.dseal_buf) >= 512:
                        self._flush_evt.set()
            if lazy:
                if self._ready_cbs:
                    for res in results:
                        for f in self._ready_cbs.pop(res[0], None) or ():
                            f()
                return
        kinds = result_kinds(results, self.node_hex)
        with r.cv:
            for (oid, kind, payload) in kinds:
                if kind is None:
                    continue  # resolved through the head once sealed
                r.owned.discard(oid)
                if oid in r.counts:
                    r.ready[oid] = (kind, payload)
            r.cv.notify_all()
            # registered with the head in batches by the flush thread (_flush_dseals)
            r.dseal_buf.append((spec.task_id, spec.fn_name, results, spec.return_ids, timing))
            if len(r.dseal_buf) >= 512:
                self._flush_evt.set()
        if self._ready_cbs:
            for (oid, kind, _p) in kinds:
                if kind is not None:
                    for f in self._ready_cbs.pop(oid, None) or ():
                        f()

    def _on_direct_lost(self, actor_id, specs):
        """The actor's direct connection broke: resubmit through the head when the
        call may be retried, else fail it with ActorDiedError."""
        from ..exceptions import ActorDiedError

        self.actor_direct[actor_id] = ("head", 0.0)
        for spec in specs:
            if spec.max_retries:
                with self._direct_lock:
                    self.actor_head_inflight.setdefault(actor_id, set()).update(spec.return_ids)
                    for o in spec.return_ids:
                        self.head_inflight_actor[o] = actor_id
                self._resubmit_via_head(spec)
                continue
            self._fail_direct(spec, ActorDiedError(actor_id.hex(),
                                                   "the actor's worker died while the call was running"))

    def _resubmit_via_head(self, spec):
        """A direct call / leased task goes (back) through the head: its return refs
        stop being direct-pending; ones dropped meanwhile are released after it."""
        r = self.refs
        with r.cv:
            dropped = [o for o in spec.return_ids if o in r.direct_dropped]
            for o in spec.return_ids:
                r.direct_pending.discard(o)
                r.direct_dropped.discard(o)
        try:
            if r.local_only or r.direct_pending:
                self._escape(spec.arg_refs)
            self.send(("submit", spec))
            if dropped:
                self.send(("decref", dropped))
        except (ConnectionClosed, OSError):
            pass

    def _submit_via_head(self, spec, keep):
        self._resubmit_via_head(spec)
        del keep

    def _fail_direct(self, spec, exc):
        blob = serialization.serialize(exc).to_bytes()
        results = [(o, blob, len(blob), None, (), True) for o in spec.return_ids]
        now = time.time()
        self._on_direct_done(spec, results, (now, now, None))

    def _local_state(self, ids):
        """None if some id is neither pushed nor owned-pending here (ask the head);
        else the list of ids already pushed."""
        r = self.refs
        ready = r.ready
        owned = r.owned
        out = []
        for i in ids:
            if i in ready:
                out.append(i)
            elif i not in owned:
                return None
        return out

    def _wait_local(self, ids, need, timeout):
        """Block until ``need`` of ``ids`` (all owned by this process) are pushed."""
        r = self.refs
        deadline = None if timeout is None else time.monotonic() + timeout
        with r.cv:
            rd = r.ready
            waiting = [i for i in ids if i not in rd]
            n_ready = len(ids) - len(waiting)
            while True:
                if waiting:
                    still = [i for i in waiting if i not in rd]
                    n_ready += len(waiting) - len(still)
                    waiting = still
                if n_ready >= need or not self.alive:
                    return [i for i in ids if i in rd]
                owned = r.owned
                if any(i not in owned and i not in rd for i in waiting):
                    return None  # a ref was dropped meanwhile: fall back to the head
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return [i for i in ids if i in rd]
                r.cv.wait(left if left is not None else 1.0)

    def close(self):
        self.alive = False
        if self.direct_server is not None:
            self.direct_server.close()
        if self.leases is not None:
            self.leases.close()
        for dc in list(self.actor_direct.values()):
            if dc is not None and not isinstance(dc, tuple):
                try:
                    dc.close()
                except Exception:
                    pass
        try:
            with self.send_lock:
                ops = self.refs.drain()
                if ops:
                    self.conn.send_many(ops)
        except Exception:
            pass
        self.conn.close()

    # ------------------------------------------------------------- objects
    def _store(self, oid: bytes, so) -> tuple:
        """-> (inline_bytes | None, size, node_hex | None)."""
        size = so.total_bytes
        if size <= INLINE_MAX:
            return so.to_bytes(), size, None
        off = self.store.create(oid, size, 0)
        if off == -1:
            self.request(lambda r: ("evict", r, size))
            off = self.store.create(oid, size, 0)
        if off < 0:
            from ..exceptions import ObjectStoreFullError

            raise ObjectStoreFullError(
                f"object of {size} bytes does not fit in the object store "
                f"(capacity {self.store.capacity}, used {self.store.used})")
        so.write_into(self.store.buffer(off, size, False),
                      lambda o, b: self.store.copy_in(off + o, b, _COPY_THREADS))
        self.store.seal(oid)
        return None, size, self.node_hex

    def put(self, value, _owner_ref=True, tensor_transport=None) -> ObjectRef:
        if isinstance(value, ObjectRef):
            raise TypeError("Calling put() on an ObjectRef is not allowed")
        so = serialization.serialize(value, tensor_transport)
        oid = ObjectID.for_put(self.worker_id)
        inline, size, node = self._store(oid, so)
        self.send(("put", oid, inline, size, node, so.contained_refs, False))
        ref = ObjectRef(oid, _owned=True)
        self.refs.cache[bytes(oid)] = ("inline", inline) if inline is not None else ("store", None)
        return ref

    def _materialize(self, oid, kind, payload):
        from ..exceptions import ObjectLostError

        if kind == "inline":
            return serialization.deserialize(payload)
        if kind == "store":
            pb = self.store.get_pinned(oid)
            if pb is None:
                raise ObjectLostError(oid.hex(), "object is not in the local object store")
            return serialization.deserialize(memoryview(pb))
        if kind in ("remote", "err_remote"):
            from .object_server import pull

            try:
                data = pull(payload[0], oid)
            except OSError as e:
                raise ObjectLostError(oid.hex(), f"object's node {payload[0]} is unreachable: {e}")
            if data is None:
                raise ObjectLostError(oid.hex(), f"object is gone from its node ({payload[0]})")
            if kind == "remote":
                return serialization.deserialize(memoryview(data))
            raise _as_raisable(serialization.deserialize(memoryview(data)))
        if kind in ("err", "err_store"):
            if kind == "err":
                err = serialization.deserialize(payload)
            else:
                err = serialization.deserialize(memoryview(self.store.get_pinned(oid)))
            raise _as_raisable(err)
        if kind == "lost":
            raise ObjectLostError(oid.hex())
        raise RuntimeError(kind)

    def get(self, refs, timeout=None):
        from ..exceptions import GetTimeoutError

        single = isinstance(refs, ObjectRef)
        if single:
            refs = [refs]
        for r in refs:
            if not isinstance(r, ObjectRef):
                raise TypeError(f"get() expects ObjectRefs, got {type(r).__name__}")
        ids = [r._id for r in refs]
        out = self._get_cached(ids)
        if out is not None:
            return out[0] if single else out
        st = self._local_state(ids)
        if st is not None:
            blocked = self._maybe_blocked(True) if len(st) < len(ids) else False
            try:
                got = self._wait_local(ids, len(ids), timeout) if len(st) < len(ids) else st
            finally:
                if blocked:
                    self._maybe_blocked(False)
            if got is not None and len(got) == len(ids):
                ready = self.refs.ready
                res = [(o, *ready[o]) for o in ids if o in ready]
                # remote copies go through the head, which knows whether their node is alive
                if len(res) == len(ids) and all(k in ("inline", "store", "err", "err_store") for _, k, _ in res):
                    cache, counts = self.refs.cache, self.refs.counts
                    for (o, k, p) in res:
                        if k in ("inline", "store") and o in counts:
                            cache[o] = (k, p)
                    out = [self._materialize_or_recover(o, k, p, timeout) for (o, k, p) in res]
                    return out[0] if single else out
            elif got is not None and timeout is not None:
                from ..exceptions import GetTimeoutError

                raise GetTimeoutError(f"get() timed out after {timeout}s")
        if self.refs.local_only or self.refs.direct_pending:
            self._escape(ids)
        blocked = self._maybe_blocked(True)
        try:
            res = self.request(lambda req: ("get", req, ids, timeout))
        finally:
            if blocked:
                self._maybe_blocked(False)
        if res is None:
            raise GetTimeoutError(f"get() timed out after {timeout}s")
        cache, counts = self.refs.cache, self.refs.counts
        for (o, k, p) in res:
            if k in ("inline", "store") and o in counts:
                cache[o] = (k, p)
        out = [self._materialize_or_recover(o, k, p, timeout) for (o, k, p) in res]
        return out[0] if single else out

    def _materialize_or_recover(self, oid, kind, payload, timeout, attempts=3):
        """Materialize; when the copy's node vanished, ask the head to re-execute the
        object's lineage and wait for the new copy (reference: object recovery)."""
        from ..exceptions import ObjectLostError

        while True:
            try:
                return self._materialize(oid, kind, payload)
            except ObjectLostError:
                if attempts <= 0:
                    raise
                if kind in ("store", "err_store"):
                    # evicted (spilled) between the head's reply and our mapping:
                    # ask again, the head restores it
                    attempts -= 1
                    self.refs.cache.pop(oid, None)
                    res = self.request(lambda req: ("get", req, [oid], timeout))
                    if res is None:
                        from ..exceptions import GetTimeoutError

                        raise GetTimeoutError(f"get() timed out after {timeout}s")
                    _o, kind, payload = res[0]
                    continue
                if kind not in ("remote", "err_remote", "lost"):
                    raise
                attempts -= 1
                if not self.request(lambda req: ("report_lost", req, oid)):
                    raise
                self.refs.cache.pop(oid, None)
                res = self.request(lambda req: ("get", req, [oid], timeout))
                if res is None:
                    from ..exceptions import GetTimeoutError

                    raise GetTimeoutError(f"get() timed out after {timeout}s")
                _o, kind, payload = res[0]

    def _get_cached(self, ids):
        cache = self.refs.cache
        ent = [cache.get(i) for i in ids]
        if any(e is None for e in ent):
            return None
        out = []
        for i, (k, p) in zip(ids, ent):
            if k == "store":
                pb = self.store.get_pinned(i)
                if pb is None:  # spilled / evicted since: ask the head
                    cache.pop(i, None)
                    return None
                out.append(serialization.deserialize(memoryview(pb)))
            else:
                out.append(serialization.deserialize(p))
        return out

    def get_future(self, ref: ObjectRef) -> concurrent.futures.Future:
        out = concurrent.futures.Future()
        oid = ref.binary()
        r = self.refs

        def local(_keep=ref):  # the closure keeps the ref (and so its result) alive
            try:
                k, p = r.ready[oid]
                out.set_result(self._materialize(oid, k, p))
            except BaseException as e:  # noqa
                out.set_exception(e)

        with r.cv:
            ent = r.ready.get(oid)
            pending_here = ent is None and oid in r.owned
            if pending_here:  # completes here (owner-side store): no head round trip
                self._ready_cbs.setdefault(oid, []).append(local)
        if ent is not None and ent[0] in ("inline", "store", "err", "err_store"):
            local()
            return out
        if pending_here:
            return out
        if r.local_only or r.direct_pending:
            self._escape([oid])
        inner = self.request_async(lambda req: ("get", req, [oid], None))

        def done(f):
            try:
                res = f.result()
                o, k, p = res[0]
                out.set_result(self._materialize(o, k, p))
            except BaseException as e:
                out.set_exception(e)

        inner.add_done_callback(done)
        return out

    def wait(self, refs, num_returns=1, timeout=None, fetch_local=True):
        ids = list(map(_ref_id, refs))
        if len(set(ids)) != len(ids):
            raise ValueError("wait() requires a list of unique object refs")
        if num_returns > len(ids):
            raise ValueError("num_returns cannot exceed the number of refs")
        # fast path: enough of them already completed here (owner-side store);
        # stops scanning at the num_returns-th ready ref
        rd = self.refs.ready
        if num_returns == 1:
            for idx, i in enumerate(ids):
                if i in rd:
                    refs = list(refs)
                    return [refs[idx]], refs[:idx] + refs[idx + 1:]
        else:
            got = []
            for i in ids:
                if i in rd:
                    got.append(i)
                    if len(got) >= num_returns:
                        gs = set(got)
                        return [x for x in refs if x._id in gs], [x for x in refs if x._id not in gs]
        st = self._local_state(ids)
        if st is not None:
            got = st if (len(st) >= num_returns or timeout == 0) else None
            if got is None:
                blocked = self._maybe_blocked(True)
                try:
                    got = self._wait_local(ids, num_returns, timeout)
                finally:
                    if blocked:
                        self._maybe_blocked(False)
            if got is not None:
                ready = set(got[:num_returns]) if len(got) >= num_returns else set(got)
                return [x for x in refs if x.binary() in ready], [x for x in refs if x.binary() not in ready]
        if self.refs.local_only or self.refs.direct_pending:
            self._escape(ids)
        blocked = self._maybe_blocked(True)
        try:
            ready = set(self.request(lambda req: ("wait", req, ids, num_returns, timeout)))
        finally:
            if blocked:
                self._maybe_blocked(False)
        r = [x for x in refs if x.binary() in ready]
        nr = [x for x in refs if x.binary() not in ready]
        return r, nr

    def _maybe_blocked(self, on: bool) -> bool:
        ctx = context.current_task()
        if self.kind != "worker" or ctx is None or ctx.actor_id is not None:
            return False
        if on:
            self._n_blocked += 1
            # a leased worker must not sit on tasks queued behind a blocked one: one of
            # them may be what unblocks it (their owners re-dispatch them elsewhere)
            self._return_unstarted_leased()
        else:
            self._n_blocked = max(0, self._n_blocked - 1)
        self.send(("blocked" if on else "unblocked", ctx.task_id))
        return True

    def _return_unstarted_leased(self, exclude: Optional[bytes] = None) -> int:
        """Hand queued-but-unstarted leased normal tasks back to their owners
        (``dreturn``): the owner re-queues them without counting an attempt."""
        q = self.task_queue
        back = []
        with q.mutex:
            keep = []
            for item in q.queue:
                if (item is not None and item[0].kind == NORMAL and item[0].task_id != exclude
                        and item[0].task_id in self.direct_origin):
                    back.append(item[0].task_id)
                else:
                    keep.append(item)
            if back:
                q.queue.clear()
                q.queue.extend(keep)
        for tid in back:
            out = self.direct_origin.pop(tid, None)
            if out is not None:
                try:
                    out.put(("dreturn", tid))
                except (ConnectionClosed, OSError):
                    pass
        return len(back)

    def free(self, refs):
        self.send(("free", [r.binary() for r in refs]))

    def cancel(self, task_id: bytes, force: bool, recursive: bool):
        if self.leases is not None and self.leases.cancel(task_id, force):
            return
        self.send(("cancel", task_id, force, recursive))

    def gen_next(self, task_id, index):
        return self.request(lambda req: ("gen_next", req, task_id, index))

    # ------------------------------------------------------------- submission
    def register_function(self, fn_id: bytes, blob_fn):
        if fn_id not in self.sent_fns:
            blob = blob_fn()
            self.fn_blobs[fn_id] = blob
            self.send(("fn", fn_id, blob))
            self.sent_fns.add(fn_id)

    def _pack_args(self, args, kwargs):
        arg_refs, pinned = [], []
        keep = []

        def pack(v):
            if isinstance(v, ObjectRef):
                arg_refs.append(v.binary())
                keep.append(v)
                return ("r", v.binary())
            so = serialization.serialize(v)
            pinned.extend(so.contained_refs)
            if so.total_bytes > INLINE_MAX:
                ref = self.put(v)
                keep.append(ref)
                arg_refs.append(ref.binary())
                return ("r", ref.binary())
            return ("v", so.to_bytes())

        pa = [pack(a) for a in args]
        pk = {k: pack(v) for k, v in kwargs.items()}
        return pa, pk, arg_refs, pinned, keep

    def submit(self, kind, fn_id, fn_name, args, kwargs, num_returns=1, resources=None,
               strategy=None, max_retries=0, retry_exceptions=False, actor_id=None, method=None,
               actor_opts=None, runtime_env=None, name=None, concurrency_group=None, gen_bp=None):
        task_id = os.urandom(16)
        pa, pk, arg_refs, pinned, keep = self._pack_args(args, kwargs)
        generator = None
        if num_returns == "streaming":
            generator = "streaming"
            return_ids = []
        elif num_returns == "dynamic":
            generator = "dynamic"
            return_ids = [ObjectID.for_task_return(task_id, 0)]
        else:
            return_ids = [ObjectID.for_task_return(task_id, i) for i in range(int(num_returns))]
        ctx = context.current_task()
        spec = TaskSpec(task_id=task_id, kind=kind, fn_id=fn_id, fn_name=fn_name, args=pa,
                        kwargs=pk, arg_refs=arg_refs, pinned_refs=pinned, num_returns=num_returns,
                        return_ids=return_ids, resources=resources or {}, strategy=strategy,
                        max_retries=max_retries, retry_exceptions=retry_exceptions,
                        actor_id=actor_id, method=method, actor_opts=actor_opts,
                        runtime_env=runtime_env, name=name, job_id=self.job_id,
                        generator=generator, parent=ctx.task_id if ctx else None,
                        concurrency_group=concurrency_group,
                        gen_bp=int(gen_bp) if gen_bp and generator == "streaming" else None)
        refs = [] if generator == "streaming" else [ObjectRef(o, _owned=True) for o in return_ids]
        r = self.refs
        busy = bool(r.owned)
        if generator is None:
            with r.lock:
                r.owned.update(return_ids)
        if kind == NORMAL and self.leases is not None and generator is None:
            from .lease import eligible, resolved_args

            resolved = resolved_args(r, arg_refs) if arg_refs else {}
            if resolved is not None and eligible(spec):
                with r.lock:
                    r.direct_pending.update(return_ids)
                if self.leases.submit(spec, (keep, [ObjectRef(o) for o in arg_refs + pinned]), resolved, busy):
                    return refs
                with r.lock:
                    r.direct_pending.difference_update(return_ids)
        elif kind == ACTOR_METHOD:
            if generator is not None:
                self._to_head_path(actor_id)
            elif self.actor_direct is not None:
                dc = self._direct_for(actor_id)
                if dc is not None:
                    resolved = None
                    if arg_refs:
                        from .lease import resolved_args

                        resolved = resolved_args(r, arg_refs)
                        if resolved is None and (r.local_only or r.direct_pending):
                            self._escape(arg_refs)  # the actor resolves them through the head
                    with r.lock:
                        r.direct_pending.update(return_ids)
                    if dc.submit(spec, (keep, [ObjectRef(o) for o in arg_refs]), resolved):
                        return refs
                    with r.lock:
                        r.direct_pending.difference_update(return_ids)
            with self._direct_lock:
                self.actor_head_inflight.setdefault(actor_id, set()).update(return_ids)
                for o in return_ids:
                    self.head_inflight_actor[o] = actor_id
        if arg_refs and (r.local_only or r.direct_pending):
            self._escape(arg_refs)
        self._track_head_spec(spec)
        self.send(("submit", spec))
        del keep
        if generator == "streaming":
            return ObjectRefGenerator(task_id)
        return refs

    # ------------------------------------------------------------- execution
    def _on_execute(self, payload):
        spec, fn_blob, resolved = payload
        if fn_blob is not None and spec.fn_id not in self.fn_cache:
            self.fn_cache[spec.fn_id] = serialization.loads_function(fn_blob)
        if spec.kind == ACTOR_METHOD and self.actor_instance is not None:
            if self.async_loop is not None:
                asyncio.run_coroutine_threadsafe(self._run_async(payload), self.async_loop)
                return
            if self.thread_pool is not None:
                self.thread_pool.submit(self.execute, payload)
                return
        self.task_queue.put(payload)

    def _on_cancel(self, task_id):
        self.cancelled_tasks.add(task_id)
        t = self.running_tasks.get(task_id)
        if isinstance(t, threading.Thread):
            ctypes.pythonapi.PyThreadState_SetAsyncExc(ctypes.c_ulong(t.ident), ctypes.py_object(_Cancelled))
        elif t is not None and hasattr(t, "cancel"):
            self.async_loop.call_soon_threadsafe(t.cancel)

    def _resolve_args(self, spec, resolved):
        if resolved is None:
            resolved = {}
        # a direct call / leased task: ref arguments the caller did not send resolved
        ids = [a[1] for a in list(spec.args) + list(spec.kwargs.values()) if a[0] != "v" and a[1] not in resolved]
        if ids:
            res = self.request(lambda req: ("get", req, ids, None))
            resolved = dict(resolved)
            resolved.update({o: (k, p) for (o, k, p) in res})

        def unpack(a):
            if a[0] == "v":
                return serialization.deserialize(a[1])
            kind, payload = resolved[a[1]]
            return self._materialize_or_recover(a[1], kind, payload, None)

        args = [unpack(a) for a in spec.args]
        kwargs = {k: unpack(v) for k, v in spec.kwargs.items()}
        return args, kwargs

    def _function(self, spec):
        fn = self.fn_cache.get(spec.fn_id)
        if fn is None:
            blob = self.request(lambda r: ("fetch_fn", r, spec.fn_id))
            fn = serialization.loads_function(blob)
            self.fn_cache[spec.fn_id] = fn
        return fn

    def _set_ctx(self, spec):
        gpu_env = os.environ.get("CAAMD_GPU_IDS", "")
        context.set_current_task(context.TaskContext(
            task_id=spec.task_id, actor_id=self.actor_id if spec.kind != NORMAL else None,
            fn_name=spec.fn_name, attempt=spec.attempt,
            gpu_ids=[int(g) for g in gpu_env.split(",") if g != ""],
            resources=spec.resources, pg=spec.strategy if spec.strategy and spec.strategy[0] == "pg" else None,
        ))

    def execute(self, payload):
        spec, _, resolved = payload
        if spec.task_id in self.direct_origin:
            self.__dict__.setdefault("_t_start", {})[spec.task_id] = time.time()
        elif spec.kind == NORMAL and self.reconnect_s > 0:
            self._running_res[spec.task_id] = dict(spec.resources or {})
        self.running_tasks[spec.task_id] = threading.current_thread()
        self._set_ctx(spec)
        error_kind, retryable = None, False
        try:
            if spec.task_id in self.cancelled_tasks:
                raise _Cancelled()
            try:
                args, kwargs = self._resolve_args(spec, resolved)
            except Exception as dep_err:
                from ..exceptions import RayError

                if isinstance(dep_err, RayError):
                    # a failed dependency: propagate the ORIGINAL error unchanged
                    results = self._error_results(spec, dep_err, raw=True)
                    self.running_tasks.pop(spec.task_id, None)
                    self._reply_done(spec, results, "dep", False)
                    context.set_current_task(None)
                    return
                raise
            if spec.kind == ACTOR_CREATE:
                cls = self._function(spec)
                self.actor_id = spec.actor_id
                self.actor_opts = spec.actor_opts or {}
                context.actor_pg = spec.strategy if spec.strategy and spec.strategy[0] == "pg" else None
                context.current_task().actor_id = spec.actor_id
                self.actor_instance = cls(*args, **kwargs)
                self._setup_actor_concurrency(cls)
                result = None
            elif spec.kind == ACTOR_METHOD:
                if self.actor_instance is None:
                    raise RuntimeError("actor is not initialised")
                if spec.method == "__ray_terminate__":
                    self._exit_actor_after = True
                    result = None
                else:
                    result = getattr(self.actor_instance, spec.method)(*args, **kwargs)
            else:
                result = self._function(spec)(*args, **kwargs)
            results = self._package_results(spec, result)
        except _Cancelled:
            from ..exceptions import TaskCancelledError

            results = self._error_results(spec, TaskCancelledError(spec.task_id.hex()), raw=True)
            error_kind = "cancel"
        except SystemExit as e:
            if getattr(e, "_caamd_exit_actor", False):
                results = self._package_results(spec, None)
                self._reply_done(spec, results, None, False)
                self.running_tasks.pop(spec.task_id, None)
                self.send(("actor_exit", self.actor_id))
                self._hard_exit()
            results = self._error_results(spec, e)
            error_kind = "app"
        except BaseException as e:  # noqa
            results = self._error_results(spec, e)
            error_kind = "app"
            retryable = _retryable(spec.retry_exceptions, e)
        self.running_tasks.pop(spec.task_id, None)
        if spec.task_id in self.cancelled_tasks and error_kind is None:
            from ..exceptions import TaskCancelledError

            results = self._error_results(spec, TaskCancelledError(spec.task_id.hex()), raw=True)
            error_kind = "cancel"
        self.cancelled_tasks.discard(spec.task_id)
        self._reply_done(spec, results, error_kind, retryable)
        context.set_current_task(None)
        if getattr(self, "_exit_actor_after", False):
            try:  # an intentional exit: the head must not restart the actor
                self.send(("actor_exit", self.actor_id))
            except (ConnectionClosed, OSError):
                pass
            self._hard_exit()

    def _hard_exit(self):
        try:
            self.close()
        finally:
            os._exit(0)

    def _reply_done(self, spec, results, error_kind, retryable):
        dc = self.direct_origin.pop(spec.task_id, None)
        if dc is not None:
            nested = [r for res in results for r in (res[4] or ())]
            try:
                if nested:  # keep nested refs alive until the caller seals the results
                    self.send(("dpin", spec.task_id, nested))
                t0 = getattr(self, "_t_start", {}).pop(spec.task_id, time.time())
                dc.put(("ddone", spec.task_id, results, error_kind, t0, time.time(), os.getpid(), retryable))
            except (ConnectionClosed, OSError):
                pass
            return
        self._unsent_done.add(spec.task_id)  # reported on re-attach while this send waits
        try:
            self.send(("task_done", spec.task_id, results, error_kind, retryable))
        except ConnectionClosed:
            pass
        finally:
            self._unsent_done.discard(spec.task_id)
            self._running_res.pop(spec.task_id, None)

    def _setup_actor_concurrency(self, cls):
        is_async = any(inspect.iscoroutinefunction(m) or inspect.isasyncgenfunction(m)
                       for _, m in inspect.getmembers(cls, predicate=inspect.isfunction))
        mc = self.actor_opts.get("max_concurrency")
        if is_async:
            self.async_loop = asyncio.new_event_loop()
            self._async_sem = None
            limit = mc or 1000
            th = threading.Thread(target=self._run_loop, args=(limit,), daemon=True)
            th.start()
        elif mc and mc > 1:
            self.thread_pool = concurrent.futures.ThreadPoolExecutor(mc)

    def _run_loop(self, limit):
        asyncio.set_event_loop(self.async_loop)
        self._async_sem = asyncio.Semaphore(limit)
        self.async_loop.run_forever()

    async def _run_async(self, payload):
        spec, _, resolved = payload
        while self._async_sem is None:
            await asyncio.sleep(0.001)
        async with self._async_sem:
            self._set_ctx(spec)
            error_kind, retryable = None, False
            task = asyncio.current_task()
            self.running_tasks[spec.task_id] = task
            try:
                args, kwargs = self._resolve_args(spec, resolved)
                m = getattr(self.actor_instance, spec.method)
                if inspect.isasyncgenfunction(m) and spec.generator == "streaming":
                    # stream items to the owner as they are produced
                    i = 0
                    try:
                        async for x in m(*args, **kwargs):
                            self._stream_item(spec, i, x)
                            i += 1
                    except asyncio.CancelledError:
                        raise
                    except BaseException as e:  # noqa
                        self._stream_error(spec, i, e)
                    result = iter(())
                elif inspect.isasyncgenfunction(m):
                    items = []
                    async for x in m(*args, **kwargs):
                        items.append(x)
                    result = items
                    if spec.generator is not None:
                        result = iter(items)
                else:
                    result = m(*args, **kwargs)
                    if inspect.isawaitable(result):
                        result = await result
                results = self._package_results(spec, result)
            except asyncio.CancelledError:
                from ..exceptions import TaskCancelledError

                results = self._error_results(spec, TaskCancelledError(spec.task_id.hex()), raw=True)
                error_kind = "cancel"
            except SystemExit as e:
                if getattr(e, "_caamd_exit_actor", False):
                    self._reply_done(spec, self._package_results(spec, None), None, False)
                    self.send(("actor_exit", self.actor_id))
                    self._hard_exit()
                results = self._error_results(spec, e)
                error_kind = "app"
            except BaseException as e:  # noqa
                results = self._error_results(spec, e)
                error_kind = "app"
                retryable = _retryable(spec.retry_exceptions, e)
            self.running_tasks.pop(spec.task_id, None)
            self._reply_done(spec, results, error_kind, retryable)

    def _package_results(self, spec, result):
        if spec.generator == "streaming":
            return self._stream(spec, result)
        if spec.generator == "dynamic":
            refs = []
            for i, item in enumerate(result):
                oid = ObjectID.for_task_return(spec.task_id, i + 1)
                so = serialization.serialize(item)
                inline, size, node = self._store(oid, so)
                self.send(("put", oid, inline, size, node, so.contained_refs, False))
                refs.append(ObjectRef(oid, _owned=True))
            result = DynamicObjectRefGenerator(refs)
            return [self._result_entry(spec.return_ids[0], result)]
        n = spec.num_returns
        tt = None
        if spec.kind == ACTOR_METHOD and self.actor_instance is not None:
            tt = getattr(getattr(type(self.actor_instance), spec.method, None), "__ray_tensor_transport__", None)
        if n == 1 and type(result).__name__ == "TransportResult":
            from .actor import TransportResult

            if isinstance(result, TransportResult):  # the method chose its transport for this call
                tt, result = result.transport or tt, result.value
        if n == 1:
            return [self._result_entry(spec.return_ids[0], result, tt)]
        if n == 0:
            return []
        vals = tuple(result) if result is not None else None
        if vals is None or len(vals) != n:
            raise ValueError(f"task declared num_returns={n} but returned {result!r}")
        return [self._result_entry(o, v, tt) for o, v in zip(spec.return_ids, vals)]

    def _stream_item(self, spec, i, item):
        oid = ObjectID.for_task_return(spec.task_id, i)
        so = serialization.serialize(item)
        inline, size, node = self._store(oid, so)
        self.send(("gen_item", spec.task_id, i, oid, inline, size, node, so.contained_refs, False))

    def _stream_error(self, spec, i, e):
        from ..exceptions import RayTaskError

        err = RayTaskError.from_exception(spec.fn_name, e)
        oid = ObjectID.for_task_return(spec.task_id, i)
        blob = serialization.serialize(err).to_bytes()
        self.send(("gen_item", spec.task_id, i, oid, blob, len(blob), None, [], True))

    def _stream(self, spec, gen):
        i = 0
        bp = spec.gen_bp or 0
        consumed = 0
        try:
            it = iter(gen)
            while True:
                if bp > 0 and i - consumed >= bp:
                    # backpressure: the generator body does not run ahead of its
                    # consumer by more than bp items
                    consumed = self.request(lambda r, n=i - bp + 1: ("gen_wait", r, spec.task_id, n))
                try:
                    item = next(it)
                except StopIteration:
                    break
                self._stream_item(spec, i, item)
                i += 1
        except BaseException as e:  # noqa
            self._stream_error(spec, i, e)
        return []

    def _result_entry(self, oid, value, tensor_transport=None):
        so = serialization.serialize(value, tensor_transport)
        inline, size, node = self._store(oid, so)
        return (oid, inline, size, node, so.contained_refs, False)

    def _error_results(self, spec, exc, raw=False):
        from ..exceptions import RayTaskError

        err = exc if raw else RayTaskError.from_exception(
            f"{spec.fn_name}" + (f".{spec.method}" if spec.method else ""), exc)
        blob = serialization.serialize(err).to_bytes()
        ids = list(spec.return_ids or [])
        if spec.generator == "streaming":
            oid = ObjectID.for_task_return(spec.task_id, 0)
            self.send(("gen_item", spec.task_id, 0, oid, blob, len(blob), None, [], True))
            return []
        return [(oid, blob, len(blob), None, [], True) for oid in ids]

    # ------------------------------------------------------------- worker main
    def run_worker_loop(self):
        while True:
            item = self.task_queue.get()
            if item is None:
                break
            self.execute(item)


_ref_id = operator.attrgetter("_id")


def _retryable(retry_exceptions, e) -> bool:
    if retry_exceptions is True:
        return True
    if isinstance(retry_exceptions, (list, tuple)):
        return isinstance(e, tuple(retry_exceptions))
    return False


def _as_raisable(err):
    from ..exceptions import RayTaskError

    if isinstance(err, RayTaskError):
        return err.as_instanceof_cause()
    return err


def function_id(fn) -> bytes:
    name = f"{getattr(fn, '__module__', '')}.{getattr(fn, '__qualname__', repr(fn))}"
    try:
        src = inspect.getsource(fn)
    except Exception:
        src = ""
    return hashlib.blake2b((name + src + str(id(fn))).encode(), digest_size=16).digest()
