"""Normal-task worker leases: the submitting process pushes tasks straight to
leased workers; the head only grants and takes back leases.

Reference roles: ``src/ray/core_worker/transport/direct_task_transport.cc``
(``CoreWorkerDirectTaskSubmitter``: per-SchedulingKey backlog, RequestNewWorkerIfNeeded,
lease reuse, ReturnWorker) and the raylet's ``HandleRequestWorkerLease``.
Design for one MI355X node:

* a scheduling key is (resource shape, placement-group bundle, runtime env) — the
  reference's SchedulingKey; GPU tasks lease GPU-pinned workers (the GPU ids stay
  with the lease until it is returned), placement-group tasks lease against their
  bundle's resources on the owner's node, runtime-env tasks lease workers of that
  env's pool (node-affinity / SPREAD / label strategies keep the head path);
* the FIRST task of a key goes through the head as before (a synchronous
  ``get(f.remote())`` loop never pays for a lease); once the owner has tasks in
  flight, further tasks of that key queue locally and the owner asks the head for
  up to ``ceil(backlog / DEPTH)`` workers of its own node in one ``lease`` request;
  the head grants idle workers (spawning more up to its pool limit), parks the
  request FIFO when the node is full, answers ``spill`` when another node has
  room (those tasks then take the head path) and ``never`` when the node cannot
  run the shape at all;
* ONE event-loop thread per owner process (a selector over every leased
  worker's Unix socket) does all lease I/O: it takes submissions from a lock-free
  deque, keeps up to ``DEPTH`` tasks in flight per lease, writes each lease's
  tasks in one non-blocking send, reads completions and publishes them to the
  owner-side store in batches. Submitting costs a deque append (plus a pipe
  write when the loop sleeps); there is no per-connection thread and no lock
  shared with the submitting thread, so the GIL is handed over rarely;
* argument refs the owner already holds resolved travel with the task, the
  function blob travels once per connection;
* a lease goes back to the head after ``LINGER`` s without work, and a busy lease
  is drained and returned after ``SLICE`` s so that parked requests of other
  owners get their turn (the owner re-requests if its backlog remains);
* results come back to the owner (``CoreWorker._on_direct_done``): small inline
  results stay owner-local until their ref escapes the process (then they are
  sealed at the head, ``lseal``), larger ones are registered in batched seals;
* a retryable application error is resubmitted through the head; a lost worker
  fails its in-flight tasks with ``WorkerCrashedError`` / ``OutOfMemoryError``
  (the head says which) or resubmits them while retries remain; cancel goes
  straight to the worker (``force`` ends the worker process).
"""
from __future__ import annotations

import collections
import os
import pickle
import selectors
import socket
import struct
import threading
import time
from typing import Dict, List, Optional

from .head import NORMAL

DEPTH = int(os.environ.get("CAAMD_LEASE_DEPTH", "64"))
LINGER = float(os.environ.get("CAAMD_LEASE_LINGER_S", "0.02"))
SLICE = float(os.environ.get("CAAMD_LEASE_SLICE_S", "0.25"))
MAX_WANT = int(os.environ.get("CAAMD_LEASE_MAX_WANT", "16"))
# tasks that run longer than this (or not measured yet) go one at a time per lease, so a
# backlog of them asks for (and spreads over) as many workers as it can use instead
# of queueing behind one another on a few (reference: max_tasks_in_flight_per_worker=1);
# short ones keep DEEP pipelines that hide the owner<->worker round trip
LONG_TASK_S = float(os.environ.get("CAAMD_LEASE_LONG_TASK_S", "0.002"))
SHORT_DEPTH = 1
RETRY_S = 0.02
_LEN = struct.Struct("<Q")


def enabled() -> bool:
    return os.environ.get("CAAMD_TASK_LEASES", "1") == "1"


def eligible(spec) -> bool:
    if spec.kind != NORMAL or spec.generator is not None:
        return False
    return spec.strategy is None or spec.strategy[0] in ("default", "pg")


def _env_sig(renv):
    if not renv:
        return None
    try:
        import json

        return json.dumps(renv, sort_keys=True, default=str)
    except (TypeError, ValueError):
        return repr(sorted(renv.items()))


def scheduling_key(spec):
    st = spec.strategy if (spec.strategy is not None and spec.strategy[0] == "pg") else None
    return (tuple(sorted(spec.resources.items())), st, _env_sig(spec.runtime_env))


def _frame(msg) -> bytes:
    d = pickle.dumps(msg, protocol=5)
    return _LEN.pack(len(d)) + d


class _Key:
    __slots__ = ("resources", "strategy", "env", "queue", "leases", "requesting", "mode", "retry_at", "active",
                 "avg_run_s")

    def __init__(self, resources, strategy=None, env=None):
        self.resources = dict(resources)
        self.strategy = strategy  # ("pg", pg_id, bundle, ...) or None
        self.env = env  # runtime env dict or None
        self.queue: collections.deque = collections.deque()  # (spec, keep, resolved)
        self.leases: List["_Lease"] = []
        self.requesting = False
        self.mode = "lease"  # "never": this shape cannot run on our node (head path)
        self.retry_at = 0.0
        self.active = False  # leases / queue / request outstanding (read by submitters)
        self.avg_run_s: Optional[float] = None  # EWMA of the key's task run time (None: not seen yet)

    def depth(self) -> int:
        """Tasks in flight per lease: deep pipelines for short tasks (hide the
        round trip), shallow ones for long or not-yet-measured tasks (parallelism)."""
        a = self.avg_run_s
        return DEPTH if (a is not None and a < LONG_TASK_S) else min(DEPTH, SHORT_DEPTH)


class _Lease:
    __slots__ = ("worker_id", "sock", "key", "pending", "out", "sent_fns", "granted_at", "last_used",
                 "alive", "rbuf", "writing", "blocked")

    def __init__(self, worker_id, sock, key):
        self.worker_id = worker_id
        self.sock = sock
        self.key = key
        self.pending: Dict[bytes, tuple] = {}  # task_id -> (spec, keep, t_submit, resolved)
        self.out = bytearray()
        self.sent_fns = set()
        self.granted_at = self.last_used = time.monotonic()
        self.alive = True
        self.rbuf = bytearray()
        self.writing = False
        self.blocked = False  # its running task blocked in get(): no new tasks until it ends


class LeaseManager:
    def __init__(self, worker):
        self.w = worker
        self.keys: Dict[tuple, _Key] = {}
        self.inq: collections.deque = collections.deque()
        self.events: collections.deque = collections.deque()  # grants / cancels from other threads
        self.tasks = set()  # task ids submitted here and not finished (any thread may read)
        self.by_task: Dict[bytes, _Lease] = {}
        self.cancelled = set()
        self.n_leased_tasks = 0
        self.alive = True
        self.sleeping = False
        self._thread = None
        self._start_lock = threading.Lock()

    # ------------------------------------------------------------ any thread
    def _ensure_thread(self):
        with self._start_lock:
            if self._thread is not None:
                return
            self.sel = selectors.DefaultSelector()
            self.wake_r, self.wake_w = os.pipe()
            os.set_blocking(self.wake_r, False)
            os.set_blocking(self.wake_w, False)
            self.sel.register(self.wake_r, selectors.EVENT_READ, None)
            self._thread = threading.Thread(target=self._loop, name="caamd-leases", daemon=True)
            self._thread.start()

    def _wake(self):
        if self.sleeping:
            self.sleeping = False
            try:
                os.write(self.wake_w, b"x")
            except (BlockingIOError, OSError):
                pass

    def submit(self, spec, keep, resolved, busy: bool) -> bool:
        """Queue ``spec`` for a leased worker; False = use the head path."""
        key = scheduling_key(spec)
        st = self.keys.get(key)
        if st is None:
            st = self.keys.setdefault(key, _Key(spec.resources, key[1], spec.runtime_env or None))
        if st.mode == "never":
            return False
        if not st.active and not busy:
            return False  # a lone task: the head path costs one hop less than a lease
        if self._thread is None:
            self._ensure_thread()
        st.active = True
        self.tasks.add(spec.task_id)
        self.inq.append((st, spec, keep, resolved))
        self._wake()
        return True

    def cancel(self, task_id: bytes, force: bool) -> bool:
        """True if the task is ours (queued here or running on a leased worker)."""
        if task_id not in self.tasks:
            return False
        self.events.append(("cancel", task_id, force))
        self._wake()
        return True

    def _granted_cb(self, st, res):
        self.events.append(("grant", st, res))
        self._wake()

    def close(self):
        self.alive = False
        if self._thread is not None:
            self.sleeping = True
            self._wake()

    # ------------------------------------------------------------ loop thread
    def _loop(self):
        last_tick = 0.0
        while self.alive:
            done: List[tuple] = []
            inq = self.inq
            while inq:
                st, spec, keep, resolved = inq.popleft()
                st.queue.append((spec, keep, resolved))
            ev = self.events
            while ev:
                e = ev.popleft()
                if e[0] == "grant":
                    self._on_grant(e[1], e[2])
                else:
                    self._on_cancel(e[1], e[2])
            now = time.monotonic()
            for st in self.keys.values():
                if st.queue:
                    self._pump(st, now)
            if now - last_tick >= 0.004:
                last_tick = now
                self._tick(now)
            # sleep until a socket / the wake pipe is readable
            busy = any(st.leases or st.queue for st in self.keys.values())
            self.sleeping = True
            if self.inq or self.events:
                self.sleeping = False
                timeout = 0
            else:
                timeout = 0.005 if busy else 0.25
            try:
                ready = self.sel.select(timeout)
            except OSError:
                ready = []
            self.sleeping = False
            for skey, mask in ready:
                lc = skey.data
                if lc is None:
                    try:
                        os.read(self.wake_r, 4096)
                    except (BlockingIOError, OSError):
                        pass
                    continue
                if mask & selectors.EVENT_WRITE:
                    self._flush(lc)
                if mask & selectors.EVENT_READ:
                    self._read(lc, done)
            if done:
                now = time.monotonic()
                for st in {lc.key for (lc, *_r) in done}:
                    if st.queue:
                        self._pump(st, now)  # refill the pipelines before publishing results
                for (lc, spec, results, error_kind, retryable, timing) in done:
                    self._complete(spec, results, error_kind, retryable, timing)

    def _read(self, lc: _Lease, done):
        try:
            data = lc.sock.recv(1 << 18)
        except BlockingIOError:
            return
        except OSError:
            data = b""
        if not data:
            self._lost(lc)
            return
        buf = lc.rbuf
        buf += data
        off = 0
        n_buf = len(buf)
        returned = []
        while n_buf - off >= 8:
            (n,) = _LEN.unpack_from(buf, off)
            if n_buf - off - 8 < n:
                break
            msg = pickle.loads(bytes(buf[off + 8: off + 8 + n]))
            off += 8 + n
            if msg[0] == "dreturn":
                # not started: the worker's running task is blocked (see worker
                # _return_unstarted_leased); dispatch it elsewhere, no attempt spent
                rec = lc.pending.pop(msg[1], None)
                lc.blocked = True
                if rec is not None:
                    self.by_task.pop(msg[1], None)
                    returned.append(rec)
                continue
            if msg[0] != "ddone":
                continue
            task_id, results, error_kind, t0, t1, pid = msg[1:7]
            retryable = msg[7] if len(msg) > 7 else False
            try:
                run = max(0.0, float(t1) - float(t0))
                st = lc.key
                # a long run flips the key to long at once; short runs decay it back
                st.avg_run_s = run if (st.avg_run_s is None or run > st.avg_run_s) else 0.8 * st.avg_run_s + 0.2 * run
            except (TypeError, ValueError):
                pass
            rec = lc.pending.pop(task_id, None)
            lc.blocked = False
            if rec is None:
                continue
            self.by_task.pop(task_id, None)
            done.append((lc, rec[0], results, error_kind, retryable, (t0, t1, pid)))
        if off:
            del buf[:off]
        lc.last_used = time.monotonic()
        if returned:
            self._requeue(lc.key, returned)

    def _requeue(self, st: _Key, recs):
        from ..exceptions import TaskCancelledError

        for rec in sorted(recs, key=lambda r: r[2], reverse=True):  # oldest ends up first
            spec, keep, _t, resolved = rec
            if spec.task_id in self.cancelled:
                self.cancelled.discard(spec.task_id)
                self.tasks.discard(spec.task_id)
                self.w._fail_direct(spec, TaskCancelledError(spec.task_id.hex()))
                continue
            st.queue.appendleft((spec, keep, resolved))
        self._pump(st, time.monotonic())

    def _complete(self, spec, results, error_kind, retryable, timing):
        tid = spec.task_id
        cancelled = tid in self.cancelled
        self.cancelled.discard(tid)
        self.tasks.discard(tid)
        if (error_kind == "app" and retryable and not cancelled
                and spec.attempt < (spec.max_retries or 0)):
            spec.attempt += 1
            self.w._resubmit_via_head(spec)
            return
        self.w._on_direct_done(spec, results, timing)

    def _pump(self, st: _Key, now: float):
        q = st.queue
        live = [lc for lc in st.leases if lc.alive and not lc.blocked and now - lc.granted_at < SLICE]
        depth = st.depth()
        touched = []
        while q and live:
            lc = min(live, key=lambda x: len(x.pending))
            if len(lc.pending) >= depth:
                break
            spec, keep, resolved = q.popleft()
            fn_blob = None
            if spec.fn_id not in lc.sent_fns:
                fn_blob = self.w.fn_blobs.get(spec.fn_id)
                lc.sent_fns.add(spec.fn_id)
            lc.pending[spec.task_id] = (spec, keep, now, resolved)
            self.by_task[spec.task_id] = lc
            self.n_leased_tasks += 1
            lc.out += _frame(("dexec", spec, resolved, fn_blob))
            if not lc.writing and lc not in touched:
                touched.append(lc)
        for lc in touched:
            self._flush(lc)
        if q and not st.requesting and now >= st.retry_at:
            cap = sum(max(0, depth - len(lc.pending)) for lc in live)
            need = len(q) - cap
            if need > 0:
                st.requesting = True
                want = min(MAX_WANT, (need + depth - 1) // depth)
                opts = {"strategy": st.strategy, "env": st.env} if (st.strategy or st.env) else None
                self.w.request_cb(lambda r: ("lease", r, st.resources, want, opts),
                                  lambda res, st=st: self._granted_cb(st, res))
        st.active = bool(st.leases or st.queue or st.requesting)

    def _flush(self, lc: _Lease):
        if not lc.out or not lc.alive:
            return
        try:
            n = lc.sock.send(lc.out)
        except BlockingIOError:
            n = 0
        except OSError:
            self._lost(lc)
            return
        if n:
            del lc.out[:n]
        want_write = bool(lc.out)
        if want_write != lc.writing:
            lc.writing = want_write
            ev = selectors.EVENT_READ | (selectors.EVENT_WRITE if want_write else 0)
            try:
                self.sel.modify(lc.sock, ev, lc)
            except (KeyError, ValueError, OSError):
                pass

    def _on_grant(self, st: _Key, res):
        from .direct import addr_usable

        st.requesting = False
        if isinstance(res, list):
            for (wid, addr) in res:
                sock = None
                if addr_usable(addr):
                    try:
                        sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                        sock.connect(addr)
                        sock.setblocking(False)
                    except OSError:
                        sock = None
                if sock is None:
                    self.w.send(("lease_return", [wid]))
                    continue
                lc = _Lease(wid, sock, st)
                self.sel.register(sock, selectors.EVENT_READ, lc)
                st.leases.append(lc)
        else:
            if res == "never" or res is None:
                st.mode = "never"
            st.retry_at = time.monotonic() + RETRY_S
            if not st.leases:  # nobody here to run them: hand the backlog to the head
                while st.queue:
                    spec, keep, _resolved = st.queue.popleft()
                    self.tasks.discard(spec.task_id)
                    self.w._submit_via_head(spec, keep)
        st.active = bool(st.leases or st.queue or st.requesting)

    def _close_lease(self, lc: _Lease):
        lc.alive = False
        try:
            self.sel.unregister(lc.sock)
        except (KeyError, ValueError, OSError):
            pass
        try:
            lc.sock.close()
        except OSError:
            pass

    def _lost(self, lc: _Lease):
        from ..exceptions import OutOfMemoryError, TaskCancelledError, WorkerCrashedError

        if not lc.alive:
            return
        self._close_lease(lc)
        st = lc.key
        if lc in st.leases:
            st.leases.remove(lc)
        specs = [rec[0] for rec in sorted(lc.pending.values(), key=lambda r: r[2])]
        lc.pending.clear()
        fate = None
        for spec in specs:
            tid = spec.task_id
            self.by_task.pop(tid, None)
            mr = spec.max_retries if spec.max_retries is not None else 3
            if tid in self.cancelled:
                self.cancelled.discard(tid)
                self.tasks.discard(tid)
                self.w._fail_direct(spec, TaskCancelledError(tid.hex()))
            elif mr < 0 or spec.attempt < mr:
                spec.attempt += 1
                self.tasks.discard(tid)
                self.w._resubmit_via_head(spec)
            else:
                if fate is None:
                    try:
                        fate = self.w.request(lambda r: ("worker_fate", r, lc.worker_id), timeout=10)
                    except Exception:
                        fate = "crash"
                if fate == "oom":
                    err = OutOfMemoryError("Task was killed due to the node running low on memory; "
                                           "retries exhausted.")
                else:
                    err = WorkerCrashedError("the worker died while running the task")
                self.tasks.discard(tid)
                self.w._fail_direct(spec, err)
        st.active = bool(st.leases or st.queue or st.requesting)

    def _on_cancel(self, task_id: bytes, force: bool):
        from ..exceptions import TaskCancelledError

        lc = self.by_task.get(task_id)
        if lc is not None:
            self.cancelled.add(task_id)
            lc.out += _frame(("dcancel", task_id, force))
            self._flush(lc)
            return
        for st in self.keys.values():
            for ent in st.queue:
                if ent[0].task_id == task_id:
                    st.queue.remove(ent)
                    self.tasks.discard(task_id)
                    self.w._fail_direct(ent[0], TaskCancelledError(task_id.hex()))
                    return

    def _tick(self, now: float):
        """Return idle leases (and drained ones whose time slice is over)."""
        back = []
        for st in self.keys.values():
            for lc in list(st.leases):
                if lc.pending or lc.out:
                    continue
                if not lc.alive or now - lc.granted_at >= SLICE or (
                        not st.queue and now - lc.last_used >= LINGER):
                    st.leases.remove(lc)
                    back.append(lc)
            st.active = bool(st.leases or st.queue or st.requesting)
        if back:
            try:
                self.w.send(("lease_return", [lc.worker_id for lc in back]))
            finally:
                for lc in back:
                    self._close_lease(lc)


def resolved_args(refs, arg_refs) -> Optional[dict]:
    """Payloads of ``arg_refs`` this process already holds (a leased worker on
    the same node can materialize them without asking the head), or None if any
    is not resolved here yet."""
    out = {}
    ready, cache = refs.ready, refs.cache
    for o in arg_refs:
        ent = ready.get(o) or cache.get(o)
        if ent is None or ent[0] not in ("inline", "err", "store", "err_store"):
            return None
        out[o] = ent
    return out
