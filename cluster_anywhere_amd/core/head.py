"""The head: GCS tables + raylet scheduling loop + object directory + worker pool.

Reference roles: ``src/ray/gcs/gcs_server`` (actor / node / job / placement-group
tables, internal KV, health checks) and ``src/ray/raylet`` (NodeManager,
LocalTaskManager, WorkerPool, DependencyManager, WaitManager). Here they are one
single-threaded event loop (selectors) so all control state is mutated without
locks; resource accounting and placement are done by the native
``ClusterScheduler`` and object payloads live in the native shared-memory
``ObjectStore`` (workers read/write it directly; only small objects are inlined
in control messages).

The head runs as a thread inside the driver (``init()``) or as a standalone
process (``python -m cluster_anywhere_amd.core.head``) that drivers and other
nodes connect to over TCP.
"""
from __future__ import annotations

import collections
import itertools
import os
import selectors
import signal
import socket
import subprocess
import sys
import threading
import time
import traceback
from typing import Any, Dict, List, Optional, Set

from . import serialization
from .ids import ObjectID
from .protocol import Conn, ConnectionClosed

# cap on retained lineage (reference: RAY_max_lineage_bytes); beyond it objects
# created by further tasks are simply not recoverable
LINEAGE_MAX_TASKS = int(os.environ.get("CAAMD_LINEAGE_MAX_TASKS", "200000"))
INLINE_MAX = int(os.environ.get("CAAMD_INLINE_MAX", str(100 * 1024)))

# task kinds
NORMAL, ACTOR_CREATE, ACTOR_METHOD = 0, 1, 2
# object states
PENDING, READY, FREED = 0, 1, 2


def _node_labels(node_hex, gpu_ids, labels):
    """Labels of a node: user labels plus the built-in ones (reference:
    ray.io/node-id and ray.io/accelerator-type node labels)."""
    out = {"ray.io/node-id": node_hex}
    if gpu_ids:
        out["ray.io/accelerator-type"] = "AMD-Instinct-MI355X"
    out.update({str(k): str(v) for k, v in (labels or {}).items()})
    return out



# Environment variables read when an interpreter (or a library it imports at
# start-up: torch, OpenMP, MKL, the dynamic loader) starts. A worker forked from the
# zygote already runs with the zygote's values, so a runtime_env that sets any of
# them gets a fresh process.
_START_TIME_ENV = ("PYTHON", "LD_", "OMP_", "MKL_", "OPENBLAS_", "GOMP_", "KMP_", "MALLOC_", "TORCH_")


def _env_key(renv) -> Optional[str]:
    """Worker-pool key of a task's runtime env (None: the job's default workers).
    Tasks only reuse workers started with the same env (reference: worker_pool.cc
    keys idle workers by runtime-env hash)."""
    if not renv:
        return None
    import hashlib
    import json

    return hashlib.sha1(json.dumps(renv, sort_keys=True, default=str).encode()).hexdigest()[:16]


def _needs_fresh_interpreter(renv) -> bool:
    if not renv:
        return False
    if renv.get("pip") or renv.get("uv") or renv.get("conda") or renv.get("py_executable"):
        return True
    return any(k.startswith(_START_TIME_ENV) for k in (renv.get("env_vars") or {}))

class TaskSpec:
    """Everything the head needs to schedule, run, retry and report a task."""

    __slots__ = (
        "task_id", "kind", "fn_id", "fn_name", "args", "kwargs", "arg_refs", "num_returns",
        "return_ids", "resources", "strategy", "max_retries", "retry_exceptions", "owner",
        "actor_id", "method", "actor_opts", "runtime_env", "name", "job_id", "attempt",
        "generator", "node", "worker", "gpu_ids", "state", "submit_time", "start_time",
        "acquired", "pg_id", "cancelled", "parent", "concurrency_group", "pinned_refs",
        "blocked", "gen_bp",
    )

    def __init__(self, **kw):
        for s in self.__slots__:
            setattr(self, s, kw.get(s))
        self.attempt = self.attempt or 0
        self.arg_refs = self.arg_refs or []
        self.resources = self.resources or {}
        self.cancelled = False


class ObjEntry:
    __slots__ = ("state", "inline", "size", "node", "refcount", "pins", "waiters", "contained",
                 "is_error", "owner_task", "spilled_path", "gen_end", "lost", "lineage_refs")

    def __init__(self):
        self.state = PENDING
        self.lineage_refs = 0
        self.inline = None
        self.size = 0
        self.node = None
        self.refcount = 0
        self.pins = 0
        self.waiters = []
        self.contained = ()
        self.is_error = False
        self.owner_task = None
        self.spilled_path = None
        self.gen_end = None
        self.lost = False


class WorkerInfo:
    __slots__ = ("worker_id", "conn", "pid", "node", "gpu_key", "idle", "actor_id", "task",
                 "proc", "fns", "alive", "kind", "started", "tasks_inflight", "env_key", "client_id",
                 "oom_killed", "direct_addr", "lease", "lease_blocked", "lease_gpus")

    def __init__(self, **kw):
        for s in self.__slots__:
            setattr(self, s, kw.get(s))
        self.fns = set()
        self.tasks_inflight = {}


class ActorInfo:
    __slots__ = ("actor_id", "spec", "state", "worker", "name", "namespace", "restarts_left",
                 "max_task_retries", "queue", "inflight", "node", "gpu_ids", "acquired",
                 "class_name", "lifetime", "death_cause", "num_restarts", "owner", "pid", "record")

    def __init__(self, **kw):
        for s in self.__slots__:
            setattr(self, s, kw.get(s))
        self.queue = collections.deque()
        self.inflight = {}
        self.num_restarts = 0


class Head:
    def __init__(self, session_dir: str, node_id: bytes, resources: Dict[str, float],
                 store_name: str, store_capacity: int, gpu_ids: List[int],
                 listen_tcp: Optional[str] = None, namespace: str = "default",
                 worker_env: Optional[Dict[str, str]] = None, prestart: int = 0,
                 spill_dir: Optional[str] = None, labels: Optional[Dict[str, str]] = None,
                 gcs_storage: Optional[str] = None, reattach: bool = False,
                 reconnect_s: Optional[float] = None, spill_config=None):
        from .. import _native

        self.session_dir = session_dir
        os.makedirs(session_dir, exist_ok=True)
        self.node_id = node_id
        self.store_name = store_name
        self.store_capacity = store_capacity
        self.reattached = False
        if reattach:
            # a restarted head on the same node: the arena (and every sealed object in
            # it) outlived the old head; workers reconnect and re-register (see
            # _h_reregister). Its mutex is robust, so a lock held by the dead head is
            # recovered by the next locker.
            self.store = _native.ObjectStore(store_name, 0, 0, False)
            self.reattached = True
        else:
            self.store = _native.ObjectStore(store_name, store_capacity, 1 << 18, True)
            self.store.prefault_async(int(os.environ.get("CAAMD_OBJECT_STORE_PREFAULT_BYTES", str(2 << 30))))
        self.sched = _native.ClusterScheduler(0.5)
        self.sched.add_node(node_id.hex(), resources)
        self.node_labels = {node_id.hex(): _node_labels(node_id.hex(), gpu_ids, labels)}
        self.sched.set_labels(node_id.hex(), self.node_labels[node_id.hex()])
        self.node_resources = {node_id.hex(): dict(resources)}
        self.free_gpus = {node_id.hex(): list(gpu_ids)}
        self.gpu_partial: Dict[str, Dict[int, float]] = {}  # node -> gpu id -> fraction in use
        self.node_info = {node_id.hex(): {"NodeID": node_id.hex(), "Alive": True,
                                          "NodeManagerAddress": "127.0.0.1",
                                          "Resources": dict(resources), "local": True,
                                          "Labels": dict(self.node_labels[node_id.hex()])}}
        self.namespace = namespace
        self.worker_env = worker_env or {}
        self.spill_dir = spill_dir or os.path.join(session_dir, "spill")
        # where evicted objects go: the session dir, or _system_config
        # object_spilling_config (several directories round-robin, or a URI)
        from .external_storage import setup_external_storage

        self.spill_store = setup_external_storage(
            spill_config if spill_config is not None else os.environ.get("CAAMD_OBJECT_SPILLING_CONFIG"),
            os.path.basename(os.path.normpath(session_dir)) or "session", self.spill_dir)
        self.sock_path = os.path.join(session_dir, "head.sock")
        if len(self.sock_path) > 100:  # AF_UNIX path limit (108 bytes)
            import tempfile

            self.sock_path = os.path.join(tempfile.gettempdir(), f"caamd-{node_id.hex()[:12]}.sock")
        self.sel = selectors.DefaultSelector()
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            os.unlink(self.sock_path)
        except FileNotFoundError:
            pass
        self.lsock.bind(self.sock_path)
        self.lsock.listen(1024)
        self.lsock.setblocking(False)
        self.sel.register(self.lsock, selectors.EVENT_READ, ("listen", None))
        self.tcp_address = None
        if listen_tcp:
            host, port = listen_tcp.rsplit(":", 1)
            self.tsock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            self.tsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            self.tsock.bind((host, int(port)))
            self.tsock.listen(1024)
            self.tsock.setblocking(False)
            self.tcp_address = f"{host}:{self.tsock.getsockname()[1]}"
            self.sel.register(self.tsock, selectors.EVENT_READ, ("listen", None))
        # multi-node: per-node store names, object-server addresses, agent connections
        self.head_hex = node_id.hex()
        self.node_store = {self.head_hex: store_name}
        self.node_obj_addr: Dict[str, str] = {}
        self.node_conns: Dict[str, Conn] = {}
        self.obj_server = None
        if listen_tcp:
            from .object_server import ObjectServer

            bind_host = listen_tcp.rsplit(":", 1)[0]
            adv = "127.0.0.1" if bind_host in ("0.0.0.0", "") else bind_host
            self.obj_server = ObjectServer(self.store, bind_host or "0.0.0.0")
            self.node_obj_addr[self.head_hex] = self.obj_server.address(adv)
            self.node_info[self.head_hex]["NodeManagerAddress"] = adv
        # wakeup pipe for cross-thread calls
        self._wr, self._ww = socket.socketpair()
        self._wr.setblocking(False)
        self.sel.register(self._wr, selectors.EVENT_READ, ("wake", None))
        self._calls = collections.deque()

        self.objects: Dict[bytes, ObjEntry] = {}
        self.tasks: Dict[bytes, TaskSpec] = {}
        # owner notifications (reference: the owner's in-process memory store learns its
        # tasks' results without a GCS round trip): return oid -> submitting client conn
        self.owner_of = {}
        self._notify = {}
        self.dpins = {}
        self.dsealed_early = set()
        self.lease_waiters: List[tuple] = []  # parked lease requests, FIFO
        self.oom_killed_ids = set()
        self.waiting_deps: Dict[bytes, Set[bytes]] = {}  # task -> unresolved object ids
        self.lineage: Dict[bytes, TaskSpec] = {}  # finished tasks kept for object recovery
        self.num_reconstructions = 0
        self.dep_index: Dict[bytes, List[bytes]] = collections.defaultdict(list)
        # ready tasks grouped by scheduling class (demand + strategy), like the
        # reference's per-SchedulingClass queues: a blocked class costs O(1) per pass
        self.ready_queues: Dict[tuple, collections.deque] = {}
        self.infeasible: List[TaskSpec] = []
        self.workers: Dict[bytes, WorkerInfo] = {}
        self.conn_worker: Dict[Conn, WorkerInfo] = {}
        self.clients: Dict[Conn, dict] = {}
        self.idle: Dict[tuple, List[WorkerInfo]] = collections.defaultdict(list)
        self.starting: Dict[tuple, int] = collections.defaultdict(int)
        self.pending_spawn: Dict[bytes, tuple] = {}
        self.actors: Dict[bytes, ActorInfo] = {}
        self.named_actors: Dict[tuple, bytes] = {}
        self.kv: Dict[tuple, bytes] = {}
        self.functions: Dict[bytes, bytes] = {}
        self.pgs: Dict[bytes, dict] = {}
        self.pending_pgs: List[bytes] = []
        self.gen_waiters: Dict[bytes, list] = collections.defaultdict(list)
        self.gen_consumed: Dict[bytes, int] = {}  # streaming task -> items handed to its consumer
        self.gen_consume_waiters: Dict[bytes, list] = {}  # producers waiting for consumption
        self.gen_stats: Dict[bytes, dict] = {}
        self.handle_objs: Dict[bytes, bytes] = {}  # handle object id -> actor id
        self.events: collections.deque = collections.deque(maxlen=200000)
        # cluster events for the state API (reference: list_cluster_events / the
        # dashboard's event head): node / actor / job / OOM / infeasibility records
        self.cluster_events: collections.deque = collections.deque(maxlen=10000)
        self._event_seq = itertools.count(1)
        self.jobs: Dict[bytes, dict] = {}
        self.metrics: Dict[str, dict] = {}
        self.max_workers = int(max(4, resources.get("CPU", 1) * 4))
        self.running = True
        self.thread = None
        self._prestart = prestart
        self.cpu_count = resources.get("CPU", 1)
        self._last_health = time.time()
        from .memory_monitor import MemoryMonitor

        self.mem_monitor = MemoryMonitor()
        self._last_mem = 0.0
        self._oom_quiet_until = 0.0
        # durable GCS tables (head fault tolerance, core/gcs_persist.py)
        gcs_storage = gcs_storage or os.environ.get("CAAMD_GCS_STORAGE") or None
        self.gcs = None
        self._gcs_actors: Set[bytes] = set()
        self.gcs_restored = {}
        self._restored_grace: Dict[bytes, float] = {}  # restored object -> evict-protection deadline
        if gcs_storage:
            from .gcs_persist import GcsPersistence

            os.makedirs(os.path.dirname(os.path.abspath(gcs_storage)), exist_ok=True)
            self.gcs = GcsPersistence(gcs_storage)
        # with durable tables, workers and drivers that lose the head keep running and
        # reconnect for this long (a restarted head re-attaches them); 0 = die with it
        # (standalone heads: head_main; a driver-embedded head dies with its driver)
        if reconnect_s is None:
            reconnect_s = float(os.environ.get("CAAMD_HEAD_RECONNECT_S", "0"))
        self.reconnect_s = float(reconnect_s) if self.gcs is not None else 0.0
        if self.reconnect_s > 0:
            self.worker_env = dict(self.worker_env, CAAMD_HEAD_RECONNECT_S=str(self.reconnect_s))
        self.reattach_s = float(os.environ.get("CAAMD_GCS_REATTACH_S", "10"))
        self._reattaching = False
        self.subscribers: Dict[str, Set[Conn]] = {}  # pubsub channel -> subscriber connections
        self.env_failures: Dict[str, str] = {}  # runtime-env key -> setup error
        self.env_specs: Dict[str, Any] = {}  # runtime-env key -> the runtime env (state API)
        self.reattached_running: Dict[bytes, tuple] = {}  # task id -> (worker, node, demand) of a re-registered run
        self._held_resubmits: List[tuple] = []  # (conn, spec) replayed by owners during the re-attach grace
        # re-attach ordering: a lease whose worker has not re-registered yet is
        # parked under the worker id; an idle re-registered worker is held out of the idle
        # pool until its lease holder claims it or the grace ends
        self._parked_leases: Dict[bytes, tuple] = {}  # worker id -> (owner conn, lease entry)
        self._reattach_hold: List[WorkerInfo] = []
        self.reattach_stats = {"workers": 0, "actors": 0, "objects": 0, "drivers": 0, "lost_objects": 0,
                               "recreated_actors": 0, "dead_actors": 0}
        if self.gcs is not None:
            self.gcs.session_put({"session_dir": session_dir, "node_id": node_id.hex(), "store_name": store_name,
                                  "store_bytes": int(store_capacity), "tcp_address": self.tcp_address,
                                  "pid": os.getpid(), "sock_path": self.sock_path})

    # ------------------------------------------------------------------ loop
    def start(self):
        self._zygote = None
        from . import zygote

        if zygote.enabled():
            try:  # forks pre-imported workers (core/zygote.py); Popen until it is ready
                self._zygote = zygote.Zygote(self.session_dir)
            except Exception:
                self._zygote = None
        if self.gcs is not None:
            self._gcs_restore()
        self.thread = threading.Thread(target=self._loop, name="caamd-head", daemon=True)
        self.thread.start()
        # physical metrics of the head's own node (other nodes push theirs: _h_node_stats)
        self.node_info[self.head_hex]["IsHeadNode"] = True
        self._reporter = None
        try:
            from ..dashboard.reporter import NodeReporter

            info = self.node_info[self.head_hex]
            self._reporter = NodeReporter(lambda st: info.__setitem__("stats", st), self.session_dir).start()
        except Exception:
            self._reporter = None
        for _ in range(self._prestart):
            self.call(lambda: self._spawn_worker(self.node_id.hex(), ()))

    def call(self, fn):
        """Run ``fn`` on the head thread (fire-and-forget)."""
        self._calls.append(fn)
        try:
            self._ww.send(b"x")
        except OSError:
            pass

    def call_sync(self, fn, timeout=30):
        ev = threading.Event()
        box = {}

        def run():
            try:
                box["v"] = fn()
            except BaseException as e:  # pragma: no cover
                box["e"] = e
            ev.set()

        self.call(run)
        if not ev.wait(timeout):
            raise TimeoutError("head did not answer")
        if "e" in box:
            raise box["e"]
        return box.get("v")

    def _loop(self):
        prof_path = os.environ.get("CAAMD_HEAD_PROFILE")
        if prof_path:  # diagnostics: cProfile of the head's event loop, dumped at shutdown
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
            try:
                self._loop_body()
            finally:
                prof.disable()
                prof.dump_stats(prof_path)
            return
        self._loop_body()

    def _loop_body(self):
        while self.running:
            try:
                events = self.sel.select(timeout=0.2)
            except OSError:
                break
            for key, _ in events:
                kind, data = key.data
                if kind == "listen":
                    try:
                        s, _ = key.fileobj.accept()
                    except OSError:
                        continue
                    # client sockets stay BLOCKING: reads only happen when epoll reports
                    # data, and sends block exactly as they did with per-send toggling
                    # (two fcntl syscalls per message saved)
                    s.setblocking(True)
                    c = Conn(s)
                    self.clients[c] = {"id": None}
                    self.sel.register(s, selectors.EVENT_READ, ("conn", c))
                elif kind == "wake":
                    try:
                        self._wr.recv(4096)
                    except OSError:
                        pass
                elif kind == "conn":
                    self._on_readable(data)
            while self._calls:
                fn = self._calls.popleft()
                try:
                    fn()
                except Exception:
                    traceback.print_exc()
            if self._notify:
                self._flush_notify()
            now = time.time()
            if now - self._last_health > 1.0:
                self._last_health = now
                self._health_check()
            if self.mem_monitor.enabled and now - self._last_mem >= self.mem_monitor.refresh_s:
                self._last_mem = now
                self._check_memory(now)

    def _flush_notify(self):
        pending, self._notify = self._notify, {}
        for c, oids in pending.items():
            rnode = self.clients.get(c, {}).get("node") or self.head_hex
            items = []
            for o in oids:
                e = self.objects.get(o)
                if e is None or e.state != READY:
                    continue
                items.append((o, *self._obj_payload(o, rnode)))
            if items:
                self._send(c, ("ready", items))

    def _on_readable(self, c: Conn):
        # one preallocated receive buffer for the whole loop: recv(1 MiB) would
        # mmap/munmap a fresh 1 MiB object per call (~50 us at high message rates)
        buf = getattr(self, "_rx", None)
        if buf is None:
            buf = self._rx = bytearray(1 << 18)
            self._rx_mv = memoryview(buf)
        try:
            n = c.sock.recv_into(buf)
        except BlockingIOError:
            return
        except OSError:
            n = 0
        if not n:
            self._on_disconnect(c)
            return
        for msg in c.feed(self._rx_mv[:n]):
            try:
                self._dispatch(c, msg)
            except Exception:
                traceback.print_exc()

    def _send(self, c: Conn, msg):
        if c is None or c.closed:
            return
        try:
            c.send(msg)
        except ConnectionClosed:
            pass

    # -------------------------------------------------------------- dispatch
    def _dispatch(self, c: Conn, msg):
        t = msg[0]
        h = getattr(self, "_h_" + t, None)
        if h is None:
            raise ValueError(f"unknown message {t}")
        h(c, *msg[1:])

    def _reply(self, c, req, value):
        self._send(c, ("reply", req, value))

    def _h_register(self, c, kind, worker_id, pid, node_hex, extra):
        node = node_hex or self.head_hex
        self.clients[c] = {"id": worker_id, "kind": kind, "pid": pid, "node": node}
        if kind == "node":
            self._register_node(c, node_hex, extra)
            return
        self._send(c, ("registered", {"store_name": self.node_store.get(node, self.store_name),
                                      "node_id": node,
                                      "namespace": self.namespace,
                                      "session_dir": self.session_dir,
                                      "reconnect_s": self.reconnect_s}))
        if kind == "worker":
            w = self.workers.get(worker_id)
            if w is None:
                w = WorkerInfo(worker_id=worker_id, pid=pid, node=node_hex,
                               gpu_key=tuple(extra.get("gpu_ids", ())), kind="worker")
                self.workers[worker_id] = w
            w.conn = c
            w.alive = True
            w.started = time.time()
            w.client_id = worker_id
            w.direct_addr = (extra or {}).get("direct")
            self.conn_worker[c] = w
            key = (w.node, w.gpu_key, w.env_key)
            self.starting[key] = max(0, self.starting[key] - 1)
            pending = self.pending_spawn.pop(worker_id, None)
            if pending and pending[0] == "actor":
                a = self.actors.get(pending[1])
                st = a.spec.strategy if a is not None and a.spec else None
                if a is None or a.state == "DEAD" or (st and st[0] == "pg" and st[1] not in self.pgs):
                    self._kill_worker(worker_id)  # its actor died (or lost its group) meanwhile
                    return
                self._start_actor_on(a, w)
            else:
                w.idle = True
                self.idle[key].append(w)
                self._schedule()
        elif kind == "driver":
            jid = extra.get("job_id", b"")
            if jid not in self.jobs:
                self.jobs[jid] = {"start": time.time(), "pid": pid, "driver": worker_id}
                self._cluster_event("INFO", "GCS", f"job {jid.hex() if isinstance(jid, bytes) else jid} started",
                                    job_id=jid.hex() if isinstance(jid, bytes) else str(jid), pid=pid)
                if self.gcs is not None:
                    self.gcs.job_put(jid, self.jobs[jid])

    # ------------------------------------------------------------ functions/kv
    def _h_fn(self, c, fn_id, blob):
        self.functions[fn_id] = blob
        if self.gcs is not None:
            self.gcs.fn_put(fn_id, blob)

    def _h_kv(self, c, req, op, ns, key, value, overwrite):
        k = (ns, key)
        if op == "put":
            existed = k in self.kv
            if overwrite or not existed:
                self.kv[k] = value
                if self.gcs is not None:
                    self.gcs.kv_put(ns, key, value)
            self._reply(c, req, not existed)
        elif op == "get":
            self._reply(c, req, self.kv.get(k))
        elif op == "del":
            if key.endswith(b"*"):
                n = 0
                for kk in [kk for kk in self.kv if kk[0] == ns and kk[1].startswith(key[:-1])]:
                    del self.kv[kk]
                    if self.gcs is not None:
                        self.gcs.kv_del(*kk)
                    n += 1
                self._reply(c, req, n)
            else:
                gone = self.kv.pop(k, None) is not None
                if gone and self.gcs is not None:
                    self.gcs.kv_del(ns, key)
                self._reply(c, req, 1 if gone else 0)
        elif op == "exists":
            self._reply(c, req, k in self.kv)
        elif op == "keys":
            self._reply(c, req, [kk[1] for kk in self.kv if kk[0] == ns and kk[1].startswith(key)])

    # ------------------------------------------------------------------ objects
    def _obj(self, oid) -> ObjEntry:
        e = self.objects.get(oid)
        if e is None:
            e = ObjEntry()
            self.objects[oid] = e
        return e

    def _h_put(self, c, oid, inline, size, node_hex, contained, is_error=False):
        e = self._obj(oid)
        e.refcount += 1
        self._seal_object(oid, inline, size, node_hex, contained, is_error)

    def _seal_object(self, oid, inline, size, node_hex, contained, is_error=False):
        e = self._obj(oid)
        oc = self.owner_of.pop(oid, None)
        if e.state == READY:
            return
        if oc is not None and not oc.closed:
            self._notify.setdefault(oc, []).append(oid)
        e.state = READY
        e.inline = inline
        e.size = size
        e.node = node_hex
        e.is_error = is_error
        e.contained = tuple(contained or ())
        for r in e.contained:
            self._obj(r).pins += 1
        waiters, e.waiters = e.waiters, []
        for w in waiters:
            w(oid)
        self._maybe_free(oid)

    def _h_addref(self, c, oids):
        for o in oids:
            self._obj(o).refcount += 1

    def _h_decref(self, c, oids):
        for o in oids:
            e = self.objects.get(o)
            if e is None:
                continue
            e.refcount -= 1
            self._maybe_free(o)

    def _maybe_free(self, oid):
        e = self.objects.get(oid)
        if e is None or e.refcount > 0 or e.pins > 0 or e.state != READY or e.waiters:
            return
        if e.owner_task is not None:
            t = self.tasks.get(e.owner_task)
            if t is not None and t.state in ("pending", "running"):
                return
        if e.lineage_refs > 0:
            # data goes, metadata stays: a retained downstream lineage may need to
            # re-create this object (reference: lineage pinning, reference_count.cc)
            e.state = FREED
        else:
            del self.objects[oid]
        aid = self.handle_objs.pop(oid, None)
        if aid is not None:
            self._on_handles_gone(aid)
            return
        if e.inline is None and e.spilled_path is None:
            if e.node and e.node != self.head_hex:
                nc = self.node_conns.get(e.node)
                if nc is not None:
                    self._send(nc, ("free", [oid]))
            else:
                try:
                    self.store.remove(oid)
                except Exception:
                    pass
        if e.spilled_path:
            self.spill_store.delete(e.spilled_path)
        for r in e.contained:
            ce = self.objects.get(r)
            if ce is not None:
                ce.pins -= 1
                self._maybe_free(r)
        e.contained = ()
        if e.state != FREED:
            self._lineage_release_if_unused(e.owner_task)

    # ------------------------------------------------- lineage reconstruction
    # Reference: src/ray/core_worker/object_recovery_manager.cc (re-execute the task
    # that created a lost object, recursively recovering lost arguments) and
    # task_manager.cc:ResubmitTask (re-executions count against max_retries).
    # Lineage of a finished NORMAL task is retained while any of its return objects
    # still has an entry; arguments keep metadata-only entries (``lineage_refs``)
    # so their own lineage survives even after their data was freed.
    def _lineage_retain(self, spec):
        if spec.kind != NORMAL or spec.generator is not None or spec.state != "finished":
            return False
        mr = spec.max_retries if spec.max_retries is not None else 3
        if mr == 0 or (0 <= mr <= spec.attempt) or len(self.lineage) >= LINEAGE_MAX_TASKS:
            return False
        self.lineage[spec.task_id] = spec
        for r in spec.arg_refs:
            self._obj(r).lineage_refs += 1
        return True

    def _lineage_release_if_unused(self, tid):
        spec = self.lineage.get(tid) if tid is not None else None
        if spec is None or any(r in self.objects for r in spec.return_ids or ()):
            return
        del self.lineage[tid]
        for r in spec.arg_refs:
            e = self.objects.get(r)
            if e is None:
                continue
            e.lineage_refs -= 1
            if e.lineage_refs <= 0 and e.state == FREED:
                del self.objects[r]
                self._lineage_release_if_unused(e.owner_task)

    def _reconstruct(self, oid, _seen=None) -> bool:
        """Re-execute the task that created ``oid``; False if it cannot be recovered."""
        e = self.objects.get(oid)
        if e is None:
            return False
        tid = e.owner_task
        live = self.tasks.get(tid) if tid is not None else None
        if live is not None and live.state in ("pending", "running"):
            return True  # already being (re)computed
        spec = self.lineage.get(tid) if tid is not None else None
        if spec is None:
            return False
        mr = spec.max_retries if spec.max_retries is not None else 3
        if 0 <= mr <= spec.attempt:
            return False
        seen = _seen if _seen is not None else set()
        if tid in seen:
            return True
        seen.add(tid)
        # arguments whose data is gone are recovered first (recursively)
        for r in spec.arg_refs:
            ae = self.objects.get(r)
            if ae is None:
                return False
            if ae.state == FREED or ae.lost:
                if not self._reconstruct(r, seen):
                    return False
        del self.lineage[tid]
        spec.attempt += 1
        spec.state = "pending"
        spec.node = spec.worker = spec.acquired = spec.gpu_ids = None
        spec.cancelled = False
        self.tasks[tid] = spec
        for r in spec.arg_refs:
            ae = self.objects[r]
            ae.pins += 1
            ae.lineage_refs -= 1
        for r in spec.return_ids or ():
            re_ = self.objects.get(r)
            if re_ is None:
                continue
            if re_.state == READY and not re_.lost and (re_.inline is not None or re_.spilled_path):
                continue  # this copy survived (inlined / spilled on the head)
            for cr in re_.contained:
                ce = self.objects.get(cr)
                if ce is not None:
                    ce.pins -= 1
            re_.contained = ()
            re_.state = PENDING
            re_.lost = False
            re_.inline = None
            re_.node = None
        self.events.append(("reconstruct", tid, spec.fn_name, time.time()))
        self.num_reconstructions += 1
        self._enqueue_when_ready(spec)
        return True

    def _h_report_lost(self, c, req, oid):
        """A reader could not pull ``oid`` from its node (it died before the head noticed)."""
        e = self.objects.get(oid)
        if e is None:
            self._reply(c, req, False)
            return
        if e.state == PENDING:
            self._reply(c, req, True)
            return
        if e.inline is not None:
            self._reply(c, req, True)
            return
        ok = self._reconstruct(oid)
        if not ok:
            e.lost = True
        self._reply(c, req, ok)

    def _obj_payload(self, oid, node=None):
        e = self.objects.get(oid)
        if e is None or getattr(e, "lost", False):
            return ("lost", None)
        if e.inline is not None:
            return ("err" if e.is_error else "inline", e.inline)
        if e.spilled_path is not None:
            self._restore(oid, e)
            e.node = self.head_hex
            # the reader maps it after this reply: keep the next evictions off it
            self._restored_grace[oid] = time.time() + self._RESTORE_GRACE_S
        src = e.node or self.head_hex
        if node is not None and src != node:
            addr = self.node_obj_addr.get(src)
            if addr is None:
                return ("lost", None)
            # the reader pulls straight from the owning node's object server
            return ("err_remote" if e.is_error else "remote", (addr, e.size))
        return ("err_store" if e.is_error else "store", e.size)

    def _restore(self, oid, e):
        data = self.spill_store.restore(e.spilled_path)
        off = self.store.create(oid, len(data), 0)
        if off < 0:
            self._evict(len(data))
            off = self.store.create(oid, len(data), 0)
        if off >= 0:
            self.store.buffer(off, len(data), False)[:] = data
            self.store.seal(oid)
            self.spill_store.delete(e.spilled_path)
            e.spilled_path = None
            self.events.append(("restore", oid.hex(), len(data), time.time()))
        else:
            e.inline = data  # last resort: serve through the control plane

    _RESTORE_GRACE_S = 2.0

    def _evict(self, need):
        """Spill least-recently-used sealed objects to disk until ``need`` fits.
        Objects restored for a reader within the last ``_RESTORE_GRACE_S`` seconds
        are spilled only when nothing else can make room (otherwise two readers of
        spilled objects evict each other's copies between the head's reply and the
        reader's mapping)."""
        now = time.time()
        grace = self._restored_grace
        for o in [o for o, t in grace.items() if t <= now]:
            del grace[o]
        freed = self._evict_pass(need, skip=grace)
        if freed < need or self.store.largest_free() < need:
            freed += self._evict_pass(need - freed, skip=None)
        return freed

    def _evict_pass(self, need, skip):
        freed = 0
        for oid in self.store.lru_candidates(256):
            e = self.objects.get(oid)
            if e is None or (skip and oid in skip):
                continue
            pb = self.store.get_pinned(oid)
            if pb is None:
                continue
            path = self.spill_store.spill(oid.hex(), memoryview(pb))
            del pb
            self.store.remove(oid)
            e.spilled_path = path
            freed += e.size
            self.events.append(("spill", oid.hex(), e.size, time.time()))
            if freed >= need and self.store.largest_free() >= need:
                break
        return freed

    def _h_evict(self, c, req, need):
        node = self.clients.get(c, {}).get("node") or self.head_hex
        self._reply(c, req, self._evict(need) if node == self.head_hex else 0)

    def _h_get(self, c, req, oids, timeout):
        """Reply when every object is ready (or on timeout with what is ready)."""
        missing = set()
        for o in oids:
            e = self._obj(o)
            if e.state != READY:
                missing.add(o)
        rnode = self.clients.get(c, {}).get("node") or self.head_hex
        if not missing:
            self._reply(c, req, [(o, *self._obj_payload(o, rnode)) for o in oids])
            return
        state = {"missing": missing, "done": False}

        def on_ready(oid):
            state["missing"].discard(oid)
            if not state["missing"] and not state["done"]:
                state["done"] = True
                self._reply(c, req, [(o, *self._obj_payload(o, rnode)) for o in oids])

        for o in missing:
            self._obj(o).waiters.append(on_ready)
        if timeout is not None and timeout >= 0:
            def on_timeout():
                if not state["done"]:
                    state["done"] = True
                    for o in list(state["missing"]):
                        e = self.objects.get(o)
                        if e is not None and on_ready in e.waiters:
                            e.waiters.remove(on_ready)
                    self._reply(c, req, None)
            self._timer(timeout, on_timeout)

    def _h_wait(self, c, req, oids, num_returns, timeout):
        ready = [o for o in oids if self._obj(o).state == READY]
        if len(ready) >= num_returns or timeout == 0:
            self._reply(c, req, ready[: max(num_returns, 0)] if len(ready) >= num_returns else ready)
            return
        state = {"ready": set(ready), "done": False}

        def finish():
            if state["done"]:
                return
            state["done"] = True
            for o in oids:
                e = self.objects.get(o)
                if e is not None and on_ready in e.waiters:
                    e.waiters.remove(on_ready)
            rs = [o for o in oids if o in state["ready"]]
            self._reply(c, req, rs[:num_returns])

        def on_ready(oid):
            state["ready"].add(oid)
            if len(state["ready"]) >= num_returns:
                finish()

        for o in oids:
            if o not in state["ready"]:
                self._obj(o).waiters.append(on_ready)
        if timeout is not None and timeout >= 0:
            self._timer(timeout, finish)

    def _timer(self, delay, fn):
        def fire():
            time.sleep(delay)
            self.call(fn)

        threading.Thread(target=fire, daemon=True).start()

    def _h_free(self, c, oids):
        for o in oids:
            e = self.objects.get(o)
            if e is not None:
                e.refcount = 0
                e.pins = 0
                self._maybe_free(o)

    # -------------------------------------------------------------------- tasks
    def _h_submit(self, c, spec: TaskSpec):
        if self.reattached and c is not None and self._resubmitted(c, spec):
            return
        spec.owner = self.clients.get(c, {}).get("id")
        spec.state = "pending"
        spec.submit_time = time.time()
        self.tasks[spec.task_id] = spec
        for i, oid in enumerate(spec.return_ids or ()):
            e = self._obj(oid)
            e.refcount += 1
            e.owner_task = spec.task_id
            if spec.generator is None:
                self.owner_of[oid] = c
        self.events.append(("submit", spec.task_id, spec.fn_name, spec.submit_time))
        for r in spec.arg_refs:
            self._obj(r).pins += 1
        for r in spec.pinned_refs or ():
            self._obj(r).pins += 1
        if spec.kind == ACTOR_CREATE:
            self._register_actor(spec, c)
        self._enqueue_when_ready(spec)

    def _resubmitted(self, c, spec) -> bool:
        """An owner re-sends the head-path tasks it had in flight when the previous
        head died. True if this one needs no new run: its results already exist,
        its actor is known (a creation), or a re-registered worker is still running
        (or reporting) it -- then it is adopted as that worker's in-flight task."""
        if spec.kind == ACTOR_CREATE and spec.actor_id in self.actors:
            return True
        rids = spec.return_ids or ()
        if rids and all((self.objects.get(o) is not None and self.objects[o].state == READY) for o in rids):
            for o in rids:
                oc = c
                if not oc.closed:
                    self._notify.setdefault(oc, []).append(o)
            return True
        run = self.reattached_running.get(spec.task_id)
        if run is None:
            held_actor = spec.kind == ACTOR_METHOD and any(
                h[1].kind == ACTOR_METHOD and h[1].actor_id == spec.actor_id for h in self._held_resubmits)
            if self._reattaching or held_actor:
                # its worker may still re-register with it running (then it is adopted,
                # not run twice); later calls to an actor with held calls queue behind them
                self._held_resubmits.append((c, spec))
                return True
            return False
        wid, node, held = run
        spec.owner = self.clients.get(c, {}).get("id")
        spec.state = "running"
        spec.submit_time = spec.start_time = time.time()
        spec.worker, spec.node = wid, node
        spec.acquired = (node, held) if held else None
        self.tasks[spec.task_id] = spec
        for oid in rids:
            e = self._obj(oid)
            e.refcount += 1
            e.owner_task = spec.task_id
            self.owner_of[oid] = c
        w = self.workers.get(wid)
        if w is not None:
            w.tasks_inflight[spec.task_id] = spec
        if spec.kind == ACTOR_METHOD:
            a = self.actors.get(spec.actor_id)
            if a is not None:
                a.inflight[spec.task_id] = spec
        self.reattached_running.pop(spec.task_id, None)
        return True

    def _enqueue_when_ready(self, spec):
        unresolved = {r for r in spec.arg_refs if self._obj(r).state != READY}
        if not unresolved:
            self._on_deps_ready(spec)
            return
        self.waiting_deps[spec.task_id] = unresolved

        def on_ready(oid, tid=spec.task_id):
            s = self.waiting_deps.get(tid)
            if s is None:
                return
            s.discard(oid)
            if not s:
                del self.waiting_deps[tid]
                t = self.tasks.get(tid)
                if t is not None and not t.cancelled:
                    self._on_deps_ready(t)

        for r in unresolved:
            self._obj(r).waiters.append(on_ready)

    def _on_deps_ready(self, spec):
        # a dependency that failed poisons the task (reference: task dependency errors)
        for r in spec.arg_refs:
            e = self.objects.get(r)
            if e is not None and e.is_error:
                pass  # the worker re-raises the stored error when it resolves the arg
        if spec.kind == ACTOR_METHOD:
            a = self.actors.get(spec.actor_id)
            if a is None:
                self._fail_task(spec, ("ActorDiedError", "actor not found"))
                return
            a.queue.append(spec)
            self._pump_actor(a)
        else:
            self._enqueue_ready(spec)
            self._schedule()

    def _demand(self, spec):
        return self._demand_for(spec.resources, spec.strategy)

    def _demand_for(self, resources, st):
        d = dict(resources)
        if st and st[0] == "pg":
            _, pg_id, bidx = st[:3]
            pg_hex = pg_id.hex()
            nd = {}
            for k, v in d.items():
                if v <= 0:
                    continue
                if bidx is None or bidx < 0:
                    nd[f"{k}_group_{pg_hex}"] = v
                else:
                    nd[f"{k}_group_{bidx}_{pg_hex}"] = v
            if not nd:
                nd = ({f"bundle_group_{pg_hex}": 0.001} if bidx is None or bidx < 0
                      else {f"bundle_group_{bidx}_{pg_hex}": 0.001})
            return nd
        return d

    def _enqueue_ready(self, spec):
        key = (tuple(sorted(spec.resources.items())), spec.strategy, spec.kind == ACTOR_CREATE)
        q = self.ready_queues.get(key)
        if q is None:
            q = self.ready_queues[key] = collections.deque()
        q.append(spec)

    def _schedule(self):
        if not self.ready_queues:
            if self.lease_waiters:
                self._serve_lease_waiters()
            return
        for key in list(self.ready_queues):
            q = self.ready_queues[key]
            while q:
                spec = q[0]
                if spec.cancelled:
                    q.popleft()
                    continue
                if self._try_place(spec):
                    q.popleft()
                else:
                    break
            if not q:
                del self.ready_queues[key]
        if self.lease_waiters:
            self._serve_lease_waiters()

    def _pick(self, spec, demand=None):
        """Node for a task under its scheduling strategy ('' = not now, '!' = never)."""
        demand = demand if demand is not None else self._demand(spec)
        st = spec.strategy or ("default",)
        strategy, aff, soft, hard_l, soft_l = 0, "", False, [], []
        if st[0] == "spread":
            strategy = 1
        elif st[0] == "node":
            strategy, aff, soft = 2, st[1], bool(st[2])
        elif st[0] == "label":
            strategy, hard_l, soft_l = 3, list(st[1]), list(st[2])
        return self.sched.pick_node(demand, strategy, aff, soft, self.node_id.hex(), hard_l, soft_l)

    def _try_place(self, spec) -> bool:
        demand = self._demand(spec)
        st = spec.strategy or ("default",)
        if st[0] == "pg" and spec.strategy[1] not in self.pgs:
            self._fail_task(spec, ("TaskPlacementGroupRemoved", "placement group was removed"))
            return True
        node = self._pick(spec, demand)
        if node == "!":
            if spec not in self.infeasible:
                self.infeasible.append(spec)
                self.events.append(("infeasible", spec.task_id, spec.fn_name, time.time()))
                self._cluster_event("WARNING", "RAYLET", f"task {spec.fn_name} is infeasible: no node has "
                                    f"{self._demand(spec)}", task_id=spec.task_id.hex())
            return True  # parked
        if node == "":
            return False
        gamt = float(spec.resources.get("GPU", 0) or 0)
        gpu_ids = self._pick_gpus(node, gamt)
        if gpu_ids is None:
            return False
        if spec.kind == ACTOR_CREATE:
            if not self.sched.acquire(node, demand):
                return False
            self._take_gpus(node, gpu_ids, gamt)
            spec.acquired = (node, demand)
            spec.gpu_ids = gpu_ids
            a = self.actors[spec.actor_id]
            a.node, a.gpu_ids, a.acquired = node, gpu_ids, (node, demand)
            wid = os.urandom(16)
            self.pending_spawn[wid] = ("actor", spec.actor_id)
            self._spawn_worker(node, gpu_ids, worker_id=wid, env=spec.runtime_env)
            return True
        ek = _env_key(spec.runtime_env)
        if ek is not None and ek in self.env_failures:
            self._fail_task(spec, ("RuntimeEnvSetupError", f"runtime env setup failed: {self.env_failures[ek]}"))
            return True
        key = (node, gpu_ids, ek)
        idle = self.idle.get(key)
        w = None
        while idle:
            cand = idle.pop()
            if cand.alive and cand.idle:
                w = cand
                break
        if w is None:
            if self.starting[key] < max(1, int(self.cpu_count)):
                if self._num_workers(node) >= self.max_workers:
                    self._evict_idle(node, key)  # an idle worker of another env makes room
                if self._num_workers(node) < self.max_workers:
                    self._spawn_worker(node, gpu_ids, env=spec.runtime_env)
            return False
        if not self.sched.acquire(node, demand):
            w.idle = True
            self.idle[key].append(w)
            return False
        self._take_gpus(node, gpu_ids, gamt)
        spec.acquired = (node, demand)
        spec.gpu_ids = gpu_ids
        self._dispatch_to(w, spec)
        return True

    # GPU ids: whole GPUs for num_gpus >= 1; fractions pack onto one GPU (the
    # fullest one that still fits), so e.g. two num_gpus=0.5 actors share a device
    def _pick_gpus(self, node, amount):
        if amount <= 0:
            return ()
        free = self.free_gpus.get(node, [])
        if amount >= 1 - 1e-9:
            n = int(round(amount))
            return tuple(free[:n]) if len(free) >= n else None
        part = self.gpu_partial.setdefault(node, {})
        best = None
        for g, used in part.items():
            if used + amount <= 1 + 1e-9 and (best is None or used > part[best]):
                best = g
        if best is not None:
            return (best,)
        return (free[0],) if free else None

    def _take_gpus(self, node, gids, amount):
        if not gids:
            return
        if amount >= 1 - 1e-9:
            for g in gids:
                self.free_gpus[node].remove(g)
            return
        g = gids[0]
        part = self.gpu_partial.setdefault(node, {})
        if g not in part:
            self.free_gpus[node].remove(g)
            part[g] = 0.0
        part[g] += amount

    def _give_gpus(self, node, gids, amount):
        if not gids:
            return
        if amount >= 1 - 1e-9:
            self.free_gpus.setdefault(node, []).extend(gids)
            return
        part = self.gpu_partial.get(node, {})
        g = gids[0]
        if g in part:
            part[g] -= amount
            if part[g] <= 1e-9:
                del part[g]
                self.free_gpus.setdefault(node, []).append(g)

    def _num_workers(self, node):
        """Pooled (task / not-yet-actor) workers on ``node``: the soft cap
        ``max_workers`` bounds these only -- a worker that hosts an actor is
        dedicated to it and never blocks task workers (reference: the raylet's
        worker pool soft limit, worker_pool.cc, counts idle/task workers)."""
        return sum(1 for w in self.workers.values() if w.node == node and w.alive and w.actor_id is None) + sum(
            v for (n, _g, _e), v in self.starting.items() if n == node)

    def _evict_idle(self, node, keep_key):
        """Stop one idle pooled worker of another runtime env on ``node`` (reference:
        the raylet worker pool kills idle workers of other runtime envs when full)."""
        for key, lst in self.idle.items():
            if key == keep_key or key[0] != node:
                continue
            while lst:
                w = lst.pop()
                if w.alive and w.idle and w.actor_id is None and w.lease is None:
                    w.idle = False
                    self._send(w.conn, ("exit",))
                    self._kill_worker(w.worker_id)
                    return True
        return False

    def _spawn_worker(self, node, gpu_ids, worker_id=None, env=None):
        worker_id = worker_id or os.urandom(16)
        ek = _env_key(env)
        if ek is not None:
            self.env_specs.setdefault(ek, env)
        key = (node, tuple(gpu_ids), ek)
        self.starting[key] += 1
        if node != self.head_hex:
            return self._spawn_remote(node, gpu_ids, worker_id, env)
        e = dict(os.environ)
        e.update(self.worker_env)
        e["CAAMD_HEAD"] = self.sock_path if node == self.node_id.hex() else (self.tcp_address or "")
        e["CAAMD_WORKER_ID"] = worker_id.hex()
        e["CAAMD_NODE_ID"] = node
        e["CAAMD_NODE_IP"] = str((self.node_info.get(node) or {}).get("NodeManagerAddress") or "127.0.0.1")
        e["CAAMD_GPU_IDS"] = ",".join(str(g) for g in gpu_ids)
        renv = env or {}
        noset = (renv.get("env_vars") or {}).get("CAAMD_NOSET_ROCR_VISIBLE_DEVICES")
        if gpu_ids and not noset:
            # isolate the worker to its GPUs before HIP initialises (reference:
            # accelerators/amd_gpu.py ROCR_VISIBLE_DEVICES). Train worker groups opt
            # out (NOSET) so RCCL sees every peer GPU of the node for xGMI P2P.
            e["ROCR_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpu_ids)
        for k, v in (renv.get("env_vars") or {}).items():
            e[k] = str(v)
        if renv:
            import json

            e["CAAMD_RUNTIME_ENV"] = json.dumps(renv)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
        # workers import user code the way the driver does (reference: the driver's
        # code search path is propagated through the job config)
        e["CAAMD_SYS_PATH"] = os.pathsep.join(p for p in sys.path if p and os.path.isdir(p))
        log_path = os.path.join(self.session_dir, f"worker-{worker_id.hex()[:8]}.log")
        try:
            from ..runtime_env import pip as _pip

            pip_cfg = _pip.pip_field(renv)
        except Exception:  # noqa: BLE001 - a malformed pip field fails at setup below
            pip_cfg = None
        if pip_cfg is not None:
            return self._spawn_in_env(worker_id, node, gpu_ids, ek, e, log_path, pip_cfg, renv)
        zyg = getattr(self, "_zygote", None)
        if zyg is not None and _needs_fresh_interpreter(renv):
            zyg = None  # start-time variables / another interpreter: a fork cannot honour them
        proc = zyg.spawn(e, log_path, os.getcwd()) if zyg is not None else None
        if proc is None:
            log = open(log_path, "ab")
            proc = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.worker_main"],
                                    env=e, stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                    cwd=os.getcwd())
            log.close()
        w = WorkerInfo(worker_id=worker_id, pid=proc.pid, node=node, gpu_key=tuple(gpu_ids),
                       kind="worker", proc=proc, alive=False, env_key=ek)
        self.workers[worker_id] = w
        return w

    def _spawn_in_env(self, worker_id, node, gpu_ids, ek, e, log_path, cfg, renv):
        """Start a worker inside a pip / uv runtime env (runtime_env/pip.py): the env is
        built (or found in the URI cache) on a thread, then the worker is launched
        with that env's interpreter (reference: PipPlugin, pip.py:216)."""
        from ..runtime_env import pip as _pip

        w = WorkerInfo(worker_id=worker_id, pid=None, node=node, gpu_key=tuple(gpu_ids), kind="worker",
                       proc=None, alive=False, env_key=ek)
        self.workers[worker_id] = w
        if ek in self.env_failures:
            self.call(lambda: self._env_setup_failed(w, ek, self.env_failures[ek]))
            return w

        def build():
            try:
                py = _pip.ensure_env(cfg, _pip.setup_timeout(renv))
            except Exception as exc:  # noqa: BLE001
                msg = str(exc)
                self.call(lambda: self._env_setup_failed(w, ek, msg))
                return

            def launch():
                if self.workers.get(worker_id) is not w or not self.running:
                    return
                log = open(log_path, "ab")
                env_dir = os.path.dirname(os.path.dirname(py))
                proc = subprocess.Popen([py, "-m", "cluster_anywhere_amd.core.worker_main"],
                                        env=dict(e, CAAMD_PIP_ENV_DIR=env_dir), stdout=log,
                                        stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, cwd=os.getcwd())
                _pip.mark_in_use(env_dir, proc.pid)  # no eviction while this worker runs
                log.close()
                w.proc, w.pid = proc, proc.pid

            self.call(launch)

        threading.Thread(target=build, name="caamd-runtime-env", daemon=True).start()
        return w

    def _env_setup_failed(self, w, ek, msg):
        """The runtime env could not be built: fail what waits for it (reference:
        RuntimeEnvSetupError), and fail later tasks of the same env at once."""
        self.env_failures[ek] = msg
        key = (w.node, w.gpu_key, ek)
        self.starting[key] = max(0, self.starting[key] - 1)
        self.workers.pop(w.worker_id, None)
        cause = f"runtime env setup failed: {msg}"
        pending = self.pending_spawn.pop(w.worker_id, None)
        if pending and pending[0] == "actor":
            a = self.actors.get(pending[1])
            if a is not None:
                a.restarts_left = 0
                a.death_cause = cause
                self._set_actor_state(a, "DEAD")
                self._fail_actor_queue(a, "RuntimeEnvSetupError", cause)
        for q in list(self.ready_queues.values()):
            for spec in [sp for sp in q if _env_key(sp.runtime_env) == ek]:
                q.remove(spec)
                self._fail_task(spec, ("RuntimeEnvSetupError", cause))

    def _spawn_remote(self, node, gpu_ids, worker_id, env):
        """Ask the node's agent to start a worker (reference: raylet worker pool)."""
        extra = dict(self.worker_env)
        renv = env or {}
        noset = (renv.get("env_vars") or {}).get("CAAMD_NOSET_ROCR_VISIBLE_DEVICES")
        if gpu_ids and not noset:
            extra["ROCR_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpu_ids)
        for k, v in (renv.get("env_vars") or {}).items():
            extra[k] = str(v)
        if renv:
            import json

            extra["CAAMD_RUNTIME_ENV"] = json.dumps(renv)
        extra["CAAMD_GPU_IDS"] = ",".join(str(g) for g in gpu_ids)
        extra["CAAMD_SYS_PATH"] = os.pathsep.join(p for p in sys.path if p and os.path.isdir(p))
        self._send(self.node_conns.get(node), ("spawn", worker_id.hex(), list(gpu_ids), extra))
        w = WorkerInfo(worker_id=worker_id, pid=None, node=node, gpu_key=tuple(gpu_ids),
                       kind="worker", proc=None, alive=False, env_key=_env_key(env))
        self.workers[worker_id] = w
        return w

    def _dispatch_to(self, w: WorkerInfo, spec: TaskSpec):
        w.idle = False
        w.task = spec.task_id
        spec.worker = w.worker_id
        spec.node = w.node
        spec.state = "running"
        spec.start_time = time.time()
        self.events.append(("start", spec.task_id, spec.fn_name, spec.start_time, w.pid))
        w.tasks_inflight[spec.task_id] = spec
        self._send(w.conn, ("execute", self._exec_payload(w, spec)))

    def _exec_payload(self, w, spec):
        fn_blob = None
        if spec.fn_id is not None and spec.fn_id not in w.fns:
            fn_blob = self.functions.get(spec.fn_id)
            w.fns.add(spec.fn_id)
        resolved = {}
        for r in spec.arg_refs:
            resolved[r] = self._obj_payload(r, w.node)
        return (spec, fn_blob, resolved)

    def _h_fetch_fn(self, c, req, fn_id):
        self._reply(c, req, self.functions.get(fn_id))

    def _h_task_done(self, c, task_id, results, error_kind, retryable):
        spec = self.tasks.get(task_id)
        w = self.conn_worker.get(c)
        if w is not None:
            w.tasks_inflight.pop(task_id, None)
        if spec is None:
            run = self.reattached_running.pop(task_id, None)
            if run is not None:
                # finished on a worker that outlived the previous head before its owner
                # re-sent the task: keep the results for the owner's resubmission
                for (oid, inline, size, node_hex, contained, is_err) in results:
                    self._obj(oid)
                    self._seal_object(oid, inline, size, node_hex, contained, is_err)
                if run[2]:
                    self.sched.release(run[1], run[2])
                if w is not None and w.actor_id is None and not w.tasks_inflight and w.lease is None:
                    w.idle = True
                    self.idle[(w.node, w.gpu_key, w.env_key)].append(w)
                    self._schedule()
            return
        self.events.append(("end", task_id, spec.fn_name, time.time(), w.pid if w else None))
        if error_kind == "app" and retryable and spec.attempt < (spec.max_retries or 0) and not spec.cancelled:
            spec.attempt += 1
            self._release(spec)
            self._finish_worker(w, spec)
            spec.state = "pending"
            self._on_deps_ready(spec)
            return
        spec.state = "finished" if not error_kind else "failed"
        for (oid, inline, size, node_hex, contained, is_err) in results:
            self._seal_object(oid, inline, size, node_hex, contained, is_err)
        if spec.generator is not None:
            self._gen_end(task_id, len(results) if spec.generator == "dynamic" else None)
        self._release(spec)
        if spec.kind == ACTOR_METHOD:
            a = self.actors.get(spec.actor_id)
            if a is not None:
                a.inflight.pop(task_id, None)
                self._pump_actor(a)
        elif spec.kind == ACTOR_CREATE:
            a = self.actors.get(spec.actor_id)
            if a is not None:
                if error_kind:
                    detail = ""
                    for (_o, inline, _s, _n, _c, is_err) in results:
                        if is_err and inline is not None:
                            try:
                                detail = str(serialization.deserialize(inline))
                            except Exception:
                                pass
                    self._set_actor_state(a, "DEAD")
                    a.death_cause = "creation task failed" + (f": {detail}" if detail else "")
                    self._fail_actor_queue(a, "ActorDiedError",
                                           "actor constructor raised" + (f":\n{detail}" if detail else ""))
                    self._kill_worker(a.worker)
                else:
                    self._set_actor_state(a, "ALIVE")
                    self._pump_actor(a)
        else:
            self._finish_worker(w, spec)
        self._task_cleanup(spec)
        self._schedule()

    def _task_cleanup(self, spec):
        if spec.kind == ACTOR_CREATE:
            return  # creation args stay pinned for restarts; released when the actor dies
        retained = self._lineage_retain(spec)
        for r in list(spec.arg_refs) + list(spec.pinned_refs or ()):
            e = self.objects.get(r)
            if e is not None:
                e.pins -= 1
                self._maybe_free(r)
        for oid in spec.return_ids or ():
            self._maybe_free(oid)
        if spec.kind != ACTOR_CREATE:
            self.tasks.pop(spec.task_id, None)
        if retained:
            self._lineage_release_if_unused(spec.task_id)

    def _finish_worker(self, w, spec):
        if w is None or not w.alive or w.actor_id is not None:
            return
        w.task = None
        w.idle = True
        self.idle[(w.node, w.gpu_key, w.env_key)].append(w)

    def _release(self, spec):
        if spec.acquired and spec.kind != ACTOR_CREATE:
            node, demand = spec.acquired
            self.sched.release(node, demand)
            self._give_gpus(node, spec.gpu_ids or (), float(spec.resources.get("GPU", 0) or 0))
            spec.acquired = None
            self._retry_pending_pgs()
            self._retry_infeasible()

    def _retry_infeasible(self):
        if not self.infeasible:
            return
        still = []
        for spec in self.infeasible:
            node = self._pick(spec)
            if node == "!":
                still.append(spec)
            else:
                self._enqueue_ready(spec)
        self.infeasible = still

    def _fail_task(self, spec, err):
        from ..exceptions import (ActorDiedError, OutOfMemoryError, RayError, TaskCancelledError,
                                  TaskPlacementGroupRemoved, WorkerCrashedError)

        kind, msg = err
        from ..exceptions import RuntimeEnvSetupError

        cls = {"ActorDiedError": ActorDiedError, "TaskCancelledError": TaskCancelledError,
               "WorkerCrashedError": WorkerCrashedError, "OutOfMemoryError": OutOfMemoryError,
               "TaskPlacementGroupRemoved": TaskPlacementGroupRemoved,
               "RuntimeEnvSetupError": RuntimeEnvSetupError}.get(kind, RayError)
        exc = cls(msg) if cls is not TaskCancelledError else TaskCancelledError(spec.task_id.hex(), msg)
        blob = serialization.serialize(exc).to_bytes()
        spec.state = "failed"
        for oid in spec.return_ids or ():
            self._seal_object(oid, blob, len(blob), None, (), True)
        if spec.generator is not None:
            self._gen_end(spec.task_id, 0, error=blob)
        self._release(spec)
        self._task_cleanup(spec)

    # ----------------------------------------------------------- generators
    def _h_gen_item(self, c, task_id, index, oid, inline, size, node_hex, contained, is_err=False):
        st = self.gen_stats.get(task_id)
        if st is None:
            if len(self.gen_stats) > 4096:
                self.gen_stats.pop(next(iter(self.gen_stats)))
            st = self.gen_stats[task_id] = {"produced": 0, "max_outstanding": 0}
        st["produced"] = max(st["produced"], index + 1)
        st["max_outstanding"] = max(st["max_outstanding"], index + 1 - self.gen_consumed.get(task_id, 0))
        self._obj(oid).refcount += 1  # held by the generator object on the owner side
        self._seal_object(oid, inline, size, node_hex, contained, is_err)
        for cb in list(self.gen_waiters.get((task_id, index), [])):
            cb()
        self.gen_waiters.pop((task_id, index), None)

    def _gen_end(self, task_id, count, error=None):
        key = ("__gen_end__", task_id)
        self.kv[key] = (count, error)
        self.gen_consumed.pop(task_id, None)
        self.gen_consume_waiters.pop(task_id, None)
        for k in [k for k in self.gen_waiters if k[0] == task_id]:
            for cb in self.gen_waiters.pop(k):
                cb()

    # ---- generator backpressure (reference: remote_function.py:396
    # _generator_backpressure_num_objects): the consumer asking for item k has taken
    # items 0..k-1; a producer with k unconsumed items waits in gen_wait.
    def _gen_consumed_to(self, task_id, n):
        if n <= self.gen_consumed.get(task_id, 0):
            return
        self.gen_consumed[task_id] = n
        waiters = self.gen_consume_waiters.get(task_id)
        if waiters:
            keep = []
            for (wc, wreq, need) in waiters:
                if n >= need:
                    self._reply(wc, wreq, n)
                else:
                    keep.append((wc, wreq, need))
            self.gen_consume_waiters[task_id] = keep

    def _h_gen_wait(self, c, req, task_id, need):
        have = self.gen_consumed.get(task_id, 0)
        if have >= need or ("__gen_end__", task_id) in self.kv:
            self._reply(c, req, have)
        else:
            self.gen_consume_waiters.setdefault(task_id, []).append((c, req, need))

    def _h_gen_drop(self, c, task_id):
        """The consumer dropped its generator: never hold the producer back again."""
        self._gen_consumed_to(task_id, 1 << 62)

    def _h_gen_next(self, c, req, task_id, index):
        self._gen_consumed_to(task_id, index)
        oid = ObjectID.for_task_return(task_id, index)

        def answer():
            e = self.objects.get(oid)
            if e is not None and e.state == READY:
                self._reply(c, req, ("item", oid))
                return True
            end = self.kv.get(("__gen_end__", task_id))
            if end is not None:
                count, err = end
                if err is not None and index == 0:
                    self._reply(c, req, ("error", err))
                else:
                    self._reply(c, req, ("end", None))
                return True
            return False

        if not answer():
            self.gen_waiters[(task_id, index)].append(answer)

    # ------------------------------------------------------------------ pubsub
    # Reference: src/ray/pubsub/publisher.h:297 -- the GCS publishes actor and node
    # state changes to subscribers (core workers, raylets, Serve). Here a
    # subscriber sends ("subscribe", channel); every change is pushed as
    # ("pub", channel, key, info) on its control connection, in order.
    CHANNELS = ("actor", "node")

    def _h_subscribe(self, c, channel):
        if channel in self.CHANNELS:
            self.subscribers.setdefault(channel, set()).add(c)

    def _h_unsubscribe(self, c, channel):
        self.subscribers.get(channel, set()).discard(c)

    def _publish(self, channel, key, info):
        subs = self.subscribers.get(channel)
        if not subs:
            return
        for sc in list(subs):
            if sc.closed:
                subs.discard(sc)
                continue
            self._send(sc, ("pub", channel, key, info))

    def _cluster_event(self, severity: str, source: str, message: str, **fields):
        self.cluster_events.append({"event_id": next(self._event_seq), "severity": severity,
                                    "source_type": source, "message": message, "time": time.time(),
                                    "custom_fields": fields})

    def _set_actor_state(self, a, state):
        if a.state == state:
            return
        if state == "DEAD":
            self._cluster_event("WARNING" if a.death_cause else "INFO", "GCS",
                                f"actor {a.class_name} {a.actor_id.hex()[:12]} died: {a.death_cause or 'exited'}",
                                actor_id=a.actor_id.hex(), pid=a.pid, node_id=a.node)
        elif state == "RESTARTING":
            self._cluster_event("WARNING", "GCS", f"actor {a.class_name} {a.actor_id.hex()[:12]} is restarting",
                                actor_id=a.actor_id.hex())
        a.state = state
        self._publish("actor", a.actor_id, {"state": state, "name": a.name, "namespace": a.namespace,
                                            "class_name": a.class_name, "pid": a.pid, "node": a.node,
                                            "death_cause": a.death_cause if state == "DEAD" else None})

    # ------------------------------------------------------------------ actors
    def _register_actor(self, spec, c):
        opts = spec.actor_opts or {}
        a = ActorInfo(actor_id=spec.actor_id, spec=spec, state="PENDING_CREATION",
                      name=opts.get("name"), namespace=opts.get("namespace") or self.namespace,
                      restarts_left=opts.get("max_restarts", 0) or 0,
                      max_task_retries=opts.get("max_task_retries", 0) or 0,
                      class_name=spec.fn_name, lifetime=opts.get("lifetime"),
                      owner=self.clients.get(c, {}).get("id"))
        self.actors[spec.actor_id] = a
        if a.name:
            self.named_actors[(a.namespace, a.name)] = spec.actor_id
        if self.gcs is not None and spec.actor_id not in self._gcs_actors:
            # every actor: a restarted head re-attaches re-registering actor workers to it
            if self.gcs.actor_put(spec, a.owner, a.lifetime):
                self._gcs_actors.add(spec.actor_id)
        # the creator's handle: an always-READY object whose refcount = live handles
        hid = spec.actor_id + b"\xac" * 8
        he = self._obj(hid)
        he.refcount += 1
        he.state = READY
        he.inline = b""
        self.handle_objs[hid] = spec.actor_id

    # ----------------------------------------------------- direct actor calls
    def _h_actor_addr(self, c, req, actor_id):
        """Where to send direct calls (core/direct.py): (state, unix address, node)."""
        a = self.actors.get(actor_id)
        if a is None:
            self._reply(c, req, (None, None, None))
            return
        w = self.workers.get(a.worker) if a.worker is not None else None
        if a.state == "ALIVE" and w is not None and w.alive:
            self._reply(c, req, ("ALIVE", w.direct_addr, w.node))
        else:
            self._reply(c, req, (a.state, None, None))

    def _h_dpin(self, c, task_id, oids):
        if task_id in self.dsealed_early:  # the caller's seal (which pins them) came first
            self.dsealed_early.discard(task_id)
            return
        for o in oids:
            self._obj(o).pins += 1
        self.dpins.setdefault(task_id, []).extend(oids)

    def _h_dseal(self, c, task_id, fn_name, results, dropped, t0, t1, pid):
        """A caller registers the results of a direct actor call (it holds one
        reference to each return object unless it already dropped it)."""
        drop = set(dropped or ())
        self.events.append(("start", task_id, fn_name, t0, pid))
        self.events.append(("end", task_id, fn_name, t1, pid))
        for (oid, inline, size, node_hex, contained, is_err) in results:
            e = self._obj(oid)
            if oid not in drop:
                e.refcount += 1
            self._seal_object(oid, inline, size, node_hex, contained, is_err)
            self._maybe_free(oid)
        pinned = self.dpins.pop(task_id, None)
        if pinned is None:
            if any(r[4] for r in results):
                self.dsealed_early.add(task_id)
            return
        for o in pinned:
            e = self.objects.get(o)
            if e is not None:
                e.pins -= 1
                self._maybe_free(o)

    def _h_dseal_batch(self, c, items):
        for it in items:
            self._h_dseal(c, *it)

    def _h_lseal(self, c, items):
        """An owner registers results it kept local so far (core/lease.py: inline
        direct-call results are sealed at the head only when their ref escapes the
        owner process). The owner holds one reference to each."""
        for (oid, inline, size, is_err) in items:
            self._obj(oid).refcount += 1
            self._seal_object(oid, inline, size, None, (), is_err)

    # ------------------------------------------------------- task worker leases
    # Reference role: raylet HandleRequestWorkerLease / ReturnWorker
    # (src/ray/raylet/node_manager.cc) + direct_task_transport.cc. An owner with a
    # backlog of normal tasks leases workers of its own node for one resource shape
    # and pushes tasks straight to them (core/lease.py); the head only grants,
    # parks (FIFO) and takes back leases.
    def _grant_leases(self, c, node, demand, want, gamt=0.0, env=None):
        """Grant up to ``want`` workers of ``node`` for one scheduling key: the
        resource demand (placement-group bundle resources for PG tasks), whole or
        fractional GPUs pinned to the lease (the worker was spawned with those GPU
        ids visible), and the runtime env's worker pool."""
        out = []
        ek = _env_key(env)
        while len(out) < want:
            gpu_ids = self._pick_gpus(node, gamt)
            if gpu_ids is None:
                break
            key = (node, gpu_ids, ek)
            if not self.sched.acquire(node, demand):
                break
            idle = self.idle.get(key)
            w = None
            while idle:
                cand = idle.pop()
                if cand.alive and cand.idle and cand.direct_addr:
                    w = cand
                    break
            if w is None:
                # no idle worker: start as many as the rest of the request can use
                # right now (resources permitting), not one per round trip
                n_fit = 1
                while n_fit < want - len(out) and self.sched.acquire(node, demand):
                    n_fit += 1
                for _ in range(n_fit):
                    self.sched.release(node, demand)
                if gamt > 0:
                    n_fit = 1  # GPU ids are picked per worker
                for _ in range(n_fit):
                    if self.starting[key] >= max(1, int(self.cpu_count)):
                        break
                    if self._num_workers(node) >= self.max_workers and ek is not None:
                        self._evict_idle(node, key)
                    if self._num_workers(node) >= self.max_workers:
                        break
                    self._spawn_worker(node, gpu_ids, env=env)
                break
            self._take_gpus(node, gpu_ids, gamt)
            w.idle = False
            w.task = None
            w.lease = (c, demand, time.time())
            w.lease_blocked = None
            w.lease_gpus = (gpu_ids, gamt) if gpu_ids else None
            out.append((w.worker_id, w.direct_addr))
        return out

    def _h_lease(self, c, req, resources, want, opts=None):
        node = self.clients.get(c, {}).get("node") or self.head_hex
        strategy = (opts or {}).get("strategy")
        env = (opts or {}).get("env") or None
        if strategy is not None and (strategy[0] != "pg" or strategy[1] not in self.pgs):
            self._reply(c, req, "never")  # removed group / other strategy: the head path decides
            return
        ek = _env_key(env)
        if ek is not None and ek in self.env_failures:
            self._reply(c, req, "never")  # the head path fails the tasks with RuntimeEnvSetupError
            return
        gamt = float(resources.get("GPU", 0) or 0)
        demand = {k: float(v) for k, v in self._demand_for(
            {k: v for k, v in resources.items() if v}, strategy).items() if v}
        if node not in self.node_resources and node != self.head_hex:
            self._reply(c, req, "never")
            return
        if self.sched.pick_node(demand, 2, node, False, self.node_id.hex(), [], []) == "!":
            self._reply(c, req, "never")  # the owner's node can never run this shape (or bundle)
            return
        got = self._grant_leases(c, node, demand, max(1, int(want)), gamt, env)
        if got:
            self._reply(c, req, got)
            return
        if strategy is None:
            other = self.sched.pick_node(demand, 0, "", False, self.node_id.hex(), [], [])
            if other not in ("", "!") and other != node:
                self._reply(c, req, "spill")  # another node has room now: send through the head
                return
        self.lease_waiters.append((c, req, node, demand, max(1, int(want)), gamt, env))

    def _serve_lease_waiters(self):
        still = []
        for ent in self.lease_waiters:
            c, req, node, demand, want, gamt, env = ent
            if c.closed:
                continue
            got = self._grant_leases(c, node, demand, want, gamt, env)
            if got:
                self._reply(c, req, got)
            else:
                still.append(ent)
        self.lease_waiters = still

    def _lease_release(self, w):
        _c, demand, _t = w.lease
        rel = dict(demand)
        for k, v in (w.lease_blocked or {}).items():
            rel[k] = rel.get(k, 0.0) - v  # lent back while blocked in get()
        self.sched.release(w.node, rel)
        if getattr(w, "lease_gpus", None):
            self._give_gpus(w.node, *w.lease_gpus)
        w.lease = None
        w.lease_blocked = None
        w.lease_gpus = None
        self._retry_pending_pgs()
        self._retry_infeasible()

    def _h_lease_return(self, c, worker_ids):
        for wid in worker_ids:
            w = self.workers.get(wid)
            if w is None or w.lease is None or w.lease[0] is not c:
                continue
            self._lease_release(w)
            if w.alive and w.actor_id is None:
                w.idle = True
                self.idle[(w.node, w.gpu_key, w.env_key)].append(w)
        self._schedule()

    def _h_worker_fate(self, c, req, worker_id):
        self._reply(c, req, "oom" if worker_id in self.oom_killed_ids else "crash")

    def _h_check_name(self, c, req, namespace, name):
        aid = self.named_actors.get((namespace or self.namespace, name))
        if aid is not None and self.actors.get(aid) and self.actors[aid].state != "DEAD":
            a = self.actors[aid]
            self._reply(c, req, (aid, a.spec.actor_opts.get("handle_meta")))
        else:
            self._reply(c, req, None)

    def _start_actor_on(self, a: ActorInfo, w: WorkerInfo):
        w.actor_id = a.actor_id
        w.idle = False
        a.worker = w.worker_id
        a.pid = w.pid
        spec = a.spec
        spec.worker = w.worker_id
        spec.node = w.node
        spec.state = "running"
        spec.start_time = time.time()
        self._set_actor_state(a, "PENDING_CREATION" if a.num_restarts == 0 else "RESTARTING")
        self.events.append(("start", spec.task_id, spec.fn_name, spec.start_time, w.pid))
        w.tasks_inflight[spec.task_id] = spec
        self._send(w.conn, ("execute", self._exec_payload(w, spec)))

    def _pump_actor(self, a: ActorInfo):
        if a.state == "DEAD":
            self._fail_actor_queue(a, "ActorDiedError", a.death_cause or "actor is dead")
            return
        if a.state != "ALIVE":
            return
        w = self.workers.get(a.worker)
        if w is None or not w.alive:
            return
        batch = []
        while a.queue:
            spec = a.queue.popleft()
            if spec.cancelled:
                continue
            spec.worker = w.worker_id
            spec.node = w.node
            spec.state = "running"
            spec.start_time = time.time()
            a.inflight[spec.task_id] = spec
            w.tasks_inflight[spec.task_id] = spec
            self.events.append(("start", spec.task_id, spec.fn_name, spec.start_time, w.pid))
            batch.append(("execute", self._exec_payload(w, spec)))
        if batch and w.conn is not None:
            try:
                w.conn.send_many(batch)
            except (ConnectionClosed, OSError):
                pass  # the actor's connection is going away; its death handling fails the calls

    def _fail_actor_queue(self, a, kind, msg):
        while a.queue:
            self._fail_task(a.queue.popleft(), (kind, msg))
        for tid, spec in list(a.inflight.items()):
            self._fail_task(spec, (kind, msg))
        a.inflight.clear()

    def _on_handles_gone(self, actor_id):
        """No handle left: terminate an unnamed, non-detached actor once its queued
        calls have run (a __ray_terminate__ call appended to its queue)."""
        a = self.actors.get(actor_id)
        if a is None or a.name or a.lifetime == "detached" or a.state == "DEAD":
            return
        a.restarts_left = 0
        a.death_cause = "all references to the actor were removed"
        term = TaskSpec(task_id=os.urandom(16), kind=ACTOR_METHOD, fn_name="__ray_terminate__",
                        args=[], kwargs={}, arg_refs=[], num_returns=0, return_ids=[],
                        actor_id=actor_id, method="__ray_terminate__", max_retries=0)
        term.state = "pending"
        self.tasks[term.task_id] = term
        a.queue.append(term)
        self._pump_actor(a)

    def _h_kill_actor(self, c, actor_id, no_restart):
        a = self.actors.get(actor_id)
        if a is None:
            return
        if no_restart:
            a.restarts_left = 0
        a.death_cause = "killed by ray.kill"
        self._kill_worker(a.worker)

    def _kill_worker(self, worker_id):
        w = self.workers.get(worker_id)
        if w is None:
            return
        try:
            os.kill(w.pid, signal.SIGKILL)
        except (ProcessLookupError, TypeError):
            pass

    def _h_actor_exit(self, c, actor_id):
        a = self.actors.get(actor_id)
        if a is not None:
            a.restarts_left = 0
            a.death_cause = "exit_actor() was called"

    def _on_actor_worker_death(self, a: ActorInfo, w: WorkerInfo):
        if a.acquired:
            node, demand = a.acquired
            if a.restarts_left == 0 or a.restarts_left is None:
                self.sched.release(node, demand)
                self._give_gpus(node, a.gpu_ids or (), float(a.spec.resources.get("GPU", 0) or 0))
                a.acquired = None
        if a.restarts_left and a.restarts_left != 0 and a.state != "DEAD":
            if a.restarts_left > 0:
                a.restarts_left -= 1
            a.num_restarts += 1
            self._set_actor_state(a, "RESTARTING")
            retry = a.max_task_retries != 0
            for tid, spec in list(a.inflight.items()):
                if retry:
                    a.queue.appendleft(spec)
                else:
                    self._fail_task(spec, ("ActorDiedError", "actor died while running the task"))
            a.inflight.clear()
            wid = os.urandom(16)
            self.pending_spawn[wid] = ("actor", a.actor_id)
            self._spawn_worker(a.node, a.gpu_ids or (), worker_id=wid, env=a.spec.runtime_env)
            return
        # the cause first: the DEAD transition's cluster event takes its severity from it
        a.death_cause = a.death_cause or "the actor's worker process died"
        self._set_actor_state(a, "DEAD")
        self._fail_actor_queue(a, "ActorDiedError", a.death_cause)
        if a.name:
            self.named_actors.pop((a.namespace, a.name), None)
        spec = a.spec
        if spec is not None:
            for r in list(spec.arg_refs) + list(spec.pinned_refs or ()):
                e = self.objects.get(r)
                if e is not None:
                    e.pins -= 1
                    self._maybe_free(r)
            spec.arg_refs = []
            spec.pinned_refs = []

    # ------------------------------------------------------------ disconnects
    def _on_disconnect(self, c: Conn):
        try:
            self.sel.unregister(c.sock)
        except (KeyError, ValueError):
            pass
        c.close()
        for subs in self.subscribers.values():
            subs.discard(c)
        info = self.clients.pop(c, {})
        w = self.conn_worker.pop(c, None)
        for lw in [x for x in self.workers.values() if x.lease is not None and x.lease[0] is c]:
            # the owner is gone: take its leases back and stop what they were running
            self._lease_release(lw)
            self._kill_worker(lw.worker_id)
        if info.get("kind") == "node":
            self._on_node_death(info.get("node"))
            return
        if w is None:
            if info.get("kind") == "driver":
                self._on_driver_exit(info.get("id"))
            return
        w.alive = False
        w.idle = False
        if w.lease is not None:
            self._lease_release(w)
        try:
            if w.proc is not None:
                w.proc.wait(timeout=1)
        except Exception:
            pass
        if w.actor_id is not None:
            a = self.actors.get(w.actor_id)
            if a is not None and a.worker == w.worker_id:
                self._on_actor_worker_death(a, w)
        for tid, spec in list(w.tasks_inflight.items()):
            if spec.kind != NORMAL:
                continue
            self._release(spec)
            mr = spec.max_retries if spec.max_retries is not None else 3
            if spec.cancelled:
                self._fail_task(spec, ("TaskCancelledError", "task was cancelled"))
            elif mr < 0 or spec.attempt < mr:
                spec.attempt += 1
                spec.state = "pending"
                self._enqueue_ready(spec)
            elif w.oom_killed:
                self._fail_task(spec, ("OutOfMemoryError", (
                    "Task was killed due to the node running low on memory (memory monitor "
                    f"threshold {self.mem_monitor.threshold:.2f}); retries exhausted.")))
            else:
                self._fail_task(spec, ("WorkerCrashedError", "the worker died while running the task"))
                self._cluster_event("ERROR", "RAYLET", f"worker {w.pid} died while running {spec.fn_name}",
                                    worker_id=w.worker_id.hex(), task_id=spec.task_id.hex(), node_id=w.node)
        w.tasks_inflight.clear()
        self.workers.pop(w.worker_id, None)
        self._schedule()

    def _on_driver_exit(self, driver_id):
        # non-detached actors owned by the driver die with it (reference: actor lifetimes)
        for a in list(self.actors.values()):
            if a.owner == driver_id and a.lifetime != "detached" and a.state != "DEAD":
                a.restarts_left = 0
                a.death_cause = "owner exited"
                self._kill_worker(a.worker)

    # ------------------------------------------------------------ OOM killer
    def _check_memory(self, now):
        """Kill one worker when the node is over the memory threshold (see
        core/memory_monitor.py; reference: raylet MemoryMonitor + worker killing policy)."""
        if now < self._oom_quiet_until:
            return
        frac = self.mem_monitor.over_threshold()
        if frac is None:
            return
        from .memory_monitor import pick_victim

        cands = []
        for w in self.workers.values():
            if not w.alive or w.node != self.head_hex or w.oom_killed:
                continue
            if w.actor_id is not None:
                a = self.actors.get(w.actor_id)
                if a is None or a.state == "DEAD":
                    continue
                start = a.spec.start_time if a.spec is not None and a.spec.start_time else 0.0
                cands.append((w, bool(a.restarts_left), start))
            elif w.tasks_inflight:
                spec = next(iter(w.tasks_inflight.values()))
                mr = spec.max_retries if spec.max_retries is not None else 3
                cands.append((w, mr < 0 or spec.attempt < mr, spec.start_time or 0.0))
            elif w.lease is not None:
                cands.append((w, True, w.lease[2]))
        w = pick_victim(cands)
        if w is None:
            return
        w.oom_killed = True
        self.oom_killed_ids.add(w.worker_id)
        self.mem_monitor.kills += 1
        self.events.append(("oom_kill", w.worker_id.hex(), time.time(), frac))
        self._cluster_event("ERROR", "RAYLET", f"memory monitor killed worker {w.pid} at {frac:.0%} node memory",
                            worker_id=w.worker_id.hex(), node_id=w.node, memory_fraction=frac)
        if w.actor_id is not None:
            a = self.actors.get(w.actor_id)
            if a is not None:
                a.death_cause = (f"the actor's worker was killed by the memory monitor: node memory "
                                 f"usage {frac:.2f} >= threshold {self.mem_monitor.threshold:.2f}")
        self._kill_worker(w.worker_id)
        # let the kernel reclaim the victim's memory before judging again
        self._oom_quiet_until = now + max(1.0, 4 * self.mem_monitor.refresh_s)

    def _gcs_reconcile(self):
        """Drop persisted detached actors that are now permanently dead (not while the
        head is going down: its own shutdown kills every worker)."""
        if not self.running:
            return
        for aid in list(self._gcs_actors):
            a = self.actors.get(aid)
            if a is None or a.state == "DEAD":
                self._gcs_actors.discard(aid)
                self.gcs.actor_del(aid)

    def _gcs_restore(self):
        """Reload the durable tables written by a previous head with the same storage
        (reference: GcsInitData::AsyncLoad + GcsActorManager / GcsPlacementGroupManager
        Initialize on GCS restart)."""
        data = self.gcs.load()
        self.kv.update(data["kv"])
        self.functions.update(data["fn"])
        for jid, info in data["job"].items():
            self.jobs.setdefault(jid, dict(info, restored=True))
        for pg_id, pg in data["pg"].items():
            self._h_pg_create(None, pg_id, pg["bundles"], pg["strategy"], pg["name"],
                              pg_id + b"\xb7" * 4, pg["lifetime"])
        n_actors = 0
        for aid, rec in data["actor"].items():
            self._gcs_actors.add(aid)  # already persisted: keep the record, do not rewrite it
            if self.reattached:
                # the node outlived the old head: wait for the actor's worker to re-register
                self._actor_placeholder(aid, rec)
                n_actors += 1
            elif rec.get("lifetime") == "detached" and rec.get("restorable", True):
                self._recreate_actor(rec["fields"])
                n_actors += 1
            else:
                self._gcs_actors.discard(aid)
                self.gcs.actor_del(aid)
        if self.reattached:
            self._reattaching = True
            self._timer(self.reattach_s, self._reattach_expired)
        self.gcs_restored = {"kv": len(data["kv"]), "functions": len(data["fn"]), "jobs": len(data["job"]),
                             "placement_groups": len(data["pg"]), "actors": n_actors,
                             "reattach": self.reattached}

    def _recreate_actor(self, fields, queue=()):
        spec = TaskSpec(**fields)
        spec.task_id = os.urandom(16)
        spec.attempt = 0
        spec.return_ids = [os.urandom(len(r)) for r in (fields.get("return_ids") or [])]
        self._h_submit(None, spec)
        a = self.actors.get(spec.actor_id)
        if a is not None:
            a.queue.extend(queue)

    def _actor_placeholder(self, aid, rec):
        fields = rec["fields"]
        spec = TaskSpec(**fields)
        opts = spec.actor_opts or {}
        a = ActorInfo(actor_id=aid, spec=spec, state="RECONNECTING", name=opts.get("name"),
                      namespace=opts.get("namespace") or self.namespace,
                      restarts_left=opts.get("max_restarts", 0) or 0,
                      max_task_retries=opts.get("max_task_retries", 0) or 0, class_name=spec.fn_name,
                      lifetime=rec.get("lifetime"), owner=rec.get("owner"))
        a.record = rec
        self.actors[aid] = a
        if a.name:
            self.named_actors[(a.namespace, a.name)] = aid
        hid = aid + b"\xac" * 8
        he = self._obj(hid)
        he.refcount += 1
        he.state = READY
        he.inline = b""
        self.handle_objs[hid] = aid

    # ------------------------------------------------- re-attach after restart
    def _h_reregister(self, c, kind, worker_id, pid, node_hex, extra):
        """A worker / driver that outlived the previous head reconnects (reference:
        core workers and raylets re-registering with a restarted GCS): rebuild its
        worker record, re-attach its actor, take back the resources it holds, and
        rebuild the object directory entries it references."""
        extra = extra or {}
        node = node_hex or self.head_hex
        self.clients[c] = {"id": worker_id, "kind": kind, "pid": pid, "node": node}
        self._send(c, ("registered", {"store_name": self.node_store.get(node, self.store_name), "node_id": node,
                                      "namespace": self.namespace, "session_dir": self.session_dir,
                                      "reconnect_s": self.reconnect_s, "reattached": True}))
        self._reattach_refs(extra)
        if kind == "driver":
            self.reattach_stats["drivers"] += 1
            jid = extra.get("job_id", b"")
            self.jobs.setdefault(jid, {"start": time.time(), "pid": pid, "driver": worker_id})
            self._reattach_leases(c, extra.get("leases") or ())
            return
        if kind != "worker":
            return
        self.reattach_stats["workers"] += 1
        w = WorkerInfo(worker_id=worker_id, pid=pid, node=node, gpu_key=tuple(extra.get("gpu_ids") or ()),
                       kind="worker", alive=True, conn=c, env_key=_env_key(extra.get("runtime_env")))
        w.started = time.time()
        w.client_id = worker_id
        w.direct_addr = extra.get("direct")
        self.workers[worker_id] = w
        self.conn_worker[c] = w
        aid = extra.get("actor_id")
        if aid is not None:
            a = self.actors.get(aid)
            if a is None or a.state != "RECONNECTING":
                self._kill_worker(worker_id)  # an actor this head has no record of (or replaced)
                return
            demand = self._demand(a.spec)
            if self.sched.acquire(node, demand):
                a.acquired = a.spec.acquired = (node, demand)
                gamt = float(a.spec.resources.get("GPU", 0) or 0)
                try:
                    self._take_gpus(node, w.gpu_key, gamt)
                except ValueError:
                    pass
            a.gpu_ids = w.gpu_key
            a.spec.gpu_ids = w.gpu_key
            a.node, a.worker, a.pid = node, worker_id, pid
            self._set_actor_state(a, "ALIVE")
            w.actor_id = aid
            w.idle = False
            self.reattach_stats["actors"] += 1
            self._pump_actor(a)
            return
        busy = False
        for (tid, res) in extra.get("running") or ():
            busy = True
            demand = {k: float(v) for k, v in (res or {}).items() if v}
            held = demand if demand and self.sched.acquire(node, demand) else {}
            self.reattached_running[tid] = (worker_id, node, held)
        for tid in extra.get("finishing") or ():
            self.reattached_running.setdefault(tid, (worker_id, node, {}))
        self._release_held(lambda sp: sp.task_id in self.reattached_running)
        parked = self._parked_leases.pop(worker_id, None)
        if parked is not None and not parked[0].closed:
            self._apply_reattached_lease(parked[0], w, parked[1])
            return
        if not busy:
            if self._reattaching:
                self._reattach_hold.append(w)  # its lease holder may still re-register
                return
            w.idle = True
            self.idle[(node, w.gpu_key, w.env_key)].append(w)
            self._schedule()

    def _reattach_refs(self, extra):
        """Object directory entries from a re-registering process's held refs: sealed
        in this node's arena, or an inline payload the process still holds."""
        inline = extra.get("inline") or {}
        for oid, n in (extra.get("refs") or {}).items():
            e = self._obj(oid)
            e.refcount += int(n)
            if e.state == READY:
                continue
            if oid in inline:
                blob, is_err = inline[oid]
                self._seal_object(oid, blob, len(blob), None, (), bool(is_err))
                self.reattach_stats["objects"] += 1
                continue
            try:
                hit = self.store.lookup(oid)
            except Exception:
                hit = None
            if hit is not None:
                self._seal_object(oid, None, int(hit[1]), self.head_hex, ())
                self.reattach_stats["objects"] += 1

    def _reattach_leases(self, c, leases):
        for ent in leases:
            wid = ent[0]
            w = self.workers.get(wid)
            if w is None:
                if self._reattaching:
                    self._parked_leases[wid] = (c, ent)  # applied when the worker re-registers
                continue
            self._apply_reattached_lease(c, w, ent)

    def _apply_reattached_lease(self, c, w, ent):
        """Restore one lease an owner held before the restart: the worker leaves the
        idle pool (or the re-attach hold) and its resources are taken back. If they
        cannot be (the node is over-committed now), the lease ends the way a dead
        lease ends: the worker is stopped and the owner's lease loop resubmits."""
        if w.lease is not None or w.actor_id is not None:
            return
        res = ent[1]
        opts = ent[2] if len(ent) > 2 else None
        strategy = (opts or {}).get("strategy")
        if strategy is not None and strategy[1] not in self.pgs:
            strategy = None
        demand = {k: float(v) for k, v in self._demand_for(
            {k: v for k, v in (res or {}).items() if v}, strategy).items() if v}
        if w in self._reattach_hold:
            self._reattach_hold.remove(w)
        if w.idle:
            w.idle = False
            lst = self.idle.get((w.node, w.gpu_key, w.env_key))
            if lst and w in lst:
                lst.remove(w)
        if demand and not self.sched.acquire(w.node, demand):
            self._kill_worker(w.worker_id)
            return
        gamt = float((res or {}).get("GPU", 0) or 0)
        w.lease_gpus = None
        if gamt and w.gpu_key:
            try:
                self._take_gpus(w.node, tuple(w.gpu_key), gamt)
                w.lease_gpus = (tuple(w.gpu_key), gamt)
            except ValueError:
                pass
        w.lease = (c, demand, time.time())

    def _release_held(self, pred):
        keep, go = [], []
        for (hc, sp) in self._held_resubmits:
            (go if pred(sp) else keep).append((hc, sp))
        self._held_resubmits = keep
        for (hc, sp) in go:
            if not hc.closed:
                self._h_submit(hc, sp)

    def _reattach_expired(self):
        """End of the re-attach grace: actors whose worker did not come back are
        re-created (detached, restorable) or dead; referenced objects that nothing
        will produce are lost."""
        from ..exceptions import ObjectLostError  # noqa: F401  (clients raise it for "lost" payloads)

        self._reattaching = False
        self._parked_leases.clear()  # their workers never came back: the owners see the loss
        hold, self._reattach_hold = self._reattach_hold, []
        for w in hold:
            if w.alive and w.lease is None and w.actor_id is None and self.workers.get(w.worker_id) is w:
                w.idle = True
                self.idle[(w.node, w.gpu_key, w.env_key)].append(w)
        for a in list(self.actors.values()):
            if a.state != "RECONNECTING":
                continue
            rec = a.record or {}
            if a.lifetime == "detached" and rec.get("restorable", True):
                self.reattach_stats["recreated_actors"] += 1
                q = list(a.queue)
                a.queue.clear()
                del self.actors[a.actor_id]
                self._recreate_actor(rec["fields"], q)
            else:
                self.reattach_stats["dead_actors"] += 1
                self._set_actor_state(a, "DEAD")
                a.death_cause = "the actor's worker did not reconnect after a head restart"
                if a.name:
                    self.named_actors.pop((a.namespace, a.name), None)
                self._fail_actor_queue(a, "ActorDiedError", a.death_cause)
        held, self._held_resubmits = self._held_resubmits, []
        for (hc, sp) in held:  # owners' replayed tasks nobody re-registered as running: run them now
            if not hc.closed:
                self._h_submit(hc, sp)
        for oid, e in list(self.objects.items()):
            if e.state == PENDING and e.refcount > 0 and e.owner_task is None:
                e.lost = True
                self.reattach_stats["lost_objects"] += 1
                self._seal_object(oid, None, 0, None, ())
        if hold:
            self._schedule()

    def _health_check(self):
        if self.gcs is not None and self._gcs_actors:
            self._gcs_reconcile()
        for w in list(self.workers.values()):
            if w.proc is not None and w.proc.poll() is not None and not w.alive and w.conn is None:
                # died before registering
                key = (w.node, w.gpu_key, w.env_key)
                self.starting[key] = max(0, self.starting[key] - 1)
                self.workers.pop(w.worker_id, None)
                pending = self.pending_spawn.pop(w.worker_id, None)
                if pending and pending[0] == "actor":
                    a = self.actors.get(pending[1])
                    if a is not None:
                        self._set_actor_state(a, "DEAD")
                        a.death_cause = "worker process failed to start (see session logs)"
                        self._fail_actor_queue(a, "ActorDiedError", a.death_cause)
                self._schedule()

    # ------------------------------------------------ blocked in ray.get
    def _h_blocked(self, c, task_id):
        """A worker blocked in get() lends its CPUs back (reference: raylet
        HandleNotifyWorkerBlocked) so nested tasks cannot deadlock the node."""
        spec = self.tasks.get(task_id)
        if spec is None:
            w = self.conn_worker.get(c)
            if w is not None and w.lease is not None and not w.lease_blocked:
                cpu = {k: v for k, v in w.lease[1].items() if k == "CPU" or k.startswith("CPU_group_")}
                if cpu:  # a leased worker's task blocked: lend its CPUs back
                    self.sched.release(w.node, cpu)
                    w.lease_blocked = cpu
                    self._schedule()
            return
        if spec.kind != NORMAL or not spec.acquired or spec.blocked:
            return
        node, demand = spec.acquired
        cpu = {k: v for k, v in demand.items() if k == "CPU" or k.startswith("CPU_group_")}
        if cpu:
            self.sched.release(node, cpu)
            spec.blocked = cpu
            self._schedule()

    def _h_unblocked(self, c, task_id):
        spec = self.tasks.get(task_id)
        if spec is None:
            w = self.conn_worker.get(c)
            if w is not None and w.lease is not None and w.lease_blocked:
                self.sched.release(w.node, {k: -v for k, v in w.lease_blocked.items()})
                w.lease_blocked = None
            return
        if not spec.blocked:
            return
        node, _ = spec.acquired
        # take the CPUs back even if that oversubscribes the node for a moment
        self.sched.release(node, {k: -v for k, v in spec.blocked.items()})
        spec.blocked = None

    # ------------------------------------------------------------------ cancel
    def _h_cancel(self, c, task_id, force, recursive):
        spec = self.tasks.get(task_id)
        if spec is None:
            return
        spec.cancelled = True
        if spec.state == "pending":
            self.waiting_deps.pop(task_id, None)
            if spec.kind == ACTOR_METHOD:
                a = self.actors.get(spec.actor_id)
                if a is not None and spec in a.queue:
                    a.queue.remove(spec)
            self._fail_task(spec, ("TaskCancelledError", "task was cancelled before it ran"))
        elif spec.state == "running":
            w = self.workers.get(spec.worker)
            if w is None:
                return
            if force and spec.kind == NORMAL:
                self._kill_worker(w.worker_id)
            else:
                self._send(w.conn, ("cancel", task_id))

    # ------------------------------------------------------- placement groups
    def _h_pg_create(self, c, pg_id, bundles, strategy, name, ready_oid, lifetime):
        codes = {"PACK": 0, "SPREAD": 1, "STRICT_PACK": 2, "STRICT_SPREAD": 3}
        self.pgs[pg_id] = {"bundles": bundles, "strategy": strategy, "name": name, "state": "PENDING",
                           "nodes": None, "ready_oid": ready_oid, "code": codes[strategy],
                           "lifetime": lifetime}
        self._obj(ready_oid).refcount += 1
        if self.gcs is not None and lifetime == "detached":
            self.gcs.pg_put(pg_id, bundles, strategy, name, lifetime)
        if not self.sched.pg_feasible(bundles, codes[strategy]):
            self.pgs[pg_id]["state"] = "INFEASIBLE"
        self.pending_pgs.append(pg_id)
        self._retry_pending_pgs()

    def _retry_pending_pgs(self):
        still = []
        for pg_id in self.pending_pgs:
            pg = self.pgs.get(pg_id)
            if pg is None:
                continue
            nodes = self.sched.reserve_pg(pg_id.hex(), pg["bundles"], pg["code"])
            if nodes or not pg["bundles"]:
                pg["nodes"] = nodes
                pg["state"] = "CREATED"
                blob = serialization.serialize(True).to_bytes()
                self._seal_object(pg["ready_oid"], blob, len(blob), None, ())
                self._schedule()
            else:
                still.append(pg_id)
        self.pending_pgs = still

    def _h_pg_remove(self, c, pg_id):
        pg = self.pgs.pop(pg_id, None)
        if pg is None:
            return
        if self.gcs is not None and pg.get("lifetime") == "detached":
            self.gcs.pg_del(pg_id)
        if pg_id in self.pending_pgs:
            self.pending_pgs.remove(pg_id)
        # actors placed in the group die with it (reference: ActorPlacementGroupRemoved)
        for a in list(self.actors.values()):
            st = a.spec.strategy if a.spec else None
            if st and st[0] == "pg" and st[1] == pg_id and a.state != "DEAD":
                a.restarts_left = 0
                a.death_cause = "placement group removed"
                if a.acquired:
                    # group resources vanish with the group; device ids go back to the node
                    self._give_gpus(a.acquired[0], a.gpu_ids or (), float(a.spec.resources.get("GPU", 0) or 0))
                    a.acquired = None
                w = self.workers.get(a.worker) if a.worker is not None else None
                if w is None or not w.alive:
                    # still being spawned / restarted: its worker must never start the actor
                    # (the device ids above may already belong to someone else)
                    for wid, pend in list(self.pending_spawn.items()):
                        if pend == ("actor", a.actor_id):
                            del self.pending_spawn[wid]
                            self._kill_worker(wid)
                    self._set_actor_state(a, "DEAD")
                    self._fail_actor_queue(a, "ActorDiedError", "placement group removed")
                self._kill_worker(a.worker)
        self.sched.remove_pg(pg_id.hex())
        self._retry_pending_pgs()
        self._schedule()

    def _h_pg_table(self, c, req, pg_id):
        def fmt(pid, pg):
            return {"placement_group_id": pid.hex(), "name": pg["name"], "strategy": pg["strategy"],
                    "state": pg["state"], "bundles": {i: b for i, b in enumerate(pg["bundles"])},
                    "bundles_to_node_id": {i: n for i, n in enumerate(pg["nodes"] or [])}}
        if pg_id is not None:
            pg = self.pgs.get(pg_id)
            self._reply(c, req, fmt(pg_id, pg) if pg else None)
        else:
            self._reply(c, req, {pid.hex(): fmt(pid, pg) for pid, pg in self.pgs.items()})

    def _h_pg_by_name(self, c, req, name):
        for pid, pg in self.pgs.items():
            if pg["name"] == name:
                self._reply(c, req, (pid, pg["bundles"], pg["strategy"]))
                return
        self._reply(c, req, None)

    # ------------------------------------------------------------- state API
    def _h_state(self, c, req, what, arg):
        self._reply(c, req, self.state(what, arg))

    def _h_metric(self, c, name, kind, desc, tag_keys, tags, value, boundaries):
        """Application metrics (reference: python/ray/util/metrics.py -> per-node
        metrics agent); aggregated here and exported by the dashboard's /metrics."""
        m = self.metrics.get(name)
        if m is None:
            m = self.metrics[name] = {"kind": kind, "desc": desc, "tag_keys": tuple(tag_keys),
                                      "boundaries": list(boundaries or []), "series": {}}
        key = tuple(tags)
        if kind == "counter":
            m["series"][key] = m["series"].get(key, 0.0) + value
        elif kind == "gauge":
            m["series"][key] = value
        else:  # histogram: (bucket counts, sum, count)
            b = m["boundaries"]
            cur = m["series"].get(key) or [[0] * (len(b) + 1), 0.0, 0]
            i = 0
            while i < len(b) and value > b[i]:
                i += 1
            cur[0][i] += 1
            cur[1] += value
            cur[2] += 1
            m["series"][key] = cur

    def state(self, what, arg=None):
        if what == "gen_stats":
            st = self.gen_stats.get(arg)
            return dict(st, consumed=self.gen_consumed.get(arg)) if st else None
        if what == "reattach_stats":
            return dict(self.reattach_stats, reattached=self.reattached, reattaching=self._reattaching)
        if what == "metrics":
            import copy

            return copy.deepcopy(self.metrics)
        if what == "cluster_resources":
            return self.sched.cluster_total()
        if what == "available_resources":
            return {k: v for k, v in self.sched.cluster_available().items()}
        if what == "available_per_node":
            return {n: self.sched.available(n) for n in self.sched.nodes()}
        if what == "nodes":
            out = []
            for n, info in self.node_info.items():
                d = dict(info)
                d["Resources"] = self.sched.total(n)
                out.append(d)
            return out
        if what == "actors":
            return [{"actor_id": a.actor_id.hex(), "class_name": a.class_name, "state": a.state,
                     "name": a.name or "", "namespace": a.namespace, "pid": a.pid,
                     "node_id": a.node, "num_restarts": a.num_restarts,
                     "death_cause": a.death_cause} for a in self.actors.values()]
        if what == "tasks":
            live = {t.task_id: {"task_id": t.task_id.hex(), "name": t.fn_name, "state": t.state,
                                "kind": ["NORMAL_TASK", "ACTOR_CREATION_TASK", "ACTOR_TASK"][t.kind],
                                "node_id": t.node, "attempt": t.attempt} for t in self.tasks.values()}
            # tasks the head no longer tracks (finished; or run on owner leases / direct
            # actor calls, which report only their task events): from the event buffer
            done: Dict[bytes, Dict[str, Any]] = {}
            for e in self.events:
                if e[0] not in ("submit", "start", "end") or not isinstance(e[1], (bytes, bytearray)):
                    continue
                if e[1] in live:
                    continue
                r = done.get(e[1])
                if r is None:
                    r = done[e[1]] = {"task_id": e[1].hex(), "name": e[2], "state": "PENDING_SCHEDULING",
                                      "kind": "NORMAL_TASK", "node_id": None, "attempt": 0}
                if e[0] == "start":
                    r["start_time_ms"] = int(e[3] * 1000) if e[3] else None
                    if len(e) > 4:
                        r["worker_pid"] = e[4]
                    if r["state"] != "FINISHED":
                        r["state"] = "RUNNING"
                elif e[0] == "end":
                    r["end_time_ms"] = int(e[3] * 1000)
                    r["state"] = "FINISHED"
            return list(live.values()) + list(done.values())
        if what == "objects":
            return [{"object_id": o.hex(), "state": ["PENDING", "READY", "FREED"][e.state],
                     "size": e.size, "inline": e.inline is not None, "ref_count": e.refcount,
                     "pins": e.pins, "spilled": e.spilled_path is not None,
                     "node_id": "inline" if e.inline is not None else (e.node or self.head_hex)}
                    for o, e in self.objects.items()]
        if what == "workers":
            return [{"worker_id": w.worker_id.hex(), "pid": w.pid, "node_id": w.node,
                     "alive": w.alive, "idle": w.idle, "actor_id": w.actor_id.hex() if w.actor_id else None,
                     "gpu_ids": list(w.gpu_key or ())} for w in self.workers.values()]
        if what == "placement_groups":
            return [{"placement_group_id": p.hex(), "name": g["name"], "state": g["state"],
                     "strategy": g["strategy"], "bundles": g["bundles"]} for p, g in self.pgs.items()]
        if what == "jobs":
            return [{"job_id": j.hex() if isinstance(j, bytes) else str(j), **v} for j, v in self.jobs.items()]
        if what == "events":
            return list(self.events)
        if what == "object_locations":
            out = {}
            for oid in arg or ():
                e = self.objects.get(oid)
                if e is None or e.state != READY:
                    continue
                inline = e.inline is not None
                out[oid] = {"node_ids": [] if inline else [e.node or self.head_hex], "size": e.size,
                            "spilled": e.spilled_path is not None}
            return out
        if what == "cluster_events":
            return list(self.cluster_events)
        if what == "runtime_envs":
            envs: Dict[Any, Dict[str, Any]] = {}
            for w in self.workers.values():
                if w.env_key is None:
                    continue
                e = envs.setdefault(w.env_key, {"runtime_env_key": w.env_key,
                                                "runtime_env": self.env_specs.get(w.env_key),
                                                "nodes": set(), "num_workers": 0,
                                                "success": w.env_key not in self.env_failures,
                                                "error": self.env_failures.get(w.env_key)})
                e["nodes"].add(w.node)
                e["num_workers"] += 1
            for k, err in self.env_failures.items():
                envs.setdefault(k, {"runtime_env_key": k, "runtime_env": self.env_specs.get(k), "nodes": set(),
                                    "num_workers": 0, "success": False, "error": err})
            return [dict(e, nodes=sorted(e["nodes"])) for e in envs.values()]
        if what == "store":
            return {"capacity": self.store.capacity, "used": self.store.used,
                    "num_objects": self.store.num_objects}
        if what == "actor":
            a = self.actors.get(arg)
            return None if a is None else {"state": a.state, "name": a.name, "pid": a.pid,
                                           "num_restarts": a.num_restarts}
        if what == "autoscaler":
            # resource demand the cluster cannot place right now (reference: GCS
            # autoscaler state: pending tasks/actors by shape + pending PG bundles)
            demand = []
            for q in self.ready_queues.values():
                for spec in q:
                    if not spec.cancelled and not (spec.strategy and spec.strategy[0] == "pg"):
                        demand.append(dict(spec.resources))
            for spec in self.infeasible:
                if not spec.cancelled:
                    demand.append(dict(spec.resources))
            pg_bundles = []
            for pid in self.pending_pgs:
                g = self.pgs.get(pid)
                if g is not None:
                    pg_bundles.append({"strategy": g["strategy"], "bundles": [dict(b) for b in g["bundles"]]})
            busy = {}
            for w in self.workers.values():
                if w.alive and (w.tasks_inflight or w.actor_id is not None):
                    busy[w.node] = busy.get(w.node, 0) + 1
            nodes = {n: {"total": self.sched.total(n), "available": self.sched.available(n),
                         "alive": info.get("Alive", False), "busy_workers": busy.get(n, 0),
                         "head": n == self.head_hex} for n, info in self.node_info.items()}
            return {"demand": demand, "pending_placement_groups": pg_bundles, "nodes": nodes}
        if what == "named_actors":
            return [(ns, n) for (ns, n), aid in self.named_actors.items()
                    if self.actors.get(aid) and self.actors[aid].state != "DEAD"]
        raise ValueError(what)

    # -------------------------------------------------------------- nodes
    def _h_add_node(self, c, req, node_hex, resources, gpu_ids, address):
        self.sched.add_node(node_hex, resources)
        self.free_gpus[node_hex] = list(gpu_ids)
        self.node_info[node_hex] = {"NodeID": node_hex, "Alive": True, "NodeManagerAddress": address,
                                    "Resources": dict(resources), "local": False}
        self._reply(c, req, True)
        self._retry_pending_pgs()
        self._retry_infeasible()
        self._schedule()

    def _h_node_stats(self, c, stats):
        """A node agent's physical-metrics sample (dashboard/reporter.py)."""
        node = self.clients.get(c, {}).get("node")
        info = self.node_info.get(node)
        if info is not None:
            info["stats"] = stats

    def _register_node(self, c, node_hex, extra):
        """A node agent joined (reference: raylet registering with the GCS node manager)."""
        res = {k: float(v) for k, v in extra["resources"].items()}
        addr = extra.get("address", "127.0.0.1")
        res.setdefault(f"node:{addr}", 1.0)
        self.sched.add_node(node_hex, res)
        self.node_labels[node_hex] = _node_labels(node_hex, extra.get("gpu_ids", ()), extra.get("labels"))
        self.sched.set_labels(node_hex, self.node_labels[node_hex])
        self.free_gpus[node_hex] = list(extra.get("gpu_ids", ()))
        self.node_store[node_hex] = extra["store_name"]
        self.node_obj_addr[node_hex] = extra["obj_addr"]
        self.node_conns[node_hex] = c
        self.node_resources[node_hex] = dict(res)
        self.node_info[node_hex] = {"NodeID": node_hex, "Alive": True, "NodeManagerAddress": addr,
                                    "Resources": dict(res), "local": False, "pid": extra.get("pid"),
                                    "Labels": dict(self.node_labels[node_hex]), "IsHeadNode": False}
        self._send(c, ("registered", {"store_name": extra["store_name"], "node_id": node_hex,
                                      "namespace": self.namespace, "session_dir": self.session_dir,
                                      "head_tcp": self.tcp_address, "reconnect_s": self.reconnect_s}))
        self.events.append(("node_added", node_hex, time.time()))
        self._publish("node", node_hex, {"state": "ALIVE", "address": addr, "resources": dict(res)})
        self._cluster_event("INFO", "GCS", f"node {node_hex[:12]} ({addr}) joined", node_id=node_hex)
        self._retry_pending_pgs()
        self._retry_infeasible()
        self._schedule()

    def _on_node_death(self, node_hex):
        self.node_conns.pop(node_hex, None)
        self.sched.set_alive(node_hex, False)
        if node_hex in self.node_info:
            self.node_info[node_hex]["Alive"] = False
        self.events.append(("node_removed", node_hex, time.time()))
        self._publish("node", node_hex, {"state": "DEAD"})
        self._cluster_event("ERROR", "GCS", f"node {node_hex[:12]} died", node_id=node_hex)
        # objects whose only copy lived there are lost: re-execute their lineage
        # where possible (reference: object_recovery_manager.cc RecoverObject)
        for oid, e in list(self.objects.items()):
            if e.node == node_hex and e.inline is None and e.state == READY and not e.spilled_path:
                e.lost = True
        for oid, e in list(self.objects.items()):
            if e.lost and e.state == READY and e.refcount > 0:
                self._reconstruct(oid)
        # workers of that node: their control connections drop on their own; fail
        # anything still attributed to them (e.g. they never connected)
        for w in list(self.workers.values()):
            if w.node == node_hex and w.conn is None:
                self.workers.pop(w.worker_id, None)

    def _h_remove_node(self, c, node_hex):
        self.sched.set_alive(node_hex, False)
        if node_hex in self.node_info:
            self.node_info[node_hex]["Alive"] = False

    # -------------------------------------------------------------- shutdown
    def shutdown(self):
        if not self.running:
            return
        self.running = False
        if getattr(self, "_reporter", None) is not None:
            self._reporter.stop()
        for w in list(self.workers.values()):
            try:
                if w.conn is not None:
                    w.conn.close()
            except Exception:
                pass
            try:
                if w.pid:
                    os.kill(w.pid, signal.SIGKILL)
            except (ProcessLookupError, TypeError):
                pass
        for w in list(self.workers.values()):
            try:
                if w.proc is not None:
                    w.proc.wait(timeout=2)
            except Exception:
                pass
        try:
            self._ww.send(b"x")
        except OSError:
            pass
        if self.thread is not None:
            self.thread.join(timeout=5)
        if getattr(self, "_zygote", None) is not None:
            self._zygote.stop()
        try:
            self.spill_store.destroy()
        except Exception:
            pass
        try:
            self.lsock.close()
            os.unlink(self.sock_path)
        except OSError:
            pass
        try:
            self.store.unlink()
        except Exception:
            pass
