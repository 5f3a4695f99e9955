"""Public Core API (reference: python/ray/_private/worker.py — init :1275,
shutdown :1884, get :2667, put :2803, wait :2868, get_actor :3013, kill :3048,
cancel :3079, remote :3256; python/ray/_private/state.py — nodes, timeline,
cluster_resources, available_resources)."""
from __future__ import annotations

import atexit
import inspect
import json
import os
import sys
import shutil
import socket
import tempfile
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

from . import context
from .object_ref import ObjectRef

_head = None
_init_lock = threading.RLock()
_session = {}

LOCAL_MODE = 2
SCRIPT_MODE = 0
WORKER_MODE = 1


_GFX_ACCELERATOR = {  # KFD gfx_target_version -> reference accelerator type name
    90500: "AMD-Instinct-MI355X-OAM", 90402: "AMD-Instinct-MI300X-OAM", 90400: "AMD-Instinct-MI300X-OAM",
    90010: "AMD-Instinct-MI250X-MI250", 90008: "AMD-Instinct-MI100"}


def detect_accelerator_type() -> Optional[str]:
    """This node's AMD accelerator type (reference: _private/accelerators/amd_gpu.py
    get_current_node_accelerator_type), from the KFD topology; ``CAAMD_ACCELERATOR_TYPE``
    overrides. The node then advertises the resource ``accelerator_type:<type>``
    that ``@remote(accelerator_type=...)`` and ``ScalingConfig(accelerator_type=...)``
    request 0.001 of. gfx950 parts (MI350X / MI355X) report as MI355X."""
    if os.environ.get("CAAMD_ACCELERATOR_TYPE"):
        return os.environ["CAAMD_ACCELERATOR_TYPE"]
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in sorted(os.listdir(base)):
            try:
                with open(os.path.join(base, d, "properties")) as f:
                    props = dict(line.split() for line in f if len(line.split()) == 2)
            except (OSError, ValueError):
                continue
            if int(props.get("simd_count", "0")) > 0:
                v = int(props.get("gfx_target_version", "0"))
                return _GFX_ACCELERATOR.get(v, f"AMD-gfx{v // 10000}{(v // 100) % 100:x}{v % 100:x}")
    except OSError:
        pass
    return None


def accelerator_resources(gpus) -> Dict[str, float]:
    if not gpus:
        return {}
    t = detect_accelerator_type()
    return {f"accelerator_type:{t}": 1.0} if t else {}


def detect_gpus() -> List[int]:
    """MI355X GPUs visible to this process, without initialising HIP.

    Reads the KFD topology (a node with simd_count > 0 is a GPU agent) and
    honours ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CAAMD_NUM_GPUS.
    """
    if "CAAMD_NUM_GPUS" in os.environ:
        return list(range(int(os.environ["CAAMD_NUM_GPUS"])))
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in sorted(os.listdir(base), key=lambda x: int(x) if x.isdigit() else 0):
            try:
                with open(os.path.join(base, d, "properties")) as f:
                    props = dict(line.split() for line in f if len(line.split()) == 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        n = 0
    ids = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v != "":
            sel = [int(x) for x in v.split(",") if x.strip().isdigit()]
            ids = [i for i in sel if i < max(n, len(sel))] if n else sel
            ids = list(range(len(ids)))  # re-indexed inside this process
            break
    return ids


def _default_cpus() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _pid_ns() -> str:
    """This process's PID-namespace id (the inode of /proc/self/ns/pid), in hex."""
    try:
        return format(os.stat("/proc/self/ns/pid").st_ino, "x")
    except OSError:
        return "0"


def store_segment_name(node: bool = False) -> str:
    """Object-store arena name ``/caamd_[node_]<pid>_<pidns>_<8 hex>``. The PID
    namespace is part of the name because /dev/shm is often shared between containers
    (``--ipc=host``) while PIDs are not: the stale-arena sweep may only judge segments
    created in its own PID namespace."""
    return f"/caamd_{'node_' if node else ''}{os.getpid()}_{_pid_ns()}_{uuid.uuid4().hex[:8]}"


def _sweep_stale_stores() -> int:
    """Unlink ``/dev/shm/caamd_[node_]<pid>_<pidns>_*`` object-store segments created
    in THIS PID namespace whose owner pid is gone and that no live process maps (a
    head or node agent killed before its shutdown could unlink them: with tmpfs the
    pages stay charged to memory until the file is removed). Segments of live pids
    (and of reused pids) are left alone, and so is an arena that a dead head's
    workers still map: a restarted head reattaches to it
    (head_main._previous_session). Segments of other PID namespaces (another
    container sharing /dev/shm: its pids are invisible here and its mappings are not
    in this /proc) and names without a namespace are never touched. Returns the
    number removed."""
    import re

    n = 0
    try:
        names = [x for x in os.listdir("/dev/shm") if x.startswith("caamd_")]
    except OSError:
        return 0
    if not names:
        return 0
    ns = _pid_ns()
    mapped = set()
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            with open(f"/proc/{pid}/maps") as f:
                for ln in f:
                    i = ln.find("/dev/shm/caamd_")
                    if i >= 0:
                        mapped.add(ln[i + 9:].split()[0])
        except OSError:
            continue
    for name in names:
        if name in mapped:
            continue
        m = re.match(r"^caamd_(?:node_)?(\d+)_([0-9a-f]+)_[0-9a-f]{8}$", name)
        if not m or m.group(2) != ns:
            continue
        try:
            os.kill(int(m.group(1)), 0)
            continue  # owner alive
        except ProcessLookupError:
            pass
        except (PermissionError, OverflowError):
            continue  # someone else's live process, or not a pid
        try:
            os.unlink(os.path.join("/dev/shm", name))
            n += 1
        except OSError:
            pass
    return n


def _default_store_bytes() -> int:
    try:
        import psutil

        avail = psutil.virtual_memory().available
    except Exception:
        avail = 8 << 30
    try:
        shm = shutil.disk_usage("/dev/shm").free
    except OSError:
        shm = avail
    return int(max(64 << 20, min(avail * 0.3, shm * 0.8, 200 << 30)))


class RayContext(dict):
    """Returned by init(): address info (dict-like, like the reference's RayContext)."""

    def __init__(self, info):
        super().__init__(info)
        self.address_info = info
        self.dashboard_url = info.get("webui_url")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        shutdown()

    def disconnect(self):
        shutdown()


def is_initialized() -> bool:
    return context.worker is not None or context.local_mode


def _spill_config(kwargs):
    """``init(_system_config={"object_spilling_config": dict or JSON})`` (reference:
    _private/external_storage.py setup_external_storage), else CAAMD_OBJECT_SPILLING_CONFIG.
    Validated here so a bad config fails ``init`` rather than the first spill."""
    from .external_storage import parse_config

    sc = kwargs.get("_system_config") or {}
    cfg = sc.get("object_spilling_config", os.environ.get("CAAMD_OBJECT_SPILLING_CONFIG"))
    cfg = parse_config(cfg)
    if cfg is not None and cfg["type"] not in ("filesystem", "smart_open", "uri", "fsspec", "pyarrow"):
        raise ValueError(f"unsupported object_spilling_config type {cfg['type']!r}")
    return cfg


def _gcs_storage(kwargs) -> Optional[str]:
    """Durable GCS table log for head fault tolerance: ``init(_gcs_storage=path)``,
    ``init(_system_config={"gcs_storage": path})`` or ``CAAMD_GCS_STORAGE``."""
    sc = kwargs.get("_system_config") or {}
    return kwargs.get("_gcs_storage") or sc.get("gcs_storage") or os.environ.get("CAAMD_GCS_STORAGE") or None


def init(address: Optional[str] = None, *, num_cpus: Optional[int] = None,
         num_gpus: Optional[int] = None, resources: Optional[Dict[str, float]] = None,
         object_store_memory: Optional[int] = None, local_mode: bool = False,
         ignore_reinit_error: bool = False, namespace: Optional[str] = None,
         runtime_env: Optional[dict] = None, include_dashboard: Optional[bool] = None,
         dashboard_host: str = "127.0.0.1", dashboard_port: Optional[int] = None,
         job_config=None, logging_level=None, log_to_driver: bool = True,
         _temp_dir: Optional[str] = None, _node_ip_address: str = "127.0.0.1",
         **kwargs) -> RayContext:
    global _head
    logging_config = kwargs.pop("logging_config", None)
    if logging_config is not None:
        # driver now; workers started by this process's head through the environment
        logging_config._apply()
        os.environ["CAAMD_LOGGING_CONFIG"] = logging_config._to_env()
    with _init_lock:
        if is_initialized():
            if ignore_reinit_error:
                return RayContext(dict(_session))
            raise RuntimeError("Maybe you called init twice by accident? "
                               "Pass ignore_reinit_error=True to ignore this.")
        if local_mode:
            context.local_mode = True
            from .local_mode import reset_local

            reset_local()
            _session.clear()
            _session.update({"node_id": "local", "address": "local"})
            return RayContext(dict(_session))
        if job_config is not None:
            runtime_env = runtime_env or (job_config.runtime_env or None)
            namespace = namespace or job_config.ray_namespace
        if runtime_env:
            _check_runtime_env(runtime_env)
        address = address or os.environ.get("CAAMD_ADDRESS") or os.environ.get("RAY_ADDRESS")
        if address and address.startswith("ray://"):
            from ..client_builder import connect

            return RayContext(connect(address, namespace=namespace, runtime_env=runtime_env))
        if address == "local":
            address = None
        from .worker import CoreWorker

        job_id = os.urandom(4)
        if address is None:
            from .head import Head

            sess = f"session_{time.strftime('%Y%m%d-%H%M%S')}_{os.getpid()}_{uuid.uuid4().hex[:6]}"
            root = _temp_dir or os.path.join(tempfile.gettempdir(), "caamd")
            session_dir = os.path.join(root, sess)
            gpus = detect_gpus()
            if num_gpus is not None:
                gpus = list(range(num_gpus))
            res = {"CPU": float(num_cpus if num_cpus is not None else _default_cpus())}
            if gpus:
                res["GPU"] = float(len(gpus))
            res.update(accelerator_resources(gpus))
            res["memory"] = float(_mem_bytes())
            _sweep_stale_stores()  # before sizing the store from the free /dev/shm space
            store_bytes = int(object_store_memory or _default_store_bytes())
            res["object_store_memory"] = float(store_bytes)
            node_id = os.urandom(16)
            res[f"node:{_node_ip_address}"] = 1.0
            res["node:__internal_head__"] = 1.0
            for k, v in (resources or {}).items():
                res[k] = float(v)
            store_name = store_segment_name()
            if os.environ.get("CAAMD_HEAD_IN_PROCESS", "0") == "1":
                head = Head(session_dir, node_id, res, store_name, store_bytes, gpus,
                            namespace=namespace or "default",
                            worker_env=_worker_env_from(runtime_env),
                            listen_tcp=kwargs.get("_listen_tcp"), labels=kwargs.get("labels"),
                            gcs_storage=_gcs_storage(kwargs), spill_config=_spill_config(kwargs))
                head.start()
                _head = head
                address = head.sock_path
                tcp = head.tcp_address
            else:
                # the head (GCS tables + scheduler loop) runs as its own process so the
                # control plane never competes with driver code for the GIL
                info = _spawn_head_process({
                    "session_dir": session_dir, "node_id": node_id.hex(), "resources": res,
                    "store_name": store_name, "store_bytes": store_bytes, "gpus": gpus,
                    "namespace": namespace or "default", "worker_env": _worker_env_from(runtime_env),
                    "listen_tcp": kwargs.get("_listen_tcp"), "parent_pid": os.getpid(),
                    "labels": kwargs.get("labels") or {}, "gcs_storage": _gcs_storage(kwargs),
                    "spill_config": _spill_config(kwargs),
                    "sys_path": [p for p in sys.path if p and os.path.isdir(p)]})
                address = info["unix"]
                tcp = info.get("address")
            try:
                os.makedirs(root, exist_ok=True)
                with open(os.path.join(root, "latest_address"), "w") as f:
                    f.write(tcp or address)
            except OSError:
                pass
        elif address == "auto":
            root = _temp_dir or os.path.join(tempfile.gettempdir(), "caamd")
            with open(os.path.join(root, "latest_address")) as f:
                address = f.read().strip()
        cw = CoreWorker(address, "driver", os.urandom(16), job_id=job_id)
        cw.namespace = namespace or cw.namespace
        context.worker = cw
        _session.clear()
        _session.update({"address": address, "node_id": cw.node_hex, "session_dir": cw.session_dir,
                         "namespace": cw.namespace, "job_id": job_id.hex(),
                         "object_store_address": getattr(cw.store, "name", ""),
                         "webui_url": None, "gcs_address": (_head.tcp_address if _head is not None and
                                                             _head.tcp_address else
                                                             (_head_proc[1].get("address") if _head_proc
                                                              else None) or address)})
        if runtime_env:
            _session["runtime_env"] = runtime_env
        global _log_monitor
        if log_to_driver and cw.session_dir and os.path.isdir(cw.session_dir) and \
                os.environ.get("CAAMD_LOG_TO_DRIVER", "1") != "0":
            from .log_monitor import LogMonitor

            _log_monitor = LogMonitor(cw.session_dir).start()
        if include_dashboard:
            from ..dashboard import start_dashboard

            _session["webui_url"] = start_dashboard(dashboard_host, 8265 if dashboard_port is None else dashboard_port,
                                                    head=_head, control_address=address,
                                                    session_dir=cw.session_dir)
        return RayContext(dict(_session))


_log_monitor = None
_head_proc = None  # (Popen, info) of the driver-owned head process


def _spawn_head_process(cfg: dict) -> dict:
    import subprocess

    global _head_proc
    proc = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.head_main", "--embedded",
                             json.dumps(cfg)], stdout=subprocess.PIPE, stdin=subprocess.DEVNULL,
                            cwd=os.getcwd(), env=_head_env())
    line = proc.stdout.readline()
    if not line:
        proc.wait(timeout=10)
        raise RuntimeError(f"head process failed to start (exit code {proc.returncode})")
    info = json.loads(line)
    proc.stdout.close()
    _head_proc = (proc, info)
    return info


def _head_env():
    e = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    return e


def _stop_head_process():
    global _head_proc
    if _head_proc is None:
        return
    proc, _ = _head_proc
    _head_proc = None
    try:
        proc.terminate()
        proc.wait(timeout=15)
    except Exception:
        try:
            proc.kill()
            proc.wait(timeout=5)
        except Exception:
            pass


def _mem_bytes():
    try:
        import psutil

        return psutil.virtual_memory().total
    except Exception:
        return 16 << 30


def _check_runtime_env(renv):
    """Validate a runtime_env. ``pip`` / ``uv`` packages are installed into a cached
    virtualenv when a worker of that env starts (runtime_env/pip.py: offline, from
    local wheels / find-links); a failed install surfaces as RuntimeEnvSetupError on
    the task's result. ``conda`` cannot be installed here (no conda in the image), so
    its dependencies must already be importable."""
    from ..exceptions import RuntimeEnvSetupError
    from ..runtime_env import RuntimeEnv, missing_packages

    RuntimeEnv(**dict(renv))
    for key in ("conda",):
        spec = renv.get(key)
        if spec is None:
            continue
        if key == "conda":
            spec = [d for d in (spec.get("dependencies", []) if isinstance(spec, dict) else [])
                    if isinstance(d, str) and not d.startswith("python")]
        miss = missing_packages(spec)
        if miss:
            raise RuntimeEnvSetupError(
                f"runtime_env {key} packages {miss} are not installed in this image and "
                "cannot be fetched (no package index available)")


def _worker_env_from(renv):
    env = {}
    if renv:
        for k, v in (renv.get("env_vars") or {}).items():
            env[k] = str(v)
        env["CAAMD_RUNTIME_ENV"] = json.dumps(renv)
    return env


def _ensure_init():
    if not is_initialized():
        init()


def shutdown(_exiting_interpreter: bool = False):
    global _head
    with _init_lock:
        if context.local_mode:
            context.local_mode = False
            from .local_mode import reset_local

            reset_local()
        global _log_monitor
        if _log_monitor is not None:
            try:
                _log_monitor.stop()
            except Exception:
                pass
            _log_monitor = None
        w = context.worker
        context.worker = None
        if w is not None:
            try:
                w.close()
            except Exception:
                pass
        if _session.get("webui_url"):
            from ..dashboard import stop_dashboard

            stop_dashboard()
        if _head is not None:
            _head.shutdown()
            _head = None
        _stop_head_process()
        _session.clear()


atexit.register(lambda: shutdown(True))


def _w():
    _ensure_init()
    return context.worker


def put(value, *, _owner=None, _tensor_transport: Optional[str] = None) -> ObjectRef:
    """``_tensor_transport="ipc"``: GPU tensors in ``value`` are shared with
    same-node readers through HIP IPC handles (zero copy) instead of host copies
    (see experimental/gpu_objects.py)."""
    if context.local_mode:
        from .local_mode import local_put

        return local_put(value)
    return _w().put(value, tensor_transport=_tensor_transport)


def get(object_refs, *, timeout: Optional[float] = None):
    if context.local_mode:
        from .local_mode import local_get

        return local_get(object_refs)
    from .object_ref import ObjectRefGenerator

    if isinstance(object_refs, ObjectRefGenerator):
        object_refs = list(object_refs)
    if isinstance(object_refs, (list, tuple)):
        return _w().get(list(object_refs), timeout=timeout)
    if not isinstance(object_refs, ObjectRef):
        from ..dag.compiled import CompiledDAGRef

        if isinstance(object_refs, CompiledDAGRef):
            return object_refs.get(timeout)
        raise TypeError(f"get() expects an ObjectRef or a list of ObjectRefs, got {type(object_refs)}")
    return _w().get(object_refs, timeout=timeout)


def wait(object_refs: List[ObjectRef], *, num_returns: int = 1, timeout: Optional[float] = None,
         fetch_local: bool = True):
    if isinstance(object_refs, ObjectRef):
        raise TypeError("wait() expected a list of ObjectRef")
    if context.local_mode:
        return list(object_refs)[:num_returns], list(object_refs)[num_returns:]
    return _w().wait(list(object_refs), num_returns=num_returns, timeout=timeout, fetch_local=fetch_local)


def remote(*args, **kwargs):
    """``@remote`` / ``@remote(num_cpus=..., ...)`` for functions and classes."""
    from .actor import ActorClass
    from .remote_function import RemoteFunction

    def make(obj, opts):
        if inspect.isclass(obj):
            return ActorClass(obj, opts)
        if callable(obj):
            return RemoteFunction(obj, opts)
        raise TypeError("@remote can only decorate functions or classes")

    if len(args) == 1 and not kwargs and callable(args[0]):
        return make(args[0], {})
    if args:
        raise TypeError("@remote takes keyword arguments only, e.g. @remote(num_gpus=1)")
    return lambda obj: make(obj, kwargs)


def get_actor(name: str, namespace: Optional[str] = None):
    from .actor import ActorHandle

    w = _w()
    res = w.request(lambda r: ("check_name", r, namespace or w.namespace, name))
    if res is None:
        raise ValueError(f"Failed to look up actor with name '{name}'.")
    return ActorHandle(res[0], res[1] or {})


def kill(actor, *, no_restart: bool = True):
    from .actor import ActorHandle

    if not isinstance(actor, ActorHandle):
        raise ValueError("kill() only supports actor handles")
    if context.local_mode:
        return
    w = _w()
    w.send(("kill_actor", actor._actor_id, no_restart))
    # later calls from this process go through the head, which orders them after the
    # kill (a still-open direct connection would reach the actor before it dies)
    if getattr(w, "actor_head_only", None) is not None:
        w._to_head_path(actor._actor_id, drop=True)


def cancel(ref, *, force: bool = False, recursive: bool = True):
    from .object_ref import ObjectRefGenerator

    if isinstance(ref, ObjectRefGenerator):
        tid = ref._task_id
    elif isinstance(ref, ObjectRef):
        tid = ref.binary()[:16]
    else:
        raise TypeError("cancel() expects an ObjectRef")
    if context.local_mode:
        return
    _w().cancel(tid, force, recursive)


def free(refs):
    _w().free(refs)


def _state(what, arg=None):
    w = _w()
    return w.request(lambda r: ("state", r, what, arg))


def nodes():
    return _state("nodes")


def cluster_resources():
    return _state("cluster_resources")


def available_resources():
    return _state("available_resources")


def available_resources_per_node():
    return _state("available_per_node")


def get_gpu_ids():
    ctx = context.current_task()
    if ctx is not None and ctx.gpu_ids is not None:
        return list(range(len(ctx.gpu_ids))) if os.environ.get("ROCR_VISIBLE_DEVICES") else ctx.gpu_ids
    env = os.environ.get("CAAMD_GPU_IDS", "")
    ids = [int(x) for x in env.split(",") if x]
    # a leased GPU worker (core/lease.py) runs with its lease's GPUs visible: same
    # numbering as the head path (device indices when ROCR_VISIBLE_DEVICES is set)
    return list(range(len(ids))) if os.environ.get("ROCR_VISIBLE_DEVICES") else ids


def _timeline_events(ev):
    starts = {}
    out = []
    for e in ev:
        if e[0] == "start":
            starts[e[1]] = e
        elif e[0] == "end" and e[1] in starts:
            s = starts.pop(e[1])
            out.append({"cat": "task", "name": s[2], "ph": "X", "ts": s[3] * 1e6,
                        "dur": (e[3] - s[3]) * 1e6, "pid": "node", "tid": s[4] or 0,
                        "args": {"task_id": e[1].hex()}})
    return out


def timeline(filename: Optional[str] = None):
    """Chrome-trace events of task execution (reference: state.py:965)."""
    out = _timeline_events(_state("events"))
    if filename:
        with open(filename, "w") as f:
            json.dump(out, f)
        return None
    return out


def show_in_dashboard(message: str, key: str = "", dtype: str = "text"):
    pass


def head():
    return _head
