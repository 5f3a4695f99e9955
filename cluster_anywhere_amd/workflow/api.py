"""Workflow API + executor (reference: python/ray/workflow/api.py,
workflow_executor.py, workflow_storage.py). See package docstring."""
from __future__ import annotations

import asyncio
import enum
import json
import os
import shutil
import tempfile
import time
from typing import Any, Dict, List, Optional, Tuple

import cloudpickle

from .. import exceptions as _exc
from ..core import api as _core
from ..dag import ClassMethodNode, DAGNode, FunctionNode, InputNode, MultiOutputNode


class WorkflowStatus(str, enum.Enum):
    NONE = "NONE"
    RUNNING = "RUNNING"
    CANCELED = "CANCELED"
    SUCCESSFUL = "SUCCESSFUL"
    FAILED = "FAILED"
    RESUMABLE = "RESUMABLE"
    PENDING = "PENDING"


class WorkflowError(_exc.RayError):
    pass


class WorkflowExecutionError(WorkflowError):
    def __init__(self, workflow_id: str, cause: Optional[BaseException] = None):
        self.workflow_id = workflow_id
        self.cause = cause
        super().__init__(f"Workflow[id={workflow_id}] failed during execution: {cause!r}")


class WorkflowCancellationError(WorkflowError):
    def __init__(self, workflow_id: str):
        self.workflow_id = workflow_id
        super().__init__(f"Workflow[id={workflow_id}] is cancelled during execution.")


class WorkflowNotFoundError(WorkflowError):
    def __init__(self, workflow_id: str):
        self.workflow_id = workflow_id
        super().__init__(f"Workflow[id={workflow_id}] was referenced but doesn't exist.")


class EventListener:
    """Subclass and implement ``poll_for_event`` (reference: event_listener.py)."""

    async def poll_for_event(self, *args, **kwargs) -> Any:
        raise NotImplementedError

    async def event_checkpointed(self, event: Any) -> None:
        pass


# ----------------------------------------------------------------- storage
_STORAGE: Optional[str] = None


def init(storage: Optional[str] = None, *, max_running_workflows: Optional[int] = None,
         max_pending_workflows: Optional[int] = None) -> None:
    global _STORAGE
    storage = storage or os.environ.get("CAAMD_WORKFLOW_STORAGE")
    if storage and storage.startswith("file://"):
        storage = storage[len("file://"):]
    _STORAGE = storage or os.path.join(tempfile.gettempdir(), "caamd", "workflows")
    os.makedirs(_STORAGE, exist_ok=True)
    if not _core.is_initialized():
        _core.init()


def _storage() -> str:
    if _STORAGE is None:
        init()
    return _STORAGE


class _Store:
    """One workflow's directory: meta.json, dag.pkl, tasks/<task_id>.pkl, output.pkl."""

    def __init__(self, root: str, wf_id: str):
        self.dir = os.path.join(root, wf_id)
        self.wf_id = wf_id

    def exists(self):
        return os.path.isfile(os.path.join(self.dir, "meta.json"))

    def _atomic(self, name, data: bytes):
        path = os.path.join(self.dir, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = f"{path}.tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)

    def meta(self) -> Dict[str, Any]:
        with open(os.path.join(self.dir, "meta.json")) as f:
            return json.load(f)

    def update_meta(self, **kw):
        m = self.meta() if self.exists() else {}
        m.update(kw)
        self._atomic("meta.json", json.dumps(m).encode())

    def save(self, name, value):
        self._atomic(name, cloudpickle.dumps(value))

    def load(self, name):
        with open(os.path.join(self.dir, name), "rb") as f:
            return cloudpickle.loads(f.read())

    def has(self, name):
        return os.path.isfile(os.path.join(self.dir, name))

    def task_file(self, task_id):
        return f"tasks/{task_id}.pkl"

    def cancel_requested(self):
        return os.path.exists(os.path.join(self.dir, "CANCEL"))


# ------------------------------------------------------------ DAG helpers
_WF_OPTS = "_workflow_options"


def options(*, task_id: Optional[str] = None, metadata: Optional[Dict] = None,
            catch_exceptions: Optional[bool] = None, checkpoint: Optional[bool] = None,
            max_retries: Optional[int] = None, retry_exceptions: Optional[bool] = None,
            **_ignored) -> Dict[str, Any]:
    """Use as ``f.options(**workflow.options(task_id="x")).bind(...)``."""
    o = {k: v for k, v in dict(task_id=task_id, metadata=metadata, catch_exceptions=catch_exceptions,
                                checkpoint=checkpoint, max_retries=max_retries,
                                retry_exceptions=retry_exceptions).items() if v is not None}
    return {_WF_OPTS: o}


class _Continuation:
    def __init__(self, dag):
        self.dag = dag


def continuation(dag_node):
    """Returned from inside a workflow task: the task's output is that sub-DAG's output."""
    if not isinstance(dag_node, DAGNode):
        return dag_node
    return _Continuation(dag_node)


def _wf_opts(node: FunctionNode) -> Dict[str, Any]:
    return dict(getattr(node._rf, "_workflow_opts", {}) or {})


def _assign_ids(root: DAGNode, prefix: str = "") -> Tuple[List[DAGNode], Dict[int, str]]:
    """Deterministic post-order + task ids (user ``task_id`` or ``<fn name>[_<n>]``)."""
    order, seen, ids, counts = [], set(), {}, {}

    def visit(n):
        if id(n) in seen:
            return
        seen.add(id(n))
        for c in n._children():
            visit(c)
        if isinstance(n, ClassMethodNode):
            raise WorkflowError("actor methods are not supported inside workflows")
        order.append(n)
        if isinstance(n, FunctionNode):
            tid = _wf_opts(n).get("task_id") or n._rf.__name__
            k = counts.get(tid, 0)
            counts[tid] = k + 1
            ids[id(n)] = prefix + (tid if k == 0 else f"{tid}_{k}")

    visit(root)
    return order, ids


# -------------------------------------------------------------- executor
def _run_dag(store: _Store, root: DAGNode, inputs, prefix: str = ""):
    from ..core.api import get as rget
    from ..core.api import put as rput
    from ..core.api import wait as rwait

    order, ids = _assign_ids(root, prefix)
    val: Dict[int, Any] = {}    # node -> ("ref", ObjectRef) | ("val", value)
    pending: Dict[Any, DAGNode] = {}
    todo = [n for n in order]

    def arg(x):
        if not isinstance(x, DAGNode):
            return x
        kind, v = val[id(x)]
        return v

    def resolved(n):
        return all(id(c) in val for c in n._children())

    def finish(n, value):
        o = _wf_opts(n)
        if o.get("checkpoint", True):
            store.save(store.task_file(ids[id(n)]), value)
        val[id(n)] = ("val", value)

    def step():
        nonlocal todo
        rest = []
        for n in todo:
            if not resolved(n):
                rest.append(n)
                continue
            if isinstance(n, InputNode):
                val[id(n)] = ("val", inputs)
            elif isinstance(n, MultiOutputNode):
                val[id(n)] = ("val", [arg(c) for c in n._args])
            elif isinstance(n, FunctionNode):
                tid = ids[id(n)]
                if store.has(store.task_file(tid)):
                    val[id(n)] = ("val", store.load(store.task_file(tid)))
                    continue
                o = _wf_opts(n)
                ropts = {k: v for k, v in (n._options or {}).items() if k != _WF_OPTS}
                ropts.setdefault("max_retries", o.get("max_retries", 3))
                ropts.setdefault("retry_exceptions", o.get("retry_exceptions", False))
                a = [arg(x) for x in n._args]
                k = {kk: arg(v) for kk, v in n._kwargs.items()}
                ref = n._rf.options(**ropts).remote(*a, **k)
                pending[ref] = n
            else:
                val[id(n)] = ("val", n._run({}, None))
        todo = rest

    step()
    while pending or todo:
        if store.cancel_requested():
            for r in list(pending):
                try:
                    _core.cancel(r, force=True)
                except Exception:
                    pass
            raise WorkflowCancellationError(store.wf_id)
        if not pending:
            raise WorkflowError("workflow DAG has unresolvable nodes")
        ready, _ = rwait(list(pending), num_returns=1, timeout=0.2)
        for r in ready:
            n = pending.pop(r)
            o = _wf_opts(n)
            try:
                out = rget(r)
                if isinstance(out, _Continuation):
                    out = _run_dag(store, out.dag, inputs, prefix=ids[id(n)] + ".")
                if o.get("catch_exceptions"):
                    out = (out, None)
            except WorkflowCancellationError:
                raise
            except Exception as e:  # noqa: BLE001
                if not o.get("catch_exceptions"):
                    raise WorkflowExecutionError(store.wf_id, e) from e
                out = (None, e)
            finish(n, out)
        step()
    kind, v = val[id(root)]
    return v


def _execute(root_dir: str, wf_id: str):
    store = _Store(root_dir, wf_id)
    dag, inputs = store.load("dag.pkl")
    store.update_meta(status=WorkflowStatus.RUNNING.value, start_time=time.time(), end_time=None)
    if store.has("output.pkl"):
        os.unlink(os.path.join(store.dir, "output.pkl"))
    try:
        out = _run_dag(store, dag, inputs)
    except WorkflowCancellationError:
        store.update_meta(status=WorkflowStatus.CANCELED.value, end_time=time.time())
        raise
    except BaseException as e:
        store.update_meta(status=WorkflowStatus.FAILED.value, end_time=time.time(), error=repr(e))
        raise
    store.save("output.pkl", out)
    store.update_meta(status=WorkflowStatus.SUCCESSFUL.value, end_time=time.time())
    return out


def _executor_task():
    from ..core.api import remote

    global _EXEC
    if _EXEC is None:
        _EXEC = remote(num_cpus=0, max_retries=0)(_execute)
    return _EXEC


_EXEC = None


# -------------------------------------------------------------------- API
def run_async(dag: DAGNode, *args, workflow_id: Optional[str] = None,
              metadata: Optional[Dict[str, Any]] = None, **kwargs):
    root = _storage()
    wf_id = workflow_id or f"workflow_{int(time.time() * 1e3)}_{os.urandom(3).hex()}"
    store = _Store(root, wf_id)
    if store.exists():
        st = store.meta().get("status")
        if st == WorkflowStatus.SUCCESSFUL.value:
            return _core.put(store.load("output.pkl"))
        if st == WorkflowStatus.RUNNING.value:
            raise WorkflowError(f"Workflow[id={wf_id}] is already running")
    os.makedirs(store.dir, exist_ok=True)
    store.save("dag.pkl", (dag, (args, kwargs) if (args or kwargs) else None))
    store.update_meta(workflow_id=wf_id, status=WorkflowStatus.PENDING.value,
                      user_metadata=dict(metadata or {}), created=time.time(), driver_pid=os.getpid())
    return _executor_task().remote(root, wf_id)


def run(dag: DAGNode, *args, workflow_id: Optional[str] = None,
        metadata: Optional[Dict[str, Any]] = None, **kwargs) -> Any:
    return _unwrap(run_async(dag, *args, workflow_id=workflow_id, metadata=metadata, **kwargs))


def _unwrap(ref):
    try:
        return _core.get(ref)
    except _exc.RayTaskError as e:
        cause = getattr(e, "cause", None)
        if isinstance(cause, WorkflowError):
            raise cause from None
        raise


def resume_async(workflow_id: str):
    root = _storage()
    store = _Store(root, workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    st = store.meta().get("status")
    if st == WorkflowStatus.SUCCESSFUL.value:
        return _core.put(store.load("output.pkl"))
    try:
        os.unlink(os.path.join(store.dir, "CANCEL"))
    except FileNotFoundError:
        pass
    store.update_meta(status=WorkflowStatus.PENDING.value, driver_pid=os.getpid())
    return _executor_task().remote(root, workflow_id)


def resume(workflow_id: str) -> Any:
    return _unwrap(resume_async(workflow_id))


def resume_all(include_failed: bool = False) -> List[Tuple[str, Any]]:
    want = {WorkflowStatus.RESUMABLE}
    if include_failed:
        want.add(WorkflowStatus.FAILED)
    return [(wid, resume_async(wid)) for wid, st in list_all(want)]


def get_output_async(workflow_id: str, *, task_id: Optional[str] = None):
    return _core.put(get_output(workflow_id, task_id=task_id))


def get_output(workflow_id: str, *, task_id: Optional[str] = None) -> Any:
    store = _Store(_storage(), workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    if task_id is not None:
        if not store.has(store.task_file(task_id)):
            raise ValueError(f"task {task_id!r} of workflow {workflow_id!r} has no checkpointed output")
        return store.load(store.task_file(task_id))
    deadline = None
    while not store.has("output.pkl"):
        st = get_status(workflow_id)
        if st in (WorkflowStatus.FAILED, WorkflowStatus.CANCELED, WorkflowStatus.RESUMABLE):
            if st == WorkflowStatus.CANCELED:
                raise WorkflowCancellationError(workflow_id)
            raise WorkflowExecutionError(workflow_id, RuntimeError(store.meta().get("error")))
        deadline = deadline or time.time()
        time.sleep(0.05)
    return store.load("output.pkl")


def get_status(workflow_id: str) -> WorkflowStatus:
    store = _Store(_storage(), workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    st = WorkflowStatus(store.meta().get("status", "NONE"))
    if st in (WorkflowStatus.RUNNING, WorkflowStatus.PENDING):
        # an executor that died with its driver leaves the workflow resumable
        if store.meta().get("driver_pid") not in (None, os.getpid()) and not _pid_alive(store.meta()["driver_pid"]):
            return WorkflowStatus.RESUMABLE
    return st


def _pid_alive(pid):
    try:
        os.kill(pid, 0)
        return True
    except OSError:
        return False


def get_metadata(workflow_id: str, task_id: Optional[str] = None) -> Dict[str, Any]:
    store = _Store(_storage(), workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    m = store.meta()
    if task_id is not None:
        return {"task_id": task_id, "checkpointed": store.has(store.task_file(task_id))}
    return {"workflow_id": workflow_id, "status": m.get("status"), "user_metadata": m.get("user_metadata", {}),
            "stats": {"start_time": m.get("start_time"), "end_time": m.get("end_time")}}


def list_all(status_filter=None) -> List[Tuple[str, WorkflowStatus]]:
    root = _storage()
    if isinstance(status_filter, (str, WorkflowStatus)):
        status_filter = {status_filter}
    want = {WorkflowStatus(s) for s in status_filter} if status_filter else None
    out = []
    for wid in sorted(os.listdir(root)):
        if not os.path.isfile(os.path.join(root, wid, "meta.json")):
            continue
        st = get_status(wid)
        if want is None or st in want:
            out.append((wid, st))
    return out


def cancel(workflow_id: str) -> None:
    store = _Store(_storage(), workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    if store.meta().get("status") in (WorkflowStatus.SUCCESSFUL.value,):
        return
    open(os.path.join(store.dir, "CANCEL"), "w").close()
    if store.meta().get("status") != WorkflowStatus.RUNNING.value:
        store.update_meta(status=WorkflowStatus.CANCELED.value)


def delete(workflow_id: str) -> None:
    store = _Store(_storage(), workflow_id)
    if not store.exists():
        raise WorkflowNotFoundError(workflow_id)
    if store.meta().get("status") == WorkflowStatus.RUNNING.value:
        raise WorkflowError(f"cannot delete running workflow {workflow_id}")
    shutil.rmtree(store.dir, ignore_errors=True)


# ------------------------------------------------------------ sleep/events
def _sleep_until(end: float):
    time.sleep(max(0.0, end - time.time()))
    return None


def _wait_event(listener_cls, args, kwargs):
    lst = listener_cls()

    async def go():
        ev = await lst.poll_for_event(*args, **kwargs)
        await lst.event_checkpointed(ev)
        return ev

    return asyncio.run(go())


def sleep(duration: float):
    """A DAG node finishing ``duration`` seconds after it starts."""
    from ..core.api import remote

    fn = remote(num_cpus=0)(lambda d: time.sleep(d))
    fn.__name__ = "workflow.sleep"
    return fn.bind(duration)


def wait_for_event(event_listener_type, *args, **kwargs):
    if not (isinstance(event_listener_type, type) and issubclass(event_listener_type, EventListener)):
        raise TypeError("wait_for_event expects an EventListener subclass")
    from ..core.api import remote

    fn = remote(num_cpus=0)(_wait_event)
    fn.__name__ = "workflow.wait_for_event"
    return fn.bind(event_listener_type, args, kwargs)
