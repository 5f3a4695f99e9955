"""Actors (reference: python/ray/actor.py: ActorClass :602, ActorHandle :1265,
``@ray.method`` :53, ``exit_actor`` :1760). Each actor runs in a dedicated worker
process; method calls from one caller execute in submission order; async
(``async def``) actors run their methods on an asyncio loop, threaded actors use
a ``max_concurrency`` thread pool."""
from __future__ import annotations

import inspect
import os
from typing import Any, Dict

from . import context, options as opt_utils, serialization
from .head import ACTOR_CREATE, ACTOR_METHOD
from .ids import ActorID


def method(*args, **kwargs):
    """``@method(num_returns=2, concurrency_group=..., tensor_transport="ipc")`` for
    actor methods. ``tensor_transport="ipc"`` returns GPU tensors as HIP IPC
    handles (zero-copy for same-node readers, experimental/gpu_objects.py)."""

    def deco(fn):
        if "num_returns" in kwargs:
            fn.__ray_num_returns__ = kwargs["num_returns"]
        if "concurrency_group" in kwargs:
            fn.__ray_concurrency_group__ = kwargs["concurrency_group"]
        if kwargs.get("tensor_transport") not in (None, "object_store", "ipc"):
            raise ValueError("tensor_transport must be 'object_store' (host copy) or 'ipc'")
        if kwargs.get("tensor_transport") == "ipc":
            fn.__ray_tensor_transport__ = "ipc"
        return fn

    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    return deco


class TransportResult:
    """Return value of an actor method that picks its tensor transport per call
    (``TransportResult(value, "ipc")``): the worker serializes ``value`` with that
    transport instead of the method's static ``@method(tensor_transport=...)``.
    Serve replicas use it to honour the annotation of the deployment method they
    dispatch to (serve/replica.py)."""

    __slots__ = ("value", "transport")

    def __init__(self, value, transport):
        if transport not in (None, "object_store", "ipc"):
            raise ValueError("tensor_transport must be 'object_store' (host copy) or 'ipc'")
        self.value, self.transport = value, transport


def _method_meta(cls) -> Dict[str, Any]:
    meta = {}
    for name, m in inspect.getmembers(cls, predicate=lambda x: inspect.isfunction(x) or inspect.ismethod(x)):
        nr = getattr(m, "__ray_num_returns__", None)
        if nr is None:
            nr = "streaming" if (inspect.isgeneratorfunction(m) or inspect.isasyncgenfunction(m)) else 1
        meta[name] = {"num_returns": nr, "concurrency_group": getattr(m, "__ray_concurrency_group__", None)}
    return meta


class ActorMethod:
    def __init__(self, handle: "ActorHandle", name: str, num_returns=1, concurrency_group=None, gen_bp=None):
        self._handle = handle
        self._name = name
        self._num_returns = num_returns
        self._cg = concurrency_group
        self._gen_bp = gen_bp

    def __call__(self, *a, **k):
        raise TypeError(f"Actor methods cannot be called directly; use '{self._name}.remote()'.")

    def options(self, **kw):
        return ActorMethod(self._handle, self._name, kw.get("num_returns", self._num_returns),
                           kw.get("concurrency_group", self._cg),
                           kw.get("_generator_backpressure_num_objects", self._gen_bp))

    def remote(self, *args, **kwargs):
        return self._handle._call(self._name, args, kwargs, self._num_returns, self._cg, self._gen_bp)

    def bind(self, *args, **kwargs):
        from ..dag import ClassMethodNode

        return ClassMethodNode(self._handle, self._name, args, kwargs, self._num_returns)


HANDLE_SUFFIX = b"\xac" * 8


def handle_ref_id(actor_id: bytes) -> bytes:
    """Object id whose reference count tracks the live handles of an actor."""
    return actor_id + HANDLE_SUFFIX


class ActorHandle:
    """Handle to an actor. Holds a reference on the actor's handle-object so an
    unnamed, non-detached actor is terminated (after its queued calls) once no
    handle to it is left anywhere (reference: actor handle ref-counting)."""

    def __init__(self, actor_id: bytes, meta: Dict[str, Any], _owned: bool = False, _ref=None):
        from .object_ref import ObjectRef

        self._actor_id = actor_id
        self._meta = meta
        self._ref = _ref if _ref is not None else ObjectRef(handle_ref_id(actor_id), _owned=_owned)

    @property
    def _ray_actor_id(self):
        return ActorID(self._actor_id)

    def __getattr__(self, name):
        if name.startswith("__") and name not in ("__ray_terminate__", "__ray_call__"):
            raise AttributeError(name)
        methods = self._meta.get("methods", {})
        if name not in methods and name not in ("__ray_terminate__", "__ray_ready__", "__ray_call__"):
            raise AttributeError(f"'{self._meta.get('class_name')}' actor has no method '{name}'")
        m = methods.get(name, {"num_returns": 1, "concurrency_group": None})
        return ActorMethod(self, name, m["num_returns"], m.get("concurrency_group"))

    def _call(self, name, args, kwargs, num_returns, cg, gen_bp=None):
        if context.local_mode:
            from .local_mode import run_local_method

            return run_local_method(self._actor_id, name, args, kwargs, num_returns)
        w = context.worker
        if name == "__ray_ready__":
            name, args, kwargs = "__ray_ready__", (), {}
        refs = w.submit(ACTOR_METHOD, None, self._meta.get("class_name", "Actor"), args, kwargs,
                        num_returns=num_returns, actor_id=self._actor_id, method=name,
                        concurrency_group=cg, max_retries=self._meta.get("max_task_retries", 0),
                        gen_bp=gen_bp)
        if num_returns == "streaming":
            return refs
        if num_returns == 1 or num_returns == "dynamic":
            return refs[0]
        return refs

    def __reduce__(self):
        # the ObjectRef travels with the handle: it is recorded as a contained
        # reference, so the actor stays alive while the handle is in flight
        return (_rebuild_handle, (self._actor_id, self._meta, self._ref))

    def __repr__(self):
        return f"Actor({self._meta.get('class_name')}, {self._actor_id.hex()})"

    def __eq__(self, other):
        return isinstance(other, ActorHandle) and other._actor_id == self._actor_id

    def __hash__(self):
        return hash(self._actor_id)


def _rebuild_handle(actor_id, meta, ref):
    return ActorHandle(actor_id, meta, _ref=ref)


class _ReadyMixin:
    def __ray_ready__(self):
        return True

    def __ray_call__(self, fn, *args, **kwargs):
        return fn(self, *args, **kwargs)


class ActorClass:
    def __init__(self, cls, opts: Dict[str, Any]):
        self._cls = cls
        self._options = opt_utils.validate(opts, opt_utils.ACTOR_DEFAULTS, "actor")
        self._name = f"{cls.__module__}.{cls.__qualname__}"
        self._blob = None
        from .worker import function_id

        self._fn_id = function_id(cls)
        self.__name__ = cls.__name__
        self.__doc__ = cls.__doc__

    def __call__(self, *a, **k):
        raise TypeError(f"Actors cannot be instantiated directly. Instead of '{self.__name__}()', "
                        f"use '{self.__name__}.remote()'.")

    def options(self, **kw) -> "ActorClass":
        ac = ActorClass.__new__(ActorClass)
        ac.__dict__.update(self.__dict__)
        merged = dict(self._options)
        merged.update(kw)
        ac._options = opt_utils.validate(merged, opt_utils.ACTOR_DEFAULTS, "actor")
        return ac

    def _blob_fn(self):
        if self._blob is None:
            wrapped = type(self._cls.__name__, (self._cls, _ReadyMixin), {"__module__": self._cls.__module__})
            wrapped.__qualname__ = self._cls.__qualname__
            self._blob = serialization.dumps_function(wrapped)
        return self._blob

    def remote(self, *args, **kwargs) -> ActorHandle:
        from .api import _ensure_init

        _ensure_init()
        o = self._options
        meta = {"methods": _method_meta(self._cls), "class_name": self._cls.__name__,
                "max_task_retries": o.get("max_task_retries") or 0}
        if context.local_mode:
            from .local_mode import create_local_actor

            return create_local_actor(self._cls, args, kwargs, meta)
        w = context.worker
        ns = o.get("namespace") or w.namespace
        if o.get("name"):
            existing = w.request(lambda r: ("check_name", r, ns, o["name"]))
            if existing is not None:
                if o.get("get_if_exists"):
                    return ActorHandle(existing[0], existing[1] or meta)
                raise ValueError(f"The name {o['name']!r} (namespace={ns!r}) is already taken.")
        w.register_function(self._fn_id, self._blob_fn)
        actor_id = os.urandom(16)
        actor_opts = {"max_restarts": o["max_restarts"], "max_task_retries": o["max_task_retries"],
                      "max_concurrency": o["max_concurrency"], "name": o["name"], "namespace": ns,
                      "lifetime": o["lifetime"], "handle_meta": meta,
                      "concurrency_groups": o.get("concurrency_groups")}
        w.submit(ACTOR_CREATE, self._fn_id, self._cls.__name__, args, kwargs, num_returns=1,
                 resources=opt_utils.resource_demand(o, actor=True),
                 strategy=opt_utils.strategy_tuple(o), actor_id=actor_id, actor_opts=actor_opts,
                 runtime_env=o.get("runtime_env"), max_retries=0)
        return ActorHandle(actor_id, meta, _owned=True)

    def bind(self, *args, **kwargs):
        from ..dag import ClassNode

        return ClassNode(self, args, kwargs)


def exit_actor():
    """Gracefully exit the current actor after the running method returns."""
    if context.worker is None or context.worker.actor_instance is None:
        raise TypeError("exit_actor() called outside of an actor")
    e = SystemExit(0)
    e._caamd_exit_actor = True
    raise e
