"""Deployment handles and the client-side router (reference:
python/ray/serve/handle.py, _private/router.py,
_private/replica_scheduler/pow_2_scheduler.py).

Routing is power-of-two-choices over the replicas' in-flight counts tracked
locally by this process's router (incremented at send, decremented when the
response future completes). Requests carrying a multiplexed model id prefer
replicas that already hold the model. Replica membership is cached and
refreshed from the controller when its version changes (polled at most every
``_REFRESH_S``) or when a replica dies."""
from __future__ import annotations

import asyncio
import concurrent.futures
import random
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

from ..core import api as core

_REFRESH_S = 0.5


def _controller():
    from .controller import CONTROLLER_NAME, NAMESPACE

    return core.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)


class _Router:
    def __init__(self, app: str, deployment: str):
        self.app, self.deployment = app, deployment
        self.replicas: List[tuple] = []  # (tag, handle, models)
        self.version = -1
        self.inflight: Dict[str, int] = {}
        self.max_ongoing = 5
        self.last_refresh = 0.0
        self.lock = threading.Lock()
        self.rng = random.Random()

    def _refresh(self, force=False):
        now = time.time()
        if not force and now - self.last_refresh < _REFRESH_S and self.replicas:
            return
        self.last_refresh = now
        try:
            snap = core.get(_controller().get_replicas.remote(self.app, self.deployment), timeout=10)
        except Exception:
            if self.replicas:
                return  # controller restarting: keep routing to the last known replicas
            raise
        if snap is None:
            raise KeyError(f"deployment {self.deployment!r} of application {self.app!r} does not exist")
        version, reps, self.max_ongoing = snap
        if version != self.version:
            self.version = version
            self.replicas = reps
            for tag, _, _ in reps:
                self.inflight.setdefault(tag, 0)

    def choose(self, model_id: str = "", timeout_s: float = 60.0):
        deadline = time.time() + timeout_s
        while True:
            try:
                self._refresh(force=not self.replicas)
            except KeyError:
                raise
            except Exception:
                if time.time() > deadline:
                    raise
            if self.replicas:
                break
            if time.time() > deadline:
                raise TimeoutError(f"no running replica of {self.app}/{self.deployment}")
            time.sleep(0.05)
        cands = self.replicas
        if model_id:
            having = [r for r in cands if model_id in r[2]]
            if having:
                cands = having
            else:
                # deterministic placement for a new model: same replica for same id
                cands = [cands[hash(model_id) % len(cands)]] if len(cands) > 1 else cands
        with self.lock:
            if len(cands) == 1:
                pick = cands[0]
            else:
                a, b = self.rng.sample(cands, 2)
                pick = a if self.inflight.get(a[0], 0) <= self.inflight.get(b[0], 0) else b
            self.inflight[pick[0]] = self.inflight.get(pick[0], 0) + 1
        return pick

    def done(self, tag):
        with self.lock:
            self.inflight[tag] = max(0, self.inflight.get(tag, 0) - 1)

    def drop_actor(self, actor_id):
        with self.lock:
            keep = [r for r in self.replicas if getattr(r[1], "_actor_id", None) != actor_id]
            if len(keep) != len(self.replicas):
                self.replicas = keep
                self.version = -1  # take the controller's next snapshot whatever its version

    def invalidate(self):
        self.last_refresh = 0.0
        self.version = -1
        self.replicas = []


_routers: Dict[tuple, _Router] = {}
_routers_lock = threading.Lock()
_actor_sub = False


def _on_actor_event(actor_id, info):
    """Head pubsub (core/head.py ``_publish``): a replica that died leaves every
    router of this process at once, before the controller's next health check."""
    if info.get("state") != "DEAD":
        return
    for r in list(_routers.values()):
        r.drop_actor(actor_id)


def _ensure_actor_sub():
    global _actor_sub
    if _actor_sub:
        return
    from ..core import context

    w = context.worker
    if w is not None and hasattr(w, "subscribe"):
        try:
            w.subscribe("actor", _on_actor_event)
            _actor_sub = True
        except Exception:
            pass


def _router(app, dep) -> _Router:
    _ensure_actor_sub()
    with _routers_lock:
        r = _routers.get((app, dep))
        if r is None:
            r = _routers[(app, dep)] = _Router(app, dep)
        return r


def _unwrap(x):
    if isinstance(x, DeploymentResponse):
        return x._to_object_ref()
    return x


class DeploymentResponse:
    def __init__(self, router: _Router, tag: str, ref, resend):
        self._router = router
        self._tag = tag
        self._ref = ref
        self._resend = resend
        self._fut = None
        self._lock = threading.Lock()

    def _future(self) -> concurrent.futures.Future:
        with self._lock:
            if self._fut is None:
                self._fut = self._ref.future()
                self._fut.add_done_callback(lambda f, t=self._tag, r=self._router: r.done(t))
            return self._fut

    def result(self, timeout_s: Optional[float] = None, _retries: int = 1):
        from ..exceptions import RayActorError

        try:
            return self._future().result(timeout_s)
        except concurrent.futures.TimeoutError:
            from ..exceptions import GetTimeoutError

            raise GetTimeoutError(f"response not ready after {timeout_s}s")
        except RayActorError:
            if _retries <= 0:
                raise
            self._router.invalidate()
            again = self._resend()
            return again.result(timeout_s, _retries - 1)

    def __await__(self):
        return self._await_retrying(1).__await__()

    async def _await_retrying(self, retries: int):
        from ..exceptions import RayActorError

        try:
            return await asyncio.wrap_future(self._future())
        except RayActorError:
            if retries <= 0:
                raise
            self._router.invalidate()  # the replica died (e.g. redeploy): pick again
            return await self._resend()._await_retrying(retries - 1)

    def _to_object_ref(self):
        return self._ref

    async def _to_object_ref_async(self):
        return self._ref

    def _to_object_ref_sync(self):
        return self._ref

    def cancel(self):
        try:
            core.cancel(self._ref)
        except Exception:
            pass

    @property
    def request_id(self):
        return self._ref.hex()


class DeploymentResponseGenerator:
    def __init__(self, router: _Router, tag: str, gen):
        self._router = router
        self._tag = tag
        self._gen = gen
        self._done = False

    def _finish(self):
        if not self._done:
            self._done = True
            self._router.done(self._tag)

    def __iter__(self):
        return self

    def __next__(self):
        try:
            ref = next(self._gen)
        except StopIteration:
            self._finish()
            raise
        return core.get(ref)

    def __aiter__(self):
        return self

    async def __anext__(self):
        try:
            ref = await self._gen.__anext__()
        except StopAsyncIteration:
            self._finish()
            raise
        return await ref

    def cancel(self):
        self._finish()


class DeploymentHandle:
    def __init__(self, deployment_name: str, app_name: str = "default", *, method_name: str = "__call__",
                 multiplexed_model_id: str = "", stream: bool = False, _grpc: Optional[tuple] = None):
        self.deployment_name = deployment_name
        self.app_name = app_name
        self._method = method_name
        self._model_id = multiplexed_model_id
        self._stream = stream
        self._grpc = _grpc  # (request type name, request id): serialized protobuf in/out (grpc_proxy.py)

    def options(self, *, method_name: Optional[str] = None, multiplexed_model_id: Optional[str] = None,
                stream: Optional[bool] = None, use_new_handle_api: bool = True, _grpc: Optional[tuple] = None,
                **_ignored) -> "DeploymentHandle":
        return DeploymentHandle(self.deployment_name, self.app_name,
                                method_name=method_name if method_name is not None else self._method,
                                multiplexed_model_id=multiplexed_model_id if multiplexed_model_id is not None
                                else self._model_id,
                                stream=self._stream if stream is None else stream,
                                _grpc=_grpc if _grpc is not None else self._grpc)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return self.options(method_name=name)

    def remote(self, *args, **kwargs):
        router = _router(self.app_name, self.deployment_name)
        args = tuple(_unwrap(a) for a in args)
        kwargs = {k: _unwrap(v) for k, v in kwargs.items()}
        meta = {"method": self._method, "model_id": self._model_id, "request_id": uuid.uuid4().hex[:12]}
        if self._grpc is not None:
            meta["grpc"] = self._grpc[0]
            if self._grpc[1]:
                meta["request_id"] = self._grpc[1]

        if self._stream:
            tag, h, _ = router.choose(self._model_id)
            gen = h.handle_request_streaming.options(num_returns="streaming").remote(meta, *args, **kwargs)
            return DeploymentResponseGenerator(router, tag, gen)

        def send():
            tag, h, _ = router.choose(self._model_id)
            ref = h.handle_request.remote(meta, *args, **kwargs)
            return DeploymentResponse(router, tag, ref, send)

        resp = send()
        resp._future()  # start tracking completion now (in-flight accounting)
        return resp

    def __reduce__(self):
        return (DeploymentHandle, (self.deployment_name, self.app_name),
                {"_method": self._method, "_model_id": self._model_id, "_stream": self._stream})

    def __setstate__(self, st):
        self.__dict__.update(st)

    def __repr__(self):
        return f"DeploymentHandle(deployment={self.deployment_name!r}, app={self.app_name!r})"
