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
import collections
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
    """Per-process router of one deployment. A request takes a replica slot only
    while that replica has fewer than ``max_ongoing_requests`` requests of this
    router in flight; otherwise it waits in the router's queue (FIFO) and is
    assigned by the router's drain thread when a slot frees or replicas are added.
    With ``max_queued_requests`` != -1 a request that would make the queue longer
    than that is rejected at once with :class:`BackPressureError` (reference:
    serve/_private/router.py:125-136)."""

    def __init__(self, app: str, deployment: str):
        self.app, self.deployment = app, deployment
        self.replicas: List[tuple] = []  # (tag, handle, models)
        self.version = -1
        self.inflight: Dict[str, int] = {}
        self.max_ongoing = 5
        self.max_queued = -1
        self.last_refresh = 0.0
        self.lock = threading.Lock()
        self.wake = threading.Condition(self.lock)
        self.pending: "collections.deque" = collections.deque()  # (model_id, Future)
        self.drainer: Optional[threading.Thread] = None
        self.rng = random.Random()
        self.router_id = uuid.uuid4().hex[:8]
        self._reported = (0, 0.0)

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
        version, reps, self.max_ongoing = snap[:3]
        self.max_queued = snap[3] if len(snap) > 3 else -1
        if version != self.version:
            with self.lock:
                self.version = version
                self.replicas = reps
                for tag, _, _ in reps:
                    self.inflight.setdefault(tag, 0)
                self.wake.notify_all()

    def _wait_for_replicas(self, timeout_s: float):
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
                return
            if time.time() > deadline:
                raise TimeoutError(f"no running replica of {self.app}/{self.deployment}")
            time.sleep(0.05)

    def _pick_locked(self, model_id: str):
        """A replica with a free slot (power of two choices over those), or None."""
        cands = self.replicas
        if not cands:
            return None
        if model_id:
            having = [r for r in cands if model_id in r[2]]
            if having:
                cands = having
            elif len(cands) > 1:
                # deterministic placement for a new model: same replica for same id
                cands = [cands[hash(model_id) % len(cands)]]
        cap = max(1, int(self.max_ongoing or 1))
        free = [r for r in cands if self.inflight.get(r[0], 0) < cap]
        if not free:
            return None
        if len(free) == 1:
            pick = free[0]
        else:
            a, b = self.rng.sample(free, 2)
            pick = a if self.inflight.get(a[0], 0) <= self.inflight.get(b[0], 0) else b
        self.inflight[pick[0]] = self.inflight.get(pick[0], 0) + 1
        return pick

    def assign(self, model_id: str = "", timeout_s: float = 60.0) -> concurrent.futures.Future:
        """Future of ``(tag, handle, models)``: resolved at once when a replica has a
        free slot and nothing is queued, else when the drain thread assigns it."""
        from .exceptions import BackPressureError

        self._wait_for_replicas(timeout_s)
        self._refresh()
        fut: concurrent.futures.Future = concurrent.futures.Future()
        with self.lock:
            if not self.pending:
                pick = self._pick_locked(model_id)
                if pick is not None:
                    fut.set_result(pick)
                    return fut
            if self.max_queued is not None and self.max_queued >= 0 and len(self.pending) >= self.max_queued:
                raise BackPressureError(len(self.pending), self.max_queued)
            self.pending.append((model_id, fut))
            if self.drainer is None or not self.drainer.is_alive():
                self.drainer = threading.Thread(target=self._drain_loop, daemon=True,
                                                name=f"serve-router-{self.deployment}")
                self.drainer.start()
            self.wake.notify_all()
        return fut

    def choose(self, model_id: str = "", timeout_s: float = 60.0):
        return self.assign(model_id, timeout_s).result(timeout_s)

    def num_queued(self) -> int:
        with self.lock:
            return sum(1 for _, f in self.pending if not f.done())

    def _report_queued(self, n: int):
        """Tell the controller how many requests wait here (autoscaling input)."""
        now = time.time()
        if n == self._reported[0] and now - self._reported[1] < 0.5:
            return
        self._reported = (n, now)
        try:
            _controller().record_handle_metrics.remote(self.app, self.deployment, n, self.router_id)
        except Exception:
            pass

    def _drain_loop(self):
        # assignments are handed out here, never in the thread that completed a
        # response (a core callback thread), so callers' submissions run off it
        while True:
            self._report_queued(len(self.pending))
            ready = []
            with self.lock:
                while self.pending:
                    model_id, f = self.pending[0]
                    if f.done():  # cancelled while queued
                        self.pending.popleft()
                        continue
                    pick = self._pick_locked(model_id)
                    if pick is None:
                        break
                    self.pending.popleft()
                    ready.append((f, pick))
                if not self.pending and not ready:
                    self.drainer = None
                    done = True
                else:
                    done = False
                if not ready and not done:
                    self.wake.wait(0.05)
            if done:
                self._report_queued(0)
                return
            for f, pick in ready:
                if f.set_running_or_notify_cancel():
                    f.set_result(pick)
                else:
                    self.done(pick[0])
            if not ready:
                try:
                    self._refresh()  # replicas added by autoscaling / recovery free slots too
                except Exception:
                    pass

    def done(self, tag):
        with self.lock:
            self.inflight[tag] = max(0, self.inflight.get(tag, 0) - 1)
            if self.pending:
                self.wake.notify_all()

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
    """Result of ``handle.remote()``. ``_assigned`` resolves to ``(tag, ref)`` once the
    router gave the request a replica slot (at once, or later from its queue)."""

    def __init__(self, router: _Router, assigned: concurrent.futures.Future, resend, request_id: str = ""):
        self._router = router
        self._assigned = assigned
        self._resend = resend
        self._request_id = request_id
        self._fut = None
        self._lock = threading.Lock()

    def _future(self) -> concurrent.futures.Future:
        with self._lock:
            if self._fut is None:
                outer: concurrent.futures.Future = concurrent.futures.Future()
                router = self._router

                def on_ref(af):
                    try:
                        tag, ref = af.result()
                    except BaseException as e:  # noqa: BLE001 (cancelled / submission failed)
                        if isinstance(e, concurrent.futures.CancelledError):
                            from .exceptions import RequestCancelledError

                            e = RequestCancelledError(self._request_id)
                        outer.set_exception(e)
                        return

                    def fin(g, t=tag):
                        router.done(t)
                        try:
                            outer.set_result(g.result())
                        except BaseException as e:  # noqa: BLE001
                            outer.set_exception(e)

                    ref.future().add_done_callback(fin)

                self._assigned.add_done_callback(on_ref)
                self._fut = outer
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
        return self._assigned.result()[1]

    async def _to_object_ref_async(self):
        return (await asyncio.wrap_future(self._assigned))[1]

    def _to_object_ref_sync(self):
        return self._to_object_ref()

    def cancel(self):
        """Cancel a queued request (it never reaches a replica) or the replica call."""
        if self._assigned.cancel():
            return
        try:
            if self._assigned.done() and self._assigned.exception() is None:
                core.cancel(self._assigned.result()[1])
        except Exception:
            pass

    @property
    def request_id(self):
        return self._request_id


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
            assigned = router.assign(self._model_id)  # BackPressureError when the queue is full
            out: concurrent.futures.Future = concurrent.futures.Future()

            def submit(af):
                try:
                    tag, h, _ = af.result()
                except BaseException as e:  # noqa: BLE001 (cancelled while queued)
                    if isinstance(e, concurrent.futures.CancelledError):
                        out.cancel()
                    else:
                        out.set_exception(e)
                    return
                if not out.set_running_or_notify_cancel():  # cancelled meanwhile
                    router.done(tag)
                    return
                try:
                    out.set_result((tag, h.handle_request.remote(meta, *args, **kwargs)))
                except BaseException as e:  # noqa: BLE001
                    router.done(tag)
                    out.set_exception(e)

            assigned.add_done_callback(submit)
            resp = DeploymentResponse(router, out, send, meta["request_id"])
            if not assigned.done():
                # cancelling the response cancels the queued assignment
                out.add_done_callback(lambda f, a=assigned: f.cancelled() and a.cancel())
            return resp

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
