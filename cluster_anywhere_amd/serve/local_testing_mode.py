"""``serve.run(app, _local_testing_mode=True)``: every deployment of the app runs in
THIS process, with no controller, proxy or replica actors (reference:
python/ray/serve/api.py:438-454, serve/_private/local_testing_mode.py).

Each deployment gets one in-process :class:`~.replica.ServeReplica` -- the same
request path real replicas run (sync methods on its thread pool, coroutines,
generators, ``@serve.batch``, multiplexing, ``reconfigure(user_config)``) -- on a
private asyncio loop thread. Its constructor runs eagerly, so errors surface in
``serve.run``. Bound child deployments are passed to their parents as local
handles, and a :class:`LocalDeploymentResponse` passed as an argument is resolved
before the call, as the reference router does."""
from __future__ import annotations

import asyncio
import concurrent.futures
import threading
import uuid
import warnings
from typing import Any, Dict, Optional

from .handle import DeploymentHandle


class _Loop:
    """One asyncio loop on a daemon thread, shared by the app's local replicas."""

    def __init__(self):
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self.loop.run_forever, name="serve-local-testing", daemon=True)
        self.thread.start()

    def submit(self, coro) -> concurrent.futures.Future:
        return asyncio.run_coroutine_threadsafe(coro, self.loop)


async def _resolve(x):
    if isinstance(x, LocalDeploymentResponse):
        return await x
    if isinstance(x, list):
        return [await _resolve(v) for v in x]
    if isinstance(x, tuple):
        return tuple([await _resolve(v) for v in x])
    if isinstance(x, dict):
        return {k: await _resolve(v) for k, v in x.items()}
    return x


class LocalDeploymentResponse:
    def __init__(self, fut: concurrent.futures.Future, request_id: str):
        self._fut = fut
        self._request_id = request_id

    def result(self, timeout_s: Optional[float] = None):
        try:
            return self._fut.result(timeout_s)
        except concurrent.futures.TimeoutError:
            from ..exceptions import GetTimeoutError

            raise GetTimeoutError(f"response not ready after {timeout_s}s")
        except concurrent.futures.CancelledError:
            from .exceptions import RequestCancelledError

            raise RequestCancelledError(self._request_id)

    def __await__(self):
        return asyncio.wrap_future(self._fut).__await__()

    def cancel(self):
        self._fut.cancel()

    def _to_object_ref(self, *a, **k):
        raise RuntimeError("Converting DeploymentResponses to ObjectRefs is not supported in local testing mode.")

    _to_object_ref_sync = _to_object_ref

    async def _to_object_ref_async(self, *a, **k):
        self._to_object_ref()

    @property
    def request_id(self):
        return self._request_id


class LocalDeploymentResponseGenerator:
    """Items of a streaming call. The generator runs to completion inside ONE task on
    the replica loop (its request context lives in that task) and hands items over
    through a queue."""

    _END = object()

    def __init__(self, loop: _Loop, agen):
        import queue

        self._q: "queue.Queue" = queue.Queue()
        self._task = loop.submit(self._pump(agen))

    async def _pump(self, agen):
        try:
            async for x in agen:
                self._q.put((True, x))
        except BaseException as e:  # noqa: BLE001 (re-raised in the consumer)
            self._q.put((False, e))
            return
        self._q.put((True, self._END))

    def _take(self):
        ok, x = self._q.get()
        if not ok:
            raise x
        return x

    def __iter__(self):
        return self

    def __next__(self):
        x = self._take()
        if x is self._END:
            raise StopIteration
        return x

    def __aiter__(self):
        return self

    async def __anext__(self):
        x = await asyncio.get_event_loop().run_in_executor(None, self._take)
        if x is self._END:
            raise StopAsyncIteration
        return x

    def cancel(self):
        self._task.cancel()


class LocalDeploymentHandle(DeploymentHandle):
    """A DeploymentHandle whose requests run on an in-process replica."""

    def __init__(self, replica, loop: _Loop, deployment_name: str, app_name: str, *,
                 method_name: str = "__call__", multiplexed_model_id: str = "", stream: bool = False):
        super().__init__(deployment_name, app_name, method_name=method_name,
                         multiplexed_model_id=multiplexed_model_id, stream=stream)
        self._replica = replica
        self._loop = loop

    def options(self, *, method_name: Optional[str] = None, multiplexed_model_id: Optional[str] = None,
                stream: Optional[bool] = None, **_ignored) -> "LocalDeploymentHandle":
        return LocalDeploymentHandle(
            self._replica, self._loop, self.deployment_name, self.app_name,
            method_name=method_name if method_name is not None else self._method,
            multiplexed_model_id=multiplexed_model_id if multiplexed_model_id is not None else self._model_id,
            stream=self._stream if stream is None else stream)

    def remote(self, *args, **kwargs):
        meta = {"method": self._method, "model_id": self._model_id, "request_id": uuid.uuid4().hex[:12]}
        rep = self._replica
        if self._stream:
            async def agen():
                a, kw = await _resolve(args), await _resolve(kwargs)
                async for x in rep.handle_request_streaming(meta, *a, **kw):
                    yield x

            return LocalDeploymentResponseGenerator(self._loop, agen())

        async def call():
            a, kw = await _resolve(args), await _resolve(kwargs)
            return await rep.handle_request(meta, *a, **kw)

        return LocalDeploymentResponse(self._loop.submit(call()), meta["request_id"])

    def __reduce__(self):
        raise TypeError("local testing mode handles cannot leave the process")

    def __repr__(self):
        return f"LocalDeploymentHandle(deployment={self.deployment_name!r}, app={self.app_name!r})"


def run_local(app, app_name: str) -> LocalDeploymentHandle:
    """Construct every deployment of ``app`` in this process; return the ingress handle."""
    from .deployment import Application
    from .replica import ServeReplica

    loop = _Loop()
    handles: Dict[int, LocalDeploymentHandle] = {}
    used: Dict[str, Any] = {}

    def sub(x):
        if isinstance(x, Application):
            return handles[id(x)]
        if isinstance(x, list):
            return [sub(v) for v in x]
        if isinstance(x, tuple):
            return tuple(sub(v) for v in x)
        if isinstance(x, dict):
            return {k: sub(v) for k, v in x.items()}
        return x

    for node in app._walk():  # children first
        d = node.deployment
        name = d.name
        k = 1
        while name in used and used[name] is not node:
            name = f"{d.name}_{k}"
            k += 1
        used[name] = node
        opts = d.config.ray_actor_options or {}
        if "num_gpus" in opts:
            warnings.warn(f"Deployment {name} has num_gpus configured; HIP_VISIBLE_DEVICES is not managed "
                          "in local testing mode.")
        if "runtime_env" in opts:
            warnings.warn(f"Deployment {name} has runtime_env configured; it is ignored in local testing mode.")
        replica = ServeReplica(app_name, name, f"{app_name}#{name}#local", d.func_or_class, sub(node.args),
                               sub(node.kwargs), d.config.user_config, d.config.max_ongoing_requests)
        loop.submit(replica.ready()).result()  # user_config -> reconfigure, eagerly
        handles[id(node)] = LocalDeploymentHandle(replica, loop, name, app_name)
    return handles[id(app)]
