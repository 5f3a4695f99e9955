"""Replica actor (reference: python/ray/serve/_private/replica.py).

One async actor per replica. ``handle_request`` runs coroutine methods on the
actor's event loop and synchronous ones on a thread pool (so a slow sync
method never blocks other in-flight requests); ``handle_request_streaming``
streams generator outputs item by item; ``handle_http`` runs the deployment's
ASGI app (``@serve.ingress``) or calls ``__call__(starlette.Request)``."""
from __future__ import annotations

import asyncio
import concurrent.futures
import contextvars
import functools
import inspect
import json
import time
from typing import Any, Dict, List, Optional, Tuple

from .context import ReplicaContext, RequestContext, _request_context, _set_replica_context
from .multiplex import loaded_model_ids


def _bind_class_routes(app, instance, cls):
    """Re-create the ASGI app with class-method endpoints bound to ``instance``."""
    try:
        from fastapi import FastAPI
        from fastapi.routing import APIRoute
    except ImportError:  # starlette app: routes are plain callables
        return app
    if not isinstance(app, FastAPI):
        return app
    new = FastAPI(title=app.title)
    owned = {v for v in vars(cls).values() if inspect.isfunction(v)}
    for base in cls.__mro__[1:]:
        owned |= {v for v in vars(base).values() if inspect.isfunction(v)}
    for r in app.router.routes:
        if isinstance(r, APIRoute) and r.endpoint in owned:
            bound = getattr(instance, r.endpoint.__name__)
            new.add_api_route(r.path, bound, methods=list(r.methods), response_model=r.response_model,
                              status_code=r.status_code, name=r.name, response_class=r.response_class)
        else:
            new.router.routes.append(r)
    return new


def _to_http(result) -> Tuple[int, List[Tuple[str, str]], bytes]:
    try:
        from starlette.responses import Response
    except ImportError:  # pragma: no cover
        Response = ()
    if Response and isinstance(result, Response):
        return result.status_code, [(k.decode(), v.decode()) for k, v in result.raw_headers], result.body
    if isinstance(result, bytes):
        return 200, [("content-type", "application/octet-stream")], result
    if isinstance(result, str):
        return 200, [("content-type", "text/plain; charset=utf-8")], result.encode()
    if result is None:
        return 200, [("content-type", "text/plain")], b""
    try:
        return 200, [("content-type", "application/json")], json.dumps(result).encode()
    except TypeError:
        return 200, [("content-type", "text/plain; charset=utf-8")], str(result).encode()


class ServeReplica:
    def __init__(self, app_name: str, deployment_name: str, replica_tag: str, target, init_args,
                 init_kwargs, user_config, max_ongoing: int):
        self.app_name = app_name
        self.deployment_name = deployment_name
        self.replica_tag = replica_tag
        self.ongoing = 0
        self.total = 0
        self.pool = concurrent.futures.ThreadPoolExecutor(max(4, max_ongoing))
        self.is_function = not inspect.isclass(target)
        if self.is_function:
            self.callable = target
            self.asgi = None
        else:
            self.callable = target.__new__(target)
            _set_replica_context(ReplicaContext(app_name, deployment_name, replica_tag, self.callable))
            target.__init__(self.callable, *init_args, **init_kwargs)
            app = getattr(target, "_serve_asgi_app", None)
            self.asgi = _bind_class_routes(app, self.callable, target) if app is not None else None
        _set_replica_context(ReplicaContext(app_name, deployment_name, replica_tag, self.callable))
        self._pending_user_config = user_config
        self._ready = False

    async def ready(self):
        if not self._ready:
            if self._pending_user_config is not None:
                await self.reconfigure(self._pending_user_config)
            self._ready = True
        return self.replica_tag

    async def reconfigure(self, user_config):
        fn = getattr(self.callable, "reconfigure", None)
        if fn is None:
            if user_config is not None:
                raise ValueError("user_config set but the deployment has no reconfigure() method")
            return True
        r = fn(user_config)
        if inspect.isawaitable(r):
            await r
        return True

    def _method(self, name):
        if self.is_function:
            return self.callable
        if name == "__call__" and not hasattr(self.callable, "__call__"):
            raise AttributeError(f"deployment {self.deployment_name} has no __call__")
        return getattr(self.callable, name)

    async def _invoke(self, m, args, kwargs):
        if inspect.iscoroutinefunction(m) or getattr(m, "_serve_batch", False):
            return await m(*args, **kwargs)
        loop = asyncio.get_event_loop()
        ctx = contextvars.copy_context()
        r = await loop.run_in_executor(self.pool, functools.partial(ctx.run, m, *args, **kwargs))
        if inspect.isawaitable(r):
            r = await r
        return r

    async def handle_request(self, meta: Dict, *args, **kwargs):
        self.ongoing += 1
        self.total += 1
        tok = _request_context.set(RequestContext(meta.get("route", ""), meta.get("request_id", ""),
                                                  self.app_name, meta.get("model_id", "")))
        try:
            grpc_t = meta.get("grpc")
            if grpc_t:  # serialized protobuf request from the gRPC proxy
                from .grpc_proxy import decode_request

                args = (decode_request(grpc_t, args[0]),) + tuple(args[1:])
            m = self._method(meta.get("method", "__call__"))
            r = await self._invoke(m, args, kwargs)
            if inspect.isgenerator(r) or inspect.isasyncgen(r):
                raise TypeError("method returned a generator: call it with handle.options(stream=True)")
            if grpc_t:
                from .grpc_proxy import encode_response

                return encode_response(r)
            if getattr(m, "__ray_tensor_transport__", None) == "ipc":
                # @ray.method(tensor_transport="ipc") on the deployment method: GPU
                # tensors in the result go to the caller as HIP IPC handles (no host copy)
                from ..core.actor import TransportResult

                return TransportResult(r, "ipc")
            return r
        finally:
            _request_context.reset(tok)
            self.ongoing -= 1

    async def handle_request_streaming(self, meta: Dict, *args, **kwargs):
        self.ongoing += 1
        self.total += 1
        tok = _request_context.set(RequestContext(meta.get("route", ""), meta.get("request_id", ""),
                                                  self.app_name, meta.get("model_id", "")))
        try:
            m = self._method(meta.get("method", "__call__"))
            grpc_t = meta.get("grpc")
            if grpc_t:  # serialized protobuf in, each streamed message serialized out
                from .grpc_proxy import decode_request, encode_response

                args = (decode_request(grpc_t, args[0]),) + tuple(args[1:])
                async for x in self._stream_items(m, args, kwargs):
                    yield encode_response(x)
                return
            if inspect.isasyncgenfunction(m):
                async for x in m(*args, **kwargs):
                    yield x
            else:
                r = await self._invoke(m, args, kwargs)
                if inspect.isasyncgen(r):
                    async for x in r:
                        yield x
                elif inspect.isgenerator(r):
                    loop = asyncio.get_event_loop()
                    sentinel = object()
                    while True:
                        x = await loop.run_in_executor(self.pool, next, r, sentinel)
                        if x is sentinel:
                            break
                        yield x
                else:
                    yield r
        finally:
            _request_context.reset(tok)
            self.ongoing -= 1

    async def _stream_items(self, m, args, kwargs):
        if inspect.isasyncgenfunction(m):
            async for x in m(*args, **kwargs):
                yield x
            return
        r = await self._invoke(m, args, kwargs)
        if inspect.isasyncgen(r):
            async for x in r:
                yield x
        elif inspect.isgenerator(r):
            loop = asyncio.get_event_loop()
            sentinel = object()
            while True:
                x = await loop.run_in_executor(self.pool, next, r, sentinel)
                if x is sentinel:
                    break
                yield x
        else:
            yield r

    async def handle_http_stream(self, req: Dict):
        """Streaming form of :meth:`handle_http` for the proxy: yields
        ``("full", status, headers, body)`` when the response is complete in one
        message, else ``("start", status, headers)`` then ``("body", bytes)`` chunks
        as the app sends them (Server-Sent Events, StreamingResponse, generator
        results of plain ``__call__`` deployments) -- nothing is buffered to the end."""
        self.ongoing += 1
        self.total += 1
        tok = _request_context.set(RequestContext(req.get("route_prefix", ""), req.get("request_id", ""),
                                                  self.app_name, req.get("model_id", "")))
        try:
            if self.asgi is None:
                from starlette.requests import Request

                scope, receive = self._asgi_scope(req)
                r = await self._invoke(self._method("__call__"), (Request(scope, receive),), {})
                if inspect.isasyncgen(r) or inspect.isgenerator(r):
                    yield ("start", 200, [("content-type", "text/plain; charset=utf-8")])
                    if inspect.isasyncgen(r):
                        async for x in r:
                            yield ("body", x if isinstance(x, bytes) else str(x).encode())
                    else:
                        for x in r:
                            yield ("body", x if isinstance(x, bytes) else str(x).encode())
                    return
                yield ("full",) + tuple(_to_http(r))
                return
            q: asyncio.Queue = asyncio.Queue()
            scope, receive = self._asgi_scope(req)

            async def send(msg):
                await q.put(msg)

            async def run_app():
                try:
                    await self.asgi(scope, receive, send)
                except Exception as e:  # noqa: BLE001 - surfaced as a 500 below
                    await q.put({"type": "caamd.error", "error": e})
                finally:
                    await q.put(None)

            runner = asyncio.ensure_future(run_app())
            status, headers, started = 500, [], False
            try:
                while True:
                    msg = await q.get()
                    if msg is None:
                        break
                    kind = msg["type"]
                    if kind == "http.response.start":
                        status = msg["status"]
                        headers = [(k.decode(), v.decode()) for k, v in msg.get("headers", [])]
                    elif kind == "http.response.body":
                        body, more = msg.get("body", b""), msg.get("more_body", False)
                        if not started and not more:
                            yield ("full", status, headers, body)
                            return
                        if not started:
                            started = True
                            yield ("start", status, headers)
                        if body:
                            yield ("body", body)
                        if not more:
                            return
                    elif kind == "caamd.error" and not started:
                        e = msg["error"]
                        yield ("full", 500, [("content-type", "text/plain; charset=utf-8")],
                               f"{type(e).__name__}: {e}".encode())
                        return
                if not started:
                    yield ("full", status, headers, b"")
            finally:
                if not runner.done():
                    runner.cancel()
        finally:
            self.ongoing -= 1
            _request_context.reset(tok)

    def _asgi_scope(self, req: Dict):
        scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1",
                 "method": req["method"], "scheme": "http",
                 "path": req["path"], "raw_path": req["path"].encode(),
                 "root_path": "", "query_string": req.get("query_string", b""),
                 "headers": [(k.encode().lower(), v.encode()) for k, v in req.get("headers", [])],
                 "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 80)}
        body = req.get("body", b"")
        sent = {"done": False}

        async def receive():
            if not sent["done"]:
                sent["done"] = True
                return {"type": "http.request", "body": body, "more_body": False}
            await asyncio.sleep(3600)
            return {"type": "http.disconnect"}

        return scope, receive

    async def handle_http(self, req: Dict):
        """``req``: method, path, query_string, headers, body, route_prefix."""
        self.ongoing += 1
        self.total += 1
        tok = _request_context.set(RequestContext(req.get("route_prefix", ""), req.get("request_id", ""),
                                                  self.app_name, req.get("model_id", "")))
        try:
            scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1",
                     "method": req["method"], "scheme": "http",
                     "path": req["path"], "raw_path": req["path"].encode(),
                     "root_path": "", "query_string": req.get("query_string", b""),
                     "headers": [(k.encode().lower(), v.encode()) for k, v in req.get("headers", [])],
                     "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 80)}
            body = req.get("body", b"")
            sent = {"done": False}

            async def receive():
                if not sent["done"]:
                    sent["done"] = True
                    return {"type": "http.request", "body": body, "more_body": False}
                await asyncio.sleep(3600)
                return {"type": "http.disconnect"}

            if self.asgi is not None:
                out = {"status": 500, "headers": [], "body": []}

                async def send(msg):
                    if msg["type"] == "http.response.start":
                        out["status"] = msg["status"]
                        out["headers"] = [(k.decode(), v.decode()) for k, v in msg.get("headers", [])]
                    elif msg["type"] == "http.response.body":
                        out["body"].append(msg.get("body", b""))

                await self.asgi(scope, receive, send)
                return out["status"], out["headers"], b"".join(out["body"])
            from starlette.requests import Request

            request = Request(scope, receive)
            r = await self._invoke(self._method("__call__"), (request,), {})
            if inspect.isasyncgen(r) or inspect.isgenerator(r):
                chunks = []
                if inspect.isasyncgen(r):
                    async for x in r:
                        chunks.append(x if isinstance(x, bytes) else str(x).encode())
                else:
                    for x in r:
                        chunks.append(x if isinstance(x, bytes) else str(x).encode())
                return 200, [("content-type", "text/plain; charset=utf-8")], b"".join(chunks)
            return _to_http(r)
        finally:
            _request_context.reset(tok)
            self.ongoing -= 1

    async def get_metrics(self):
        if not hasattr(self, "_node_id"):
            try:
                from ..runtime_context import get_runtime_context

                self._node_id = get_runtime_context().get_node_id()
            except Exception:
                self._node_id = None
        return {"ongoing": self.ongoing, "total": self.total, "models": loaded_model_ids(self.callable),
                "time": time.time(), "node_id": self._node_id}

    async def check_health(self):
        fn = getattr(self.callable, "check_health", None)
        if fn is not None and not self.is_function:
            r = fn()
            if inspect.isawaitable(r):
                await r
        return True

    async def prepare_for_shutdown(self, timeout_s: float = 5.0, loop_s: float = 0.2):
        deadline = time.time() + timeout_s
        while self.ongoing > 0 and time.time() < deadline:
            await asyncio.sleep(loop_s)
        fn = getattr(self.callable, "__del__", None)
        if fn is not None and not self.is_function:
            try:
                fn()
            except Exception:
                pass
        return True
