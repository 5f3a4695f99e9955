"""HTTP proxy actor (reference: python/ray/serve/_private/proxy.py,
proxy_router.py).

A uvicorn server on its own thread inside an actor. Requests are matched to the
longest ``route_prefix``; the body is read fully and shipped with method / path
(relative to the prefix) / query / headers to the ingress deployment's
``handle_http_stream`` through the same power-of-two router handles use; the
response comes back as a stream (one item when it is complete at once). Routes are
refreshed from the controller every 0.5 s. ``/-/healthz`` and ``/-/routes`` are
built-in."""
from __future__ import annotations

import asyncio
import json
import socket
import threading
import time
import uuid


def _free_port(host="127.0.0.1"):
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


class HTTPProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 8000, request_timeout_s=None):
        import os

        import uvicorn

        # end-to-end limit per request (reference: proxy.py:143-147, 1026-1033: 408 and
        # the replica call cancelled); also from RAY_SERVE_REQUEST_PROCESSING_TIMEOUT_S
        if request_timeout_s is None:
            request_timeout_s = float(os.environ.get("RAY_SERVE_REQUEST_PROCESSING_TIMEOUT_S", "0")) or None
        self.request_timeout_s = request_timeout_s if request_timeout_s and request_timeout_s > 0 else None
        self.host = host
        self.port = port or _free_port(host)
        self.routes = {}
        self.alive = True
        self.num_requests = 0
        cfg = uvicorn.Config(self._app, host=self.host, port=self.port, log_level="warning",
                             lifespan="off", access_log=False, interface="asgi3")
        self.server = uvicorn.Server(cfg)
        self.thread = threading.Thread(target=self.server.run, name="serve-http", daemon=True)
        self.thread.start()
        self.refresher = threading.Thread(target=self._refresh_loop, daemon=True)
        self.refresher.start()
        deadline = time.time() + 30
        while not self.server.started and time.time() < deadline:
            time.sleep(0.02)

    def ready(self):
        return self.port

    def refresh(self):
        from ..core import api as core
        from .handle import _controller

        self.routes = core.get(_controller().get_routes.remote(), timeout=30)
        return list(self.routes)

    def _refresh_loop(self):
        from ..core import api as core
        from .handle import _controller

        while self.alive:
            try:
                self.routes = core.get(_controller().get_routes.remote(), timeout=5)
            except Exception:
                pass
            time.sleep(0.5)

    def _match(self, path: str):
        best = None
        for prefix, target in self.routes.items():
            p = prefix.rstrip("/")
            if path == p or path.startswith(p + "/") or p == "":
                if best is None or len(p) > len(best[0]):
                    best = (p, target)
        return best

    async def _app(self, scope, receive, send):
        if scope["type"] != "http":
            return
        path = scope["path"]
        if path == "/-/healthz":
            return await _respond(send, 200, b"success")
        if path == "/-/routes":
            body = json.dumps({k: v[0] for k, v in self.routes.items()}).encode()
            return await _respond(send, 200, body, "application/json")
        m = self._match(path)
        if m is None:
            return await _respond(send, 404, f"Path '{path}' not found. Routes: {list(self.routes)}".encode())
        prefix, (app_name, ingress) = m
        chunks = []
        while True:
            msg = await receive()
            chunks.append(msg.get("body", b""))
            if not msg.get("more_body"):
                break
        rel = path[len(prefix):] or "/"
        headers = [(k.decode(), v.decode()) for k, v in scope.get("headers", [])]
        model_id = next((v for k, v in headers if k.lower() == "serve_multiplexed_model_id"), "")
        req = {"method": scope["method"], "path": rel, "query_string": scope.get("query_string", b""),
               "headers": headers, "body": b"".join(chunks), "route_prefix": prefix or "/",
               "request_id": uuid.uuid4().hex[:12], "model_id": model_id}
        self.num_requests += 1
        timeout = self.request_timeout_s
        state = {"started": False}
        work = asyncio.ensure_future(self._forward(app_name, ingress, model_id, req, send, state))
        try:
            await asyncio.wait_for(asyncio.shield(work), timeout)
        except asyncio.TimeoutError:
            # cancel the queued assignment / replica call, then answer 408 if nothing
            # was sent yet (a streaming response already under way is just ended)
            work.cancel()
            try:
                await work
            except BaseException:  # noqa: BLE001
                pass
            msg = f"Request {req['request_id']} timed out after {timeout}s.".encode()
            if not state["started"]:
                await _respond(send, 408, msg)
            else:
                await send({"type": "http.response.body", "body": b"", "more_body": False})

    async def _forward(self, app_name, ingress, model_id, req, send, state):
        from ..exceptions import RayActorError
        from .exceptions import BackPressureError, DeploymentUnavailableError
        from .handle import _router

        router = _router(app_name, ingress)
        loop = asyncio.get_event_loop()
        # the replica streams the response back (handle_http_stream): a complete
        # response is one item; a streaming one (SSE, StreamingResponse) is relayed
        # chunk by chunk as the app produces it
        gen = first = tag = af = None
        try:
            for attempt in range(3):
                # a slot on a replica with fewer than max_ongoing_requests in flight;
                # queued in the router otherwise (BackPressureError when its queue is full)
                af = await loop.run_in_executor(None, router.assign, model_id)
                tag, h, _ = await asyncio.wrap_future(af)
                try:
                    gen = h.handle_http_stream.options(num_returns="streaming").remote(req)
                    first = await (await gen.__anext__())
                    break
                except RayActorError:
                    # the replica went away (redeploy / downscale / crash): re-resolve and retry
                    router.done(tag)
                    tag = gen = None
                    if attempt == 2:
                        raise
                    router.invalidate()
        except asyncio.CancelledError:
            self._cancel(router, af, tag, gen)
            raise
        except (BackPressureError, DeploymentUnavailableError) as e:
            if tag is not None:
                router.done(tag)
            return await _respond(send, 503, e.message.encode())
        except Exception as e:  # noqa
            if tag is not None:
                router.done(tag)
            return await _respond(send, 500, f"{type(e).__name__}: {e}".encode())
        try:
            if first[0] == "full":
                _, status, hdrs, body = first
                state["started"] = True
                await send({"type": "http.response.start", "status": status,
                            "headers": [(k.encode(), v.encode()) for k, v in hdrs
                                        if k.lower() != "content-length"]
                            + [(b"content-length", str(len(body)).encode())]})
                await send({"type": "http.response.body", "body": body})
                return
            _, status, hdrs = first
            state["started"] = True
            await send({"type": "http.response.start", "status": status,
                        "headers": [(k.encode(), v.encode()) for k, v in hdrs if k.lower() != "content-length"]})
            try:
                async for ref in gen:
                    item = await ref
                    await send({"type": "http.response.body", "body": item[1], "more_body": True})
            except asyncio.CancelledError:
                self._cancel(router, None, None, gen)
                raise
            await send({"type": "http.response.body", "body": b"", "more_body": False})
        finally:
            router.done(tag)

    @staticmethod
    def _cancel(router, af, tag, gen):
        from ..core import api as core

        if af is not None and not af.cancel():
            # assigned meanwhile: the slot is ours to give back
            if tag is None and not af.cancelled() and af.exception() is None:
                tag = af.result()[0]
        elif af is not None:
            return  # still queued: it never reached a replica
        if gen is not None:
            try:
                core.cancel(gen)
            except Exception:
                pass
        if tag is not None:
            router.done(tag)

    def stats(self):
        return {"num_requests": self.num_requests, "port": self.port}

    def shutdown(self):
        self.alive = False
        self.server.should_exit = True
        return True


async def _respond(send, status, body: bytes, ctype="text/plain; charset=utf-8"):
    await send({"type": "http.response.start", "status": status,
                "headers": [(b"content-type", ctype.encode()), (b"content-length", str(len(body)).encode())]})
    await send({"type": "http.response.body", "body": body})
