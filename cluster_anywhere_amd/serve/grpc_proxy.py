"""gRPC ingress (reference roles: python/ray/serve/_private/proxy.py:532 ``gRPCProxy``,
python/ray/serve/_private/grpc_util.py ``gRPCGenericServer``, serve/config.py
``gRPCOptions``).

``serve.start(grpc_options=gRPCOptions(port=..., grpc_servicer_functions=[...]))``
starts a ``grpc.server`` inside a proxy actor. Each entry of
``grpc_servicer_functions`` is a protoc-style ``add_<Service>Servicer_to_server``
function (or its import path). The proxy calls it against a *capturing*
server, which records every method's handler (its request type, response
serializer and whether it streams), and registers in its place a BYTES-IN /
BYTES-OUT handler on the real server:

* the request stays serialized: the proxy never needs the user's message
  classes. It forwards ``(method, request type name, bytes)`` to the ingress
  deployment of the target application, chosen by the ``application`` metadata
  key (or the only running application);
* the replica rebuilds the request from the descriptor pool (the deployment's
  module imports its ``*_pb2``), calls the deployment method of the same name
  (``multiplexed_model_id`` / ``request_id`` metadata become the request
  context), and serializes the returned message (or each streamed message);
* unary->unary and unary->stream methods are supported; errors map to gRPC
  status codes (NOT_FOUND for an unknown application, DEADLINE_EXCEEDED,
  INTERNAL with the exception text).

The built-in ``ray.serve.RayServeAPIService`` (``ListApplications``,
``Healthz``) is always served.
"""
from __future__ import annotations

import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple, Union


@dataclass
class gRPCOptions:
    port: int = 9000
    grpc_servicer_functions: List[Union[str, Callable]] = field(default_factory=list)
    request_timeout_s: Optional[float] = None
    host: str = "127.0.0.1"


def _resolve(fn):
    if callable(fn):
        return fn
    mod, _, name = str(fn).rpartition(".")
    import importlib

    return getattr(importlib.import_module(mod), name)


class _Capture:
    """Stands in for ``grpc.Server`` while a servicer-registration function runs."""

    def __init__(self):
        self.methods: Dict[str, Any] = {}  # "/pkg.Service/Method" -> RpcMethodHandler

    def add_generic_rpc_handlers(self, handlers):
        for h in handlers:
            name = getattr(h, "_name", None) or getattr(h, "service_name", lambda: None)()
            table = getattr(h, "_method_handlers", None)
            if table is None or name is None:
                raise TypeError("unsupported generic handler; pass a protoc-generated add_*_to_server")
            for mname, mh in table.items():
                full = mname if mname.startswith("/") else f"/{name}/{mname}"
                self.methods[full] = mh

    def add_registered_method_handlers(self, service_name, method_handlers):
        for mname, mh in method_handlers.items():
            self.methods[f"/{service_name}/{mname}"] = mh


class _Dummy:
    """Servicer placeholder: registration functions only take bound attributes."""

    def __getattr__(self, name):
        return lambda *a, **k: None


def _type_name(mh) -> Optional[str]:
    deser = mh.request_deserializer
    owner = getattr(deser, "__self__", None)
    desc = getattr(owner, "DESCRIPTOR", None)
    return desc.full_name if desc is not None else None


class gRPCProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 9000, servicer_functions=(),
                 request_timeout_s: Optional[float] = None):
        import grpc

        from . import _serve_api_pb2 as api

        self.timeout = request_timeout_s
        self.apps: Dict[str, str] = {}
        self.num_requests = 0
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=64))
        cap = _Capture()
        for fn in servicer_functions:
            _resolve(fn)(_Dummy(), cap)
        by_service: Dict[str, Dict[str, Any]] = {}
        for full, mh in cap.methods.items():
            _, svc, meth = full.split("/")
            if mh.request_streaming:
                raise ValueError(f"{full}: client-streaming gRPC methods are not supported")
            tname = _type_name(mh)
            ident = lambda b: b  # noqa: E731 - bytes pass through the proxy untouched
            if mh.response_streaming:
                h = grpc.unary_stream_rpc_method_handler(self._streamer(meth, tname), request_deserializer=ident,
                                                         response_serializer=ident)
            else:
                h = grpc.unary_unary_rpc_method_handler(self._unary(meth, tname), request_deserializer=ident,
                                                        response_serializer=ident)
            by_service.setdefault(svc, {})[meth] = h
        for svc, table in by_service.items():
            self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(svc, table),))
        api.add_RayServeAPIServiceServicer_to_server(self, self.server)
        self.port = self.server.add_insecure_port(f"{host}:{port}")
        if not self.port:
            raise RuntimeError(f"gRPC proxy could not bind {host}:{port}")
        self.server.start()
        self._refresh()
        threading.Thread(target=self._refresh_loop, name="serve-grpc-refresh", daemon=True).start()

    # ------------------------------------------------------------ control
    def ready(self):
        return self.port

    def _refresh(self):
        from ..core import api as core
        from .handle import _controller

        ctl = _controller()
        st = core.get(ctl.status.remote(), timeout=30)
        self.apps = {n: core.get(ctl.get_ingress.remote(n), timeout=30) for n, a in st.items()
                     if a["status"] in ("RUNNING", "DEPLOYING")}
        return list(self.apps)

    def refresh(self):
        return self._refresh()

    def _refresh_loop(self):
        while True:
            time.sleep(0.5)
            try:
                self._refresh()
            except Exception:
                pass

    def stop(self):
        self.server.stop(grace=1.0)
        return True

    # ------------------------------------------------------------ built-in API
    def ListApplications(self, request, context):
        from . import _serve_api_pb2 as api

        return api.ListApplicationsResponse(application_names=sorted(self.apps))

    def Healthz(self, request, context):
        from . import _serve_api_pb2 as api

        return api.HealthzResponse(message="success")

    # ------------------------------------------------------------ routing
    def _target(self, context) -> Tuple[str, str, Dict[str, str]]:
        import grpc

        md = {k: v for k, v in (context.invocation_metadata() or ())}
        app = md.get("application")
        if app is None:
            if len(self.apps) != 1:
                context.abort(grpc.StatusCode.NOT_FOUND,
                              f"set the 'application' metadata key; running applications: {sorted(self.apps)}")
            app = next(iter(self.apps))
        ingress = self.apps.get(app)
        if ingress is None:
            self._refresh()
            ingress = self.apps.get(app)
        if ingress is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"application {app!r} not found; running: {sorted(self.apps)}")
        return app, ingress, md

    def _handle(self, context, meth, tname, stream):
        from .handle import DeploymentHandle

        app, ingress, md = self._target(context)
        self.num_requests += 1
        return DeploymentHandle(ingress, app).options(
            method_name=meth, multiplexed_model_id=md.get("multiplexed_model_id", ""), stream=stream,
            _grpc=(tname, md.get("request_id", "")))

    def _unary(self, meth, tname):
        def call(req_bytes, context):
            import grpc

            h = self._handle(context, meth, tname, False)
            try:
                return h.remote(req_bytes).result(timeout_s=self.timeout)
            except TimeoutError:
                context.abort(grpc.StatusCode.DEADLINE_EXCEEDED, f"request exceeded {self.timeout}s")
            except Exception as e:  # noqa: BLE001 - surfaced as a gRPC status
                context.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")
        return call

    def _streamer(self, meth, tname):
        def call(req_bytes, context):
            import grpc

            h = self._handle(context, meth, tname, True)
            try:
                for b in h.remote(req_bytes):
                    yield b
            except Exception as e:  # noqa: BLE001
                context.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")
        return call


def decode_request(tname: str, payload: bytes):
    """Replica side: rebuild the request message from the default descriptor pool."""
    from google.protobuf import descriptor_pool, message_factory

    cls = message_factory.GetMessageClass(descriptor_pool.Default().FindMessageTypeByName(tname))
    return cls.FromString(payload)


def encode_response(msg) -> bytes:
    if isinstance(msg, (bytes, bytearray)):
        return bytes(msg)
    ser = getattr(msg, "SerializeToString", None)
    if ser is None:
        raise TypeError(f"gRPC deployment methods must return protobuf messages, got {type(msg).__name__}")
    return ser()
