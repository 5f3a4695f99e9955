"""Public Serve API (reference: python/ray/serve/api.py: start :64, shutdown :118,
run :499, delete :556, status :736, get_app_handle :764,
get_deployment_handle :800)."""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Union

from ..core import api as core
from .config import HTTPOptions
from .controller import CONTROLLER_NAME, NAMESPACE, ServeController
from .deployment import Application, Deployment
from .handle import DeploymentHandle, _routers


def _get_controller(create: bool = True):
    core._ensure_init()
    try:
        return core.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
    except ValueError:
        if not create:
            return None
    from ..core.actor import ActorClass

    Ctl = ActorClass(ServeController, {})
    # restarted without limit (reference: serve/_private/api.py:101 max_restarts=-1); calls
    # that hit a restart are retried; the state comes back from the KV checkpoint
    h = Ctl.options(name=CONTROLLER_NAME, namespace=NAMESPACE, lifetime="detached", get_if_exists=True,
                    num_cpus=0, max_concurrency=64, max_restarts=-1, max_task_retries=-1).remote()
    core.get(h.list_apps.remote())
    return h


def start(http_options: Union[None, dict, HTTPOptions] = None, detached: bool = True,
          proxy_location: str = "HeadOnly", grpc_options=None, **_ignored):
    """Start the controller and (unless ``proxy_location='Disabled'``) the HTTP proxy;
    with ``grpc_options`` (a ``gRPCOptions`` or dict) also the gRPC proxy."""
    ctl = _get_controller()
    if grpc_options is not None:
        _start_grpc(ctl, grpc_options)
    if proxy_location in ("Disabled", "disabled", None):
        return ctl
    proxy, port = core.get(ctl.get_proxy.remote())
    if proxy is None:
        from ..core.actor import ActorClass
        from .proxy import HTTPProxy

        if isinstance(http_options, dict):
            http_options = HTTPOptions(**http_options)
        http_options = http_options or HTTPOptions()
        P = ActorClass(HTTPProxy, {})
        proxy = P.options(num_cpus=0, max_concurrency=8, name="SERVE_PROXY", namespace=NAMESPACE,
                          lifetime="detached").remote(http_options.host, http_options.port,
                                                      http_options.request_timeout_s)
        port = core.get(proxy.ready.remote())
        core.get(ctl.set_proxy.remote(proxy, port))
    return ctl


def _start_grpc(ctl, grpc_options):
    from .grpc_proxy import gRPCOptions, gRPCProxy

    if isinstance(grpc_options, dict):
        grpc_options = gRPCOptions(**grpc_options)
    proxy, port = core.get(ctl.get_grpc_proxy.remote())
    if proxy is not None:
        return port
    from ..core.actor import ActorClass

    fns = [f if isinstance(f, str) else f"{f.__module__}.{f.__qualname__}" if f.__module__ != "__main__" else f
           for f in grpc_options.grpc_servicer_functions]
    P = ActorClass(gRPCProxy, {})
    proxy = P.options(num_cpus=0, max_concurrency=8, name="SERVE_GRPC_PROXY", namespace=NAMESPACE,
                      lifetime="detached").remote(grpc_options.host, grpc_options.port, fns,
                                                  grpc_options.request_timeout_s)
    port = core.get(proxy.ready.remote())
    core.get(ctl.set_grpc_proxy.remote(proxy, port))
    return port


def grpc_port() -> Optional[int]:
    ctl = _get_controller(create=False)
    if ctl is None:
        return None
    return core.get(ctl.get_grpc_proxy.remote())[1]


def http_port() -> Optional[int]:
    ctl = _get_controller(create=False)
    if ctl is None:
        return None
    return core.get(ctl.get_proxy.remote())[1]


def _build(app: Application, app_name: str):
    nodes = app._walk()
    names: Dict[int, str] = {}
    used = {}
    for node in nodes:
        n = node.deployment.name
        if n in used and used[n] is not node:
            k = 1
            while f"{n}_{k}" in used:
                k += 1
            n = f"{n}_{k}"
        used[n] = node
        names[id(node)] = n

    def sub(x):
        if isinstance(x, Application):
            return DeploymentHandle(names[id(x)], app_name)
        if isinstance(x, list):
            return [sub(v) for v in x]
        if isinstance(x, tuple):
            return tuple(sub(v) for v in x)
        if isinstance(x, dict):
            return {k: sub(v) for k, v in x.items()}
        return x

    deps = []
    for node in nodes:
        d: Deployment = node.deployment
        deps.append({"name": names[id(node)], "target": d.func_or_class, "args": sub(node.args),
                     "kwargs": sub(node.kwargs), "config": d.config})
    return deps, names[id(app)]


def run(target: Union[Application, Deployment], *, name: str = "default", route_prefix: Optional[str] = "/",
        blocking: bool = False, timeout_s: float = 120.0, _local_testing_mode: bool = False,
        http: bool = True) -> DeploymentHandle:
    if isinstance(target, Deployment):
        target = target.bind()
    if not isinstance(target, Application):
        raise TypeError("serve.run() expects an Application (Deployment.bind(...))")
    if not name:
        from .exceptions import RayServeException

        raise RayServeException("Application name must a non-empty string.")
    import os

    if os.environ.get("RAY_SERVE_FORCE_LOCAL_TESTING_MODE", "0") == "1":
        _local_testing_mode = True
    if _local_testing_mode:
        # every deployment in this process, no cluster needed (api.py:438-454)
        from .local_testing_mode import run_local

        return run_local(target, name)
    if target.deployment.route_prefix is not None and route_prefix == "/":
        route_prefix = target.deployment.route_prefix
    ctl = start(proxy_location="HeadOnly" if http and route_prefix is not None else "Disabled")
    deps, ingress = _build(target, name)
    core.get(ctl.deploy_application.remote(name, route_prefix, ingress, deps))
    deadline = time.time() + timeout_s
    while True:
        st = core.get(ctl.status.remote()).get(name)
        if st and st["status"] == "RUNNING":
            break
        if st and st["status"] == "DEPLOY_FAILED":
            msgs = "; ".join(d["message"] for d in st["deployments"].values() if d["message"])
            raise RuntimeError(f"application {name!r} failed to deploy: {msgs}")
        if time.time() > deadline:
            raise TimeoutError(f"application {name!r} not running after {timeout_s}s: {st}")
        time.sleep(0.05)
    for key in [k for k in _routers if k[0] == name]:
        _routers[key].invalidate()
    for getter in (ctl.get_proxy, ctl.get_grpc_proxy):
        proxy, _ = core.get(getter.remote())
        if proxy is not None:
            core.get(proxy.refresh.remote())
    handle = DeploymentHandle(ingress, name)
    if blocking:
        try:
            while True:
                time.sleep(1)
        except KeyboardInterrupt:
            pass
    return handle


def delete(name: str, _blocking: bool = True):
    ctl = _get_controller(create=False)
    if ctl is None:
        return
    core.get(ctl.delete_application.remote(name))
    proxy, _ = core.get(ctl.get_proxy.remote())
    if proxy is not None:
        core.get(proxy.refresh.remote())
    if _blocking:
        deadline = time.time() + 30
        while time.time() < deadline and name in core.get(ctl.status.remote()):
            time.sleep(0.05)
    for key in [k for k in _routers if k[0] == name]:
        _routers.pop(key, None)


@dataclass
class DeploymentStatus:
    name: str
    status: str
    replica_states: Dict[str, str] = field(default_factory=dict)
    message: str = ""
    target_replicas: int = 0
    running_replicas: int = 0


@dataclass
class ApplicationStatus:
    status: str
    route_prefix: Optional[str]
    deployments: Dict[str, DeploymentStatus]


@dataclass
class ServeStatus:
    applications: Dict[str, ApplicationStatus]
    proxies: Dict[str, str] = field(default_factory=dict)


def status() -> ServeStatus:
    ctl = _get_controller(create=False)
    if ctl is None:
        return ServeStatus({})
    raw = core.get(ctl.status.remote())
    apps = {}
    for n, a in raw.items():
        deps = {dn: DeploymentStatus(dn, d["status"], d["replica_states"], d["message"], d["target_replicas"],
                                     d["running_replicas"]) for dn, d in a["deployments"].items()}
        apps[n] = ApplicationStatus(a["status"], a["route_prefix"], deps)
    proxy, port = core.get(ctl.get_proxy.remote())
    return ServeStatus(apps, {"head": "HEALTHY"} if proxy is not None else {})


def shutdown():
    ctl = _get_controller(create=False)
    if ctl is None:
        return
    try:
        core.get(ctl.shutdown.remote(), timeout=60)
    except Exception:
        pass
    try:
        core.kill(ctl)
    except Exception:
        pass
    _routers.clear()


def get_app_handle(name: str) -> DeploymentHandle:
    ctl = _get_controller(create=False)
    ingress = core.get(ctl.get_ingress.remote(name)) if ctl is not None else None
    if ingress is None:
        raise KeyError(f"application {name!r} does not exist")
    return DeploymentHandle(ingress, name)


def get_deployment_handle(deployment_name: str, app_name: Optional[str] = None) -> DeploymentHandle:
    if app_name is None:
        from .context import _replica_context

        app_name = _replica_context.app_name if _replica_context is not None else "default"
    return DeploymentHandle(deployment_name, app_name)
