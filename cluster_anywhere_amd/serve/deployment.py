"""Deployments and applications (reference: python/ray/serve/deployment.py,
api.py:deployment :246, ingress :170)."""
from __future__ import annotations

import copy
import inspect
from dataclasses import fields, replace
from typing import Any, Callable, Dict, List, Optional

from .config import AutoscalingConfig, DeploymentConfig

_CONFIG_KEYS = {f.name for f in fields(DeploymentConfig)}


class Application:
    """A bound deployment graph node: ``Deployment.bind(*args, **kwargs)``."""

    def __init__(self, deployment: "Deployment", args: tuple, kwargs: dict):
        self.deployment = deployment
        self.args = args
        self.kwargs = kwargs

    def _walk(self, seen=None):
        """All applications reachable through bound arguments (children first)."""
        seen = seen if seen is not None else {}
        for a in list(self.args) + list(self.kwargs.values()):
            for child in _find_apps(a):
                if id(child) not in seen:
                    child._walk(seen)
        seen.setdefault(id(self), self)
        return list(seen.values())


def _find_apps(x):
    if isinstance(x, Application):
        return [x]
    if isinstance(x, (list, tuple)):
        return [a for v in x for a in _find_apps(v)]
    if isinstance(x, dict):
        return [a for v in x.values() for a in _find_apps(v)]
    return []


class Deployment:
    def __init__(self, func_or_class: Callable, name: str, config: DeploymentConfig,
                 route_prefix: Optional[str] = None):
        self.func_or_class = func_or_class
        self.name = name
        self.config = config
        self.route_prefix = route_prefix

    @property
    def num_replicas(self):
        return self.config.num_replicas

    @property
    def user_config(self):
        return self.config.user_config

    @property
    def max_ongoing_requests(self):
        return self.config.max_ongoing_requests

    @property
    def ray_actor_options(self):
        return self.config.ray_actor_options

    def options(self, *, name: Optional[str] = None, route_prefix: Optional[str] = None, **kw) -> "Deployment":
        unknown = set(kw) - _CONFIG_KEYS
        if unknown:
            raise TypeError(f"unknown deployment option(s): {sorted(unknown)}")
        if "autoscaling_config" in kw:
            kw["autoscaling_config"] = AutoscalingConfig.coerce(kw["autoscaling_config"])
            if kw["autoscaling_config"] is not None and "num_replicas" not in kw:
                kw["num_replicas"] = None
        if kw.get("num_replicas") == "auto":
            kw["num_replicas"] = None
            kw.setdefault("autoscaling_config", AutoscalingConfig(min_replicas=1, max_replicas=100))
        cfg = replace(self.config, **kw)
        return Deployment(self.func_or_class, name or self.name, cfg,
                          route_prefix if route_prefix is not None else self.route_prefix)

    def bind(self, *args, **kwargs) -> Application:
        return Application(self, args, kwargs)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be called directly; use .bind() and serve.run()")

    def __repr__(self):
        return f"Deployment(name={self.name})"


def deployment(_func_or_class: Optional[Callable] = None, name: Optional[str] = None,
               version: Optional[str] = None, num_replicas=None, route_prefix: Optional[str] = None,
               ray_actor_options: Optional[Dict] = None, placement_group_bundles=None,
               placement_group_strategy: Optional[str] = None, max_replicas_per_node=None,
               user_config: Any = None, max_ongoing_requests: Optional[int] = None,
               max_queued_requests: Optional[int] = None, autoscaling_config=None,
               graceful_shutdown_wait_loop_s: Optional[float] = None,
               graceful_shutdown_timeout_s: Optional[float] = None,
               health_check_period_s: Optional[float] = None,
               health_check_timeout_s: Optional[float] = None, logging_config=None):
    if num_replicas is not None and autoscaling_config is not None and num_replicas != "auto":
        raise ValueError("num_replicas and autoscaling_config cannot both be set")

    def deco(target):
        kw = {}
        for k, v in dict(version=version, ray_actor_options=ray_actor_options,
                         placement_group_bundles=placement_group_bundles,
                         placement_group_strategy=placement_group_strategy,
                         max_replicas_per_node=max_replicas_per_node, user_config=user_config,
                         max_ongoing_requests=max_ongoing_requests, max_queued_requests=max_queued_requests,
                         graceful_shutdown_wait_loop_s=graceful_shutdown_wait_loop_s,
                         graceful_shutdown_timeout_s=graceful_shutdown_timeout_s,
                         health_check_period_s=health_check_period_s,
                         health_check_timeout_s=health_check_timeout_s).items():
            if v is not None:
                kw[k] = v
        cfg = DeploymentConfig(**kw)
        if num_replicas == "auto":
            cfg.num_replicas = None
            cfg.autoscaling_config = AutoscalingConfig.coerce(autoscaling_config) or \
                AutoscalingConfig(min_replicas=1, max_replicas=100)
        elif autoscaling_config is not None:
            cfg.num_replicas = None
            cfg.autoscaling_config = AutoscalingConfig.coerce(autoscaling_config)
        elif num_replicas is not None:
            cfg.num_replicas = num_replicas
        return Deployment(target, name or target.__name__, cfg, route_prefix)

    if _func_or_class is not None and callable(_func_or_class):
        return deco(_func_or_class)
    return deco


def ingress(app):
    """Class decorator: serve HTTP traffic of this deployment through a FastAPI /
    Starlette ASGI ``app`` whose routes may be methods of the class."""

    def deco(cls):
        if not inspect.isclass(cls):
            raise TypeError("@serve.ingress must decorate a class")
        cls._serve_asgi_app = app
        return cls

    return deco
