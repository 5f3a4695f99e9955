"""Declarative Serve config (reference: python/ray/serve/schema.py — ``ServeDeploySchema``
:689, ``ServeApplicationSchema``, ``DeploymentSchema``, ``HTTPOptionsSchema``,
``gRPCOptionsSchema``) and the code that applies it.

A config file lists applications by ``import_path`` (``module:attr`` or
``module.attr``; the attribute is a bound ``Application``, a ``Deployment``, or
an application *builder* ``fn(args) -> Application``) plus per-deployment
overrides (replicas, autoscaling, user_config, actor options, ...).
``deploy_config`` imports each application, applies the overrides to the
matching deployments of its graph, deploys it, deletes applications that are
no longer listed, and records the config in the controller (``serve config``).
``build_config`` does the reverse: the config YAML for importable apps.
"""
from __future__ import annotations

import importlib
import sys
from typing import Any, Dict, List, Literal, Optional, Union

from pydantic import BaseModel, ConfigDict, Field, field_validator, model_validator

_DEPLOYMENT_OPTION_KEYS = ("num_replicas", "max_ongoing_requests", "max_queued_requests", "user_config",
                           "autoscaling_config", "graceful_shutdown_wait_loop_s", "graceful_shutdown_timeout_s",
                           "health_check_period_s", "health_check_timeout_s", "ray_actor_options",
                           "placement_group_bundles", "placement_group_strategy", "max_replicas_per_node")


class DeploymentSchema(BaseModel):
    model_config = ConfigDict(extra="forbid")
    name: str
    num_replicas: Optional[Union[int, Literal["auto"]]] = None
    max_ongoing_requests: Optional[int] = Field(default=None, gt=0)
    max_queued_requests: Optional[int] = None
    user_config: Optional[Any] = None
    autoscaling_config: Optional[Dict[str, Any]] = None
    graceful_shutdown_wait_loop_s: Optional[float] = Field(default=None, ge=0)
    graceful_shutdown_timeout_s: Optional[float] = Field(default=None, ge=0)
    health_check_period_s: Optional[float] = Field(default=None, gt=0)
    health_check_timeout_s: Optional[float] = Field(default=None, gt=0)
    ray_actor_options: Optional[Dict[str, Any]] = None
    placement_group_bundles: Optional[List[Dict[str, float]]] = None
    placement_group_strategy: Optional[str] = None
    max_replicas_per_node: Optional[int] = None

    @model_validator(mode="after")
    def _replicas_xor_autoscaling(self):
        if isinstance(self.num_replicas, int) and self.autoscaling_config is not None:
            raise ValueError(f"deployment {self.name!r}: num_replicas and autoscaling_config are exclusive")
        return self

    def overrides(self) -> Dict[str, Any]:
        return {k: getattr(self, k) for k in _DEPLOYMENT_OPTION_KEYS if k in self.model_fields_set}


class ServeApplicationSchema(BaseModel):
    model_config = ConfigDict(extra="forbid")
    name: str = "default"
    route_prefix: Optional[str] = "/"
    import_path: str
    runtime_env: Dict[str, Any] = Field(default_factory=dict)
    deployments: List[DeploymentSchema] = Field(default_factory=list)
    args: Dict[str, Any] = Field(default_factory=dict)

    @field_validator("route_prefix")
    @classmethod
    def _prefix(cls, v):
        if v is not None and (not v.startswith("/") or (len(v) > 1 and v.endswith("/"))):
            raise ValueError(f"route_prefix {v!r} must start with '/' and not end with '/'")
        return v

    @field_validator("import_path")
    @classmethod
    def _import_path(cls, v):
        if ":" not in v and "." not in v:
            raise ValueError(f"import_path {v!r} must look like 'module:attr' or 'module.attr'")
        return v


class HTTPOptionsSchema(BaseModel):
    model_config = ConfigDict(extra="forbid")
    host: str = "127.0.0.1"
    port: int = 8000
    root_path: str = ""
    request_timeout_s: Optional[float] = None
    keep_alive_timeout_s: int = 5


class gRPCOptionsSchema(BaseModel):
    model_config = ConfigDict(extra="forbid")
    port: int = 9000
    grpc_servicer_functions: List[str] = Field(default_factory=list)
    request_timeout_s: Optional[float] = None


class ServeDeploySchema(BaseModel):
    model_config = ConfigDict(extra="forbid")
    proxy_location: str = "HeadOnly"
    http_options: HTTPOptionsSchema = Field(default_factory=HTTPOptionsSchema)
    grpc_options: gRPCOptionsSchema = Field(default_factory=gRPCOptionsSchema)
    logging_config: Optional[Dict[str, Any]] = None
    applications: List[ServeApplicationSchema]

    @model_validator(mode="after")
    def _unique(self):
        names = [a.name for a in self.applications]
        if len(set(names)) != len(names):
            raise ValueError(f"application names must be unique: {names}")
        prefixes = [a.route_prefix for a in self.applications if a.route_prefix is not None]
        if len(set(prefixes)) != len(prefixes):
            raise ValueError(f"route prefixes must be unique: {prefixes}")
        return self


# ---------------------------------------------------------------- import / apply
def import_attr(path: str):
    if ":" in path:
        mod, attr = path.split(":", 1)
    else:
        mod, _, attr = path.rpartition(".")
    if "" not in sys.path and "." not in sys.path:
        sys.path.insert(0, "")  # like the reference CLI: the cwd is importable
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def build_app(app: ServeApplicationSchema):
    """Import one application and apply its per-deployment overrides."""
    from .deployment import Application, Deployment

    target = import_attr(app.import_path)
    if isinstance(target, Deployment):
        target = target.bind()
    elif not isinstance(target, Application) and callable(target):
        target = target(dict(app.args))  # application builder
    if not isinstance(target, Application):
        raise TypeError(f"{app.import_path} is not an Application, Deployment or application builder")
    nodes = {n.deployment.name: n for n in target._walk()}
    for d in app.deployments:
        if d.name not in nodes:
            raise ValueError(f"application {app.name!r} has no deployment {d.name!r} "
                             f"(deployments: {sorted(nodes)})")
        ov = d.overrides()
        if ov:
            nodes[d.name].deployment = nodes[d.name].deployment.options(**ov)
    return target


def deploy_config(config: Union[ServeDeploySchema, dict], *, wait: bool = True):
    from . import api

    if isinstance(config, dict):
        config = ServeDeploySchema.model_validate(config)
    grpc_opts = None
    if config.grpc_options.grpc_servicer_functions:
        grpc_opts = config.grpc_options.model_dump()
    api.start(http_options=config.http_options.model_dump(), proxy_location=config.proxy_location,
              grpc_options=grpc_opts)
    wanted = {a.name for a in config.applications}
    ctl = api._get_controller()
    from ..core import api as core

    for name in core.get(ctl.list_apps.remote()):
        if name not in wanted:
            api.delete(name)
    for app in config.applications:
        api.run(build_app(app), name=app.name, route_prefix=app.route_prefix,
                http=config.proxy_location not in ("Disabled", "disabled"))
    core.get(ctl.set_deploy_config.remote(config.model_dump(mode="json")))
    return True


def build_config(import_paths: List[str], *, app_names: Optional[List[str]] = None) -> Dict[str, Any]:
    """``serve build``: a deploy config for importable applications, listing every
    deployment with its current options."""
    from .deployment import Application, Deployment

    apps = []
    for i, path in enumerate(import_paths):
        target = import_attr(path)
        if isinstance(target, Deployment):
            target = target.bind()
        if not isinstance(target, Application):
            raise TypeError(f"{path} is not an Application or Deployment")
        deps = []
        for node in target._walk():
            c = node.deployment.config
            d: Dict[str, Any] = {"name": node.deployment.name}
            if c.autoscaling_config is not None:
                d["autoscaling_config"] = {k: v for k, v in vars(c.autoscaling_config).items() if v is not None}
            else:
                d["num_replicas"] = c.num_replicas
            d["max_ongoing_requests"] = c.max_ongoing_requests
            if c.user_config is not None:
                d["user_config"] = c.user_config
            if c.ray_actor_options:
                d["ray_actor_options"] = dict(c.ray_actor_options)
            deps.append(d)
        name = (app_names[i] if app_names and i < len(app_names) else
                ("default" if len(import_paths) == 1 else f"app{i + 1}"))
        prefix = target.deployment.route_prefix or ("/" if len(import_paths) == 1 else f"/{name}")
        apps.append({"name": name, "route_prefix": prefix, "import_path": path, "deployments": deps})
    cfg = ServeDeploySchema.model_validate({"applications": apps})
    return cfg.model_dump(mode="json", exclude_none=True)
