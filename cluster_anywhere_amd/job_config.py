"""Per-job configuration (reference: python/ray/job_config.py)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class JobConfig:
    def __init__(self, jvm_options: Optional[List[str]] = None, code_search_path=None,
                 runtime_env: Optional[dict] = None, _client_job: bool = False,
                 metadata: Optional[Dict[str, str]] = None, ray_namespace: Optional[str] = None,
                 default_actor_lifetime: str = "non_detached", _py_driver_sys_path=None):
        if default_actor_lifetime not in ("detached", "non_detached"):
            raise ValueError("default_actor_lifetime must be 'detached' or 'non_detached'")
        self.jvm_options = list(jvm_options or [])
        self.code_search_path = list(code_search_path or [])
        self.runtime_env = dict(runtime_env or {})
        self.metadata = dict(metadata or {})
        self.ray_namespace = ray_namespace
        self.default_actor_lifetime = default_actor_lifetime
        self._py_driver_sys_path = list(_py_driver_sys_path or [])

    def set_metadata(self, key: str, value: str) -> None:
        self.metadata[key] = value

    def set_runtime_env(self, runtime_env: Optional[dict], validate: bool = False) -> None:
        if validate and runtime_env:
            from .runtime_env import RuntimeEnv

            RuntimeEnv(**runtime_env)
        self.runtime_env = dict(runtime_env or {})

    def set_ray_namespace(self, ray_namespace: str) -> None:
        self.ray_namespace = ray_namespace

    def set_default_actor_lifetime(self, default_actor_lifetime: str) -> None:
        if default_actor_lifetime not in ("detached", "non_detached"):
            raise ValueError("default_actor_lifetime must be 'detached' or 'non_detached'")
        self.default_actor_lifetime = default_actor_lifetime

    def _validate_runtime_env(self):
        from .runtime_env import RuntimeEnv

        return RuntimeEnv(**self.runtime_env)

    def to_json(self) -> Dict[str, Any]:
        return {"runtime_env": self.runtime_env, "metadata": self.metadata,
                "ray_namespace": self.ray_namespace, "default_actor_lifetime": self.default_actor_lifetime}

    @classmethod
    def from_json(cls, d: Dict[str, Any]) -> "JobConfig":
        return cls(runtime_env=d.get("runtime_env"), metadata=d.get("metadata"),
                   ray_namespace=d.get("ray_namespace"),
                   default_actor_lifetime=d.get("default_actor_lifetime", "non_detached"))
