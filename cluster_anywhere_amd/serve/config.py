"""Serve configs (reference: python/ray/serve/config.py: AutoscalingConfig :33,
HTTPOptions; _private/config.py: DeploymentConfig)."""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, List, Optional


@dataclass
class AutoscalingConfig:
    min_replicas: int = 1
    initial_replicas: Optional[int] = None
    max_replicas: int = 1
    target_ongoing_requests: float = 2.0
    metrics_interval_s: float = 0.5
    look_back_period_s: float = 2.0
    smoothing_factor: float = 1.0
    upscaling_factor: Optional[float] = None
    downscaling_factor: Optional[float] = None
    upscale_delay_s: float = 0.5
    downscale_delay_s: float = 5.0

    def __post_init__(self):
        if self.min_replicas > self.max_replicas:
            raise ValueError("min_replicas must be <= max_replicas")
        if self.target_ongoing_requests <= 0:
            raise ValueError("target_ongoing_requests must be > 0")

    @classmethod
    def coerce(cls, v) -> Optional["AutoscalingConfig"]:
        if v is None or isinstance(v, AutoscalingConfig):
            return v
        names = {f.name for f in fields(cls)}
        return cls(**{k: x for k, x in dict(v).items() if k in names})

    def desired(self, total_ongoing: float, current: int) -> int:
        """Replicas needed so each carries ``target_ongoing_requests``, with the
        change scaled by the up/down factors (reference autoscaling_policy.py)."""
        raw = total_ongoing / self.target_ongoing_requests
        if current > 0:
            delta = raw - current
            f = (self.upscaling_factor if delta > 0 else self.downscaling_factor) or self.smoothing_factor
            raw = current + delta * f
        n = int(math.ceil(raw - 1e-9))
        return max(self.min_replicas, min(self.max_replicas, n))


@dataclass
class HTTPOptions:
    host: str = "127.0.0.1"
    port: int = 8000
    root_path: str = ""
    request_timeout_s: Optional[float] = None
    keep_alive_timeout_s: int = 5


@dataclass
class DeploymentConfig:
    num_replicas: Optional[int] = 1
    max_ongoing_requests: int = 5
    max_queued_requests: int = -1
    user_config: Any = None
    autoscaling_config: Optional[AutoscalingConfig] = None
    graceful_shutdown_wait_loop_s: float = 0.2
    graceful_shutdown_timeout_s: float = 5.0
    health_check_period_s: float = 2.0
    health_check_timeout_s: float = 10.0
    ray_actor_options: Dict[str, Any] = field(default_factory=dict)
    placement_group_bundles: Optional[List[Dict[str, float]]] = None
    placement_group_strategy: str = "PACK"
    max_replicas_per_node: Optional[int] = None
    version: Optional[str] = None

    def __post_init__(self):
        # reference: serve/_private/config.py:432 (_validate_max_replicas_per_node),
        # schema.py:411-420 (not together with placement_group_bundles)
        if self.max_queued_requests is not None and self.max_queued_requests != -1 and self.max_queued_requests < 1:
            raise ValueError("max_queued_requests must be -1 (no limit) or a positive integer")
        if self.max_ongoing_requests is not None and self.max_ongoing_requests < 1:
            raise ValueError("max_ongoing_requests must be a positive integer")
        if self.max_replicas_per_node is not None:
            if not (1 <= int(self.max_replicas_per_node) <= 100):
                raise ValueError("max_replicas_per_node must be between 1 and 100")
            if self.placement_group_bundles is not None:
                raise ValueError("Setting max_replicas_per_node is not allowed when "
                                 "placement_group_bundles is provided.")
        if self.placement_group_bundles is not None:
            from ..util.placement_group import VALID_STRATEGIES, _validate_bundles

            _validate_bundles(self.placement_group_bundles)
            if self.placement_group_strategy not in VALID_STRATEGIES:
                raise ValueError(f"Invalid placement group strategy {self.placement_group_strategy}")

    def initial_replicas(self) -> int:
        a = self.autoscaling_config
        if a is not None:
            return a.initial_replicas if a.initial_replicas is not None else a.min_replicas
        return self.num_replicas if self.num_replicas is not None else 1
