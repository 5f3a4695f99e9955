"""Scaling policies for the v2 controller (reference:
python/ray/train/v2/_internal/execution/scaling_policy/{scaling_policy,fixed}.py).

* :class:`FixedScalingPolicy` - always ``ScalingConfig.num_workers``.
* :class:`ElasticScalingPolicy` - ``ScalingConfig(num_workers=(min, max))``: start
  with as many workers as the cluster can place now (at least ``min``), and while
  running, every ``check_interval_s`` ask for a RESIZE to a larger size when the
  free resources would fit more workers (the controller restarts the group from
  the latest checkpoint at the new size).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

from ..config import ScalingConfig


class ScalingDecision:
    pass


@dataclass
class ResizeDecision(ScalingDecision):
    num_workers: int
    resources_per_worker: Dict[str, float] = field(default_factory=dict)


class NoopDecision(ScalingDecision):
    pass


class ScalingPolicy:
    def __init__(self, scaling_config: ScalingConfig):
        self.scaling_config = scaling_config

    def make_decision_for_non_running_worker_group(self) -> ScalingDecision:
        raise NotImplementedError

    def make_decision_for_running_worker_group(self, num_workers: int) -> ScalingDecision:
        return NoopDecision()

    # controller-callback hooks (the policy observes the controller like any callback)
    def after_controller_state_update(self, previous, current):
        pass


class FixedScalingPolicy(ScalingPolicy):
    def make_decision_for_non_running_worker_group(self):
        return ResizeDecision(self.scaling_config.total_workers, self.scaling_config._resources_per_worker_not_none)


class ElasticScalingPolicy(ScalingPolicy):
    def __init__(self, scaling_config: ScalingConfig, min_workers: int, max_workers: int,
                 check_interval_s: float = 5.0):
        super().__init__(scaling_config)
        if not 1 <= min_workers <= max_workers:
            raise ValueError("need 1 <= min_workers <= max_workers")
        self.min_workers, self.max_workers = min_workers, max_workers
        self.check_interval_s = check_interval_s
        self._last_check = 0.0

    def _fits(self, extra_free: Optional[Dict[str, float]] = None) -> int:
        """Workers the free resources (plus what the running group holds) can place."""
        from ...core import api as core

        free = dict(core.available_resources())
        for k, v in (extra_free or {}).items():
            free[k] = free.get(k, 0.0) + v
        per = self.scaling_config._resources_per_worker_not_none
        n = min((int(free.get(k, 0.0) // v) for k, v in per.items() if v > 0), default=self.max_workers)
        return max(0, min(n, self.max_workers))

    def make_decision_for_non_running_worker_group(self):
        n = max(self.min_workers, self._fits())
        return ResizeDecision(n, self.scaling_config._resources_per_worker_not_none)

    def make_decision_for_running_worker_group(self, num_workers):
        now = time.monotonic()
        if now - self._last_check < self.check_interval_s or num_workers >= self.max_workers:
            return NoopDecision()
        self._last_check = now
        per = self.scaling_config._resources_per_worker_not_none
        held = {k: v * num_workers for k, v in per.items()}
        n = self._fits(held)
        if n > num_workers:
            return ResizeDecision(n, per)
        return NoopDecision()


def create_scaling_policy(scaling_config: ScalingConfig) -> ScalingPolicy:
    nw = scaling_config.num_workers
    if isinstance(nw, (tuple, list)):
        lo, hi = int(nw[0]), int(nw[1])
        sc = ScalingConfig(num_workers=hi, use_gpu=scaling_config.use_gpu,
                           resources_per_worker=scaling_config.resources_per_worker,
                           placement_strategy=scaling_config.placement_strategy)
        return ElasticScalingPolicy(sc, lo, hi)
    return FixedScalingPolicy(scaling_config)


def elastic_bounds(scaling_config: ScalingConfig) -> Optional[Tuple[int, int]]:
    nw = scaling_config.num_workers
    return (int(nw[0]), int(nw[1])) if isinstance(nw, (tuple, list)) else None
