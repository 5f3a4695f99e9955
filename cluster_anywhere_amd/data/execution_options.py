"""Execution options of the streaming executor (reference roles:
``python/ray/data/_internal/execution/interfaces/execution_options.py:9``
ExecutionResources and ``:210`` ExecutionOptions).

Set on the context: ``DataContext.get_current().execution_options =
ExecutionOptions(resource_limits=ExecutionResources(cpu=4))``. What each field
does here:

* ``resource_limits.cpu`` caps the tasks one operator keeps in flight (and the
  CPUs the executor assumes it may use), ``.gpu`` caps GPU actor pools, and
  ``.object_store_memory`` is the execution's object-store budget (the
  reserved + shared pools of ``resource_manager.py``).
* ``exclude_resources`` is subtracted from the cluster's resources before the
  defaults are derived (e.g. CPUs a concurrent trainer holds).
* ``preserve_order`` = ``DataContext.execution_preserve_order``.
* ``locality_with_output`` / ``actor_locality_enabled`` are accepted; on one node
  every block already sits in the node's shared arena, and multi-node pulls go
  node to node, so there is no placement to steer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional


@dataclass
class ExecutionResources:
    cpu: Optional[float] = None
    gpu: Optional[float] = None
    object_store_memory: Optional[float] = None

    @classmethod
    def for_limits(cls, cpu=None, gpu=None, object_store_memory=None) -> "ExecutionResources":
        inf = float("inf")
        return cls(cpu if cpu is not None else inf, gpu if gpu is not None else inf,
                   object_store_memory if object_store_memory is not None else inf)

    @classmethod
    def zero(cls) -> "ExecutionResources":
        return cls(0.0, 0.0, 0.0)

    def is_zero(self) -> bool:
        return not (self.cpu or self.gpu or self.object_store_memory)

    def _pair(self, other, op):
        def f(a, b):
            if a is None and b is None:
                return None
            return op(a or 0.0, b or 0.0)
        return ExecutionResources(f(self.cpu, other.cpu), f(self.gpu, other.gpu),
                                  f(self.object_store_memory, other.object_store_memory))

    def add(self, other: "ExecutionResources") -> "ExecutionResources":
        return self._pair(other, lambda a, b: a + b)

    def subtract(self, other: "ExecutionResources") -> "ExecutionResources":
        return self._pair(other, lambda a, b: a - b)

    def min(self, other: "ExecutionResources") -> "ExecutionResources":
        def f(a, b):
            if a is None:
                return b
            if b is None:
                return a
            return min(a, b)
        return ExecutionResources(f(self.cpu, other.cpu), f(self.gpu, other.gpu),
                                  f(self.object_store_memory, other.object_store_memory))

    def satisfies_limit(self, limit: "ExecutionResources") -> bool:
        for mine, lim in ((self.cpu, limit.cpu), (self.gpu, limit.gpu),
                          (self.object_store_memory, limit.object_store_memory)):
            if lim is not None and (mine or 0.0) > lim:
                return False
        return True

    def object_store_memory_str(self) -> str:
        v = self.object_store_memory
        return "None" if v is None else f"{v / (1 << 20):.1f}MB"


@dataclass
class ExecutionOptions:
    resource_limits: ExecutionResources = field(default_factory=ExecutionResources)
    exclude_resources: ExecutionResources = field(default_factory=ExecutionResources.zero)
    locality_with_output: bool = False
    preserve_order: bool = True
    actor_locality_enabled: bool = True
    verbose_progress: bool = False

    def validate(self) -> None:
        for name in ("cpu", "gpu", "object_store_memory"):
            for res in (self.resource_limits, self.exclude_resources):
                v = getattr(res, name)
                if v is not None and v < 0:
                    raise ValueError(f"execution resources must be >= 0, got {name}={v}")
