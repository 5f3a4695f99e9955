"""Per-execution resource accounting for the streaming executor (reference roles:
python/ray/data/_internal/execution/resource_manager.py:25 (ResourceManager),
:296 (ReservationOpResourceAllocator), execution/autoscaler/).

One ``ResourceManager`` per Dataset execution. Each operator (a fused task
stage or an actor-pool stage) gets an ``OpState``:

* **object-store budget** — the execution may use
  ``DataContext.execution_object_store_fraction`` of the object store; half of
  it is reserved evenly per operator and the other half is a shared pool any
  operator may borrow from. An operator's usage is the estimated size of its
  in-flight task outputs (tasks x running mean of observed output block size)
  plus the outputs it has produced that its consumer has not pulled yet.
  ``can_submit`` gates new tasks on that budget (one task is always allowed so
  the pipeline cannot deadlock), on top of the per-op in-flight task cap.
* **stats** — tasks, rows, bytes, busy time, peak memory and (actor pools)
  the actor count over time, rendered by ``Dataset.stats()``.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional


class OpState:
    def __init__(self, mgr: "ResourceManager", name: str):
        self.mgr = mgr
        self.name = name
        self.inflight = 0
        self.pending_output_bytes = 0  # produced, not yet pulled downstream
        self.avg_out_bytes = 0.0
        self.n_out = 0
        self.tasks = 0
        self.rows = 0
        self.bytes = 0
        self.t_first: Optional[float] = None
        self.t_last: Optional[float] = None
        self.peak_bytes = 0
        self.actors_now = 0
        self.actors_peak = 0
        self.actors_min: Optional[int] = None
        self.scale_ups = 0
        self.scale_downs = 0
        self.throttled = 0
        self.warmup_cap = 4  # tasks allowed before the first output size is known

    # accounting --------------------------------------------------------------
    @property
    def usage(self) -> float:
        return self.inflight * self.avg_out_bytes + self.pending_output_bytes

    def on_submit(self):
        self.inflight += 1
        self.tasks += 1
        if self.t_first is None:
            self.t_first = time.perf_counter()
        self.peak_bytes = max(self.peak_bytes, int(self.usage))

    def on_output(self, meta: dict):
        self.inflight = max(0, self.inflight - 1)
        nb = int(meta.get("size_bytes", 0))
        self.n_out += 1
        self.avg_out_bytes += (nb - self.avg_out_bytes) / self.n_out
        self.rows += int(meta.get("num_rows", 0))
        self.bytes += nb
        self.pending_output_bytes += nb
        self.t_last = time.perf_counter()
        self.peak_bytes = max(self.peak_bytes, int(self.usage))

    def on_pulled(self, meta: dict):
        self.pending_output_bytes = max(0, self.pending_output_bytes - int(meta.get("size_bytes", 0)))

    def set_actors(self, n: int):
        self.actors_now = n
        self.actors_peak = max(self.actors_peak, n)
        self.actors_min = n if self.actors_min is None else min(self.actors_min, n)

    # admission ---------------------------------------------------------------
    def can_submit(self) -> bool:
        if self.inflight == 0:
            return True
        if self.n_out == 0 and self.mgr.budget != float("inf"):
            # no output size observed yet: hold at the warm-up width until one lands
            ok = self.inflight < self.warmup_cap
            if not ok:
                self.throttled += 1
            return ok
        ok = self.mgr.admit(self, self.usage + max(self.avg_out_bytes, 1.0))
        if not ok:
            self.throttled += 1
        return ok


class ResourceManager:
    def __init__(self, budget_bytes: float):
        self.budget = float(budget_bytes)
        self.ops: List[OpState] = []
        self.lock = threading.Lock()

    @staticmethod
    def for_execution() -> "ResourceManager":
        from .context import DataContext

        ctx = DataContext.get_current()
        cap = ctx.execution_object_store_bytes
        limit = ctx.resource_limits()[2]
        if limit is not None and limit != float("inf"):
            cap = float(limit)  # ExecutionOptions(resource_limits=ExecutionResources(object_store_memory=...))
        if not cap:
            try:
                from ..core.api import cluster_resources

                cap = float(cluster_resources().get("object_store_memory", 0)) * ctx.execution_object_store_fraction
            except Exception:
                cap = 0
        return ResourceManager(cap or float("inf"))

    def op(self, name: str) -> OpState:
        st = OpState(self, name)
        self.ops.append(st)
        return st

    def admit(self, op: OpState, want: float) -> bool:
        if self.budget == float("inf"):
            return True
        n = max(1, len(self.ops))
        reserved = 0.5 * self.budget / n
        if want <= reserved:
            return True
        shared = 0.5 * self.budget
        borrowed = sum(max(0.0, o.usage - reserved) for o in self.ops if o is not op)
        return want - reserved <= shared - borrowed

    def summary(self) -> str:
        lines = []
        for i, o in enumerate(self.ops):
            wall = (o.t_last - o.t_first) if (o.t_first is not None and o.t_last is not None) else 0.0
            s = (f"Operator {i} {o.name}: {o.tasks} tasks, {o.rows} rows, {o.bytes / 2**20:.1f} MiB out, "
                 f"{wall:.3f}s active, peak object-store use {o.peak_bytes / 2**20:.1f} MiB")
            if o.actors_peak:
                s += (f", actors min/peak {o.actors_min}/{o.actors_peak} "
                      f"(+{o.scale_ups}/-{o.scale_downs})")
            if o.throttled:
                s += f", throttled {o.throttled}x by the memory budget"
            lines.append(s)
        if self.budget != float("inf"):
            lines.append(f"object-store budget for this execution: {self.budget / 2**30:.2f} GiB")
        return "\n".join(lines)
