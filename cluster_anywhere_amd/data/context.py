"""DataContext (reference: python/ray/data/context.py)."""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field


@dataclass
class DataContext:
    target_max_block_size: int = 128 * 1024 * 1024
    target_min_block_size: int = 1 * 1024 * 1024
    max_tasks_in_flight_per_op: int = int(os.environ.get("CAAMD_DATA_MAX_INFLIGHT", "0"))
    actor_max_tasks_in_flight: int = 4
    execution_preserve_order: bool = True
    # object-store budget of one execution (resource_manager.py): a fraction of the
    # store, or an absolute byte count when set
    execution_object_store_fraction: float = 0.5
    execution_object_store_bytes: int = 0
    enable_progress_bars: bool = False
    read_op_min_num_blocks: int = 8
    eager_free: bool = True
    verbose_stats_logs: bool = False

    _lock = threading.Lock()
    _current = None

    @staticmethod
    def get_current() -> "DataContext":
        with DataContext._lock:
            if DataContext._current is None:
                DataContext._current = DataContext()
            return DataContext._current

    @staticmethod
    def _set_current(ctx: "DataContext"):
        DataContext._current = ctx

    @property
    def execution_options(self):
        """The :class:`~.execution_options.ExecutionOptions` of executions started
        from this context (``preserve_order`` is ``execution_preserve_order``)."""
        from .execution_options import ExecutionOptions

        opts = self.__dict__.get("_execution_options")
        if opts is None:
            opts = self.__dict__["_execution_options"] = ExecutionOptions()
        opts.preserve_order = self.execution_preserve_order
        return opts

    @execution_options.setter
    def execution_options(self, opts):
        opts.validate()
        self.__dict__["_execution_options"] = opts
        self.execution_preserve_order = bool(opts.preserve_order)

    @property
    def preserve_order(self) -> bool:
        return self.execution_preserve_order

    @preserve_order.setter
    def preserve_order(self, v: bool):
        self.execution_preserve_order = bool(v)

    def resource_limits(self):
        """(cpu, gpu, object_store_memory) limits of an execution; None = no limit."""
        opts = self.__dict__.get("_execution_options")
        if opts is None:
            return None, None, None
        r = opts.resource_limits
        return r.cpu, r.gpu, r.object_store_memory

    def excluded_cpus(self) -> float:
        opts = self.__dict__.get("_execution_options")
        return float((opts.exclude_resources.cpu or 0.0) if opts is not None else 0.0)
