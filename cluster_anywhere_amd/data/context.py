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
        return self

    @property
    def preserve_order(self) -> bool:
        return self.execution_preserve_order

    @preserve_order.setter
    def preserve_order(self, v: bool):
        self.execution_preserve_order = bool(v)
