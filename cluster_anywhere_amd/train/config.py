"""Run / scaling / failure / checkpoint configs (reference: python/ray/air/config.py:
ScalingConfig :102, FailureConfig :397, CheckpointConfig :447, RunConfig :596)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Union


@dataclass
class ScalingConfig:
    num_workers: Optional[int] = None
    use_gpu: Union[bool, None] = False
    resources_per_worker: Optional[Dict[str, float]] = None
    placement_strategy: str = "PACK"
    trainer_resources: Optional[Dict[str, float]] = None
    accelerator_type: Optional[str] = None

    def __post_init__(self):
        nw = self.num_workers
        if isinstance(nw, (tuple, list)):  # elastic (min, max): the v2 controller's ElasticScalingPolicy
            if len(nw) != 2 or not 1 <= int(nw[0]) <= int(nw[1]):
                raise ValueError("elastic num_workers must be (min, max) with 1 <= min <= max")
        elif nw is not None and nw < 1:
            raise ValueError("num_workers must be >= 1")
        if self.resources_per_worker:
            if "GPU" in self.resources_per_worker and not self.use_gpu and self.resources_per_worker["GPU"] > 0:
                raise ValueError("use_gpu=False but resources_per_worker requests GPUs")

    @property
    def total_workers(self) -> int:
        nw = self.num_workers
        if isinstance(nw, (tuple, list)):
            return int(nw[1])
        return nw or 1

    @property
    def _resources_per_worker_not_none(self) -> Dict[str, float]:
        r = dict(self.resources_per_worker or {})
        r.setdefault("CPU", 1.0)
        if self.use_gpu:
            r.setdefault("GPU", 1.0)
        return {k: float(v) for k, v in r.items()}

    def as_placement_group_bundles(self) -> List[Dict[str, float]]:
        return [self._resources_per_worker_not_none for _ in range(self.total_workers)]

    @property
    def num_cpus_per_worker(self):
        return self._resources_per_worker_not_none.get("CPU", 0)

    @property
    def num_gpus_per_worker(self):
        return self._resources_per_worker_not_none.get("GPU", 0)


@dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: Union[bool, str] = False


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None

    def __post_init__(self):
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError("num_to_keep must be positive or None")
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be 'max' or 'min'")


@dataclass
class DataConfig:
    datasets_to_split: Union[str, List[str]] = "all"


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    storage_filesystem: Any = None
    failure_config: Optional[FailureConfig] = None
    checkpoint_config: Optional[CheckpointConfig] = None
    stop: Any = None
    callbacks: Optional[List[Any]] = None
    verbose: int = 1
    log_to_file: bool = False
    sync_config: Any = None
    progress_reporter: Any = None

    def __post_init__(self):
        self.failure_config = self.failure_config or FailureConfig()
        self.checkpoint_config = self.checkpoint_config or CheckpointConfig()
        if self.storage_path is None:
            self.storage_path = os.environ.get("CAAMD_STORAGE_PATH",
                                               os.path.join(os.path.expanduser("~"), "caamd_results"))
