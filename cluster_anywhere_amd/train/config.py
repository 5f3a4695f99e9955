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
        if self.accelerator_type:
            # a node advertising accelerator_type:<X> (core/api.py detect_accelerator_type)
            # -- reference: air/config.py:209-215
            r.setdefault(f"accelerator_type:{self.accelerator_type}", 0.001)
        return {k: float(v) for k, v in r.items() if v != 0 or k == "CPU"}

    @property
    def _trainer_resources_not_none(self) -> Dict[str, float]:
        """What the run's coordinator reserves next to its workers (reference:
        air/config.py:217-233): ``trainer_resources`` as given; by default nothing
        when the run has workers (the coordinator is the driver / a light actor)."""
        if self.trainer_resources is None:
            return {} if self.num_workers else {"CPU": 1.0}
        return {k: float(v) for k, v in self.trainer_resources.items() if v}

    def as_placement_group_bundles(self) -> List[Dict[str, float]]:
        """The run's gang: the coordinator's bundle first when it reserves anything
        (reference: ScalingConfig.as_placement_group_factory), then one per worker."""
        head = [self._trainer_resources_not_none] if self._trainer_resources_not_none else []
        return head + [self._resources_per_worker_not_none for _ in range(self.total_workers)]

    @property
    def total_resources(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for b in self.as_placement_group_bundles():
            for k, v in b.items():
                out[k] = out.get(k, 0.0) + v
        return out

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
