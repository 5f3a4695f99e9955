"""Distributed training (reference: python/ray/train/__init__.py)."""
from .checkpoint import Checkpoint
from .config import CheckpointConfig, DataConfig, FailureConfig, RunConfig, ScalingConfig
from .session import TrainContext, get_checkpoint, get_context, get_dataset_shard, report
from .trainer import Backend, DataParallelTrainer, Result, TrainingFailedError

BackendConfig = Backend
TRAIN_DATASET_KEY = "train"


class SyncConfig:
    """Checkpoint / artifact sync options (reference: train/_internal/syncer.py).
    Train workers upload checkpoints to the run's storage filesystem themselves
    (train/storage.py); Tune mirrors its locally staged experiment directory to a
    remote storage every ``sync_period`` seconds and at the end (tune/tuner.py)."""

    def __init__(self, sync_period: int = 300, sync_timeout: int = 1800, sync_artifacts: bool = False,
                 sync_artifacts_on_checkpoint: bool = True, **_kw):
        self.sync_period, self.sync_timeout = sync_period, sync_timeout
        self.sync_artifacts = sync_artifacts
        self.sync_artifacts_on_checkpoint = sync_artifacts_on_checkpoint


class TrainingIterator:
    """Iterate the per-report results of a trainer run (reference: train/trainer.py)."""

    def __init__(self, trainer):
        self._result = None
        self._trainer = trainer

    def __iter__(self):
        self._result = self._trainer.fit()
        for m in getattr(self._result, "_history", None) or [self._result.metrics]:
            yield m

    def get_final_results(self):
        return self._result

__all__ = [
    "Checkpoint", "CheckpointConfig", "DataConfig", "FailureConfig", "RunConfig", "ScalingConfig",
    "TrainContext", "get_checkpoint", "get_context", "get_dataset_shard", "report", "Backend",
    "DataParallelTrainer", "Result", "TrainingFailedError", "torch", "BackendConfig", "SyncConfig",
    "TRAIN_DATASET_KEY", "TrainingIterator",
]


def __getattr__(name):
    if name == "torch":
        import importlib

        return importlib.import_module(".torch", __name__)
    raise AttributeError(name)
