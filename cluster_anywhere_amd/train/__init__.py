"""Distributed training (reference: python/ray/train/__init__.py)."""
from .checkpoint import Checkpoint
from .config import CheckpointConfig, DataConfig, FailureConfig, RunConfig, ScalingConfig
from .session import TrainContext, get_checkpoint, get_context, get_dataset_shard, report
from .trainer import Backend, DataParallelTrainer, Result, TrainingFailedError

__all__ = [
    "Checkpoint", "CheckpointConfig", "DataConfig", "FailureConfig", "RunConfig", "ScalingConfig",
    "TrainContext", "get_checkpoint", "get_context", "get_dataset_shard", "report", "Backend",
    "DataParallelTrainer", "Result", "TrainingFailedError", "torch",
]


def __getattr__(name):
    if name == "torch":
        import importlib

        return importlib.import_module(".torch", __name__)
    raise AttributeError(name)
