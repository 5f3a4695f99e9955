"""Legacy ``ray.air.session`` entry points (reference: python/ray/air/session.py)
forwarding to the Train/Tune session of the current worker."""
from ..train.session import get_checkpoint, get_context, get_dataset_shard, report


def get_world_size() -> int:
    return get_context().get_world_size()


def get_world_rank() -> int:
    return get_context().get_world_rank()


def get_local_rank() -> int:
    return get_context().get_local_rank()


def get_trial_name():
    return get_context().get_trial_name()


def get_experiment_name():
    return get_context().get_experiment_name()


__all__ = ["report", "get_checkpoint", "get_context", "get_dataset_shard", "get_world_size",
           "get_world_rank", "get_local_rank", "get_trial_name", "get_experiment_name"]
