"""Old API stack sampling (reference: rllib/evaluation/)."""
from .rollout_worker import RolloutWorker

__all__ = ["RolloutWorker"]
