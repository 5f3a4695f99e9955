"""Failure handling for the v2 controller (reference:
python/ray/train/v2/_internal/execution/failure_handling/default.py)."""
from __future__ import annotations

import enum
from typing import Dict

from ..config import FailureConfig


class FailureDecision(enum.Enum):
    RESTART = "RESTART"
    RAISE = "RAISE"
    NOOP = "NOOP"


class FailurePolicy:
    def __init__(self, failure_config: FailureConfig):
        self.failure_config = failure_config

    def make_decision(self, errors: Dict[int, BaseException]) -> FailureDecision:
        raise NotImplementedError


class DefaultFailurePolicy(FailurePolicy):
    """Restart while the run's failure count stays within
    ``FailureConfig.max_failures`` (-1: always), then raise."""

    def __init__(self, failure_config: FailureConfig):
        super().__init__(failure_config)
        self.total_failures = 0

    def make_decision(self, errors):
        if not errors:
            return FailureDecision.NOOP
        self.total_failures += 1
        mf = self.failure_config.max_failures
        if mf == -1 or self.total_failures <= mf:
            return FailureDecision.RESTART
        return FailureDecision.RAISE
