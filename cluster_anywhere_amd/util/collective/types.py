"""Backend / reduce-op enums (reference: python/ray/util/collective/types.py)."""
from __future__ import annotations

from enum import Enum


class Backend(str, Enum):
    """``NCCL`` is RCCL on ROCm: ring/tree collectives over the point-to-point
    xGMI links between MI355X GPUs. ``"rccl"`` is accepted as an alias."""

    NCCL = "nccl"
    GLOO = "gloo"

    @classmethod
    def _missing_(cls, value):
        v = str(value).lower()
        if v in ("nccl", "rccl"):
            return cls.NCCL
        if v == "gloo":
            return cls.GLOO
        return None


class ReduceOp(Enum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3
