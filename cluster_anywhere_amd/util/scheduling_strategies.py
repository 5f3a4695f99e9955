"""Scheduling strategies (reference: python/ray/util/scheduling_strategies.py)."""
from __future__ import annotations

from typing import Dict, List, Optional, Union


class PlacementGroupSchedulingStrategy:
    def __init__(self, placement_group, placement_group_bundle_index: int = -1,
                 placement_group_capture_child_tasks: Optional[bool] = None):
        self.placement_group = placement_group
        self.placement_group_bundle_index = placement_group_bundle_index
        self.placement_group_capture_child_tasks = placement_group_capture_child_tasks


class NodeAffinitySchedulingStrategy:
    def __init__(self, node_id, soft: bool, _spill_on_unavailable: bool = False,
                 _fail_on_unavailable: bool = False):
        self.node_id = node_id
        self.soft = soft
        self._spill_on_unavailable = _spill_on_unavailable
        self._fail_on_unavailable = _fail_on_unavailable


class In:
    def __init__(self, *values):
        self.values = list(values)


class NotIn:
    def __init__(self, *values):
        self.values = list(values)


class Exists:
    pass


class DoesNotExist:
    pass


class NodeLabelSchedulingStrategy:
    """Schedule on nodes whose labels satisfy every ``hard`` condition; among those
    prefer nodes that also satisfy ``soft``. Values: ``In(...)``, ``NotIn(...)``,
    ``Exists()``, ``DoesNotExist()``. Enforced by the native ClusterScheduler
    (csrc/runtime/scheduler.cc ``labels_match``); a task no node can ever satisfy
    is reported infeasible."""

    def __init__(self, hard: Dict, *, soft: Optional[Dict] = None):
        self.hard = hard
        self.soft = soft or {}


SchedulingStrategyT = Union[None, str, PlacementGroupSchedulingStrategy, NodeAffinitySchedulingStrategy,
                            NodeLabelSchedulingStrategy]
