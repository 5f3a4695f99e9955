"""Placement groups (reference: python/ray/util/placement_group.py:145).
Bundles are reserved atomically by the native ClusterScheduler (PACK / SPREAD /
STRICT_PACK / STRICT_SPREAD); ``ready()`` is an ObjectRef sealed once reserved."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from ..core import context
from ..core.ids import ObjectID, PlacementGroupID

VALID_STRATEGIES = ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD")


class PlacementGroup:
    def __init__(self, id: PlacementGroupID, bundles: Optional[List[Dict]] = None,
                 strategy: str = "PACK", ready_oid: Optional[bytes] = None, name: str = ""):
        self.id = id
        self._bundles = bundles or []
        self._strategy = strategy
        self._ready_oid = ready_oid
        self._ready_ref = None
        self._name = name

    @staticmethod
    def empty():
        return PlacementGroup(PlacementGroupID.nil())

    @property
    def bundle_specs(self) -> List[Dict]:
        return list(self._bundles)

    @property
    def bundle_count(self) -> int:
        return len(self._bundles)

    @property
    def strategy(self) -> str:
        return self._strategy

    def ready(self):
        from ..core.object_ref import ObjectRef

        if self._ready_ref is None:
            if self._ready_oid is None:
                raise ValueError("placement group handle has no readiness object")
            self._ready_ref = ObjectRef(self._ready_oid)
        return self._ready_ref

    def wait(self, timeout_seconds: float = 30) -> bool:
        from ..core.api import wait

        ready, _ = wait([self.ready()], timeout=timeout_seconds)
        return bool(ready)

    def __eq__(self, other):
        return isinstance(other, PlacementGroup) and other.id == self.id

    def __hash__(self):
        return hash(self.id)

    def __reduce__(self):
        return (PlacementGroup, (self.id, self._bundles, self._strategy, self._ready_oid, self._name))


def _validate_bundles(bundles):
    if not isinstance(bundles, list) or not bundles:
        raise ValueError("bundles must be a non-empty list of resource dicts")
    for b in bundles:
        if not isinstance(b, dict) or not b:
            raise ValueError(f"invalid bundle {b!r}: must be a non-empty dict")
        if all(v == 0 for v in b.values()):
            raise ValueError(f"bundle {b!r} requests no resources")
        for k, v in b.items():
            if v < 0:
                raise ValueError("bundle resources must be non-negative")


def placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", name: str = "",
                    lifetime: Optional[str] = None, _max_cpu_fraction_per_node=None,
                    _soft_target_node_id=None) -> PlacementGroup:
    from ..core.api import _ensure_init

    _ensure_init()
    _validate_bundles(bundles)
    if strategy not in VALID_STRATEGIES:
        raise ValueError(f"Invalid placement group strategy {strategy}. Supported: {VALID_STRATEGIES}")
    if lifetime not in (None, "detached"):
        raise ValueError("lifetime must be None or 'detached'")
    pg_id = PlacementGroupID.from_random()
    ready_oid = ObjectID.for_put(pg_id.binary())
    bundles = [{k: float(v) for k, v in b.items()} for b in bundles]
    if context.local_mode:
        return PlacementGroup(pg_id, bundles, strategy, None, name)
    context.worker.send(("pg_create", pg_id.binary(), bundles, strategy, name, ready_oid, lifetime))
    return PlacementGroup(pg_id, bundles, strategy, ready_oid, name)


def remove_placement_group(pg: PlacementGroup) -> None:
    if context.local_mode:
        return
    context.worker.send(("pg_remove", pg.id.binary()))


def get_placement_group(name: str) -> PlacementGroup:
    w = context.worker
    res = w.request(lambda r: ("pg_by_name", r, name))
    if res is None:
        raise ValueError(f"Failed to look up placement group with name: {name}")
    pid, bundles, strategy = res
    return PlacementGroup(PlacementGroupID(pid), bundles, strategy, None, name)


def placement_group_table(pg: Optional[PlacementGroup] = None) -> dict:
    w = context.worker
    return w.request(lambda r: ("pg_table", r, pg.id.binary() if pg is not None else None))


def get_current_placement_group() -> Optional[PlacementGroup]:
    """The placement group of the running task, or of this actor (also inside its
    methods' thread pools / event loops)."""
    cur = context.current_pg()
    if not cur:
        return None
    return PlacementGroup(PlacementGroupID(cur[1]))


def check_placement_group_index(pg: PlacementGroup, bundle_index: int):
    if bundle_index >= pg.bundle_count or bundle_index < -1:
        raise ValueError(f"placement_group_bundle_index {bundle_index} out of range for "
                         f"{pg.bundle_count} bundles")
