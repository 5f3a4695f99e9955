"""Utilities (reference: python/ray/util/): ActorPool, Queue, placement groups,
scheduling strategies, state API, metrics, collective, multiprocessing Pool."""
from .actor_pool import ActorPool
from .placement_group import (
    PlacementGroup,
    get_current_placement_group,
    get_placement_group,
    placement_group,
    placement_group_table,
    remove_placement_group,
)
from .queue import Empty, Full, Queue
from .scheduling_strategies import (
    NodeAffinitySchedulingStrategy,
    NodeLabelSchedulingStrategy,
    PlacementGroupSchedulingStrategy,
)


def get_node_ip_address() -> str:
    return "127.0.0.1"


def list_named_actors(all_namespaces: bool = False):
    from ..core.api import _state
    from ..core import context

    names = _state("named_actors")
    if all_namespaces:
        return [{"name": n, "namespace": ns} for ns, n in names]
    ns = context.worker.namespace
    return [n for (s, n) in names if s == ns]


__all__ = [
    "ActorPool", "Queue", "Empty", "Full", "PlacementGroup", "placement_group",
    "remove_placement_group", "get_placement_group", "placement_group_table",
    "get_current_placement_group", "PlacementGroupSchedulingStrategy",
    "NodeAffinitySchedulingStrategy", "NodeLabelSchedulingStrategy", "get_node_ip_address",
    "list_named_actors",
]


def inspect_serializability(*a, **k):
    from .check_serialize import inspect_serializability as _i

    return _i(*a, **k)
