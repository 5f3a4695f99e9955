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
    """IP address of the node this process runs on (workers: the address their node
    registered with; drivers: the head's advertised address when attached, else
    loopback)."""
    import os

    ip = os.environ.get("CAAMD_NODE_IP")
    if ip:
        return ip
    try:
        from ..core import context

        w = context.worker
        if w is not None and getattr(w, "node_hex", None):
            from ..core.api import nodes

            for n in nodes():
                if n.get("NodeID") == w.node_hex and n.get("NodeManagerAddress"):
                    return n["NodeManagerAddress"]
    except Exception:
        pass
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


from .debug import disable_log_once_globally, enable_periodic_logging, log_once  # noqa: E402
from .serialization import deregister_serializer, register_serializer  # noqa: E402
from . import accelerators, iter  # noqa: E402
from . import rpdb as pdb  # noqa: E402


def connect(conn_str, secure=False, metadata=None, connection_retries=3, job_config=None,
            namespace=None, ignore_version=False, _credentials=None, ray_init_kwargs=None):
    """Client-mode connect (reference: util/client_connect.py)."""
    from ..core.api import init

    addr = conn_str if conn_str.startswith("ray://") else "ray://" + conn_str
    return init(addr, namespace=namespace, job_config=job_config, **(ray_init_kwargs or {}))


def disconnect():
    from ..core.api import shutdown

    shutdown()


def ray_debugpy(*a, **k):
    raise ImportError("debugpy is not installed in this image; use util.pdb.set_trace()")


def __getattr__(name):
    if name == "collective":
        import importlib

        return importlib.import_module(".collective", __name__)
    raise AttributeError(name)
