"""``util.collective`` (reference: python/ray/util/collective/__init__.py)."""
from .collective import (
    allgather,
    allreduce,
    barrier,
    broadcast,
    create_collective_group,
    destroy_collective_group,
    get_collective_group_size,
    get_rank,
    gloo_available,
    init_collective_group,
    is_group_initialized,
    nccl_available,
    rccl_available,
    recv,
    reduce,
    reducescatter,
    send,
    synchronize,
)
from .types import Backend, ReduceOp

__all__ = [
    "allgather", "allreduce", "barrier", "broadcast", "create_collective_group",
    "destroy_collective_group", "get_collective_group_size", "get_rank", "gloo_available",
    "init_collective_group", "is_group_initialized", "nccl_available", "rccl_available", "recv",
    "reduce", "reducescatter", "send", "synchronize", "Backend", "ReduceOp",
]
