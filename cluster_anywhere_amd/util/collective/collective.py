"""Collective communication between actors / tasks (reference:
python/ray/util/collective/collective.py — ``init_collective_group`` :120,
``create_collective_group`` :151, ``allreduce`` :258, ``broadcast`` :373,
``allgather`` :423, ``reducescatter`` :472, ``send``/``recv`` :531/:594).

MI355X-first design: every group is its OWN torch.distributed process group,
constructed directly (``ProcessGroupNCCL`` = RCCL over xGMI for GPU tensors,
``ProcessGroupGloo`` for CPU tensors / numpy arrays) instead of going through
the process-global default group, so one actor can sit in any number of groups
(e.g. a DP group and a weight-sync group). Rendezvous: rank 0 opens a
``TCPStore`` on a free port and publishes ``host:port`` in the cluster's
internal KV under the group name; the other ranks read it from there. Groups
declared from the driver with :func:`create_collective_group` are joined lazily
by each member actor on its first collective call.
"""
from __future__ import annotations

import datetime
import json
import os
import time
from typing import Dict, List, Optional

from .types import Backend, ReduceOp

_NS = "collective"
_groups: Dict[str, "CollectiveGroup"] = {}


def _torch_op(op):
    import torch.distributed as dist

    return {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.PRODUCT: dist.ReduceOp.PRODUCT,
            ReduceOp.MIN: dist.ReduceOp.MIN, ReduceOp.MAX: dist.ReduceOp.MAX}[ReduceOp(op)]


def _node_ip() -> str:
    return os.environ.get("CAAMD_NODE_IP", "127.0.0.1")


def _store_key(name: str) -> str:
    return f"{name}/store"


def _info_key(name: str) -> str:
    return f"{name}/info"


def _rendezvous(name: str, rank: int, world: int, timeout: datetime.timedelta):
    import torch.distributed as dist

    from ...experimental import internal_kv as kv

    if rank == 0:
        host = _node_ip()
        store = dist.TCPStore(host, 0, world, True, timeout, wait_for_workers=False)
        kv._internal_kv_put(_store_key(name), f"{host}:{store.port}", True, namespace=_NS)
        return store
    deadline = time.time() + timeout.total_seconds()
    while True:
        v = kv._internal_kv_get(_store_key(name), namespace=_NS)
        if v:
            break
        if time.time() > deadline:
            raise TimeoutError(f"collective group {name!r}: rank 0 never published its store")
        time.sleep(0.02)
    host, port = v.decode().rsplit(":", 1)
    return dist.TCPStore(host, int(port), world, False, timeout)


class CollectiveGroup:
    """One communicator: ``world_size`` members, this process is ``rank``."""

    def __init__(self, world_size: int, rank: int, backend: Backend, group_name: str,
                 timeout_s: float = 300.0):
        import torch.distributed as dist

        self.world_size, self.rank = world_size, rank
        self.backend, self.group_name = Backend(backend), group_name
        timeout = datetime.timedelta(seconds=timeout_s)
        self._store = _rendezvous(group_name, rank, world_size, timeout)
        if self.backend == Backend.GLOO:
            self.pg = dist.ProcessGroupGloo(self._store, rank, world_size, timeout)
            self.device = "cpu"
        else:
            import torch

            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = timeout
            opts.group_name = group_name
            self.pg = dist.ProcessGroupNCCL(self._store, rank, world_size, opts)
            self.device = f"cuda:{torch.cuda.current_device()}"
            # build the RCCL communicator now (what init_process_group(device_id=..)
            # does), not lazily inside the first collective
            self.pg.eager_connect_single_device(torch.device(self.device))

    # -- collectives (every call blocks until the result is in place) ----------
    def allreduce(self, t, op=ReduceOp.SUM):
        import torch.distributed as dist

        o = dist.AllreduceOptions()
        o.reduceOp = _torch_op(op)
        self.pg.allreduce([t], o).wait()

    def reduce(self, t, dst_rank: int, op=ReduceOp.SUM):
        import torch.distributed as dist

        o = dist.ReduceOptions()
        o.reduceOp = _torch_op(op)
        o.rootRank = dst_rank
        o.rootTensor = 0
        self.pg.reduce([t], o).wait()

    def broadcast(self, t, src_rank: int):
        import torch.distributed as dist

        o = dist.BroadcastOptions()
        o.rootRank = src_rank
        o.rootTensor = 0
        self.pg.broadcast([t], o).wait()

    def allgather(self, tensor_list, t):
        self.pg.allgather([list(tensor_list)], [t]).wait()

    def reducescatter(self, t, tensor_list, op=ReduceOp.SUM):
        import torch.distributed as dist

        o = dist.ReduceScatterOptions()
        o.reduceOp = _torch_op(op)
        self.pg.reduce_scatter([t], [list(tensor_list)], o).wait()

    def send(self, t, dst_rank: int):
        self.pg.send([t], dst_rank, 0).wait()

    def recv(self, t, src_rank: int):
        self.pg.recv([t], src_rank, 0).wait()

    def barrier(self):
        import torch

        x = torch.zeros(1, device=self.device)
        self.allreduce(x)
        if self.device != "cpu":
            torch.cuda.synchronize()

    def destroy(self):
        if self.rank == 0:
            try:
                from ...experimental import internal_kv as kv

                kv._internal_kv_del(_store_key(self.group_name), namespace=_NS)
            except Exception:
                pass
        self.pg = None
        self._store = None


# ------------------------------------------------------------------ group API
def nccl_available() -> bool:
    try:
        import torch
        import torch.distributed as dist

        return dist.is_nccl_available() and torch.cuda.is_available()
    except Exception:
        return False


rccl_available = nccl_available


def gloo_available() -> bool:
    try:
        import torch.distributed as dist

        return dist.is_gloo_available()
    except Exception:
        return False


def is_group_initialized(group_name: str = "default") -> bool:
    return group_name in _groups


def init_collective_group(world_size: int, rank: int, backend=Backend.NCCL, group_name: str = "default",
                          timeout_s: float = 300.0) -> None:
    """Join (or create) ``group_name`` from inside an actor / task."""
    backend = Backend(backend)
    if not group_name:
        raise ValueError(f"group_name '{group_name}' needs to be a non-empty string.")
    if group_name in _groups:
        raise RuntimeError("Trying to initialize a group twice.")
    if not (world_size > 0 and 0 <= rank < world_size):
        raise ValueError(f"invalid rank {rank} for world_size {world_size}")
    if backend == Backend.NCCL and not nccl_available():
        raise RuntimeError("RCCL (backend 'nccl') needs a GPU process; use backend='gloo' on CPU")
    _groups[group_name] = CollectiveGroup(world_size, rank, backend, group_name, timeout_s)


def create_collective_group(actors, world_size: int, ranks: List[int], backend=Backend.NCCL,
                            group_name: str = "default") -> None:
    """Declare ``actors`` a collective group from the driver; each member joins
    lazily on its first collective call."""
    from ...experimental import internal_kv as kv

    backend = Backend(backend)
    if len(ranks) != len(actors):
        raise RuntimeError(f"Each actor should correspond to one rank. Got '{len(ranks)}' ranks "
                           f"but '{len(actors)}' actors")
    if set(ranks) != set(range(len(ranks))):
        raise RuntimeError(f"Ranks must be a permutation from 0 to '{len(ranks)}'. Got '{ranks}'.")
    if world_size <= 0:
        raise RuntimeError(f"World size must be greater than zero. Got '{world_size}'.")
    info = {"actor_ids": [a._actor_id.hex() for a in actors], "world_size": world_size,
            "ranks": list(ranks), "backend": backend.value}
    if kv._internal_kv_put(_info_key(group_name), json.dumps(info), False, namespace=_NS):
        raise RuntimeError("Trying to initialize a group twice.")


def destroy_collective_group(group_name: str = "default") -> None:
    g = _groups.pop(group_name, None)
    if g is not None:
        g.destroy()
        if g.rank == 0:
            try:
                from ...experimental import internal_kv as kv

                kv._internal_kv_del(_info_key(group_name), namespace=_NS)
            except Exception:
                pass


def _check_and_get_group(group_name: str) -> CollectiveGroup:
    g = _groups.get(group_name)
    if g is not None:
        return g
    from ...experimental import internal_kv as kv
    from ...runtime_context import get_runtime_context

    v = kv._internal_kv_get(_info_key(group_name), namespace=_NS)
    if v is None:
        raise RuntimeError(f"The collective group '{group_name}' is not initialized in the process.")
    info = json.loads(v)
    me = get_runtime_context().get_actor_id()
    if me not in info["actor_ids"]:
        raise RuntimeError(f"This process is not a member of collective group '{group_name}'.")
    rank = info["ranks"][info["actor_ids"].index(me)]
    init_collective_group(info["world_size"], rank, info["backend"], group_name)
    return _groups[group_name]


def get_rank(group_name: str = "default") -> int:
    g = _groups.get(group_name)
    return -1 if g is None else g.rank


def get_collective_group_size(group_name: str = "default") -> int:
    g = _groups.get(group_name)
    return -1 if g is None else g.world_size


def _t(x):
    """numpy arrays are reduced in place through a zero-copy torch view."""
    import numpy as np

    if isinstance(x, np.ndarray):
        import torch

        return torch.from_numpy(x)
    return x


def allreduce(tensor, group_name: str = "default", op=ReduceOp.SUM):
    _check_and_get_group(group_name).allreduce(_t(tensor), op)


def barrier(group_name: str = "default"):
    _check_and_get_group(group_name).barrier()


def reduce(tensor, dst_rank: int = 0, group_name: str = "default", op=ReduceOp.SUM):
    g = _check_and_get_group(group_name)
    _check_rank(g, dst_rank)
    g.reduce(_t(tensor), dst_rank, op)


def broadcast(tensor, src_rank: int = 0, group_name: str = "default"):
    g = _check_and_get_group(group_name)
    _check_rank(g, src_rank)
    g.broadcast(_t(tensor), src_rank)


def allgather(tensor_list: list, tensor, group_name: str = "default"):
    g = _check_and_get_group(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("The length of the tensor list operands to allgather must be equal to world_size.")
    g.allgather([_t(x) for x in tensor_list], _t(tensor))


def reducescatter(tensor, tensor_list: list, group_name: str = "default", op=ReduceOp.SUM):
    g = _check_and_get_group(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("The length of the tensor list operands to reducescatter must be equal to world_size.")
    g.reducescatter(_t(tensor), [_t(x) for x in tensor_list], op)


def send(tensor, dst_rank: int, group_name: str = "default"):
    g = _check_and_get_group(group_name)
    _check_rank(g, dst_rank)
    if dst_rank == g.rank:
        raise RuntimeError(f"The destination rank '{dst_rank}' is self.")
    g.send(_t(tensor), dst_rank)


def recv(tensor, src_rank: int, group_name: str = "default"):
    g = _check_and_get_group(group_name)
    _check_rank(g, src_rank)
    if src_rank == g.rank:
        raise RuntimeError(f"The source rank '{src_rank}' is self.")
    g.recv(_t(tensor), src_rank)


def synchronize(gpu_id: Optional[int] = None):
    import torch

    torch.cuda.synchronize(gpu_id)


def _check_rank(g, rank):
    if not 0 <= rank < g.world_size:
        raise ValueError(f"rank '{rank}' is out of range for group '{g.group_name}' (size {g.world_size})")
