"""Zero-copy GPU tensor hand-off between processes of one node
(``tensor_transport="ipc"``).

By default a GPU tensor inside an object is copied to host memory when it is
serialised and copied back to the reader's GPU — correct everywhere, but two
PCIe/xGMI round trips per hand-off. With ``tensor_transport="ipc"`` the object
instead carries a HIP IPC handle (dmabuf-backed on this stack; keep
``HSA_ENABLE_IPC_MODE_LEGACY=0`` in the environment) to the producer's HBM
allocation: a reader on the same node maps the SAME memory — no copy at all.
The producer's caching allocator keeps the block alive until every reader has
released it (torch's CUDA-IPC reference counting).

Use it per object or per actor method::

    ref = ray.put(gpu_tensor, _tensor_transport="ipc")

    @ray.remote(num_gpus=1)
    class Producer:
        @ray.method(tensor_transport="ipc")
        def weights(self):
            return self.w          # readers on this node get a view, not a copy

Device mapping: the handle records the producer's PHYSICAL GPU id; the reader
opens it on its local index of that GPU when the GPU is visible to it, else on
its current device (a peer mapping over xGMI — the reader must not be isolated
from the producer's GPU by ``ROCR_VISIBLE_DEVICES``). Readers on other nodes
cannot map the handle and get an error: use the default transport there.
(The reference exposes the same idea for actors as GPU objects /
``tensor_transport`` in later Ray releases; Ray 2.42's CPU path is
``python/ray/_private/serialization.py``.)
"""
from __future__ import annotations

import os
from typing import List, Optional

_DEVICE_ARG = 6  # position of the device index in torch's rebuild_cuda_tensor args


def _visible_physical() -> Optional[List[int]]:
    """Physical GPU ids visible to this process in local-index order, or None if
    the process is not isolated (local index == physical id)."""
    rocr = os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
    if rocr:
        try:
            return [int(x) for x in rocr.split(",") if x.strip()]
        except ValueError:
            pass
    return None


def physical_gpu(local_index: int) -> int:
    vis = _visible_physical()
    return vis[local_index] if vis is not None and local_index < len(vis) else local_index


def local_gpu(physical: int) -> Optional[int]:
    vis = _visible_physical()
    if vis is None:
        import torch

        return physical if physical < torch.cuda.device_count() else None
    return vis.index(physical) if physical in vis else None


def reduce_ipc(t):
    """Pickle reducer for a GPU tensor under ``tensor_transport="ipc"``."""
    from torch.multiprocessing.reductions import reduce_tensor

    rebuild, args = reduce_tensor(t.detach())
    return _rebuild_ipc, (rebuild, args, physical_gpu(t.device.index), os.getpid())


def _producer_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def _rebuild_ipc(rebuild, args, phys: int, producer_pid: int):
    import torch

    if producer_pid != os.getpid() and not _producer_alive(producer_pid):
        # the HBM behind the handle belonged to a process that has exited: mapping it
        # would read freed memory. Readers must finish with IPC views before the
        # producer is killed (keep the producer actor alive, or use the default
        # host-copy transport for objects that outlive it).
        from ..exceptions import ObjectLostError

        raise ObjectLostError("", f"the producer (pid {producer_pid}) of this tensor_transport='ipc' "
                                  "object has exited; its GPU memory is gone")
    if not torch.cuda.is_available():
        raise RuntimeError("an object sent with tensor_transport='ipc' can only be read by a GPU "
                           "process on the producer's node")
    args = list(args)
    loc = local_gpu(phys)
    args[_DEVICE_ARG] = loc if loc is not None else torch.cuda.current_device()
    return rebuild(*args)
