"""PyTorch-ROCm training (reference: python/ray/train/torch/: torch_trainer.py:11,
config.py:36/66, train_loop_utils.py: get_device :46, prepare_model :162,
prepare_data_loader :204, accelerate :278, prepare_optimizer :299, backward :312,
enable_reproducibility :322).

MI355X specifics: the process group is RCCL (``"nccl"``) over xGMI with
``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC); ``prepare_model`` uses DDP buckets
sized for per-link-bound xGMI rings (64 MiB, gradients as bucket views);
``prepare_data_parallel_step`` returns the fused fast path (flat bf16 weights +
fp32 master, bucketed all-reduce or ZeRO-1, one fused HIP AdamW launch).
"""
from __future__ import annotations

import os
import random
from datetime import timedelta
from typing import Any, Dict, Optional

from ..checkpoint import Checkpoint
from ..config import RunConfig, ScalingConfig
from ..session import get_context
from ..trainer import Backend, DataParallelTrainer, Result


_PREFLIGHT = os.environ.get("CAAMD_RCCL_PREFLIGHT", "1") == "1"


def rccl_transports(lines) -> Dict[str, int]:
    """Count the transports RCCL reported for its channels ("Channel 00/0 : 0[0] ->
    1[1] via P2P/IPC", "... via SHM/direct/direct", "... via NET/IB/0")."""
    import re

    out: Dict[str, int] = {}
    pat = re.compile(r"Channel \S+ : .* via (\S+)")
    for ln in lines:
        m = pat.search(ln)
        if m:
            t = m.group(1).split("/")[0] if m.group(1).startswith("NET") else m.group(1)
            out[t] = out.get(t, 0) + 1
    return out


def rccl_preflight(rank: int, world_size: int, device_id: Optional[int], debug_file: Optional[str] = None,
                   nbytes: int = 4 << 20) -> Dict[str, Any]:
    """RCCL pre-flight after the process group comes up: a checked 4 MiB all-reduce
    (every rank must see the sum), its time, and the transports RCCL picked (xGMI
    peers show as P2P/IPC; SHM or NET inside one MI355X node means P2P is off, e.g.
    IPC not in dmabuf mode). Rank 0 prints one line."""
    import time

    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", device_id if device_id is not None else torch.cuda.current_device())
    t = torch.full((nbytes // 4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize(dev)
    t.fill_(1.0)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    dist.all_reduce(t)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3
    ok = bool(torch.all(t == float(world_size)).item())
    transports: Dict[str, int] = {}
    if debug_file and os.path.exists(debug_file):
        try:
            with open(debug_file, errors="replace") as f:
                transports = rccl_transports(f)
        except OSError:
            pass
    info = {"world_size": world_size, "allreduce_ms": round(ms, 3), "allreduce_MiB": nbytes >> 20,
            "correct": ok, "transports": transports}
    if rank == 0:
        print(f"RCCL pre-flight: {info}", flush=True)
    if not ok:
        raise RuntimeError(f"RCCL pre-flight all-reduce returned wrong sums on rank {rank}: {info}")
    return info


class TorchConfig(Backend):
    def __init__(self, backend: Optional[str] = None, init_method: str = "env", timeout_s: int = 1800):
        self.backend = backend
        self.init_method = init_method
        self.timeout_s = timeout_s

    def on_start(self, rank, world_size, master_addr, master_port, device_id):
        import torch
        import torch.distributed as dist

        backend = self.backend
        if device_id is not None and torch.cuda.is_available():
            torch.cuda.set_device(int(device_id))
        if backend is None:
            backend = "nccl" if (device_id is not None and torch.cuda.is_available()) else "gloo"
        if dist.is_initialized():
            return
        kw = {}
        debug_file = None
        if backend == "nccl" and device_id is not None:
            kw["device_id"] = torch.device("cuda", int(device_id))
            if world_size > 1 and _PREFLIGHT and "NCCL_DEBUG" not in os.environ:
                # RCCL logs the transport of every channel at communicator set-up
                # ("... via P2P/IPC"); keep that log in a file of its own
                import tempfile

                debug_file = os.path.join(tempfile.gettempdir(), f"caamd-rccl-{os.getpid()}.log")
                os.environ.update({"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,P2P,SHM,NET,GRAPH",
                                   "NCCL_DEBUG_FILE": debug_file})
        dist.init_process_group(backend, init_method=f"tcp://{master_addr}:{master_port}", rank=rank,
                                world_size=world_size, timeout=timedelta(seconds=self.timeout_s), **kw)
        if backend == "nccl" and world_size > 1 and _PREFLIGHT:
            self.preflight = rccl_preflight(rank, world_size, int(device_id) if device_id is not None else None,
                                            debug_file)

    def on_shutdown(self):
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


class TorchTrainer(DataParallelTrainer):
    _default_backend = TorchConfig

    def __init__(self, train_loop_per_worker, *, train_loop_config=None, torch_config=None,
                 scaling_config=None, run_config=None, datasets=None, dataset_config=None,
                 resume_from_checkpoint=None, metadata=None):
        super().__init__(train_loop_per_worker, train_loop_config=train_loop_config,
                         backend_config=torch_config or TorchConfig(), scaling_config=scaling_config,
                         run_config=run_config, datasets=datasets, dataset_config=dataset_config,
                         resume_from_checkpoint=resume_from_checkpoint, metadata=metadata)

    def _fit_spmd(self):
        import torch
        import torch.distributed as dist

        if not dist.is_initialized():
            lr = int(os.environ.get("LOCAL_RANK", "0"))
            if torch.cuda.is_available():
                torch.cuda.set_device(lr)
                os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
                dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
            else:
                dist.init_process_group("gloo")
        return super()._fit_spmd()


def get_device():
    import torch

    if torch.cuda.is_available():
        ids = [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]
        if ids and not os.environ.get("ROCR_VISIBLE_DEVICES"):
            return torch.device("cuda", ids[0])
        if "LOCAL_RANK" in os.environ and not ids:
            return torch.device("cuda", int(os.environ["LOCAL_RANK"]) % torch.cuda.device_count())
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def get_devices():
    return [get_device()]


class _Accelerator:
    """Process-wide settings of ``accelerate()`` (reference: train_loop_utils.py:278
    ``accelerate`` / ``_TorchAccelerator``): automatic mixed precision for
    ``prepare_model`` / ``prepare_optimizer`` / ``backward``."""

    def __init__(self):
        self.amp = False
        self.dtype = None
        self.scaler = None

    def autocast_dtype(self, device):
        if self.dtype is not None:
            return self.dtype
        import torch

        # MI355X: bf16 autocast (fp32 range, no loss scaling); fp16 needs GradScaler
        return torch.bfloat16


_ACCEL = _Accelerator()


def accelerate(amp: bool = False, amp_dtype=None):
    """Enable automatic mixed precision for models / optimizers prepared afterwards.
    ``amp_dtype`` defaults to bfloat16 (no loss scaling needed); ``torch.float16``
    adds dynamic loss scaling through ``prepare_optimizer`` + ``backward``."""
    _ACCEL.amp = bool(amp)
    _ACCEL.dtype = amp_dtype
    _ACCEL.scaler = None


class _AmpForward:
    """Wraps a module's forward in autocast and returns fp32 floating outputs
    (the reference's _WrappedModel does the same)."""

    def __init__(self, fwd, device, dtype):
        self.fwd, self.device, self.dtype = fwd, device, dtype

    def __call__(self, *args, **kwargs):
        import torch

        with torch.autocast(self.device.type, dtype=self.dtype):
            out = self.fwd(*args, **kwargs)
        return _to_fp32(out)


def _to_fp32(x):
    import torch

    if isinstance(x, torch.Tensor):
        return x.float() if x.is_floating_point() and x.dtype != torch.float32 else x
    if isinstance(x, (list, tuple)):
        return type(x)(_to_fp32(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_fp32(v) for k, v in x.items()}
    return x


def prepare_model(model, move_to_device: bool = True, parallel_strategy: Optional[str] = "ddp",
                  parallel_strategy_kwargs: Optional[Dict[str, Any]] = None):
    import torch
    import torch.distributed as dist

    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    if _ACCEL.amp:
        model.forward = _AmpForward(model.forward, dev, _ACCEL.autocast_dtype(dev))
    if not dist.is_initialized() or dist.get_world_size() == 1 or parallel_strategy is None:
        return model
    kw = dict(parallel_strategy_kwargs or {})
    if parallel_strategy == "fsdp":
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP

        return FSDP(model, device_id=dev if dev.type == "cuda" else None, **kw)
    from torch.nn.parallel import DistributedDataParallel as DDP

    kw.setdefault("bucket_cap_mb", float(os.environ.get("CAAMD_BUCKET_MB", "64")))
    kw.setdefault("gradient_as_bucket_view", True)
    if dev.type == "cuda":
        kw.setdefault("device_ids", [dev.index])
    return DDP(model, **kw)


def prepare_data_parallel_step(model, **kwargs):
    """The fused MI355X training step (see :class:`cluster_anywhere_amd.train.loop.DataParallelStep`)."""
    from ..loop import DataParallelStep

    return DataParallelStep(model.to(get_device()), **kwargs)


class _DeviceLoader:
    """Wraps a DataLoader: moves every batch to the device on a side HIP stream,
    one batch ahead, so host->HBM copies overlap compute."""

    def __init__(self, loader, device):
        self.loader = loader
        self.device = device

    def __len__(self):
        return len(self.loader)

    def _move(self, b):
        import torch

        if isinstance(b, torch.Tensor):
            return b.to(self.device, non_blocking=True)
        if isinstance(b, (list, tuple)):
            return type(b)(self._move(x) for x in b)
        if isinstance(b, dict):
            return {k: self._move(v) for k, v in b.items()}
        return b

    def __iter__(self):
        if self.device.type != "cuda":
            for b in self.loader:
                yield self._move(b)
            return
        # side-stream copies one batch ahead; hand_over() = wait_stream + record_stream
        # on every moved tensor (train_loop_utils.py:688-703): without the record, a
        # batch the loop drops goes back to the side stream's pool while the compute
        # stream may still read it, and the next prefetch copy overwrites it
        from ...util.device_transfer import SideStreamMover

        mover = SideStreamMover(self.device)
        it = iter(self.loader)
        try:
            try:
                nxt = mover.stage(next(it))
            except StopIteration:
                return
            while nxt is not None:
                cur = mover.hand_over(nxt)  # before the next copy is enqueued
                try:
                    nxt = mover.stage(next(it))
                except StopIteration:
                    nxt = None
                yield cur
        finally:
            mover.close()


def prepare_data_loader(data_loader, add_dist_sampler: bool = True, move_to_device: bool = True,
                        auto_transfer: bool = True):
    import torch
    import torch.distributed as dist
    from torch.utils.data import DataLoader, DistributedSampler

    if add_dist_sampler and dist.is_initialized() and dist.get_world_size() > 1 and \
            not isinstance(getattr(data_loader, "sampler", None), DistributedSampler):
        sampler = DistributedSampler(data_loader.dataset, shuffle=isinstance(
            data_loader.sampler, torch.utils.data.RandomSampler))
        data_loader = DataLoader(data_loader.dataset, batch_size=data_loader.batch_size, sampler=sampler,
                                 num_workers=data_loader.num_workers, collate_fn=data_loader.collate_fn,
                                 pin_memory=torch.cuda.is_available(), drop_last=data_loader.drop_last)
    if move_to_device:
        return _DeviceLoader(data_loader, get_device())
    return data_loader


class _ScaledOptimizer:
    """fp16 AMP: steps through a GradScaler (skips steps with inf/nan grads)."""

    def __init__(self, optimizer, scaler):
        self.optimizer, self.scaler = optimizer, scaler

    def step(self, closure=None):
        self.scaler.step(self.optimizer)
        self.scaler.update()

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


def prepare_optimizer(optimizer):
    """With ``accelerate(amp=True, amp_dtype=torch.float16)`` the optimizer steps
    through a dynamic loss scaler; bf16 / no AMP returns it unchanged."""
    import torch

    if _ACCEL.amp and _ACCEL.dtype == torch.float16:
        dev = get_device()
        _ACCEL.scaler = torch.amp.GradScaler(dev.type)
        return _ScaledOptimizer(optimizer, _ACCEL.scaler)
    return optimizer


def backward(tensor):
    """``loss.backward()``, scaled when fp16 AMP is active."""
    if _ACCEL.scaler is not None:
        _ACCEL.scaler.scale(tensor).backward()
    else:
        tensor.backward()


def enable_reproducibility(seed: int = 0):
    import numpy as np
    import torch

    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.use_deterministic_algorithms(True, warn_only=True)


__all__ = ["TorchTrainer", "TorchConfig", "get_device", "get_devices", "prepare_model",
           "prepare_data_loader", "prepare_optimizer", "prepare_data_parallel_step", "backward",
           "accelerate", "enable_reproducibility"]


# ----------------------------------------------------------- checkpoint / predict
class TorchCheckpoint(Checkpoint):
    """Directory checkpoint holding a model state dict (reference:
    train/torch/torch_checkpoint.py). The state dict is stored with
    ``torch.save`` and read back with ``weights_only=True``; the module class is
    supplied by the caller on load (no pickled code in the checkpoint)."""

    MODEL_FILENAME = "model.pt"

    @classmethod
    def from_state_dict(cls, state_dict, *, preprocessor=None) -> "TorchCheckpoint":
        import tempfile

        import torch

        d = tempfile.mkdtemp(prefix="torch_ckpt_")
        torch.save({k: v.detach().cpu() for k, v in state_dict.items()}, os.path.join(d, cls.MODEL_FILENAME))
        return cls(d)

    @classmethod
    def from_model(cls, model, *, preprocessor=None) -> "TorchCheckpoint":
        return cls.from_state_dict(model.state_dict())

    def get_state_dict(self):
        import torch

        return torch.load(os.path.join(self.path, self.MODEL_FILENAME), weights_only=True, map_location="cpu")

    def get_model(self, model=None):
        if model is None:
            raise ValueError("pass the (uninitialised) nn.Module to load the state dict into")
        model.load_state_dict(self.get_state_dict())
        return model


class TorchPredictor:
    """Batch inference with a torch module (reference: train/torch/torch_predictor.py);
    bf16 autocast on the GPU when ``use_gpu``."""

    def __init__(self, model, preprocessor=None, use_gpu: bool = False):
        import torch

        self.use_gpu = use_gpu and torch.cuda.is_available()
        self.device = torch.device("cuda" if self.use_gpu else "cpu")
        self.model = model.to(self.device).eval()
        self.preprocessor = preprocessor

    @classmethod
    def from_checkpoint(cls, checkpoint: "TorchCheckpoint", model=None, use_gpu: bool = False):
        ck = checkpoint if isinstance(checkpoint, TorchCheckpoint) else TorchCheckpoint(checkpoint.path)
        return cls(ck.get_model(model), use_gpu=use_gpu)

    def _to_tensor(self, x):
        import numpy as np
        import torch

        return torch.as_tensor(np.asarray(x)).to(self.device)

    def call_model(self, inputs):
        return self.model(inputs)

    def predict(self, data, dtype=None):
        import torch

        if self.preprocessor is not None:
            data = self.preprocessor.transform_batch(data)
        if isinstance(data, dict):
            cols = list(data)
            x = self._to_tensor(data[cols[0]]) if len(cols) == 1 else {k: self._to_tensor(v) for k, v in data.items()}
        else:
            x = self._to_tensor(data)
        if dtype is not None and not isinstance(x, dict):
            x = x.to(dtype)
        with torch.no_grad(), torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.use_gpu):
            out = self.call_model(x)
        if isinstance(out, dict):
            return {k: v.float().cpu().numpy() for k, v in out.items()}
        return {"predictions": out.float().cpu().numpy()}


class TorchDetectionPredictor(TorchPredictor):
    """Detection models take a list of CHW images and return a list of dicts."""

    def call_model(self, inputs):
        imgs = [im for im in (inputs if isinstance(inputs, (list, tuple)) else inputs.unbind(0))]
        outs = self.model(imgs)
        keys = outs[0].keys() if outs else []
        return {k: [o[k] for o in outs] for k in keys}

    def predict(self, data, dtype=None):
        import numpy as np
        import torch

        x = data["image"] if isinstance(data, dict) else data
        x = self._to_tensor(x)
        if dtype is not None:
            x = x.to(dtype)
        with torch.no_grad():
            outs = self.call_model(x)
        return {k: np.array([v.cpu().numpy() for v in vs], dtype=object) for k, vs in outs.items()}


__all__ += ["TorchCheckpoint", "TorchPredictor", "TorchDetectionPredictor"]
