"""The per-worker data-parallel training step used by ``TorchTrainer`` workers.

``DataParallelStep(model)`` converts the model to flat bf16 weights (+ fp32
master), attaches the bucketed RCCL reducer (plain all-reduce DDP, or ZeRO-1
reduce-scatter/all-gather) and the fused AdamW, and exposes
``step(inputs, targets) -> loss``. Works on one GPU, on N GPUs over RCCL, and
on CPU over gloo (reference math path) for tests.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..ops.optim import FusedAdamW
from ..parallel.ddp import DEFAULT_BUCKET_MB, BucketedDDP
from ..parallel.flat import FlatParamSpace


class DataParallelStep:
    def __init__(
        self,
        model: torch.nn.Module,
        lr: float = 1e-4,
        betas=(0.9, 0.95),
        eps: float = 1e-8,
        weight_decay: float = 0.1,
        max_grad_norm: Optional[float] = 1.0,
        bucket_cap_mb: Optional[float] = None,
        zero: bool = False,
        compute_dtype: Optional[torch.dtype] = None,
        process_group=None,
        loss_fn: Optional[Callable] = None,
    ):
        bucket_cap_mb = bucket_cap_mb or DEFAULT_BUCKET_MB
        world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.world = world
        # ZeRO-1 only pays with more than one rank; zero="always" runs the sharded
        # path on any initialised group (world-1 RCCL test of the ZeRO machinery)
        self.zero = bool(zero and (world > 1 or (zero == "always" and dist.is_initialized())))
        p0 = next(model.parameters())
        if p0.is_cuda:
            from ..ops.gemm_tuning import use_tuned_gemms

            use_tuned_gemms()  # shipped per-shape hipBLASLt/rocBLAS selections (lookup only)
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if p0.is_cuda else torch.float32
        align = 64
        if self.zero:
            while align % (8 * world):
                align += 64
        self.model = model
        self.flat = FlatParamSpace(model, dtype=compute_dtype, align=align)
        self.loss_fn = loss_fn
        if self.zero:
            from ..parallel.zero import Zero1Reducer

            self.reducer = Zero1Reducer(
                self.flat, process_group, bucket_cap_mb, lr=lr, betas=betas, eps=eps,
                weight_decay=weight_decay, max_grad_norm=max_grad_norm or 0.0, module=model,
            )
            self.optimizer = self.reducer.optimizer
        else:
            self.reducer = BucketedDDP(self.flat, process_group, bucket_cap_mb)
            self.optimizer = FusedAdamW(
                self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                max_grad_norm=max_grad_norm,
            )

    def wait_params(self):
        """Weights are up to date on the current stream after this (ZeRO-1 defers
        the all-gather into the next forward)."""
        if self.zero:
            self.reducer.wait_params()

    def set_lr(self, lr: float):
        self.optimizer.lr = lr

    def __call__(self, inputs, targets):
        self.flat.zero_grad()
        self.reducer.start()
        if self.loss_fn is None:
            loss = self.model(inputs, targets)
        else:
            loss = self.loss_fn(self.model(inputs), targets)
        loss.backward()
        self.reducer.finish()
        if self.zero:
            self.reducer.step()
        else:
            self.optimizer.step(inv_world=self.reducer.inv_world)
        return loss.detach()
