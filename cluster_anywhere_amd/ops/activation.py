"""Fused bias + GELU(tanh) backed by ``bias_gelu.hip`` (dbias fused into backward)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel


def bias_gelu_ref(h, b=None):
    x = h.float() + (b.float() if b is not None else 0.0)
    return F.gelu(x, approximate="tanh").to(h.dtype)


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, b):
        h = h.contiguous()
        ctx.save_for_backward(h, b)
        return kernels().bias_gelu_fwd(h, b)

    @staticmethod
    def backward(ctx, dy):
        h, b = ctx.saved_tensors
        dh, db = kernels().bias_gelu_bwd(dy.contiguous(), h, b)
        return dh, (db if b is not None else None)


def bias_gelu(h: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if use_gpu_kernel(h, b) and h.dtype == torch.bfloat16 and h.shape[-1] % 8 == 0:
        return _BiasGeluFn.apply(h, b)
    x = h + b if b is not None else h
    return F.gelu(x, approximate="tanh")
