"""Linear layer whose weight/bias gradients are written straight into the flat
data-parallel gradient buffer ("main grad").

Forward is a plain hipBLASLt GEMM with the bias epilogue. Backward computes
``dX = dY @ W`` and accumulates ``dW += dY^T X`` with ``addmm_`` (GEMM with
beta = 1) directly into ``weight.main_grad`` — a view of the flat grad buffer —
and ``db += colsum(dY)`` with the HIP ``bias_grad_`` kernel, then signals the
bucketed reducer that the parameter is ready. Autograd's AccumulateGrad (a
read-modify-write of every gradient) and torch's generic bias reduction are
skipped entirely.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel


def _ready(p):
    h = getattr(p, "_ca_grad_ready", None)
    if h is not None:
        h(p)


class _MainGradLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        b = ctx.bias
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ w).view(*dy.shape[:-1], w.shape[1])
        gw = gb = None
        mg = getattr(w, "main_grad", None)
        if mg is not None:
            mg.addmm_(dy2.t(), x2)
            _ready(w)
        elif ctx.needs_input_grad[1]:
            gw = dy2.t() @ x2
        if b is not None:
            bmg = getattr(b, "main_grad", None)
            if bmg is not None and dy2.shape[1] % 8 == 0:
                kernels().bias_grad_(dy2.contiguous(), bmg, True)
                _ready(b)
            elif ctx.needs_input_grad[2]:
                gb = dy2.float().sum(0).to(b.dtype)
        return dx, gw, gb


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    if use_gpu_kernel(x, weight) and getattr(weight, "main_grad", None) is not None and x.requires_grad:
        return _MainGradLinear.apply(x, weight, bias)
    return F.linear(x, weight, bias)
