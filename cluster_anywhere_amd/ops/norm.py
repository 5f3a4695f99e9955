"""LayerNorm (optionally fused with the residual add) backed by ``layernorm.hip``."""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel


def layer_norm_ref(x, g, b, eps=1e-5):
    return F.layer_norm(x.float(), (x.shape[-1],), g.float(), b.float(), eps).to(x.dtype)


def ln_bias_fusion_ok(x: torch.Tensor) -> bool:
    """Whether the LayerNorm backward can also produce the column sums of its input
    gradient (the bias gradient of the layer that produced the residual branch)."""
    return use_gpu_kernel(x) and x.dtype == torch.bfloat16 and bool(kernels().ln_bwd_dxsum_ok(x.shape[-1]))


def _main_ok(mg, g) -> bool:
    return (mg.dtype == torch.bfloat16 and mg.is_contiguous() and mg.numel() == g.numel()
            and mg.device == g.device)


class _Use:
    """One pending forward use of a LayerNorm's parameters. The backward writes
    dgamma / dbeta straight into their main-grad views and signals readiness itself,
    which is only right when the norm ran ONCE in the step: a shared norm (the same
    module applied twice) must let autograd sum every use before the one
    post-accumulate hook fires. The count of pending uses lives on the weight; a use
    ends at its backward, or when its graph is freed without one (``__del__``)."""

    __slots__ = ("p", "live")

    def __init__(self, p):
        self.p = p
        self.live = True
        p._ca_ln_uses = getattr(p, "_ca_ln_uses", 0) + 1

    def shared(self) -> bool:
        """Called in the backward, before finish(): was the norm used more than once?"""
        p = self.p
        if getattr(p, "_ca_ln_uses", 0) > 1:
            p._ca_ln_shared = True
        return getattr(p, "_ca_ln_shared", False)

    def finish(self):
        if self.live:
            self.live = False
            p = self.p
            p._ca_ln_uses = max(0, getattr(p, "_ca_ln_uses", 1) - 1)
            if p._ca_ln_uses == 0:
                p._ca_ln_shared = False

    def __del__(self):
        try:
            self.finish()
        except Exception:
            pass


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, g, b, eps, res_bias=None):
        ctx.res_bias = res_bias
        ctx.gb = (g, b)
        ctx.use = _Use(g) if torch.is_grad_enabled() and getattr(g, "main_grad", None) is not None else None
        C = kernels()
        x = x.contiguous()
        if res is not None:
            res = res.contiguous()
        y, mean, rstd, s = C.layernorm_fwd(x, res, g, b, eps)
        saved = s if res is not None else x
        ctx.save_for_backward(saved, g, mean, rstd)
        ctx.has_res = res is not None
        if res is not None:
            return s, y
        return y

    @staticmethod
    def backward(ctx, *grads):
        C = kernels()
        saved, g, mean, rstd = ctx.saved_tensors
        if ctx.has_res:
            ds, dy = grads
            dres = ds.contiguous() if ds is not None else None
        else:
            (dy,) = grads
            dres = None
        if dy is None:
            dy = torch.zeros_like(saved)
        rb = ctx.res_bias
        from .linear import _ready

        # the LayerNorm's own weight / bias gradients go straight into their main-grad
        # views (flat DDP buffer) when both have one: no per-tensor accumulate launch
        gm, bm = (getattr(p, "main_grad", None) for p in ctx.gb)
        own = gm is not None and bm is not None and _main_ok(gm, g) and _main_ok(bm, g)
        if ctx.use is not None:
            own = own and not ctx.use.shared()  # shared norm: autograd sums the uses
            ctx.use.finish()
        dx, dg, db = C.layernorm_bwd(dy.contiguous(), saved, g, mean, rstd, dres,
                                     rb.main_grad if rb is not None else None,
                                     gm if own else None, bm if own else None)
        if rb is not None:
            _ready(rb)  # bias gradient of the residual branch's producer (its main-grad view)
        if own:
            for p in ctx.gb:
                _ready(p)
        if ctx.has_res:
            return dx, dx, dg, db, None, None
        return dx, None, dg, db, None, None


def layer_norm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float = 1e-5):
    if use_gpu_kernel(x, g, b) and x.dtype == torch.bfloat16:
        return _LayerNormFn.apply(x, None, g, b, eps)
    return F.layer_norm(x, (x.shape[-1],), g, b, eps)


def add_layer_norm(
    x: torch.Tensor, res: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float = 1e-5, res_bias=None
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return ``(s, LN(s))`` with ``s = x + res`` in one HBM pass. ``res_bias``: the
    bias (with a ``main_grad``) of the layer that produced ``res``; its gradient is
    then accumulated by this backward (see :func:`ln_bias_fusion_ok`)."""
    if use_gpu_kernel(x, res, g, b) and x.dtype == torch.bfloat16:
        return _LayerNormFn.apply(x, res, g, b, eps, res_bias)
    if res_bias is not None:
        raise ValueError("res_bias needs the fused LayerNorm path")
    s = x + res
    return s, F.layer_norm(s, (s.shape[-1],), g, b, eps)
