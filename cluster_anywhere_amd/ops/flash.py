"""Autograd wrapper of the MFMA flash attention (``flash_attention.hip``).

Takes the packed projection ``qkv [B, T, 3*H*D]`` and returns ``o [B, T, H*D]``;
backward writes one packed ``dqkv`` (dQ, dK, dV interleaved exactly like qkv),
so there is no permute / cat / contiguous copy on either side of the kernels.
"""
from __future__ import annotations

import torch

from ._lib import kernels


class _FlashQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_head, causal, qkv_bias):
        qkv = qkv.contiguous()
        out, lse = kernels().flash_attn_fwd(qkv, n_head, causal)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_head, ctx.causal = n_head, causal
        ctx.qkv_bias = qkv_bias
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        b = ctx.qkv_bias
        if b is None:
            return kernels().flash_attn_bwd(qkv, out, dout.contiguous(), lse, ctx.n_head, ctx.causal), None, None, None
        # the qkv projection's bias gradient = column sums of dqkv, taken from the
        # backward kernels' registers (fp32 atomics) instead of a re-read of dqkv
        from .linear import _dbias_acc, _ready

        mg = getattr(b, "main_grad", None)
        # bf16 main gradient: accumulate into the persistent zeroed fp32 vector that
        # drain_f32_ empties (one launch) instead of zeros() + add_ (two)
        drain = (mg is not None and mg.dtype == torch.bfloat16 and mg.is_contiguous()
                 and mg.device == qkv.device)
        db = (_dbias_acc(qkv.device, qkv.shape[-1]) if drain
              else torch.zeros(qkv.shape[-1], device=qkv.device, dtype=torch.float32))
        dqkv = kernels().flash_attn_bwd(qkv, out, dout.contiguous(), lse, ctx.n_head, ctx.causal, db)
        if mg is not None:
            if drain:
                kernels().drain_f32_(db, mg)
            else:
                mg.add_(db)
            _ready(b)
            return dqkv, None, None, None
        return dqkv, None, None, (db.to(b.dtype) if ctx.needs_input_grad[3] else None)


def flash_attention_qkv(qkv: torch.Tensor, n_head: int, causal: bool = True, qkv_bias=None) -> torch.Tensor:
    """``qkv_bias``: the projection bias that produced ``qkv``; its gradient is then
    computed here (the caller's linear must skip its own bias gradient)."""
    return _FlashQKV.apply(qkv, n_head, causal, qkv_bias)


def flash_attention_lse(qkv: torch.Tensor, n_head: int, causal: bool = True):
    """Forward only, also returning the natural-log LSE [B, H, T] (for tests/serving)."""
    return kernels().flash_attn_fwd(qkv.contiguous(), n_head, causal)
