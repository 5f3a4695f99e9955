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
    def forward(ctx, qkv, n_head, causal):
        qkv = qkv.contiguous()
        out, lse = kernels().flash_attn_fwd(qkv, n_head, causal)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_head, ctx.causal = n_head, causal
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dqkv = kernels().flash_attn_bwd(qkv, out, dout.contiguous(), lse, ctx.n_head, ctx.causal)
        return dqkv, None, None


def flash_attention_qkv(qkv: torch.Tensor, n_head: int, causal: bool = True) -> torch.Tensor:
    return _FlashQKV.apply(qkv, n_head, causal)


def flash_attention_lse(qkv: torch.Tensor, n_head: int, causal: bool = True):
    """Forward only, also returning the natural-log LSE [B, H, T] (for tests/serving)."""
    return kernels().flash_attn_fwd(qkv.contiguous(), n_head, causal)
