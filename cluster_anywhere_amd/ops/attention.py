"""Causal multi-head attention entry point.

``attention(qkv, n_head)`` takes the fused QKV projection output laid out as
``[B, T, 3, H, Dh]`` (exactly what ``x @ W_qkv^T`` produces) and returns
``[B, T, H*Dh]``. On MI355X it dispatches to the hand-written MFMA flash
attention (``attention.hip``) when it is built for this head dim; otherwise it
uses torch's fused SDPA. CPU tensors use the math reference.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel

_FORCE_SDPA = os.environ.get("CAAMD_ATTN", "") == "sdpa"


def attention_ref(q, k, v, causal=True):
    """q,k,v: [B, H, T, Dh] -> [B, H, T, Dh] (fp32 math)."""
    d = q.shape[-1]
    s = (q.float() @ k.float().transpose(-1, -2)) / (d ** 0.5)
    if causal:
        T, S = q.shape[-2], k.shape[-2]
        mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(S - T)
        s = s.masked_fill(~mask, float("-inf"))
    return (torch.softmax(s, -1) @ v.float()).to(q.dtype)


def _have_flash(dh: int) -> bool:
    if _FORCE_SDPA:
        return False
    try:
        return hasattr(kernels(), "flash_attn_fwd") and dh in (64, 128)
    except Exception:
        return False


def flash_path(x: torch.Tensor, d_model: int, n_head: int) -> bool:
    """Whether :func:`attention` on a qkv projection of ``x`` takes the flash kernels
    (then it can also produce the projection's bias gradient, ``qkv_bias``)."""
    return use_gpu_kernel(x) and x.dtype == torch.bfloat16 and _have_flash(d_model // n_head)


def attention(qkv: torch.Tensor, n_head: int, causal: bool = True, qkv_bias=None) -> torch.Tensor:
    """``qkv_bias`` (flash path only, see :func:`flash_path`): the bias of the qkv
    projection, whose gradient the attention backward then computes."""
    B, T, three_d = qkv.shape
    D = three_d // 3
    dh = D // n_head
    if use_gpu_kernel(qkv) and qkv.dtype == torch.bfloat16 and _have_flash(dh):
        from .flash import flash_attention_qkv

        return flash_attention_qkv(qkv, n_head, causal, qkv_bias)
    if qkv_bias is not None:
        raise ValueError("qkv_bias is only taken on the flash path (check flash_path first)")
    q, k, v = qkv.view(B, T, 3, n_head, dh).permute(2, 0, 3, 1, 4).unbind(0)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
    return o.transpose(1, 2).reshape(B, T, D)
