"""Fused vocab-wide softmax cross-entropy backed by ``cross_entropy.hip``.

``cross_entropy(logits, target, vocab)`` takes 2-D bf16 logits whose row stride
may be padded beyond ``vocab`` (GPT-2: 50257 -> 50304 for MFMA-friendly GEMMs),
returns per-row fp32 losses, and in backward overwrites the logits buffer with
the gradient (no second N x V buffer).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel


def cross_entropy_ref(logits, target, vocab=None):
    vocab = vocab or logits.shape[-1]
    return F.cross_entropy(
        logits[:, :vocab].float(), target, reduction="none", ignore_index=-100
    )


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vocab):
        loss, lse = kernels().xent_fwd(logits, target, vocab)
        ctx.save_for_backward(logits, target, lse)
        ctx.vocab = vocab
        ctx.mark_non_differentiable(lse)
        return loss

    @staticmethod
    def backward(ctx, dl):
        logits, target, lse = ctx.saved_tensors
        # in-place: the logits buffer is dead after this backward
        kernels().xent_bwd_(logits, target, lse, dl.contiguous().float(), ctx.vocab)
        return logits, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, vocab: int = None) -> torch.Tensor:
    """Per-row loss; ignore_index is any negative target."""
    vocab = vocab or logits.shape[-1]
    if (
        use_gpu_kernel(logits, target)
        and logits.dtype == torch.bfloat16
        and logits.is_contiguous()
        and logits.shape[-1] % 8 == 0
    ):
        return _XentFn.apply(logits, target.contiguous().long(), vocab)
    t = target.clone()
    t[t < 0] = -100
    return F.cross_entropy(logits[:, :vocab].float(), t, reduction="none", ignore_index=-100)
