"""Fused vocab-wide softmax cross-entropy backed by ``cross_entropy.hip``.

``cross_entropy(logits, target, vocab)`` takes 2-D bf16 logits whose row stride
may be padded beyond ``vocab`` (GPT-2: 50257 -> 50432 for MFMA-friendly GEMMs),
returns per-row fp32 losses, and in backward overwrites the logits buffer with
the gradient (no second N x V buffer).

``linear_cross_entropy(h, w, target, vocab)`` is the whole LM head: mean loss of
``softmax(h @ w^T)`` without ever materialising the [tokens, vocab] logits. The
tokens are cut into chunks (16,384 rows = a 1.65 GB logits buffer for GPT-2-XL,
reused); per chunk, in the FORWARD pass: logits GEMM -> one register-resident
softmax/loss/gradient kernel that overwrites the logits with dlogits (scaled by
1/#valid, a device scalar) -> dh = dlogits @ w (NT GEMM against w^T) -> dw (+)=
dlogits^T h (weight-gradient kernel). All three GEMMs run on ``gemm.hip``. The
backward only scales the stored dh / dw by the incoming gradient (and adds dw into
the flat-buffer ``main_grad`` when the weight has one), so a 3.3 GB logits tensor
is neither written nor kept alive across the step. Role reference: the model's
loss in ``python/ray/train/examples`` GPT-2 / HF trainers (torch cross_entropy over
full logits); the chunked fused form is this framework's own.
"""
from __future__ import annotations

import os

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


FUSED_HEAD = os.environ.get("CAAMD_FUSED_HEAD", "1") == "1"
HEAD_CHUNK = int(os.environ.get("CAAMD_HEAD_CHUNK", "16384"))


def linear_cross_entropy_ok(h2: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the chunked head takes: tokens % 256, hidden % 320, vocab % 256 (the
    fwd / dgrad / wgrad tiles of gemm.hip) and a row short enough for the
    register-resident softmax (<= 131,072 columns)."""
    from . import gemm as _g

    if not (FUSED_HEAD and use_gpu_kernel(h2, w) and _g._ok(h2, w) and h2.dim() == 2 and w.dim() == 2):
        return False
    N, D = h2.shape
    V = w.shape[0]
    C = min(N, HEAD_CHUNK)
    return (N % 256 == 0 and C % 256 == 0 and V % 256 == 0 and D % 320 == 0 and V <= 131072
            and _g.tile_for(C, V, D) is not None and _g.tile_for(C, D, V) is not None)


class _LinearXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h2, w, target, vocab, chunk):
        from . import gemm as _g

        N, D = h2.shape
        V = w.shape[0]
        k = kernels()
        scale = (1.0 / (target >= 0).sum().clamp(min=1).float()).reshape(1)
        C = min(N, chunk)
        logits = torch.empty(C, V, device=h2.device, dtype=torch.bfloat16)
        dh = torch.empty_like(h2)
        dw = torch.empty_like(w)
        # dh = dlogits @ w: on the NN kernel with w read as stored, else against a
        # transposed copy [D, V] on the NT kernel (both operands K-major)
        nn = _g.nn_ok(min(N, chunk), D, V) and (N % min(N, chunk)) % 256 == 0 and _g._ok(h2, w)
        wt = None if nn else _g.transpose(w)
        losses = []
        for c0 in range(0, N, C):
            c1 = min(N, c0 + C)
            hc, lg = h2[c0:c1], logits[: c1 - c0]
            _g._run(hc, w, lg, _g.EPI_BF16)                          # logits = h w^T
            loss_c, _ = k.xent_fused_(lg, target[c0:c1], scale, vocab)  # lg <- scale*(p - onehot)
            losses.append(loss_c)
            if nn:
                _g.linear_nn64(lg, w, out=dh[c0:c1])                    # dh = dlogits w
            else:
                _g._run(lg, wt, dh[c0:c1], _g.EPI_BF16)
            tn = _g.tn_plan(V, D, c1 - c0)
            if tn is not None:
                _g.run_tn(lg, hc, dw, c0 > 0, *tn)                   # dw (+)= dlogits^T h
            else:
                _g.run_sk(lg, hc, dw, 2, accumulate=c0 > 0)
        ctx.save_for_backward(dh, dw)
        ctx.w = w
        return torch.cat(losses).sum() * scale[0]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        # dh / dw were computed in forward and are scaled in place here: a second
        # backward through the same graph would scale them twice
        if getattr(ctx, "consumed", False):
            raise RuntimeError("linear_cross_entropy: backward ran twice through one forward "
                               "(retain_graph=True is not supported by the fused LM head)")
        ctx.consumed = True
        dh, dw = ctx.saved_tensors
        w = ctx.w
        gb = g.to(torch.bfloat16)
        dx = dh.mul_(gb)
        mg = getattr(w, "main_grad", None)
        if mg is not None:
            # the embedding's AccumulateGrad adds the other half of the tied gradient
            # later and fires the bucket hook, so no readiness signal here
            mg.addcmul_(dw, gb)
            gw = None
        else:
            gw = dw.mul_(gb) if ctx.needs_input_grad[1] else None
        return dx, gw, None, None, None


def linear_cross_entropy(h2: torch.Tensor, w: torch.Tensor, target: torch.Tensor, vocab: int,
                         chunk: int = None) -> torch.Tensor:
    """Mean cross-entropy of ``h2 @ w^T`` (columns >= vocab masked; negative targets
    ignored) without materialising the logits when the shapes tile, else the
    plain logits + fused cross-entropy path."""
    target = target.reshape(-1)
    # the fused head computes the dgrad / wgrad GEMMs inside forward: only worth it
    # when a backward will follow (eval and no_grad take the plain logits path)
    wants_grad = torch.is_grad_enabled() and (h2.requires_grad or w.requires_grad)
    if wants_grad and linear_cross_entropy_ok(h2, w):
        return _LinearXentFn.apply(h2, w, target.contiguous().long(), vocab, chunk or HEAD_CHUNK)
    logits = F.linear(h2, w)
    losses = cross_entropy(logits, target, vocab)
    valid = (target >= 0).sum().clamp(min=1)
    return losses.sum() / valid
