"""RLlib learner ops on the gfx950 kernels of ``csrc/kernels/rl_encoder.hip``.

* ``nature_cnn(x_u8, params)`` — the Nature-CNN encoder (three NHWC valid convs +
  fc, ReLU) forward AND backward on MFMA: im2col gather (uint8 frames scaled by
  1/255 in the gather), GEMM with fused bias+ReLU, wgrad by split-M fp32 atomics,
  dgrad GEMM + col2im with the ReLU mask fused. Weights are fp32 masters cast to
  bf16 per call; gradients come back fp32.
* ``mlp_tanh(x, params)`` — tanh MLP layers (the default vector-obs encoder) on
  the same GEMM (bias+tanh epilogue, tanh' fused into the dgrad).
* ``ppo_loss_categorical(...)`` — PPO's clipped surrogate + clipped value loss +
  entropy + KL(old||new) for Categorical heads in ONE kernel that writes
  d(loss)/dlogits and d(loss)/dvalue directly.

Every op has a plain fp32 PyTorch reference (``*_ref``) with the same parameter
layout; CPU tensors (env runners, CPU tests) use it, and the GPU numerics tests
compare the kernels against it. Parameter layout: conv weight ``[Cout, KH*KW*Cin]``
with k ordered (kh, kw, ci) — NHWC windows — and the fc input flattened in NHWC
order (h, w, c).

Reference role: rllib/core/models/torch/encoder.py (CNN / MLP encoders) and
rllib/algorithms/ppo/torch/ppo_torch_learner.py (the loss).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from ._lib import kernels

RE_BF16, RE_BIAS_RELU, RE_BIAS_TANH, RE_F32_ATOMIC, RE_DRELU, RE_DTANH = range(6)
ENABLED = os.environ.get("CAAMD_RL_KERNELS", "1") == "1"
_WGRAD_ROWS = 2048  # reduction rows per split-K slice of a wgrad


def use_kernels(x: torch.Tensor) -> bool:
    return ENABLED and x.is_cuda


# ------------------------------------------------------------------ geometry
NATURE_CONVS: Tuple[Tuple[int, int, int], ...] = ((32, 8, 4), (64, 4, 2), (64, 3, 1))  # (Cout, K, stride)


def conv_out(h: int, k: int, s: int) -> int:
    return (h - k) // s + 1


def nature_shapes(h: int, w: int, c: int):
    """Per conv layer: (H, W, Cin, Cout, K, S, OH, OW)."""
    out = []
    for cout, k, s in NATURE_CONVS:
        oh, ow = conv_out(h, k, s), conv_out(w, k, s)
        out.append((h, w, c, cout, k, s, oh, ow))
        h, w, c = oh, ow, cout
    return out, h * w * c


# ------------------------------------------------------------------ references
def nature_cnn_ref(x: torch.Tensor, params: Sequence[torch.Tensor]) -> torch.Tensor:
    """fp32 reference: x uint8 / float NHWC [B,H,W,C] -> [B, F]."""
    B, H, W, C = x.shape
    shapes, _ = nature_shapes(H, W, C)
    y = x.float() * (1.0 / 255.0) if x.dtype == torch.uint8 else x.float()
    y = y.permute(0, 3, 1, 2)
    for li, (h, w, cin, cout, k, s, oh, ow) in enumerate(shapes):
        wgt = params[2 * li].view(cout, k, k, cin).permute(0, 3, 1, 2)
        y = F.relu(F.conv2d(y, wgt, params[2 * li + 1], stride=s))
    y = y.permute(0, 2, 3, 1).reshape(B, -1)  # NHWC flatten
    return F.relu(F.linear(y, params[6], params[7]))


def mlp_tanh_ref(x: torch.Tensor, params: Sequence[torch.Tensor]) -> torch.Tensor:
    y = x.float().reshape(x.shape[0], -1)
    for i in range(0, len(params), 2):
        y = torch.tanh(F.linear(y, params[i], params[i + 1]))
    return y


# ------------------------------------------------------------------ kernel helpers
def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.bfloat16).contiguous()


def _gemm(a, b, c, layout, epi, M, N, K, lda, ldb, ldc, bias=None, aux=None, splits=1):
    kernels().rl_gemm(a, b, c, layout, epi, bias, aux, M, N, K, lda, ldb, ldc, splits)
    return c


class _Flag:
    on = False


# process-wide, not thread-local: CUDA backward runs on autograd's device threads
_ACCUM = _Flag()


class accumulate_into_grad:
    """Within this context the encoder backward adds its fp32 weight gradients
    straight into ``param.grad`` (the learner's flat gradient buffer, zeroed
    before each step) instead of returning fresh tensors for autograd to add: no
    per-parameter memset / add kernels. Only for ``loss.backward()`` — never
    around ``torch.autograd.grad``, which must not touch ``.grad``."""

    def __enter__(self):
        _ACCUM.on = True

    def __exit__(self, *exc):
        _ACCUM.on = False


def _target(param: torch.Tensor, shape) -> Tuple[torch.Tensor, bool]:
    g = param.grad if getattr(_ACCUM, "on", False) else None
    if g is not None and g.dtype == torch.float32 and g.is_contiguous() and tuple(g.shape) == tuple(shape):
        return g, True
    return torch.zeros(shape, device=param.device, dtype=torch.float32), False


def _wgrad(dz: torch.Tensor, x: torch.Tensor, n_out: int, k_in: int, rows: int, param: torch.Tensor):
    """dW[n_out, k_in] (+)= dz[rows, n_out]^T . x[rows, k_in] (fp32). Returns the
    gradient for autograd, or None when it went straight into ``param.grad``."""
    dw, into = _target(param, (n_out, k_in))
    splits = max(1, (rows + _WGRAD_ROWS - 1) // _WGRAD_ROWS)
    _gemm(dz, x, dw, 2, RE_F32_ATOMIC, n_out, k_in, rows, n_out, k_in, k_in, splits=splits)
    return None if into else dw


def _colsum(dz: torch.Tensor, n: int, param: torch.Tensor):
    db, into = _target(param, (n,))
    kernels().rl_colsum(dz.view(-1, n), db)
    return None if into else db


class _NatureCNN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3, wf, bf):
        B, H, W, C = x.shape
        shapes, flat = nature_shapes(H, W, C)
        dev = x.device
        ws = [_bf(w) for w in (w1, w2, w3, wf)]
        bs = [_bf(b) for b in (b1, b2, b3, bf)]
        cols, ys = [], []
        inp = x.contiguous()
        for li, (h, w, cin, cout, k, s, oh, ow) in enumerate(shapes):
            M, K = B * oh * ow, k * k * cin
            col = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
            kernels().rl_im2col(inp, col, k, k, s, 1.0 / 255.0 if li == 0 else 1.0)
            y = torch.empty(B, oh, ow, cout, device=dev, dtype=torch.bfloat16)
            _gemm(col, ws[li], y, 0, RE_BIAS_RELU, M, cout, K, K, K, cout, bias=bs[li])
            cols.append(col)
            ys.append(y)
            inp = y
        nf = wf.shape[0]
        z = torch.empty(B, nf, device=dev, dtype=torch.bfloat16)
        _gemm(ys[-1].view(B, flat), ws[3], z, 0, RE_BIAS_RELU, B, nf, flat, flat, flat, nf, bias=bs[3])
        ctx.save_for_backward(*cols, *ys, z, *ws)
        ctx.geom = (B, H, W, C, shapes, flat, nf, x.requires_grad)
        ctx.params = (w1, b1, w2, b2, w3, b3, wf, bf)
        return z

    @staticmethod
    def backward(ctx, gz):
        col1, col2, col3, y1, y2, y3, z, w1, w2, w3, wf = ctx.saved_tensors
        B, H, W, C, shapes, flat, nf, _ = ctx.geom
        cols, ys, ws = (col1, col2, col3), (y1, y2, y3), (w1, w2, w3)
        P = ctx.params
        dzf = (gz * (z > 0)).to(torch.bfloat16).contiguous()  # fc ReLU'
        dwf = _wgrad(dzf, ys[-1].view(B, flat), nf, flat, B, P[6])
        dbf = _colsum(dzf, nf, P[7])
        dz = torch.empty(B, flat, device=gz.device, dtype=torch.bfloat16)
        # d(conv3 out) with conv3's ReLU' fused: dz3 = (dzf . Wf) * (y3 > 0)
        _gemm(dzf, wf, dz, 1, RE_DRELU, B, flat, nf, nf, flat, flat, aux=ys[-1].view(B, flat))
        grads = [None] * 6
        for li in range(len(shapes) - 1, -1, -1):
            h, w, cin, cout, k, s, oh, ow = shapes[li]
            M, K = B * oh * ow, k * k * cin
            dz2d = dz.view(M, cout)
            grads[2 * li] = _wgrad(dz2d, cols[li], cout, K, M, P[2 * li])
            grads[2 * li + 1] = _colsum(dz2d, cout, P[2 * li + 1])
            if li == 0:
                break
            dcol = torch.empty(M, K, device=gz.device, dtype=torch.bfloat16)
            _gemm(dz2d, ws[li], dcol, 1, RE_BF16, M, K, cout, cout, K, K)
            dprev = torch.empty(B, h, w, cin, device=gz.device, dtype=torch.bfloat16)
            kernels().rl_col2im(dcol, ys[li - 1], dprev, k, k, s, 1)  # previous layer's ReLU'
            dz = dprev
        return (None, grads[0], grads[1], grads[2], grads[3], grads[4], grads[5], dwf, dbf)


def nature_kernel_ok(h: int, w: int, c: int) -> bool:
    """The im2col / col2im kernels move 8-element runs: KW*C, S*C and W*C must be
    multiples of 8 on every layer (true for 84x84x4 Atari frames)."""
    shapes, flat = nature_shapes(h, w, c)
    return flat % 8 == 0 and all(
        (k * cin) % 8 == 0 and (s * cin) % 8 == 0 and (w_ * cin) % 8 == 0 and oh > 0 and ow > 0
        for (h_, w_, cin, cout, k, s, oh, ow) in shapes)


def nature_cnn(x: torch.Tensor, params: Sequence[torch.Tensor]) -> torch.Tensor:
    """Nature-CNN encoder. GPU: MFMA kernels (bf16 compute, fp32 grads); CPU: reference."""
    if not use_kernels(x) or not nature_kernel_ok(*x.shape[1:]):
        return nature_cnn_ref(x, params)
    if x.dtype != torch.uint8:
        x = x.to(torch.bfloat16)
    return _NatureCNN.apply(x.contiguous(), *params).float()


class _MLPTanh(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        B = x.shape[0]
        h = x.reshape(B, -1).to(torch.bfloat16).contiguous()
        acts = [h]
        ws = []
        for i in range(0, len(params), 2):
            wt, b = _bf(params[i]), _bf(params[i + 1])
            n, k = wt.shape
            y = torch.empty(B, n, device=x.device, dtype=torch.bfloat16)
            _gemm(h, wt, y, 0, RE_BIAS_TANH, B, n, k, k, k, n, bias=b)
            acts.append(y)
            ws.append(wt)
            h = y
        ctx.save_for_backward(*acts, *ws)
        ctx.n = len(ws)
        ctx.params = params
        return h

    @staticmethod
    def backward(ctx, gy):
        saved = ctx.saved_tensors
        n = ctx.n
        acts, ws = saved[:n + 1], saved[n + 1:]
        B = gy.shape[0]
        # tanh' of the last layer: dz = gy * (1 - y^2)
        y = acts[-1].float()
        dz = (gy * (1.0 - y * y)).to(torch.bfloat16).contiguous()
        grads: List[torch.Tensor] = [None] * (2 * n)
        for li in range(n - 1, -1, -1):
            nout, kin = ws[li].shape
            grads[2 * li] = _wgrad(dz, acts[li], nout, kin, B, ctx.params[2 * li])
            grads[2 * li + 1] = _colsum(dz, nout, ctx.params[2 * li + 1])
            if li == 0:
                break
            dprev = torch.empty(B, kin, device=gy.device, dtype=torch.bfloat16)
            _gemm(dz, ws[li], dprev, 1, RE_DTANH, B, kin, nout, nout, kin, kin, aux=acts[li])
            dz = dprev
        return (None, *grads)


def mlp_kernel_ok(in_dim: int, hiddens: Sequence[int]) -> bool:
    return all(d % 8 == 0 for d in [in_dim, *hiddens])


def mlp_tanh(x: torch.Tensor, params: Sequence[torch.Tensor]) -> torch.Tensor:
    if not use_kernels(x):
        return mlp_tanh_ref(x, params)
    return _MLPTanh.apply(x, *params).float()


# ------------------------------------------------------------------ fused PPO loss
class _PPOLossCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, vf, actions, old_logp, adv, vt, old_logits, clip, vf_clip, vf_coeff, ent_coeff,
                kl_coeff, kl_dev):
        dl, dv, stats = kernels().ppo_loss_cat(
            logits.float().contiguous(), vf.float().contiguous(), actions.long().contiguous(),
            old_logp.float().contiguous(), adv.float().contiguous(), vt.float().contiguous(),
            old_logits.float().contiguous(), clip, vf_clip, vf_coeff, ent_coeff, kl_coeff, kl_dev)
        inv_b = 1.0 / logits.shape[0]
        # no host->device copies here: the whole step may be captured in a HIP graph
        loss = (stats[1] * vf_coeff - stats[0] - stats[2] * ent_coeff) * inv_b
        loss = loss + (kl_dev[0] if kl_dev is not None else kl_coeff) * stats[3] * inv_b
        ctx.save_for_backward(dl, dv)
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, gloss, _gstats):
        dl, dv = ctx.saved_tensors
        return dl * gloss, dv * gloss, None, None, None, None, None, None, None, None, None, None, None


def ppo_loss_categorical_ref(logits, vf, actions, old_logp, adv, vt, old_logits, clip, vf_clip, vf_coeff,
                             ent_coeff, kl_coeff):
    lp = logits.float().log_softmax(-1)
    lpo = old_logits.float().log_softmax(-1)
    logp = lp.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
    r = torch.exp(logp - old_logp)
    surr = torch.min(r * adv, r.clamp(1 - clip, 1 + clip) * adv)
    vfl = ((vf - vt) ** 2).clamp(max=vf_clip)
    ent = -(lp.exp() * lp).sum(-1)
    kl = (lpo.exp() * (lpo - lp)).sum(-1)
    loss = -surr.mean() + vf_coeff * vfl.mean() - ent_coeff * ent.mean() + kl_coeff * kl.mean()
    stats = torch.stack([surr.sum(), vfl.sum(), ent.sum(), kl.sum()]).detach()
    return loss, stats


def ppo_loss_categorical(logits, vf, actions, old_logp, adv, vt, old_logits, clip, vf_clip, vf_coeff, ent_coeff,
                         kl_coeff, kl_dev: Optional[torch.Tensor] = None):
    """Returns (loss, stats[4] = sums of surrogate, clipped vf loss, entropy, KL).
    ``kl_dev`` (GPU, 1 float) overrides ``kl_coeff`` from device memory, so a
    captured HIP graph of the learner step follows the adaptive KL coefficient."""
    if not use_kernels(logits):
        if kl_dev is not None:
            kl_coeff = float(kl_dev[0])
        return ppo_loss_categorical_ref(logits, vf, actions, old_logp, adv, vt, old_logits, clip, vf_clip,
                                        vf_coeff, ent_coeff, kl_coeff)
    return _PPOLossCat.apply(logits, vf, actions, old_logp, adv, vt, old_logits, float(clip), float(vf_clip),
                             float(vf_coeff), float(ent_coeff), float(kl_coeff), kl_dev)
