"""Linear layer whose weight/bias gradients are written straight into the flat
data-parallel gradient buffer ("main grad").

Forward and input-gradient GEMMs run on the hand-written MFMA kernels
(``ops/gemm.py`` -> ``csrc/kernels/gemm.hip``) whenever the shape tiles
(GPT-2-XL: every projection), with the bias add fused into the epilogue; the
input gradient ``dX = dY @ W`` runs on the NN kernel reading ``W`` as stored (round 6;
before, an NT GEMM against a transposed copy: one 64x64-tile transpose per weight per
step, ~1.7 ms for all of GPT-2-XL). ``dW += dY^T X`` accumulates directly into ``weight.main_grad`` — a view
of the flat grad buffer — on the split-K / stream-K weight-gradient kernel of
gemm.hip for the shapes where it measured faster (``gemm.WGRAD_WINNERS``), else
with ``addmm_`` (hipBLASLt, beta = 1); and
``db += colsum(dY)`` with the HIP ``bias_grad_`` kernel, then the parameter is
signalled ready to the bucketed reducer. Autograd's AccumulateGrad (a
read-modify-write of every gradient) and torch's generic bias reduction are
skipped entirely.

``mlp()`` is the fused GPT-2 MLP: fc GEMM with bias+GELU in its epilogue (stores
the pre-activation for backward), fc2 GEMM with bias; in backward the fc2 input
gradient GEMM applies GELU' in its epilogue and accumulates the fc bias gradient
(column sums, fp32 atomics), so no separate bias-GELU kernel runs either way.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import gemm as _g
from ._lib import kernels, use_gpu_kernel


_DBIAS_ACC: dict = {}


def _dbias_acc(dev, n: int) -> torch.Tensor:
    """Zeroed fp32 accumulator of ``n`` floats per device (left zeroed by drain_f32_)."""
    key = (dev, n)
    t = _DBIAS_ACC.get(key)
    if t is None:
        t = _DBIAS_ACC[key] = torch.zeros(n, device=dev, dtype=torch.float32)
    return t


def _ready(p):
    h = getattr(p, "_ca_grad_ready", None)
    if h is not None:
        h(p)


def _wgrad(w, dy2, x2, needs):
    mg = getattr(w, "main_grad", None)
    if mg is not None:
        a, b, c = dy2, x2, mg
        if mg.dim() == 2 and not mg.is_contiguous() and mg.t().is_contiguous():
            a, b, c = x2, dy2, mg.t()  # transposed storage: dW^T += X^T dY
        runs = tn = None
        if c.is_cuda and c.dtype == torch.bfloat16 and _g._ok(a, b, c):
            tn = _g.tn_plan(c.shape[0], c.shape[1], a.shape[0])
            runs = _g.wgrad_runs(c.shape[0], c.shape[1], a.shape[0])
        if tn is not None:
            _g.run_tn(a, b, c, True, *tn)  # c += a^T b (gemm.hip TN full-line kernel)
        elif runs is not None:
            _g.run_sk(a, b, c, 2, True, runs=runs)  # c += a^T b (gemm.hip, split-K / stream-K)
        else:
            c.addmm_(a.t(), b)
        _ready(w)
        return None
    return dy2.t() @ x2 if needs else None


def _wt(w):
    """W^T as a contiguous [K_in, N_out] (free for a transposed-storage weight)."""
    return w.t() if (not w.is_contiguous() and w.t().is_contiguous()) else _g.transpose(w)


def _wn(w):
    """W as a contiguous [N_out, K_in] (one transpose for a transposed-storage weight)."""
    return _g.transpose(w.t()) if (not w.is_contiguous() and w.t().is_contiguous()) else w


def _bgrad(b, dy2, needs):
    if b is None:
        return None
    bmg = getattr(b, "main_grad", None)
    if bmg is not None and dy2.shape[1] % 8 == 0:
        kernels().bias_grad_(dy2.contiguous(), bmg, True)
        _ready(b)
        return None
    return dy2.float().sum(0).to(b.dtype) if needs else None


def _dgrad(dy2, w, mfma):
    if mfma:
        return _g.dgrad_w(dy2.contiguous(), w)
    return dy2 @ w


class _MainGradLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, bias_grad=True):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias if bias_grad else None  # else a later op computes it (fused)
        x2 = x.reshape(-1, x.shape[-1])
        ctx.mfma = _g.supported(x2, weight)
        if ctx.mfma:
            return _g.linear_nt(x2.contiguous(), weight, bias).view(*x.shape[:-1], weight.shape[0])
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        b = ctx.bias
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy2, w, ctx.mfma).view(*dy.shape[:-1], w.shape[1])
        gw = _wgrad(w, dy2, x2, ctx.needs_input_grad[1])
        gb = _bgrad(b, dy2, ctx.needs_input_grad[2])
        return dx, gw, gb, None


class _MainGradMLP(torch.autograd.Function):
    """y = gelu(x W1^T + b1) W2^T + b2 with the GELU fused into both GEMM epilogues."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, b2_grad=True):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        u, z = _g.linear_gelu(x2, w1, b1)
        if (not w2.is_contiguous() and w2.t().is_contiguous()
                and _g.nn_ok(u.shape[0], w2.shape[0], w2.shape[1]) and _g._ok(u, b2)):
            y = _g.linear_nn64(u, w2.t(), b2)  # transposed storage read as stored (NN kernel)
        elif _FC2_NN and not w2.is_contiguous():
            y = _g.linear_nn(u, w2.t(), b2)  # transposed storage read as the NN layout
        else:
            y = _g.linear_nt(u, _wn(w2), b2)
        ctx.save_for_backward(x2, w1, w2, u, z)
        ctx.b = (b1, b2 if b2_grad else None)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, u, z = ctx.saved_tensors
        b1, b2 = ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        gw2 = _wgrad(w2, dy2, u, ctx.needs_input_grad[3])
        gb2 = _bgrad(b2, dy2, ctx.needs_input_grad[4])
        bmg = getattr(b1, "main_grad", None)
        drain = (bmg is not None and bmg.dtype == torch.bfloat16 and bmg.is_contiguous()
                 and bmg.device == dy2.device)
        # the epilogue adds its bias-gradient column sums atomically into an fp32 vector:
        # a persistent zeroed one that drain_f32_ empties into the main gradient (one
        # launch), else a fresh zeros() converted below
        db1 = (_dbias_acc(dy2.device, w1.shape[0]) if drain
               else torch.zeros(w1.shape[0], device=dy2.device, dtype=torch.float32))
        dz = _g.dgrad_dgelu(dy2, _wt(w2), z, db1)
        gb1 = None
        if drain:
            kernels().drain_f32_(db1, bmg)
            _ready(b1)
        elif bmg is not None:
            bmg.add_(db1.to(bmg.dtype))
            _ready(b1)
        elif ctx.needs_input_grad[2]:
            gb1 = db1.to(b1.dtype)
        gw1 = _wgrad(w1, dz, x2, ctx.needs_input_grad[1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _g.dgrad_w(dz, w1).view(ctx.xshape)
        return dx, gw1, gb1, gw2, gb2, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, bias_grad: bool = True) -> torch.Tensor:
    """``bias_grad=False``: the bias gradient is produced by a later fused op (the
    flash-attention backward for the qkv projection); only on the main-grad path."""
    if use_gpu_kernel(x, weight) and getattr(weight, "main_grad", None) is not None and x.requires_grad:
        return _MainGradLinear.apply(x, weight, bias, bias_grad)
    if use_gpu_kernel(x, weight) and _g.supported(x.reshape(-1, x.shape[-1]), weight):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if not torch.is_grad_enabled() or not (x.requires_grad or weight.requires_grad):
            return _g.linear_nt(x2, weight, bias).view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


# The fused epilogues run after the MFMA loop, so their VALU work is exposed: with the
# library tanhf they measured slower than plain GEMM + the streaming bias-GELU kernels
# (764 vs 700 us fwd, 878 vs 840 us bwd at 32768 x 6400); with the exp/rcp tanh the
# fused MLP wins in the real step (86.8k / 86.6k vs 85.9k / 85.8k tok/s, alternating
# runs on one box), so it is the default (CAAMD_FUSED_MLP=0 selects the unfused path).
_FUSED_MLP = os.environ.get("CAAMD_FUSED_MLP", "1") == "1"
# fc2 forward from its transposed storage on the NN layout instead of transpose + NT
_FC2_NN = os.environ.get("CAAMD_FC2_NN", "0") == "1"


def mlp(x, w1, b1, w2, b2, b2_grad: bool = True):
    """GPT-2 MLP ``fc2(gelu_tanh(fc(x)))`` (fused path when the shapes tile).
    ``b2_grad=False``: fc2's bias gradient comes from a later fused op."""
    from .activation import bias_gelu

    x2 = x.reshape(-1, x.shape[-1])
    if (_FUSED_MLP and use_gpu_kernel(x, w1, w2) and b1 is not None and getattr(w1, "main_grad", None) is not None
            and getattr(w2, "main_grad", None) is not None and x.requires_grad
            and _g.supported(x2, w1) and (w2.is_contiguous() or w2.t().is_contiguous())
            and _g.tile_for(x2.shape[0], w2.shape[0], w2.shape[1]) is not None
            and _g.tile_for(x2.shape[0], w2.shape[1], w2.shape[0]) is not None):
        return _MainGradMLP.apply(x, w1, b1, w2, b2, b2_grad)
    return linear(bias_gelu(linear(x, w1), b1), w2, b2, bias_grad=b2_grad)
