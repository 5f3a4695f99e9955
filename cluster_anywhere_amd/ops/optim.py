"""Fused AdamW over a :class:`FlatParamSpace` (``adamw.hip``).

One ``grad_sumsq`` launch (global-norm clipping, device-resident) plus one
``adamw_step`` launch update the fp32 master, both moments and the bf16 model
weights for the whole model. No host synchronisation. ``inv_world`` folds the
data-parallel gradient average (1/N of a SUM all-reduce) into the update.

Reference parity: ``python/ray/train/torch/train_loop_utils.py:299``
(`prepare_optimizer`) and the torch AdamW that Ray Train users plug in.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ._lib import kernels, use_gpu_kernel


class FusedAdamW:
    def __init__(
        self,
        flat,  # FlatParamSpace (or a shard view with the same attributes)
        lr: float = 1e-4,
        betas=(0.9, 0.95),
        eps: float = 1e-8,
        weight_decay: float = 0.1,
        max_grad_norm: Optional[float] = 1.0,
    ):
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm or 0.0
        n = flat.master.numel()
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=flat.master.device)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=flat.master.device)
        self.step_count = 0
        v = os.environ.get("CAAMD_ADAM_VARIANT")  # kernel variant override (A/B timing)
        if v is not None and flat.master.is_cuda:
            kernels().adamw_config(int(v))

    def state_dict(self):
        sd = {
            "step": self.step_count,
            "exp_avg": self.exp_avg,
            "exp_avg_sq": self.exp_avg_sq,
            "master": self.flat.master,
            "lr": self.lr,
        }
        if hasattr(self.flat, "layout"):
            # the flat buffers' element order depends on which weights are stored
            # transposed (CAAMD_FC2_T): record it so a resume can map them back
            sd["layout"] = self.flat.layout()
        return sd

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.flat.master.copy_(sd["master"])
        saved = sd.get("layout")
        if saved is not None and hasattr(self.flat, "relayout_"):
            for buf in (self.exp_avg, self.exp_avg_sq, self.flat.master):
                self.flat.relayout_(buf, saved)
        self.lr = sd.get("lr", self.lr)

    def step(self, grads: Optional[torch.Tensor] = None, param_out=None, inv_world: float = 1.0,
             sumsq: Optional[torch.Tensor] = None):
        """``grads``: flat grad (defaults to the space's grad buffer).
        ``param_out``: flat compute-dtype weights to refresh (defaults to the space's).
        ``sumsq``: precomputed global sum of squares (ZeRO passes an all-reduced one)."""
        self.step_count += 1
        g = self.flat.grad_buffer if grads is None else grads
        pout = self.flat.param_buffer if param_out is None else param_out
        p, m, v = self.flat.master, self.exp_avg, self.exp_avg_sq
        if use_gpu_kernel(p, g):
            C = kernels()
            if self.max_grad_norm > 0 and sumsq is None:
                self.sumsq.zero_()
                C.grad_sumsq(g, self.sumsq)
                sumsq = self.sumsq
            C.adamw_step(
                p, m, v, g, pout if pout is not None and pout.dtype == torch.bfloat16 else None,
                self.lr, self.beta1, self.beta2, self.eps, self.wd, self.step_count, inv_world,
                self.max_grad_norm, sumsq if self.max_grad_norm > 0 else None, self.flat.wd_mask,
            )
            if pout is not None and pout.dtype != torch.bfloat16 and pout.data_ptr() != p.data_ptr():
                pout.copy_(p)
            return
        self._step_ref(p, m, v, g, pout, inv_world, sumsq)

    @torch.no_grad()
    def _step_ref(self, p, m, v, g, pout, inv_world, sumsq):
        gf = g.float() * inv_world
        if self.max_grad_norm > 0:
            ss = sumsq if sumsq is not None else (g.float() ** 2).sum()
            norm = torch.sqrt(ss) * inv_world
            gf = gf * torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
        t = self.step_count
        m.mul_(self.beta1).add_(gf, alpha=1 - self.beta1)
        v.mul_(self.beta2).addcmul_(gf, gf, value=1 - self.beta2)
        bc1 = 1 - self.beta1**t
        bc2 = 1 - self.beta2**t
        mask = self.flat.wd_mask.repeat_interleave(8).to(p.dtype)
        p.mul_(1 - self.lr * self.wd * mask)
        denom = v.sqrt() / math.sqrt(bc2) + self.eps
        p.addcdiv_(m, denom, value=-self.lr / bc1)
        if pout is not None and pout.data_ptr() != p.data_ptr():
            pout.copy_(p.to(pout.dtype))
