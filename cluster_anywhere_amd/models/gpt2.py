"""GPT-2 family (124M … 1.5B "XL") built on the gfx950 kernels.

Pre-LN transformer. The residual stream is carried as (h, pending_delta) so every
``h = h + delta; a = LN(h)`` pair is ONE fused ``add_layer_norm`` kernel. MLP
bias+GELU is one fused kernel (dbias fused in backward); the LM head is tied to
the token embedding, the vocab is padded to a multiple of 256 for the GEMM tiles
and the cross-entropy masks the padding. The projection GEMMs (forward and
input-gradient, and the weight gradients where they win) are the hand-written
MFMA kernels of ``ops/gemm.py`` with bias / bias+GELU / GELU' fused into their
epilogues; the LM head + loss is :func:`ops.loss.linear_cross_entropy` (chunked,
logits never materialised, all three GEMMs on gemm.hip); attention goes through
:func:`ops.attention`.

This is the model behind the headline benchmark (Ray Train
TorchTrainer DDP GPT-2-XL tokens/s).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import add_layer_norm, attention, layer_norm
from ..ops.attention import flash_path
from ..ops.norm import ln_bias_fusion_ok
from ..ops.linear import linear, mlp
from ..ops.loss import linear_cross_entropy


# qkv bias gradient from the flash-attention backward's registers: opt-in
# (CAAMD_FUSED_QKV_BGRAD=1) -- it measured 88.4-88.5k vs 91.0k tok/s in alternating
# same-box runs (the backward kernels' epilogue reduction costs more than the 52 us
# column-sum pass it replaces; profiles/step_ab_r3_bias_fusion.txt)
_FUSED_QKV_BGRAD = os.environ.get("CAAMD_FUSED_QKV_BGRAD", "0") == "1"
# fc2 weight stored transposed ([4d, d] in memory, the shape stays [d, 4d]): its weight
# gradient dW^T = u^T dy is then the fc-shaped 6400 x 1600 problem whose 125 tiles x 2
# splits fill the CUs on gemm.hip, instead of 1600 x 6400 (140 ragged tiles) on
# hipBLASLt; the dgrad reads the stored layout directly and the forward transposes it
# once (CAAMD_FC2_T=0: plain layout)
_FC2_T = os.environ.get("CAAMD_FC2_T", "1") == "1"
# proj / fc2 bias gradients from the LayerNorm backward (CAAMD_NO_FUSED_LN_BGRAD=1: own passes)
_FUSED_LN_BGRAD = os.environ.get("CAAMD_NO_FUSED_LN_BGRAD", "0") != "1"


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_layer: int = 48
    n_head: int = 25
    n_embd: int = 1600
    ln_eps: float = 1e-5
    pad_vocab_to: int = 256

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_to
        return (self.vocab_size + m - 1) // m * m

    @staticmethod
    def named(name: str) -> "GPT2Config":
        presets = {
            "gpt2": dict(n_layer=12, n_head=12, n_embd=768),
            "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),
            "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),
            "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),
            "gpt2-tiny": dict(n_layer=2, n_head=4, n_embd=128, n_positions=128, vocab_size=512),
        }
        return GPT2Config(**presets[name])


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        d = cfg.n_embd
        self.n_head = cfg.n_head
        self.eps = cfg.ln_eps
        self.ln1_w = nn.Parameter(torch.ones(d))
        self.ln1_b = nn.Parameter(torch.zeros(d))
        self.attn_w = nn.Parameter(torch.empty(3 * d, d))
        self.attn_b = nn.Parameter(torch.zeros(3 * d))
        self.proj_w = nn.Parameter(torch.empty(d, d))
        self.proj_b = nn.Parameter(torch.zeros(d))
        self.ln2_w = nn.Parameter(torch.ones(d))
        self.ln2_b = nn.Parameter(torch.zeros(d))
        self.fc_w = nn.Parameter(torch.empty(4 * d, d))
        self.fc_b = nn.Parameter(torch.zeros(4 * d))
        self.fc2_w = nn.Parameter(torch.empty(4 * d, d).t() if _FC2_T else torch.empty(d, 4 * d))
        self.fc2_b = nn.Parameter(torch.zeros(d))
        std = 0.02
        nn.init.normal_(self.attn_w, std=std)
        nn.init.normal_(self.fc_w, std=std)
        nn.init.normal_(self.proj_w, std=std / math.sqrt(2 * cfg.n_layer))
        nn.init.normal_(self.fc2_w, std=std / math.sqrt(2 * cfg.n_layer))

    def forward(self, h, delta, delta_bias=None):
        """-> (h, mlp output, fc2 bias whose gradient the NEXT LayerNorm backward takes or None)."""
        if delta is None:
            a = layer_norm(h, self.ln1_w, self.ln1_b, self.eps)
        else:
            h, a = add_layer_norm(h, delta, self.ln1_w, self.ln1_b, self.eps, res_bias=delta_bias)
        # on the flash path the attention backward also takes the qkv bias gradient
        # (column sums of dqkv from its registers); only with main-grad buffers,
        # where the linear below then skips its own pass over dqkv
        fused_b = (_FUSED_QKV_BGRAD and flash_path(a, a.shape[-1], self.n_head)
                   and getattr(self.attn_w, "main_grad", None) is not None and a.requires_grad)
        qkv = linear(a, self.attn_w, self.attn_b, bias_grad=not fused_b)
        y = attention(qkv, self.n_head, causal=True, qkv_bias=self.attn_b if fused_b else None)
        # proj / fc2 bias gradients = column sums of the residual-stream gradient,
        # taken by the following LayerNorm backward (no separate pass over it)
        fuse_ln = (_FUSED_LN_BGRAD and getattr(self.proj_b, "main_grad", None) is not None
                   and getattr(self.fc2_b, "main_grad", None) is not None and h.requires_grad
                   and ln_bias_fusion_ok(h))
        attn_out = linear(y, self.proj_w, self.proj_b, bias_grad=not fuse_ln)
        h, m = add_layer_norm(h, attn_out, self.ln2_w, self.ln2_b, self.eps,
                              res_bias=self.proj_b if fuse_ln else None)
        out = mlp(m, self.fc_w, self.fc_b, self.fc2_w, self.fc2_b, b2_grad=not fuse_ln)
        return h, out, (self.fc2_b if fuse_ln else None)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd))
        nn.init.normal_(self.wte, std=0.02)
        nn.init.normal_(self.wpe, std=0.01)
        with torch.no_grad():
            self.wte[cfg.vocab_size :].zero_()
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.lnf_w = nn.Parameter(torch.ones(cfg.n_embd))
        self.lnf_b = nn.Parameter(torch.zeros(cfg.n_embd))

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def hidden(self, idx):
        B, T = idx.shape
        h = F.embedding(idx, self.wte) + self.wpe[:T]
        delta = dbias = None
        for blk in self.blocks:
            h, delta, dbias = blk(h, delta, dbias)
        _, hf = add_layer_norm(h, delta, self.lnf_w, self.lnf_b, self.cfg.ln_eps, res_bias=dbias)
        return hf

    def forward(self, idx, targets=None):
        hf = self.hidden(idx)
        B, T, D = hf.shape
        if targets is not None:
            return linear_cross_entropy(hf.reshape(B * T, D), self.wte, targets, self.cfg.vocab_size)
        logits = F.linear(hf.reshape(B * T, D), self.wte)  # [B*T, Vpad]
        return logits.view(B, T, -1)[..., : self.cfg.vocab_size]

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token (fwd+bwd = 3x fwd), PaLM-style accounting incl. attention."""
        c = self.cfg
        n = sum(p.numel() for n_, p in self.named_parameters() if n_ != "wpe")
        n -= (c.padded_vocab - c.vocab_size) * c.n_embd  # padded vocab rows are not model FLOPs
        attn = 12 * c.n_layer * c.n_embd * seq_len / 2  # causal: half the score matrix
        return 6 * n + attn
