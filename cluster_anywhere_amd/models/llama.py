"""Llama-family decoder (Llama-3 architecture: RMSNorm, RoPE with llama3
frequency scaling, grouped-query attention, SwiGLU) laid out for serving on
MI355X: one fused ``w_qkv`` and one fused ``w_gate_up`` GEMM per layer, the
paged KV cache in ``[num_blocks, KVH, block_size, D]`` bf16, and every
non-GEMM op a gfx950 kernel (``ops/llm.py``).

This is the model of the Serve LLM path (BASELINE.json config
"Ray Serve Llama-3-8B bf16, one replica per MI355X, continuous batching");
the reference serves it through vLLM (python/ray/llm/_internal/serve/...),
here the engine is ``cluster_anywhere_amd/llm/engine.py``.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import llm as L


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    d_model: int = 4096
    n_layer: int = 32
    n_head: int = 32
    n_kv_head: int = 8
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = field(default_factory=lambda: {
        "rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 8192})
    norm_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False

    @property
    def head_dim(self):
        return self.d_model // self.n_head

    @classmethod
    def named(cls, name: str) -> "LlamaConfig":
        if name in ("llama3-8b", "llama-3-8b", "Llama-3-8B"):
            return cls()
        if name in ("llama3-70b",):
            return cls(d_model=8192, n_layer=80, n_head=64, n_kv_head=8, ffn_dim=28672)
        if name in ("llama3.2-1b",):
            return cls(d_model=2048, n_layer=16, n_head=32, n_kv_head=8, ffn_dim=8192, tie_embeddings=True,
                       rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                                     "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
        if name == "llama-tiny":
            return cls(vocab_size=512, d_model=256, n_layer=2, n_head=4, n_kv_head=2, ffn_dim=512,
                       rope_theta=10000.0, rope_scaling=None, max_position=1024)
        if name == "llama-small":
            return cls(vocab_size=4096, d_model=1024, n_layer=4, n_head=8, n_kv_head=2, ffn_dim=2816,
                       max_position=4096)
        raise ValueError(f"unknown Llama config {name!r}")

    def num_params(self):
        d, f, hd = self.d_model, self.ffn_dim, self.head_dim
        per = d * (self.n_head + 2 * self.n_kv_head) * hd + self.n_head * hd * d + 3 * d * f + 2 * d
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return self.n_layer * per + emb + d


class LlamaLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        d, hd = cfg.d_model, cfg.head_dim
        self.cfg = cfg
        self.attn_norm = nn.Parameter(torch.ones(d))
        self.w_qkv = nn.Parameter(torch.empty((cfg.n_head + 2 * cfg.n_kv_head) * hd, d))
        self.w_o = nn.Parameter(torch.empty(d, cfg.n_head * hd))
        self.mlp_norm = nn.Parameter(torch.ones(d))
        self.w_gate_up = nn.Parameter(torch.empty(2 * cfg.ffn_dim, d))
        self.w_down = nn.Parameter(torch.empty(d, cfg.ffn_dim))


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed = nn.Parameter(torch.empty(cfg.vocab_size, cfg.d_model))
        self.layers = nn.ModuleList([LlamaLayer(cfg) for _ in range(cfg.n_layer)])
        self.final_norm = nn.Parameter(torch.ones(cfg.d_model))
        self.lm_head = None if cfg.tie_embeddings else nn.Parameter(torch.empty(cfg.vocab_size, cfg.d_model))
        self._cos_sin = None
        self._dec = None  # decode-GEMM weight copies (prepare_decode)
        self._shared = False  # originals released: prefill / decode / forward all read the packed copies

    @torch.no_grad()
    def init_weights(self, std: float = 0.02, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        for name, p in self.named_parameters():
            if p.dim() >= 2:
                if p.is_cuda:
                    p.normal_(0.0, std)
                else:
                    p.copy_(torch.randn(p.shape, generator=g) * std)
            else:
                p.fill_(1.0)
        return self

    def cos_sin(self, device):
        if self._cos_sin is None or self._cos_sin.device != torch.device(device):
            self._cos_sin = L.rope_cos_sin(self.cfg.head_dim, self.cfg.max_position, self.cfg.rope_theta,
                                           self.cfg.rope_scaling, device)
        return self._cos_sin

    def _head(self, x):
        if self._shared and self._dec["head"] is not None:
            return self._dg(x, self._dec["head"])
        w = self.embed if self.lm_head is None else self.lm_head
        return F.linear(x, w)

    def _dg(self, x, w, epi: int = 0, residual=None):
        """Decode GEMM on a packed weight for any row count (<= 128 rows per launch)."""
        if x.shape[0] <= 128:
            return L.decode_gemm(x, w, epi, residual=residual, packed=True)
        return torch.cat([L.decode_gemm(x[i:i + 128], w, epi, packed=True,
                                        residual=None if residual is None else residual[i:i + 128])
                          for i in range(0, x.shape[0], 128)])

    def _weight(self, i: int, name: str) -> torch.Tensor:
        """Layer i's weight in nn.Linear layout (unpacked from the shared copy if the
        original was released)."""
        layer = self.layers[i]
        if not self._shared:
            return getattr(layer, name)
        if name == "w_qkv":
            return L.unpack_decode_weight(self._dec["attn"][i][0])
        if name == "w_o":
            return L.unpack_decode_weight(self._dec["attn"][i][1])
        if name == "w_gate_up":
            gu = L.unpack_decode_weight(self._dec["layers"][i][0])
            two_f, d = gu.shape
            blk = gu.reshape(two_f // 128, 2, 64, d)
            return torch.cat([blk[:, 0].reshape(two_f // 2, d), blk[:, 1].reshape(two_f // 2, d)])
        if name == "w_down":
            return L.unpack_decode_weight(self._dec["layers"][i][1])
        raise KeyError(name)

    @torch.no_grad()
    def prepare_decode(self) -> bool:
        """Decode-side copies of the weight-streaming GEMMs for ``decode_gemm.hip``
        (batch <= 128): ``w_gate_up`` with gate/up rows interleaved in 64-row blocks
        (SwiGLU fused into the GEMM epilogue, no [B, 2F] intermediate) and
        ``w_down`` / ``w_qkv`` / ``w_o`` / the vocabulary projection, all prepacked
        in the kernel's streaming order. With the split-K partials combined by a
        separate reduce launch the kernel also beats hipBLASLt at the qkv / o
        widths (``tools/bench_decode_gemm3.py --sweep``,
        ``profiles/decode_gemm_ext_reduce_r3.jsonl``). Costs one extra copy of
        those weights in HBM (about 14 GB for Llama-3-8B), taken before the KV
        cache is sized. Returns whether the decode path uses them."""
        import os

        self._restore_originals()
        if os.environ.get("CAAMD_DECODE_GEMM", "1") == "0" or not self.embed.is_cuda \
                or self.embed.dtype != torch.bfloat16 or not L.decode_gemm_available():
            self._dec = None
            return False
        cfg = self.cfg
        if cfg.ffn_dim % 64 or cfg.d_model % 128 or cfg.d_model % 64 or cfg.ffn_dim % 64:
            self._dec = None
            return False
        head = self.embed if self.lm_head is None else self.lm_head
        attn_ok = os.environ.get("CAAMD_DECODE_ATTN_GEMM", "1") == "1" and all(
            l.w_qkv.shape[0] % 128 == 0 and l.w_o.shape[0] % 128 == 0 for l in self.layers)
        # CAAMD_DECODE_NORM_FUSED=1: RMSNorms folded into the GEMMs that consume them
        # (norm weights in the weight columns, row statistics taken by the producer
        # waves while x streams through, residual adds in the o / down epilogues: no
        # rmsnorm launches in the layer). Measured level with the separate rmsnorm
        # launches (TPOT 6.89 vs 6.88 ms, profiles/llm_decode_norm_fold_r3.txt: the
        # statistics cost gate/up 5 us of its 50), so opt-in.
        norm = attn_ok and os.environ.get("CAAMD_DECODE_NORM_FUSED", "0") == "1"
        fold = (lambda w, g: L.fold_norm(w, g)) if norm else (lambda w, g: w)
        layers = [(L.pack_decode_weight(fold(L.interleave_gate_up(l.w_gate_up), l.mlp_norm)),
                   L.pack_decode_weight(l.w_down)) for l in self.layers]
        attn = None
        if attn_ok:
            attn = [(L.pack_decode_weight(fold(l.w_qkv, l.attn_norm)), L.pack_decode_weight(l.w_o))
                    for l in self.layers]
        self._dec = {"layers": layers, "attn": attn, "norm": norm,
                     "head": L.pack_decode_weight(fold(head, self.final_norm)) if head.shape[0] % 128 == 0 else None}
        shapes = [tuple(w.shape) for l in self.layers[:1] for w in (l.w_down, l.w_qkv, l.w_o)]
        L.decode_gemm_reserve(self.embed.device, shapes)
        # One weight copy: prefill runs gemm.hip straight from the packed layout
        # (ops/gemm.py prefill_linear), so the nn.Linear-layout originals are
        # released (about 14 GB for Llama-3-8B, +1 GB untied LM head) unless the
        # norms are folded into the packed copies or a projection does not tile.
        from ..ops import gemm as G

        d, f = cfg.d_model, cfg.ffn_dim
        hd = cfg.head_dim
        tiles = all(n % 256 == 0 for n in ((cfg.n_head + 2 * cfg.n_kv_head) * hd, cfg.n_head * hd, 2 * f, d)) \
            and d % 64 == 0 and f % 64 == 0 and (cfg.n_head * hd) % 64 == 0
        self._dec["prefill"] = bool(attn and not norm and tiles and G.ENABLED
                                    and os.environ.get("CAAMD_LLM_PACKED_PREFILL", "1") == "1")
        if self._dec["prefill"] and os.environ.get("CAAMD_LLM_SHARED_WEIGHTS", "1") == "1":
            empty = lambda p: p.data.new_empty((0,) + tuple(p.shape[1:]))  # noqa: E731
            for l in self.layers:
                for n in ("w_qkv", "w_o", "w_gate_up", "w_down"):
                    getattr(l, n).data = empty(getattr(l, n))
            if self.lm_head is not None and self._dec["head"] is not None:
                self.lm_head.data = empty(self.lm_head)
            self._shared = True
            torch.cuda.empty_cache()
        return True

    @torch.no_grad()
    def _restore_originals(self):
        """Undo the weight sharing of :meth:`prepare_decode` (re-preparation,
        checkpoint export): the nn.Linear-layout weights rebuilt from the packed copies."""
        if not self._shared:
            return
        for i, l in enumerate(self.layers):
            for n in ("w_qkv", "w_o", "w_gate_up", "w_down"):
                getattr(l, n).data = self._weight(i, n)
        if self.lm_head is not None and self.lm_head.numel() == 0:
            self.lm_head.data = L.unpack_decode_weight(self._dec["head"])
        self._shared = False
        self._dec = None

    # -------------------------------------------------------------- prefill
    @torch.no_grad()
    def prefill(self, tokens: torch.Tensor, positions: torch.Tensor, slots: Optional[torch.Tensor],
                k_caches, v_caches, last_idx: torch.Tensor) -> torch.Tensor:
        """``tokens/positions [B, T]`` (right-padded), ``slots [B*T]`` cache slots
        (-1 = padding), ``last_idx [B]`` index of each sequence's last prompt
        token -> logits ``[B, vocab]`` of those positions."""
        cfg = self.cfg
        B, T = tokens.shape
        H, KVH, hd = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        cs = self.cos_sin(tokens.device)
        if self._dec is not None and self._dec.get("prefill"):
            return self._prefill_packed(tokens, positions, slots, k_caches, v_caches, last_idx)
        x = F.embedding(tokens, self.embed)  # [B, T, d]
        res = None
        pos = positions.reshape(-1).to(torch.int32)
        for i, layer in enumerate(self.layers):
            h, res = L.rms_norm(x, layer.attn_norm, cfg.norm_eps, res)
            if res is None:
                res = x
            qkv = F.linear(h, layer.w_qkv)  # [B, T, (H+2KVH)*hd]
            L.rope_cache_(qkv, cs, pos, slots, k_caches[i] if k_caches is not None else None,
                          v_caches[i] if v_caches is not None else None, H, KVH)
            q = qkv[..., : H * hd]
            k = qkv[..., H * hd: (H + KVH) * hd]
            v = qkv[..., (H + KVH) * hd:]
            o = L.prefill_attention(q, k, v, H, KVH, causal=True)
            x = F.linear(o, layer.w_o)
            h, res = L.rms_norm(x, layer.mlp_norm, cfg.norm_eps, res)
            x = F.linear(L.silu_mul(F.linear(h, layer.w_gate_up)), layer.w_down)
        h, _ = L.rms_norm(x, self.final_norm, cfg.norm_eps, res)
        last = h[torch.arange(B, device=h.device), last_idx.long()]
        return self._head(last)

    def _prefill_packed(self, tokens, positions, slots, k_caches, v_caches, last_idx):
        """Prefill on gemm.hip from the packed weights: the residual stream ``res``
        ([M rounded up to 256, d]) is updated in place by the o / down GEMM epilogues
        (``res += o W_o^T``, ``res += swiglu W_down^T``), the gate/up GEMM stores
        silu(gate) * up directly. Rows past M are padding (zero inputs, never read)."""
        from ..ops import gemm as G

        cfg = self.cfg
        B, T = tokens.shape
        H, KVH, hd = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        M = B * T
        Mp = -(-M // 256) * 256
        cs = self.cos_sin(tokens.device)
        pos = positions.reshape(-1).to(torch.int32)
        res = torch.zeros(Mp, cfg.d_model, device=tokens.device, dtype=self.embed.dtype)
        res[:M] = F.embedding(tokens.reshape(-1), self.embed)
        o_pad = torch.zeros(Mp, H * hd, device=tokens.device, dtype=res.dtype) if Mp != M else None
        for i in range(len(self.layers)):
            layer = self.layers[i]
            wq, wo = self._dec["attn"][i]
            gu, dn = self._dec["layers"][i]
            h, _ = L.rms_norm(res, layer.attn_norm, cfg.norm_eps)
            qkv = G.prefill_linear(h, wq)[:M].view(B, T, -1)
            L.rope_cache_(qkv, cs, pos, slots, k_caches[i] if k_caches is not None else None,
                          v_caches[i] if v_caches is not None else None, H, KVH)
            o = L.prefill_attention(qkv[..., : H * hd], qkv[..., H * hd: (H + KVH) * hd],
                                    qkv[..., (H + KVH) * hd:], H, KVH, causal=True).reshape(M, H * hd)
            if o_pad is not None:
                o_pad[:M] = o
                o = o_pad
            G.prefill_linear(o, wo, out=res, accumulate=True)
            h, _ = L.rms_norm(res, layer.mlp_norm, cfg.norm_eps)
            G.prefill_linear(G.prefill_linear(h, gu, epi=G.EPI_SWIGLU), dn, out=res, accumulate=True)
        h, _ = L.rms_norm(res[:M], self.final_norm, cfg.norm_eps)
        last = h.view(B, T, -1)[torch.arange(B, device=h.device), last_idx.long()]
        return self._head(last)

    # --------------------------------------------------------------- decode
    @torch.no_grad()
    def decode(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, k_caches, v_caches,
               block_tables: torch.Tensor, ctx_lens: torch.Tensor, max_ctx: int) -> torch.Tensor:
        """One new token per sequence: ``tokens/positions/slots/ctx_lens [B]``
        (ctx_lens include the new token), ``block_tables [B, max_blocks]``."""
        cfg = self.cfg
        H, KVH, hd = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        cs = self.cos_sin(tokens.device)
        x = F.embedding(tokens, self.embed)  # [B, d]
        res = None
        pos = positions.to(torch.int32)
        dec = self._dec if (self._dec is not None and (tokens.shape[0] <= 128 or self._shared)) else None
        if dec is not None and dec["norm"]:
            return self._decode_folded(x, dec, cs, pos, slots, k_caches, v_caches, block_tables, ctx_lens, max_ctx)
        if dec is not None and dec["attn"] is not None and tokens.shape[0] <= 128:
            out = self._decode_reduce_norm(x, dec, cs, pos, slots, k_caches, v_caches, block_tables, ctx_lens,
                                           max_ctx)
            if out is not None:
                return out
        for i, layer in enumerate(self.layers):
            h, res = L.rms_norm(x, layer.attn_norm, cfg.norm_eps, res)
            if res is None:
                res = x
            # decode GEMMs stream the weights once: decode_gemm.hip (<= 128 rows)
            att = dec["attn"][i] if (dec is not None and dec["attn"] is not None) else None
            qkv = L.decode_gemm_qkv_rope(h, att[0], cs, pos, slots, k_caches[i], v_caches[i], H, KVH) \
                if att else None
            if qkv is None:
                qkv = self._dg(h, att[0]) if att else L.decode_linear(h, layer.w_qkv)
                L.rope_cache_(qkv, cs, pos, slots, k_caches[i], v_caches[i], H, KVH)
            o = L.paged_decode_attention(qkv, k_caches[i], v_caches[i], block_tables, ctx_lens, max_ctx, H)
            x = self._dg(o, att[1]) if att else L.decode_linear(o, layer.w_o)
            h, res = L.rms_norm(x, layer.mlp_norm, cfg.norm_eps, res)
            if dec is not None:  # SwiGLU in the gate/up GEMM epilogue, packed weight streams
                gu, dn = dec["layers"][i]
                x = self._dg(self._dg(h, gu, 2), dn)
            else:
                x = L.decode_linear(L.silu_mul(L.decode_linear(h, layer.w_gate_up)), layer.w_down)
        h, _ = L.rms_norm(x, self.final_norm, cfg.norm_eps, res)
        if dec is not None and dec["head"] is not None:
            return self._dg(h, dec["head"])
        w = self.embed if self.lm_head is None else self.lm_head
        return L.decode_linear(h, w)

    def _decode_reduce_norm(self, x, dec, cs, pos, slots, k_caches, v_caches, block_tables, ctx_lens, max_ctx):
        """Decode layers with the o / down projections' split-K combine, residual add
        and the following RMSNorm in one launch each (``L.decode_gemm_norm``): per
        layer qkv(+RoPE +cache append) -> paged attention -> o(+res, mlp_norm) ->
        gate/up (SwiGLU) -> down(+res, next attn_norm / final_norm). ``res`` (the
        residual stream) is updated in place. Returns None before any work when the
        fused path does not apply to these shapes (the caller runs the plain loop)."""
        cfg = self.cfg
        H, KVH, eps = cfg.n_head, cfg.n_kv_head, cfg.norm_eps
        n = len(self.layers)
        res = x
        h = None
        for i, layer in enumerate(self.layers):
            wq, wo = dec["attn"][i]
            gu, dn = dec["layers"][i]
            if i == 0:
                if not (L.decode_gemm_ok(x.new_empty(x.shape[0], wo.shape[1]), wo)
                        and L.decode_gemm_splits(wo.shape[0], wo.shape[1], L._cus(x.device)) > 1
                        and L.decode_gemm_splits(dn.shape[0], dn.shape[1], L._cus(x.device)) > 1
                        and wo.shape[0] <= 8192 and os.environ.get("CAAMD_DECODE_REDUCE_NORM", "1") != "0"):
                    return None
                h, _ = L.rms_norm(x, layer.attn_norm, eps)
            qkv = L.decode_gemm_qkv_rope(h, wq, cs, pos, slots, k_caches[i], v_caches[i], H, KVH)
            if qkv is None:
                qkv = self._dg(h, wq)
                L.rope_cache_(qkv, cs, pos, slots, k_caches[i], v_caches[i], H, KVH)
            o = L.paged_decode_attention(qkv, k_caches[i], v_caches[i], block_tables, ctx_lens, max_ctx, H)
            h = L.decode_gemm_norm(o, wo, res, layer.mlp_norm, eps)
            nxt = self.layers[i + 1].attn_norm if i + 1 < n else self.final_norm
            h = L.decode_gemm_norm(L.decode_gemm(h, gu, 2, packed=True), dn, res, nxt, eps)
        if dec["head"] is not None:
            return self._dg(h, dec["head"])
        w = self.embed if self.lm_head is None else self.lm_head
        return L.decode_linear(h, w)

    def _decode_folded(self, x, dec, cs, pos, slots, k_caches, v_caches, block_tables, ctx_lens, max_ctx):
        """Decode layers with every RMSNorm folded into the GEMM that consumes it:
        per layer qkv(+RoPE +cache append) -> paged attention -> o (+residual) ->
        gate/up (SwiGLU) -> down (+residual); ``u`` is the residual stream."""
        cfg = self.cfg
        H, KVH, eps = cfg.n_head, cfg.n_kv_head, cfg.norm_eps
        u = x
        for i in range(len(self.layers)):
            wq, wo = dec["attn"][i]
            gu, dn = dec["layers"][i]
            qkv = L.decode_gemm_qkv_rope(u, wq, cs, pos, slots, k_caches[i], v_caches[i], H, KVH, norm_eps=eps)
            if qkv is None:
                qkv = L.decode_gemm(u, wq, 0, packed=True, norm_eps=eps)
                L.rope_cache_(qkv, cs, pos, slots, k_caches[i], v_caches[i], H, KVH)
            o = L.paged_decode_attention(qkv, k_caches[i], v_caches[i], block_tables, ctx_lens, max_ctx, H)
            u = L.decode_gemm(o, wo, 1, residual=u, packed=True)
            u = L.decode_gemm(L.decode_gemm(u, gu, 2, packed=True, norm_eps=eps), dn, 1, residual=u, packed=True)
        if dec["head"] is not None:
            return L.decode_gemm(u, dec["head"], 0, packed=True, norm_eps=eps)
        h, _ = L.rms_norm(u, self.final_norm, eps)
        return L.decode_linear(h, self.embed if self.lm_head is None else self.lm_head)

    # ------------------------------------------------ reference full forward
    @torch.no_grad()
    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        """Dense causal forward over ``tokens [B, T]`` (no cache) -> logits."""
        B, T = tokens.shape
        pos = torch.arange(T, device=tokens.device).expand(B, T)
        cfg = self.cfg
        H, KVH, hd = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        cs = self.cos_sin(tokens.device)
        x = F.embedding(tokens, self.embed)
        res = None
        for i, layer in enumerate(self.layers):
            h, res = L.rms_norm(x, layer.attn_norm, cfg.norm_eps, res)
            if res is None:
                res = x
            qkv = F.linear(h, self._weight(i, "w_qkv"))
            L.rope_cache_(qkv, cs, pos.reshape(-1).to(torch.int32), None, None, None, H, KVH)
            o = L.prefill_attention(qkv[..., : H * hd], qkv[..., H * hd: (H + KVH) * hd],
                                    qkv[..., (H + KVH) * hd:], H, KVH, causal=True)
            x = F.linear(o, self._weight(i, "w_o"))
            h, res = L.rms_norm(x, layer.mlp_norm, cfg.norm_eps, res)
            x = F.linear(L.silu_mul(F.linear(h, self._weight(i, "w_gate_up"))), self._weight(i, "w_down"))
        h, _ = L.rms_norm(x, self.final_norm, cfg.norm_eps, res)
        if self._shared and self._dec["head"] is not None:
            return F.linear(h, L.unpack_decode_weight(self._dec["head"]))
        return self._head(h)
