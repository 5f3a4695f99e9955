"""LLM-serving ops (``csrc/kernels/llm.hip`` + GQA flash forward) with plain
PyTorch fp32 references used on CPU and by the GPU numerics tests.

KV cache layout: ``[num_blocks, KVH, block_size, D]`` bf16 (one page of one
head is contiguous). Fused projection layout: ``qkv [N, (H + 2*KVH) * D]``.
"""
from __future__ import annotations

import math
import os as _os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ._lib import kernels, use_gpu_kernel


# ------------------------------------------------------------------ RMSNorm
def rms_norm_ref(x, w, eps, residual=None):
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        xf = s.float()
    else:
        s = None
        xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype), s


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5,
             residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns ``(norm(x [+ residual]) * w, x + residual or None)``."""
    if use_gpu_kernel(x, w, residual) and x.dtype == torch.bfloat16 and x.is_contiguous():
        y, s = kernels().rmsnorm(x, w, eps, residual)
        return y, (s if residual is not None else None)
    return rms_norm_ref(x, w, eps, residual)


# ------------------------------------------------------------------ SwiGLU
# ---------------------------------------------------------------- decode GEMM
_SKINNY_WS = {}


def skinny_workspace(device, floats: int = 8 << 20, slabs: int = 4096):
    """Per-device split-K workspace (fp32 partial tiles) and arrival counters of the
    decode GEMM. Allocated once (before any HIP-graph capture) and reused: every
    launch leaves the counters zeroed."""
    dev = torch.device(device)
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    ws = _SKINNY_WS.get(key)
    if ws is None:
        ws = (torch.empty(floats, device=dev, dtype=torch.float32), torch.zeros(slabs, device=dev, dtype=torch.int32))
        _SKINNY_WS[key] = ws
    return ws


def skinny_splits(N: int, K: int) -> int:
    """Split-K factor of the decode GEMM. Measured on MI355X at M = 128
    (tools/bench_decode_gemm.py, CAAMD_SKINNY_SPLITS sweep): 2 for N <= 8192 at
    K = 4096, else 4 where K allows (the last-arriver reduction of 8 splits costs
    more than it hides), 1 for the vocabulary projection."""
    forced = int(_os.environ.get("CAAMD_SKINNY_SPLITS", "0"))
    if forced and K % (128 * forced) == 0:
        return forced
    if N >= 65536:
        return 1
    s = 2 if (N <= 8192 and K <= 4096) else 4
    while s > 1 and K % (128 * s):
        s //= 2
    return s


def skinny_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2
            and 1 <= x.shape[0] <= 128 and x.stride(1) == 1 and w.is_contiguous() and w.shape[0] % 64 == 0
            and x.shape[1] == w.shape[1] and x.shape[1] % 128 == 0)


def skinny_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x @ w.T`` on the weight-streaming MFMA kernel (``skinny_gemm.hip``); the
    shapes must satisfy ``skinny_ok`` (raises otherwise)."""
    if not skinny_ok(x, w):
        raise ValueError(f"skinny_gemm: unsupported shapes {tuple(x.shape)} x {tuple(w.shape)}")
    M, K = x.shape
    N = w.shape[0]
    s = skinny_splits(N, K)
    part, cnt = skinny_workspace(x.device)
    if s > 1 and part.numel() < s * N * 128:
        s = 1
    out = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    kernels().skinny_gemm(x, w, out, part, cnt, s)
    return out


def decode_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x @ w.T`` for decode-sized batches: the skinny MFMA kernel when enabled
    (``CAAMD_SKINNY_GEMM=1``) and the shapes fit, else torch / hipBLASLt."""
    if _SKINNY_ON and use_gpu_kernel(x, w) and skinny_ok(x, w):
        return skinny_linear(x, w)
    return F.linear(x, w)


# opt-in: at batch 128 the kernel measured level with hipBLASLt's tuned selections
# per GEMM (PERF.md, "Decode GEMM"), so serving keeps hipBLASLt unless this is set
_SKINNY_ON = _os.environ.get("CAAMD_SKINNY_GEMM", "0") == "1"


def silu_mul_ref(gu):
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    if use_gpu_kernel(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous() and gu.shape[-1] % 16 == 0:
        return kernels().silu_mul(gu)
    return silu_mul_ref(gu)


# ------------------------------------------------------------------ RoPE tables
def rope_cos_sin(head_dim: int, max_pos: int, theta: float = 10000.0, scaling: Optional[dict] = None,
                 device=None) -> torch.Tensor:
    """``[max_pos, D/2, 2]`` fp32 (cos, sin), with Llama-3 frequency scaling."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        orig = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = orig / lo, orig / hi
        wl = 2 * math.pi / inv
        smooth = (orig / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().to(device)


def rope_cache_ref(qkv, cos_sin, positions, slots, k_cache, v_cache, H, KVH):
    N = positions.numel()
    D = qkv.numel() // (N * (H + 2 * KVH))
    x = qkv.view(N, H + 2 * KVH, D)
    half = D // 2
    cs = cos_sin[positions.long()]  # [N, D/2, 2]
    c, s = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    qk = x[:, : H + KVH].float()
    a, b = qk[..., :half], qk[..., half:]
    rot = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    x[:, : H + KVH] = rot.to(qkv.dtype)
    if k_cache is not None:
        BS = k_cache.shape[2]
        sl = slots.long()
        ok = sl >= 0
        blk, off = sl[ok] // BS, sl[ok] % BS
        k = x[ok, H: H + KVH]
        v = x[ok, H + KVH:]
        k_cache[blk, :, off] = k
        v_cache[blk, :, off] = v
    return qkv


def rope_cache_(qkv, cos_sin, positions, slots=None, k_cache=None, v_cache=None, H=1, KVH=1):
    """Rotate q/k of ``qkv`` in place and append k/v to the paged cache."""
    if use_gpu_kernel(qkv) and qkv.dtype == torch.bfloat16:
        kernels().rope_cache_(qkv, cos_sin, positions, slots, k_cache, v_cache, H, KVH)
        return qkv
    return rope_cache_ref(qkv, cos_sin, positions, slots, k_cache, v_cache, H, KVH)


# ------------------------------------------------------------------ attention
def paged_decode_ref(q, k_cache, v_cache, block_tables, ctx_lens, H, scale):
    B = q.shape[0]
    KVH, BS, D = k_cache.shape[1], k_cache.shape[2], k_cache.shape[3]
    G = H // KVH
    out = torch.empty(B, H * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        n = int(ctx_lens[b])
        nb = (n + BS - 1) // BS
        blocks = block_tables[b, :nb].long()
        k = k_cache[blocks].permute(1, 0, 2, 3).reshape(KVH, nb * BS, D)[:, :n].float()
        v = v_cache[blocks].permute(1, 0, 2, 3).reshape(KVH, nb * BS, D)[:, :n].float()
        qq = q[b, : H * D].view(KVH, G, D).float()
        s = torch.einsum("kgd,ktd->kgt", qq, k) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("kgt,ktd->kgd", p, v).reshape(H * D).to(q.dtype)
    return out


def paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, max_ctx: int, H: int,
                           scale: Optional[float] = None):
    """``q [B, >=H*D]`` (row stride free) -> ``o [B, H*D]``."""
    D = k_cache.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if use_gpu_kernel(q, k_cache) and q.dtype == torch.bfloat16:
        return kernels().paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, int(max_ctx), H, scale)
    return paged_decode_ref(q, k_cache, v_cache, block_tables, ctx_lens, H, scale)


def prefill_attention_ref(q, k, v, H, KVH, causal=True):
    B, T, _ = q.shape
    D = q.shape[-1] // H
    qq = q.reshape(B, T, H, D).transpose(1, 2).float()
    kk = k.reshape(B, T, KVH, D).transpose(1, 2).float().repeat_interleave(H // KVH, dim=1)
    vv = v.reshape(B, T, KVH, D).transpose(1, 2).float().repeat_interleave(H // KVH, dim=1)
    o = F.scaled_dot_product_attention(qq, kk, vv, is_causal=causal)
    return o.transpose(1, 2).reshape(B, T, H * D).to(q.dtype)


def prefill_attention(q, k, v, H: int, KVH: int, causal: bool = True):
    """``q [B, T, H*D]``, ``k/v [B, T, KVH*D]`` (views of one fused projection
    are fine) -> ``o [B, T, H*D]`` on the MFMA flash kernel."""
    D = q.shape[-1] // H
    if use_gpu_kernel(q, k, v) and q.dtype == torch.bfloat16 and D in (64, 128):
        out, _ = kernels().flash_attn_gqa(q, k, v, H, KVH, causal)
        return out
    return prefill_attention_ref(q, k, v, H, KVH, causal)
