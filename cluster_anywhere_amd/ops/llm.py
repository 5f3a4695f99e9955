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
# ---------------------------------------------------- decode GEMM v3 (decode_gemm.hip)
_DG_WS: dict = {}
# split-count overrides for A/B runs: CAAMD_DG_SPLITS="4096x4096:4,6144x4096:6" (N x K : splits)
_DG_SPLITS = {tuple(int(v) for v in p.split(":")[0].split("x")): int(p.split(":")[1])
              for p in _os.environ.get("CAAMD_DG_SPLITS", "").split(",") if ":" in p}


def decode_gemm_splits(N: int, K: int, cus: int = 256) -> int:
    """Split-K so the (N/128) x splits workgroups cover the CUs, >= 4 K-steps each.
    The splits are ceil(steps / s) 64-k steps long with a shorter last one, so s need
    not divide K: Llama-3-8B qkv (48 slabs, K 4096) runs 5 splits on 240 CUs instead
    of 4 on 192 (measured level, 19.4 vs 19.3-19.5 us: that GEMM is bound by each
    CU's LDS-DMA intake, not by the idle CUs; profiles/decode_ragged_split_r4.txt)."""
    forced = _DG_SPLITS.get((N, K))
    if forced:
        return forced
    slabs = N // 128
    steps = K // 64
    s = max(1, min(cus // max(1, slabs), K // 256))
    while s > 1 and (s - 1) * (-(-steps // s)) >= steps:
        s -= 1
    return s


def _dg_ws(dev, floats: int, tickets: int):
    """(partials, tickets, row statistics) of the decode GEMM; the row-statistics
    buffer holds [slabs][splits][128] sums of squares for the folded RMSNorm."""
    ws = _DG_WS.get(dev.index)
    if ws is None or ws[0].numel() < floats or ws[1].numel() < tickets:
        ws = (torch.empty(max(floats, 1), device=dev, dtype=torch.float32),
              torch.zeros(max(tickets, 1024), device=dev, dtype=torch.int32),
              torch.empty(max(floats // 128, 1024 * 128), device=dev, dtype=torch.float32))
        _DG_WS[dev.index] = ws
    return ws


def decode_gemm_available() -> bool:
    """The decode GEMM is compiled into the extension (raises on a GPU box when the
    extension itself is missing: no silent fallback there)."""
    return hasattr(kernels(), "decode_gemm")


def decode_gemm_reserve(dev, shapes) -> None:
    """Allocate the split-K workspace for every (N, K) decode shape up front, so no
    allocation happens inside a HIP-graph capture (graphs keep raw pointers)."""
    cus = _cus(dev)
    need = max([(n // 128) * decode_gemm_splits(n, k, cus) * 16384 for n, k in shapes] + [1])
    _dg_ws(dev, need, 1024)


def decode_gemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.dim() == 2 and 1 <= x.shape[0] <= 128 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.is_contiguous() and x.stride(-1) == 1 and w.shape[0] % 128 == 0 and x.shape[1] % 64 == 0
            and w.shape[1] == x.shape[1])


def decode_gemm(x: torch.Tensor, w: torch.Tensor, epi: int = 0, residual: Optional[torch.Tensor] = None,
                splits: Optional[int] = None, packed: bool = False, norm_eps: Optional[float] = None) -> torch.Tensor:
    """``x @ w.T`` (epi 0), ``+ residual`` (epi 1) or SwiGLU over a 64-row-interleaved
    gate/up weight (epi 2, see :func:`interleave_gate_up`) on the decode GEMM v3.
    ``packed``: ``w`` is in :func:`pack_decode_weight` order. ``norm_eps``: RMSNorm
    folded in — ``rmsnorm(x) @ w.T`` with the norm weight already multiplied into
    ``w``'s columns (:func:`fold_norm`); the row statistics are gathered while x
    streams through the GEMM, so no separate normalisation pass runs."""
    M, K = x.shape
    N = w.shape[0]
    s = splits or decode_gemm_splits(N, K, _cus(x.device))
    y = torch.empty(M, N // 2 if epi == 2 else N, device=x.device, dtype=torch.bfloat16)
    part, tick, ssp = _dg_ws(x.device, (N // 128) * s * 16384 if s > 1 else 1, N // 128)
    kernels().decode_gemm(x, w, y, residual, part, tick, epi, s, packed,
                          ssp if norm_eps is not None else None, float(norm_eps or 0.0))
    return y


def decode_gemm_norm(x: torch.Tensor, w: torch.Tensor, res: torch.Tensor, norm_w: torch.Tensor,
                     eps: float) -> Optional[torch.Tensor]:
    """``res += x @ w.T`` (in place) and ``h = rmsnorm(res) * norm_w`` on the decode
    GEMM (``w`` prepacked) with the split-K combine, the residual add and the norm in
    ONE launch after the GEMM (``dg_reduce_norm_kernel``) instead of the reduce +
    rmsnorm pair. The same numbers as ``rms_norm(decode_gemm(x, w), norm_w, eps, res)``
    (the GEMM's sum is rounded to bf16 before the add). Returns ``h``, or None where
    it does not apply (one split, N > 8192, ``CAAMD_DECODE_REDUCE_NORM=0``)."""
    M, K = x.shape
    N = w.shape[0]
    if (not decode_gemm_ok(x, w) or N > 8192 or res.shape != (M, N) or not res.is_contiguous()
            or res.dtype != torch.bfloat16 or norm_w.dtype != torch.bfloat16
            or _os.environ.get("CAAMD_DECODE_REDUCE_NORM", "1") == "0"):
        return None
    s = decode_gemm_splits(N, K, _cus(x.device))
    if s < 2:
        return None
    part, _, _ = _dg_ws(x.device, (N // 128) * s * 16384, N // 128)
    return kernels().decode_gemm_norm(x, w, part, s, res, norm_w.contiguous(), float(eps))


def fold_norm(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """``w [N, K]`` with the RMSNorm weight ``g [K]`` multiplied into its columns
    (``rmsnorm(x) @ w.T == rsqrt-scaled x @ fold_norm(w, g).T``), in fp32 then
    rounded once."""
    return (w.float() * g.float()[None, :]).to(w.dtype)


def decode_gemm_qkv_rope(x: torch.Tensor, w: torch.Tensor, cos_sin: torch.Tensor, positions: torch.Tensor,
                         slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, H: int,
                         KVH: int, norm_eps: Optional[float] = None) -> Optional[torch.Tensor]:
    """qkv projection on the decode GEMM (``w`` prepacked) with RoPE and the paged
    cache append fused into its split-K reduce launch: the same result as
    ``decode_gemm`` + :func:`rope_cache_` with one launch and one pass over qkv
    fewer. Returns None where it does not apply (head_dim != 128, one split, or
    int64 positions / slots): the caller then runs the two steps."""
    M, K = x.shape
    N = w.shape[0]
    if (k_cache is None or k_cache.shape[-1] != 128 or N != (H + 2 * KVH) * 128 or not decode_gemm_ok(x, w)
            or positions.dtype != torch.int32 or slots.dtype != torch.int32
            or _os.environ.get("CAAMD_DECODE_ROPE_FUSED", "1") == "0"):
        return None
    s = decode_gemm_splits(N, K, _cus(x.device))
    if s < 2:
        return None
    y = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
    part, _, ssp = _dg_ws(x.device, (N // 128) * s * 16384, N // 128)
    kernels().decode_gemm_qkv_rope(x, w, y, part, s, cos_sin, positions.contiguous(), slots.contiguous(),
                                   k_cache, v_cache, H, KVH, ssp if norm_eps is not None else None,
                                   float(norm_eps or 0.0))
    return y


_CUS: dict = {}


def _cus(dev) -> int:
    n = _CUS.get(dev.index)
    if n is None:
        n = _CUS[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n


def _swz_cols(device) -> torch.Tensor:
    """[128 rows, 8 positions] -> source 16-byte chunk (decode_gemm.hip ``swz``)."""
    row = torch.arange(128, device=device).view(128, 1)
    pos = torch.arange(8, device=device).view(1, 8)
    x = (row >> 1) & 7
    return pos ^ (x ^ ((x & 1) << 2))


def pack_decode_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> the decode kernel's streaming order (same shape and numel): for
    every 128-row slab and 64-wide k step, the 16 KiB swizzled LDS image
    contiguously (``dma_packed`` in decode_gemm.hip). Done once at load time."""
    N, K = w.shape
    assert N % 128 == 0 and K % 64 == 0
    v = w.reshape(N // 128, 128, K // 64, 8, 8).permute(0, 2, 1, 3, 4)  # [slab, kstep, row, chunk, 8]
    idx = _swz_cols(w.device).view(1, 1, 128, 8, 1).expand(N // 128, K // 64, 128, 8, 8)
    return torch.gather(v, 3, idx).contiguous().view(N, K)


def unpack_decode_weight(wp: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`pack_decode_weight` (tests, checkpoint export)."""
    N, K = wp.shape
    v = wp.reshape(N // 128, K // 64, 128, 8, 8)
    idx = _swz_cols(wp.device).view(1, 1, 128, 8, 1).expand_as(v)
    out = torch.empty_like(v)
    out.scatter_(3, idx, v)
    return out.permute(0, 2, 1, 3, 4).contiguous().view(N, K)


def interleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    """[gate; up] ([2F, d]) -> 64-row blocks [gate_b; up_b] for the SwiGLU epilogue."""
    two_f, d = w.shape
    f = two_f // 2
    assert f % 64 == 0
    g, u = w[:f].reshape(f // 64, 64, d), w[f:].reshape(f // 64, 64, d)
    return torch.stack([g, u], dim=1).reshape(two_f, d).contiguous()


def decode_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x @ w.T`` for decode-sized batches on a weight without a packed decode copy
    (torch / hipBLASLt); the packed projections run on ``decode_gemm`` (v3)."""
    return F.linear(x, w)


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
        return kernels().paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, int(max_ctx), H, scale, -1)
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
