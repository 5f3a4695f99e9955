"""Hand-written MFMA GEMMs (``csrc/kernels/gemm.hip``) for the training hot path.

Shapes the kernels take: M % 256 == 0, N % 320 == 0 (or % 256), K % 64 == 0 —
every GPT-2-XL projection at micro-batch x seq = 32768 tokens. Anything else
(small test models, odd vocab widths) goes to torch / hipBLASLt.

* ``linear_nt(x, w, b)``           y = x W^T + b  (bias fused in the epilogue)
* ``linear_gelu(x, w, b)``         z = x W^T + b, u = gelu(z)   (one kernel, both stored)
* ``dgrad(dy, wt)``                dx = dy W  using W^T (K-major B operand: wt = W^T)
* ``dgrad_dgelu(dy, wt, z, dbias)`` dz = (dy W) * gelu'(z); dbias += colsum(dz)
* ``transpose(w)``                 W^T (64x64 LDS tiles)

Tile choice: 256 x 320 (divides 1600/4800/6400) with the ping-pong pipeline
(``algo=2``: BK=32, 4-deep LDS ring, LDS-DMA two K-steps ahead, counted vmcnt, staggered wave rows), else 256 x 256.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from ._lib import kernels

ALGO = int(os.environ.get("CAAMD_GEMM_ALGO", "2"))
ENABLED = os.environ.get("CAAMD_MFMA_GEMM", "1") == "1"

EPI_BF16, EPI_BF16_ACC, EPI_F32, EPI_BIAS_GELU, EPI_DGELU = range(5)


def tile_for(M: int, N: int, K: int) -> Optional[Tuple[int, int]]:
    if not ENABLED or K % 64 or M % 256:
        return None
    if N % 320 == 0:
        return 256, 320
    if N % 256 == 0:
        return 256, 256
    return None


def _ok(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()) for t in ts)


def supported(x2: torch.Tensor, w: torch.Tensor) -> bool:
    """x2 [M,K] against an nn.Linear weight w [N,K] (forward and dgrad shapes)."""
    if not _ok(x2, w) or x2.dim() != 2 or w.dim() != 2:
        return False
    M, K = x2.shape
    N = w.shape[0]
    return tile_for(M, N, K) is not None and tile_for(M, K, N) is not None


def _run(a, b, c, epi, bias=None, z=None, zout=None, dbias=None):
    M, N = c.shape
    K = a.shape[1]
    bm, bn = tile_for(M, N, K)
    kernels().gemm_bf16(a, b, c, 0, epi, bm, bn, bias, z, zout, dbias, 1, None, False, ALGO)
    return c


def linear_nt(x2: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    out = torch.empty(x2.shape[0], w.shape[0], device=x2.device, dtype=torch.bfloat16)
    return _run(x2, w, out, EPI_BF16, bias=b)


def linear_gelu(x2: torch.Tensor, w: torch.Tensor, b: torch.Tensor):
    M, N = x2.shape[0], w.shape[0]
    u = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    z = torch.empty_like(u)
    _run(x2, w, u, EPI_BIAS_GELU, bias=b, zout=z)
    return u, z


def dgrad(dy2: torch.Tensor, wt: torch.Tensor) -> torch.Tensor:
    """dx = dy @ W given wt = W^T ([K_in, N_out], row-major)."""
    out = torch.empty(dy2.shape[0], wt.shape[0], device=dy2.device, dtype=torch.bfloat16)
    return _run(dy2, wt, out, EPI_BF16)


def dgrad_dgelu(dy2: torch.Tensor, wt: torch.Tensor, z: torch.Tensor, dbias_f32: torch.Tensor) -> torch.Tensor:
    out = torch.empty(dy2.shape[0], wt.shape[0], device=dy2.device, dtype=torch.bfloat16)
    return _run(dy2, wt, out, EPI_DGELU, z=z, dbias=dbias_f32)


def transpose(w: torch.Tensor) -> torch.Tensor:
    if w.is_cuda and w.dtype == torch.bfloat16 and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0:
        return kernels().transpose_bf16(w.contiguous())
    return w.t().contiguous()


def gemm(a: torch.Tensor, b: torch.Tensor, layout: int = 0, *, algo: Optional[int] = None,
         tile: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """General entry (tests / tools): layout 0 a[M,K] b[N,K]; 1 a[M,K] b[K,N]; 2 a[K,M] b[K,N]."""
    M = a.shape[1] if layout == 2 else a.shape[0]
    N = b.shape[0] if layout == 0 else b.shape[1]
    K = a.shape[0] if layout == 2 else a.shape[1]
    bm, bn = tile or tile_for(M, N, K) or (0, 0)
    if not bm:
        raise ValueError(f"no MFMA tile for M={M} N={N} K={K}")
    c = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    kernels().gemm_bf16(a, b, c, layout, EPI_BF16, bm, bn, None, None, None, None, 1, None, False,
                        ALGO if algo is None else algo)
    return c
