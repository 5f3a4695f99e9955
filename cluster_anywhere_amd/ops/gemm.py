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
NT GEMMs with N or K >= 1536 (fc / fc2 / qkv / proj forward and dgrad) take the
full-line kernel instead (``algo=4009``: BK=64, one 128-byte line per row and K-tile,
two LDS buffers, DMA of K-tile t+1 issued in the first of two MFMA phases of t): 2-4 %
faster on the large shapes in round 4 (``profiles/gemm_k64_r4.jsonl``); since round 6
also on the 1600 x 1600 projection (149-152 vs 154-168 us,
``profiles/gemm_algo_ab_r6.jsonl``).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ._lib import kernels

ALGO = int(os.environ.get("CAAMD_GEMM_ALGO", "2"))
ENABLED = os.environ.get("CAAMD_MFMA_GEMM", "1") == "1"
# split-K tail of the ping-pong kernel: tiles past the last full round of CUs are
# split over K-slices so that round is not half empty (N = 1600: 640 tiles = 2.5 rounds)
TAIL = os.environ.get("CAAMD_GEMM_TAIL", "1") == "1"
# full-line BK=64 kernel (algo 4009) on the large NT shapes (CAAMD_GEMM_K64=0: off)
K64 = os.environ.get("CAAMD_GEMM_K64", "1") == "1"
K64_ALGO = 4009
# smallest max(N, K) routed to the full-line kernel: the 1600 x 1600 attention projection
# (fwd and dgrad, 640 tiles) runs 149-152 us there vs 154-168 on the ping-pong kernel
# (tools/gemm_algo_ab.py, profiles/gemm_algo_ab_r6.jsonl); the rule was 4096 until round 6
K64_MIN = int(os.environ.get("CAAMD_GEMM_K64_MIN", "1536"))


# 256 x 256 tiles on the full-line kernel too (the LM-head logits GEMM: vocab 50432 is
# not a multiple of 320); CAAMD_GEMM_K64_256=0: those stay on the ping-pong kernel
K64_256 = os.environ.get("CAAMD_GEMM_K64_256", "1") == "1"


def k64_ok(layout: int, epi: int, bm: int, bn: int, N: int, K: int) -> bool:
    tiles = (bm, bn) == (256, 320) or (K64_256 and (bm, bn) == (256, 256))
    return (K64 and layout == 0 and tiles and epi != EPI_F32 and max(N, K) >= K64_MIN and K % 64 == 0)
MAX_TAIL_SPLIT = int(os.environ.get("CAAMD_GEMM_TAIL_SPLIT", "4"))

EPI_BF16, EPI_BF16_ACC, EPI_F32, EPI_BIAS_GELU, EPI_DGELU, EPI_SWIGLU = range(6)


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


_PLANS: dict = {}
_WS: dict = {}


def _workspace(dev: torch.device, floats: int, tickets: int):
    """Per-device split-K slab workspace + zeroed ticket counters (the kernel's last
    arriver resets its ticket, so the counters stay zero between launches)."""
    ws, cnt = _WS.get(dev.index, (None, None))
    if ws is None or ws.numel() < floats or cnt.numel() < tickets:
        ws = torch.empty(max(floats, 1 << 20), device=dev, dtype=torch.float32)
        cnt = torch.zeros(max(tickets, 4096), device=dev, dtype=torch.int32)
        _WS[dev.index] = (ws, cnt)
    return ws, cnt


# De-phased full-line launches (CAAMD_GEMM_DEPHASE=1, experimental): on grids that are a
# whole number of CU rounds, a quarter round of tiles is split in two K-halves and those
# half-tiles are dispatched first, so half the CUs run half a tile out of phase with the
# other half and the two groups' output-store bursts do not coincide.
DEPHASE = os.environ.get("CAAMD_GEMM_DEPHASE", "0") == "1"
_DEPHASE_SET: dict = {}


def tail_plan(M: int, N: int, K: int, bm: int, bn: int, dev: torch.device, algo: int = None):
    """(full tiles, tail split) of a ping-pong launch; split 1 = no tail split."""
    algo = ALGO if algo is None else algo
    if DEPHASE and algo % 10 == 9:
        slots = torch.cuda.get_device_properties(dev).multi_processor_count
        T = (M // bm) * (N // bn)
        if _DEPHASE_SET.get(dev.index) is None:
            kernels().gemm_set_tail_first(1)
            _DEPHASE_SET[dev.index] = True
        if T % slots == 0 and T >= 4 * slots and (K // 64) // 2 >= 8 and slots % 32 == 0:
            return (T - slots // 4, 2)
    if not TAIL or not (1 <= algo % 10 <= 3 or algo % 10 == 9) or K < 4096:
        # K = 1600: the split slices and slab round trip cost more than the half-empty
        # last round (which the chip runs at a higher clock); profiles/gemm_tail_split.jsonl
        return (0, 1)
    key = ("pp", M, N, K, bm, bn, dev.index, MAX_TAIL_SPLIT, algo % 10 == 9)
    p = _PLANS.get(key)
    if p is None:
        slots = torch.cuda.get_device_properties(dev).multi_processor_count
        ks = 64 if algo % 10 == 9 else 32
        p = _PLANS[key] = tuple(kernels().gemm_tail_plan((M // bm) * (N // bn), K, ks, slots, MAX_TAIL_SPLIT))
    return p


def run_pp(a, b, c, layout, epi, bm, bn, bias=None, z=None, zout=None, dbias=None, algo=None):
    """Ping-pong (algo 2) or full-line (algo 4009) kernel of gemm.hip with the split-K tail."""
    M, N = c.shape
    K = a.shape[0] if layout == 2 else a.shape[1]
    if algo is None and ALGO == 2 and k64_ok(layout, epi, bm, bn, N, K):
        algo = K64_ALGO
    algo = ALGO if algo is None else algo
    full, S = tail_plan(M, N, K, bm, bn, c.device, algo)
    ws = cnt = None
    if S > 1:
        ws, cnt = _workspace(c.device, ((M // bm) * (N // bn) - full) * S * bm * bn, (M // bm) * (N // bn) - full)
    kernels().gemm_bf16(a, b, c, layout, epi, bm, bn, bias, z, zout, dbias, 1, None, False, algo,
                        ws, cnt, full, S)
    return c


# weight gradients on the stream-K ping-pong kernel (algo 5): dW (+)= dY^T X
WGRAD_SK = os.environ.get("CAAMD_WGRAD_SK", "1") == "1"


# (N_out, K_in) -> runs where the kernel measured faster than hipBLASLt at 32768
# tokens (profiles/wgrad_stream_k.jsonl): GPT-2-XL fc (6400 x 1600, lockstep split-K
# 2) and attention proj (1600 x 1600, 245 runs = 35 tiles x 7 slices). qkv stays on
# hipBLASLt; fc2 is stored transposed, so its weight gradient is the fc shape.
WGRAD_WINNERS = {(6400, 1600): 250, (1600, 1600): 245}
# slice-major lockstep order (one token window per XCD at a time) for run counts
# that are a whole number of slices per tile (CAAMD_WGRAD_LOCKSTEP=0: stream-K order)
WGRAD_LOCKSTEP = os.environ.get("CAAMD_WGRAD_LOCKSTEP", "1") == "1"
# lockstep slabs combined by a separate reduce launch over all CUs (algo 15) instead
# of by each tile's last-arriving slice (CAAMD_WGRAD_EXT=0: in-kernel combine)
WGRAD_EXT = os.environ.get("CAAMD_WGRAD_EXT", "1") == "1"
# extra entries for A/B runs: CAAMD_WGRAD_EXTRA="1600x6400:420,4800x1600:190"
for _e in filter(None, os.environ.get("CAAMD_WGRAD_EXTRA", "").split(",")):
    _shape, _runs = _e.split(":")
    _m, _n = _shape.split("x")
    WGRAD_WINNERS[(int(_m), int(_n))] = int(_runs)


def wgrad_runs(M: int, N: int, K: int) -> Optional[int]:
    """Runs for dW[M=N_out, N=K_in] over K tokens on the weight-gradient kernel, or
    None to keep the library GEMM."""
    if not (ENABLED and WGRAD_SK) or M % 8 or N % 320 or K % 64 or K < 16384:
        return None
    return WGRAD_WINNERS.get((M, N))


def sk_runs(M: int, N: int, K: int, dev: torch.device) -> int:
    """Runs for the weight-gradient kernel: lockstep split-K, tiles x S <= CUs with S
    dividing the K-steps (every block then streams the same token window at the same
    time, so the dY / X panels are read from HBM once and shared through L2 / MALL);
    stream-K over all CUs scatters the runs over the tokens and measured HBM-bound
    (profiles/wgrad_stream_k.jsonl)."""
    tiles = -(-M // 256) * (N // 320)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nk = K // 32
    S = max(1, cus // tiles)
    while S > 1 and nk % S:
        S -= 1
    return tiles * S


def run_sk(a, b, c, layout: int, accumulate: bool, runs: Optional[int] = None):
    """Weight-gradient launch: layout 2 a[K,M] b[K,N] -> c[M,N] (+)= a^T b, the
    tiles x K-steps space cut into `runs` equal runs (stream-K; split-K when runs =
    tiles x S)."""
    M, N = c.shape
    K = a.shape[0] if layout == 2 else a.shape[1]
    tiles = -(-M // 256) * (N // 320)
    if runs is None:
        runs = sk_runs(M, N, K, c.device)
    ws, cnt = _workspace(c.device, 2 * runs * 256 * 320, tiles)
    slices = runs // tiles if WGRAD_LOCKSTEP and runs % tiles == 0 and runs > tiles else 0
    # (two slices: level with the in-kernel combine; 7 slices at 1600 x 1600: 225 vs 301 us)
    algo = 15 if (slices > 2 and WGRAD_EXT) else 5
    kernels().gemm_bf16(a, b, c, layout, EPI_BF16_ACC if accumulate else EPI_BF16, 256, 320, None, None,
                        None, None, 1, None, accumulate, algo, ws, cnt, slices, runs)
    return c


# weight gradients on the TN full-line kernel (gemm.hip algo 25: 64-deep K-tiles, every
# LDS / DMA address precomputed, lockstep split-K + reduce launch). (N_out, K_in) ->
# (tile rows, slices): 250 / 245 / 250 runs for 256 CUs. CAAMD_WGRAD_TN=0: stream-K kernel.
WGRAD_TN = os.environ.get("CAAMD_WGRAD_TN", "1") == "1"
TN_PLANS = {(6400, 1600): (256, 2), (4800, 1600): (192, 2), (1600, 1600): (256, 7)}


def tn_plan(M: int, N: int, K: int) -> Optional[Tuple[int, int]]:
    """(tile rows, slices) of the TN weight-gradient kernel for dW[M, N] over K tokens,
    or None (shape not tuned / not tileable). Outputs of >= 768 tiles (the LM head,
    50432 x 1600: 985 tiles) fill the CUs without a split: 256 rows, one slice
    (2.0 ms vs 2.5 ms on the stream-K kernel per 16384-token chunk,
    profiles/wgrad_tn64_r5.jsonl)."""
    if not (ENABLED and WGRAD_TN) or M % 8 or N % 320 or K % 64 or K < 16384:
        return None
    plan = TN_PLANS.get((M, N))
    if plan is None and -(-M // 256) * (N // 320) >= 768:
        plan = (256, 1)
    return plan


# two-slice splits combined inside the GEMM by each tile's last-arriving slice
# (write-through slabs + ticket, algo 26) instead of a reduce launch (algo 25): measured
# level (fc 500.7 vs 500.3 us, qkv 413.0 vs 414.2 incl. the reduce launch,
# profiles/wgrad_tn64_inkernel_r5.jsonl), so opt-in: CAAMD_WGRAD_TN_INKERNEL=1
TN_INKERNEL = os.environ.get("CAAMD_WGRAD_TN_INKERNEL", "0") == "1"


def run_tn(a, b, c, accumulate: bool, bm: int = 256, slices: int = 1, inkernel: Optional[bool] = None):
    """c[M, N] (+)= a[K, M]^T b[K, N] on gemm_tn64_kernel (``slices`` > 1: lockstep
    split-K, fp32 slabs summed in slice order -- by the tile's last arriving slice,
    or by a reduce launch with ``inkernel=False``)."""
    M, N = c.shape
    ws = cnt = None
    if slices > 1:
        tiles = -(-M // bm) * (N // 320)
        ws, cnt = _workspace(c.device, slices * tiles * bm * 320, tiles)
        if slices != 2 or not (TN_INKERNEL if inkernel is None else inkernel):
            cnt = None  # the in-kernel combine takes two slices; others use the reduce launch
    kernels().gemm_tn64(a, b, c, bm, accumulate, slices, ws, cnt)
    return c


def _run(a, b, c, epi, bias=None, z=None, zout=None, dbias=None):
    M, N = c.shape
    K = a.shape[1]
    bm, bn = tile_for(M, N, K)
    return run_pp(a, b, c, 0, epi, bm, bn, bias, z, zout, dbias)


# Plain (no-epilogue) NT GEMMs routed to the library (hipBLASLt / rocBLAS through
# torch, with the shipped TunableOp selections of ops/gemm_tuning.py): a comma list of
# "NxK" output-width x depth pairs, e.g. CAAMD_LIB_NT=1600x6400,4800x1600. Default:
# none (every GEMM of the step on gemm.hip). tools/gemm_vs_blaslt.py compares the two
# per shape; the fused-epilogue GEMMs and the weight gradients stay on gemm.hip.
_LIB_NT = {tuple(int(v) for v in p.split("x")) for p in os.environ.get("CAAMD_LIB_NT", "").split(",")
           if "x" in p}


def _lib(N: int, K: int) -> bool:
    return bool(_LIB_NT) and (N, K) in _LIB_NT


def linear_nt(x2: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _lib(w.shape[0], w.shape[1]):
        return F.linear(x2, w, b)
    out = torch.empty(x2.shape[0], w.shape[0], device=x2.device, dtype=torch.bfloat16)
    return _run(x2, w, out, EPI_BF16, bias=b)


# NN GEMMs on the TN kernel's full-line schedule with a K-major A (gemm.hip algo 27):
# x @ W for a weight W [K, N] read as stored, so the input-gradient GEMMs, the fc2
# forward from its transposed storage and the LM-head dgrad need no transpose pass.
# Opt-in (CAAMD_GEMM_NN=1): it measured slower than transpose + the k64 NT kernel on
# the 640-tile shapes (fc dgrad 571-581 vs 537-550 us: no split tail on this schedule)
# and the step 99.5k / 99.7k vs 100.9k / 101.2k (profiles/gemm_nn_ab_r6.txt)
NN = os.environ.get("CAAMD_GEMM_NN", "0") == "1"


def nn_ok(M: int, N: int, K: int) -> bool:
    return NN and ENABLED and M % 256 == 0 and N % 320 == 0 and K % 64 == 0


def linear_nn64(x2: torch.Tensor, wkn: torch.Tensor, b: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x2 [M, K] @ wkn [K, N] (+ b)`` on the NN kernel (caller checks :func:`nn_ok`)."""
    if out is None:
        out = torch.empty(x2.shape[0], wkn.shape[1], device=x2.device, dtype=torch.bfloat16)
    kernels().gemm_nn64(x2, wkn, out, b)
    return out


def dgrad_w(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx = dy @ W for an nn.Linear weight W [N_out, K_in] as stored: the NN kernel,
    else W^T by the transpose kernel + the NT path (:func:`dgrad`)."""
    if nn_ok(dy2.shape[0], w.shape[1], w.shape[0]) and _ok(dy2, w):
        return linear_nn64(dy2, w)
    return dgrad(dy2, transpose(w))


def linear_gelu(x2: torch.Tensor, w: torch.Tensor, b: torch.Tensor):
    M, N = x2.shape[0], w.shape[0]
    u = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    z = torch.empty_like(u)
    _run(x2, w, u, EPI_BIAS_GELU, bias=b, zout=z)
    return u, z


def dgrad(dy2: torch.Tensor, wt: torch.Tensor) -> torch.Tensor:
    """dx = dy @ W given wt = W^T ([K_in, N_out], row-major)."""
    if _lib(wt.shape[0], wt.shape[1]):
        return F.linear(dy2, wt)
    out = torch.empty(dy2.shape[0], wt.shape[0], device=dy2.device, dtype=torch.bfloat16)
    return _run(dy2, wt, out, EPI_BF16)


def dgrad_dgelu(dy2: torch.Tensor, wt: torch.Tensor, z: torch.Tensor, dbias_f32: torch.Tensor) -> torch.Tensor:
    out = torch.empty(dy2.shape[0], wt.shape[0], device=dy2.device, dtype=torch.bfloat16)
    return _run(dy2, wt, out, EPI_DGELU, z=z, dbias=dbias_f32)


def linear_nn(x2: torch.Tensor, wt: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x2 @ wt (+ b)`` with ``wt = W^T`` row-major [K_in, N_out] (layout 1: the
    B tile is read with the hardware transpose reads, no weight transpose pass)."""
    M, K = x2.shape
    N = wt.shape[1]
    out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    bm, bn = tile_for(M, N, K)
    return run_pp(x2, wt, out, 1, EPI_BF16, bm, bn, bias=b)


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
    return run_pp(a, b, c, layout, EPI_BF16, bm, bn, algo=algo)


# ---------------------------------------------------------------- serving prefill
# Llama prefill projections on the full-line kernel straight from the decode GEMM's
# packed weight copy (ops/llm.py pack_decode_weight): 256 x 256 tiles (every packed
# N is a multiple of 128, the slabs of a tile are contiguous), the SwiGLU of the
# 64-row-interleaved gate/up weight and the residual adds of o / down in the
# epilogues, so prefill keeps no second copy of the weights and no [M, 2F]
# intermediate.
PREFILL_ALGO = int(os.environ.get("CAAMD_PREFILL_ALGO", "9"))  # 256 x 256: four phases, DMA over two (tools/bench_prefill_gemm.py)
_PREFILL_ALGO_FORCED = "CAAMD_PREFILL_ALGO" in os.environ


def prefill_algo(M: int, N: int, K: int, epi: int) -> int:
    """Full-line kernel variant per prefill projection. Measured at the serving
    bench's 8192-token chunks (tools/bench_prefill_gemm.py --tokens 8192,
    profiles/prefill_algo_8192_r5.jsonl): qkv 380.7 -> 312.2 us and o 234.4 -> 221.5 us
    with DMA over three phases (3009), gate/up + SwiGLU 1578.9 -> 1466.9 us and down
    736.9 -> 727.2 us with two phases (4009); above 8192 tokens the round-4 choice (9)."""
    if _PREFILL_ALGO_FORCED or M > 8192:
        return PREFILL_ALGO
    if epi == EPI_SWIGLU or K >= 8192:
        return 4009
    return 3009


def prefill_ok(M: int, N: int, K: int) -> bool:
    return ENABLED and M % 256 == 0 and N % 256 == 0 and K % 64 == 0 and M > 0


def prefill_linear(x2: torch.Tensor, wp: torch.Tensor, *, epi: int = EPI_BF16, out: Optional[torch.Tensor] = None,
                   accumulate: bool = False) -> torch.Tensor:
    """``x2 [M, K] @ W^T`` with ``wp`` = W [N, K] in packed order: ``epi`` 0 -> [M, N]
    (``accumulate``: ``out += ...``, the residual add), ``EPI_SWIGLU`` -> [M, N/2] =
    silu(gate) * up for a gate/up weight interleaved in 64-row blocks."""
    M, K = x2.shape
    N = wp.shape[0]
    if not prefill_ok(M, N, K):
        raise ValueError(f"prefill_linear: M % 256, N % 256, K % 64 must be 0 (M={M} N={N} K={K})")
    if out is None:
        out = torch.empty(M, N // 2 if epi == EPI_SWIGLU else N, device=x2.device, dtype=torch.bfloat16)
    algo = prefill_algo(M, N, K, epi)
    full, S = tail_plan(M, N, K, 256, 256, x2.device, algo)
    ws = cnt = None
    if S > 1:
        ws, cnt = _workspace(x2.device, ((M // 256) * (N // 256) - full) * S * 256 * 256, (M // 256) * (N // 256) - full)
    kernels().gemm_bf16(x2, wp, out, 0, epi, 256, 256, None, None, None, None, 1, None, accumulate, algo,
                        ws, cnt, full, S, True)
    return out
