"""Vision inference ops backed by ``csrc/kernels/vision.hip``: uint8 NHWC image
normalisation straight into bf16 channels_last, and the fused residual
``y = relu(y + r)``. CPU tensors take the plain-PyTorch reference path (what the
GPU numerics tests compare against)."""
from __future__ import annotations

from typing import Sequence

import torch

from ._lib import kernels

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def image_normalize_ref(x: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                        dtype=torch.float32) -> torch.Tensor:
    m = torch.tensor(mean, dtype=torch.float32, device=x.device)
    s = torch.tensor(std, dtype=torch.float32, device=x.device)
    y = (x.float() / 255.0 - m) / s  # [N, H, W, 3]
    return y.permute(0, 3, 1, 2).to(dtype).contiguous(memory_format=torch.channels_last)


def image_normalize(x: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN,
                    std: Sequence[float] = IMAGENET_STD) -> torch.Tensor:
    """uint8 [N, H, W, 3] -> normalised [N, 3, H, W] in channels_last (bf16 on GPU)."""
    if x.is_cuda:
        return kernels().image_normalize(x.contiguous(), list(mean), list(std))
    return image_normalize_ref(x, mean, std)


def add_relu_(y: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    if (y.is_cuda and y.dtype == torch.bfloat16 and r.dtype == torch.bfloat16
            and y.stride() == r.stride() and y.numel() % 8 == 0):
        kernels().add_relu_(y, r)
        return y
    return y.add_(r).relu_()


def bias_act_(y: torch.Tensor, b: torch.Tensor, residual=None, relu: bool = True) -> torch.Tensor:
    """In place: y = act(y + b[channel] (+ residual)), y channels_last [N, C, H, W]."""
    if (y.is_cuda and y.dtype == torch.bfloat16 and y.dim() == 4 and y.size(1) % 8 == 0
            and y.is_contiguous(memory_format=torch.channels_last)
            and (residual is None or residual.stride() == y.stride())):
        kernels().bias_act_(y, b, residual, relu)
        return y
    y.add_(b.view(1, -1, 1, 1))
    if residual is not None:
        y.add_(residual)
    return y.relu_() if relu else y


# ---- implicit-GEMM NHWC convolution (csrc/kernels/conv.hip) ------------------------
# The Data ResNet path runs every convolution on its own MFMA kernel with the folded
# BN bias, the residual join and ReLU in the epilogue (no MIOpen conv, no separate
# bias / add / ReLU pass). Activations are plain contiguous NHWC [N, H, W, C].

_ZERO: dict = {}


def _zero_page(dev: torch.device) -> torch.Tensor:
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(64, dtype=torch.bfloat16, device=dev)
    return z


def conv_weight_nhwc(w: torch.Tensor, cin_pad: int = 0) -> torch.Tensor:
    """[Cout, Cin, KH, KW] -> [Cout, Kp]: k = (kh * KW + kw) * Cin' + ci, Cin padded
    with zero channels to ``cin_pad`` and K zero-padded to a multiple of 32."""
    cout, cin, kh, kw = w.shape
    w = w.permute(0, 2, 3, 1)
    if cin_pad > cin:
        w = torch.nn.functional.pad(w, (0, cin_pad - cin))
    w = w.reshape(cout, -1)
    k = w.shape[1]
    kp = (k + 31) // 32 * 32
    if kp > k:
        w = torch.nn.functional.pad(w, (0, kp - k))
    return w.contiguous()


def conv_tile(m: int, cout: int, k: int = 1 << 30, residual: bool = False) -> int:
    """0 = 256x128, 1 = 256x64 (Cout 64), 2 = 128x128. Per-shape timings over every
    ResNet-50 conv at batch 512 (tools/bench_conv.py, profiles/conv_shapes_r3.jsonl):
    the 128x128 tile wins where the epilogue dominates (a residual join, or a short
    reduction K = Cin*KS*KS < 256: more workgroups per CU overlap one's epilogue
    with another's main loop), the 256x128 tile everywhere else."""
    if cout % 128:
        return 1
    if residual or k < 256:
        return 2
    return 0


def conv2d_nhwc(x: torch.Tensor, w2d: torch.Tensor, bias: torch.Tensor, ks: int, stride: int, pad: int,
                relu: bool, residual=None, tile=None) -> torch.Tensor:
    """y = act(conv(x, w) + bias (+ residual)) on NHWC bf16 (GPU kernel only)."""
    n, h, wd, _ = x.shape
    ho = (h + 2 * pad - ks) // stride + 1
    wo = (wd + 2 * pad - ks) // stride + 1
    if tile is None:
        tile = conv_tile(n * ho * wo, w2d.shape[0], x.shape[3] * ks * ks, residual is not None)
    return kernels().conv2d_nhwc(x, w2d, bias, residual, ks, stride, pad, relu, tile, _zero_page(x.device))


def conv2d_nhwc_ex(x: torch.Tensor, w2d: torch.Tensor, bias: torch.Tensor, kh: int, kw: int, stride: int,
                   stride_w: int, pad: int, pad_w: int, relu: bool, residual=None, tile=None) -> torch.Tensor:
    """:func:`conv2d_nhwc` with a kh x kw kernel and per-direction stride / padding."""
    n, h, wd, _ = x.shape
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (wd + 2 * pad_w - kw) // stride_w + 1
    if tile is None:
        tile = conv_tile(n * ho * wo, w2d.shape[0], x.shape[3] * kh * kw, residual is not None)
    return kernels().conv2d_nhwc_ex(x, w2d, bias, residual, kh, kw, stride, stride_w, pad, pad_w, relu, tile,
                                    _zero_page(x.device))


def conv_weight_pairs(w: torch.Tensor) -> torch.Tensor:
    """Stem weight [Cout, 3, 7, 7] -> the pixel-pair form [Cout, 224] for
    :func:`normalize_pairs` input: virtual tap (kh, j) covers real taps kw = 2j, 2j+1,
    channel c8 = 4 * (kw - 2j) + c (c < 3; the 4th channel and tap kw = 7 are zero);
    k = (kh * 4 + j) * 8 + c8."""
    cout, cin, kh, kw = w.shape
    assert cin == 3 and kh == 7 and kw == 7, "pixel-pair stem: [Cout, 3, 7, 7]"
    wp = torch.zeros(cout, 7, 8, 4, dtype=w.dtype, device=w.device)  # [cout, kh, kw (8), c (4)]
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    return wp.reshape(cout, 7, 4, 2, 4).reshape(cout, 7 * 4 * 8).contiguous()


def normalize_pairs(x: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN,
                    std: Sequence[float] = IMAGENET_STD) -> torch.Tensor:
    """uint8 [N, H, W, 3] -> bf16 [N, H + 6, (W + 6) / 2, 8]: normalised RGB + a zero
    channel per pixel, a 3-pixel zero border, two horizontally adjacent pixels per
    8-channel "virtual pixel" (the pixel-pair stem's input, conv.hip)."""
    return kernels().normalize_pairs(x.contiguous(), list(mean), list(std))


def conv2d_nhwc_ref(x: torch.Tensor, w4: torch.Tensor, bias: torch.Tensor, stride: int, pad: int, relu: bool,
                    residual=None) -> torch.Tensor:
    """fp32 reference of :func:`conv2d_nhwc` with the 4-D [Cout, Cin, KH, KW] weight."""
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w4.float(), bias.float(), stride, pad)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.float()
    return y.relu() if relu else y


def normalize_pad8(x: torch.Tensor, mean: Sequence[float] = IMAGENET_MEAN,
                   std: Sequence[float] = IMAGENET_STD) -> torch.Tensor:
    """uint8 [N, H, W, 3] -> bf16 [N, H, W, 8]: normalised RGB + 5 zero channels."""
    return kernels().normalize_pad8(x.contiguous(), list(mean), list(std))


def maxpool3s2_nhwc(x: torch.Tensor) -> torch.Tensor:
    return kernels().maxpool3s2_nhwc(x)
