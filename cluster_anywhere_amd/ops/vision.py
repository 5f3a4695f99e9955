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
