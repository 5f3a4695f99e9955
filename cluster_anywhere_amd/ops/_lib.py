"""Loader for the gfx950 kernel extension (``cluster_anywhere_amd/_C*.so``).

GPU tensors always go to the HIP kernels; if the extension is missing while a
GPU is present we raise instead of silently falling back to eager PyTorch.
CPU tensors use the plain-PyTorch reference implementations (these are what the
GPU numerics tests compare against).
"""
from __future__ import annotations

import importlib
import os

import torch

_C = None
_ERR = None


def kernels():
    """Return the ``_C`` module, building it in-tree on first use if allowed."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        _C = importlib.import_module("cluster_anywhere_amd._C")
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        if os.environ.get("CAAMD_AUTOBUILD", "1") == "1":
            from .. import _build

            _build.build_kernels()
            _C = importlib.import_module("cluster_anywhere_amd._C")
        else:
            raise RuntimeError(
                "cluster_anywhere_amd HIP kernels (_C) are not built; run "
                "`python -m cluster_anywhere_amd._build`"
            ) from e
    # A/B switches for the LayerNorm backward kernel: variant and grid cap (0: the default)
    v, nb = os.environ.get("CAAMD_LN_BWD_VARIANT"), os.environ.get("CAAMD_LN_BWD_BLOCKS")
    if (v is not None or nb is not None) and hasattr(_C, "ln_bwd_config"):
        _C.ln_bwd_config(int(v or 3), int(nb or 0))
    gm = os.environ.get("CAAMD_GEMM_GROUP_M")  # A/B switch: m-tiles per tile-order group of the k64 GEMM
    if gm is not None and hasattr(_C, "gemm_set_group_m"):
        _C.gemm_set_group_m(int(gm))
    tg = os.environ.get("CAAMD_TN_GROUP_M")  # the same for the TN weight-gradient kernel
    if tg is not None and hasattr(_C, "gemm_set_tn_group_m"):
        _C.gemm_set_tn_group_m(int(tg))
    return _C


def use_gpu_kernel(*tensors) -> bool:
    return all(t is None or t.is_cuda for t in tensors) and any(
        t is not None and t.is_cuda for t in tensors
    )


def available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


def has_gpu() -> bool:
    return torch.cuda.is_available()
