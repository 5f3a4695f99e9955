"""Hand-written gfx950 HIP kernels exposed as autograd-aware torch ops."""
from ._lib import available, kernels
from .activation import bias_gelu
from .attention import attention
from .loss import cross_entropy
from .norm import add_layer_norm, layer_norm
from .optim import FusedAdamW
from .rl import gae, vtrace

__all__ = [
    "available",
    "kernels",
    "bias_gelu",
    "attention",
    "cross_entropy",
    "layer_norm",
    "add_layer_norm",
    "FusedAdamW",
    "gae",
    "vtrace",
]
