"""Flat parameter / gradient storage.

Every trainable parameter of a module becomes a view into ONE contiguous
compute-dtype buffer (bf16 on MI355X), its ``.grad`` a view into ONE contiguous
gradient buffer, and the optimizer state (fp32 master, Adam moments) lives in
matching flat fp32 buffers. This gives:

* one fused AdamW launch for the whole model (``adamw.hip``),
* gradient buckets that are plain slices of the grad buffer, so the RCCL
  all-reduce / reduce-scatter reads the grads in place (no pack/unpack copies),
* one ``memset`` to zero all gradients.

Each parameter slice is aligned to 64 elements (128 B for bf16) so the 16-byte
vector kernels never straddle two parameters and a per-8-element weight-decay
mask is exact. The total is padded to a multiple of ``pad_multiple`` so a
reduce-scatter shards evenly.

Reference parity: the role of ``python/ray/train/torch/train_loop_utils.py:162``
(`prepare_model` → DDP with `gradient_as_bucket_view`).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import torch

ALIGN = 64


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class ParamSlot:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    decay: bool
    transposed: bool = False  # stored in physical [in, out] order (see _phys)


def _phys(t: torch.Tensor) -> Optional[torch.Tensor]:
    """A 2-D parameter stored transposed (``t.t()`` contiguous, e.g. GPT-2's fc2
    weight kept as [in, out] so its weight gradient tiles the CUs): its physical
    [in, out] view; None for a contiguous parameter."""
    if t.dim() == 2 and not t.is_contiguous() and t.t().is_contiguous():
        return t.t()
    return None


def _slot_view(buf: torch.Tensor, offset: int, like: torch.Tensor) -> torch.Tensor:
    """``buf[offset:offset + like.numel()]`` viewed with ``like``'s shape AND memory
    layout (so the flat order of the param, its gradient, the fp32 master and the
    Adam moments stay elementwise aligned for transposed parameters too)."""
    flat = buf[offset: offset + like.numel()]
    ph = _phys(like)
    return flat.view(ph.shape).t() if ph is not None else flat.view_as(like)


def default_decay_rule(name: str, p: torch.Tensor) -> bool:
    """GPT-style: decay matrices/embeddings, not biases or norm gains."""
    return p.dim() >= 2


class FlatParamSpace:
    def __init__(
        self,
        module: torch.nn.Module,
        dtype: Optional[torch.dtype] = None,
        grad_dtype: Optional[torch.dtype] = None,
        pad_multiple: int = ALIGN,
        decay_rule: Callable[[str, torch.Tensor], bool] = default_decay_rule,
        master_fp32: bool = True,
        align: int = ALIGN,
    ):
        align = max(ALIGN, align)
        assert align % 8 == 0
        seen = set()
        named = []
        for n, p in module.named_parameters():
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            named.append((n, p))
        if not named:
            raise ValueError("module has no trainable parameters")
        device = named[0][1].device
        self.dtype = dtype or named[0][1].dtype
        self.grad_dtype = grad_dtype or self.dtype
        off = 0
        self.slots: List[ParamSlot] = []
        for n, p in named:
            self.slots.append(ParamSlot(n, p, off, p.numel(), decay_rule(n, p), _phys(p) is not None))
            off = _round_up(off + p.numel(), align)
        self.align = align
        self.numel = _round_up(off, max(pad_multiple, align))
        self.device = device

        self.param_buffer = torch.zeros(self.numel, dtype=self.dtype, device=device)
        self.grad_buffer = torch.zeros(self.numel, dtype=self.grad_dtype, device=device)
        master = torch.zeros(self.numel, dtype=torch.float32, device=device) if master_fp32 else None
        mask = torch.zeros(self.numel // 8, dtype=torch.uint8, device=device)
        with torch.no_grad():
            for s in self.slots:
                src = s.param.detach()
                ph = _phys(src)
                if master is not None:  # physical (storage) order, like the views below
                    master[s.offset : s.offset + s.numel].copy_((ph if ph is not None else src).reshape(-1).float())
                view = _slot_view(self.param_buffer, s.offset, src)
                view.copy_(src)
                s.param.data = view
                s.param.grad = _slot_view(self.grad_buffer, s.offset, src)
                # fused layers (ops.linear) accumulate straight into this view
                s.param.main_grad = s.param.grad
                if s.decay:
                    a, b = s.offset // 8, (s.offset + s.numel + 7) // 8
                    mask[a:b] = 1
        self.master = master
        self.wd_mask = mask

    def zero_grad(self):
        self.grad_buffer.zero_()
        # autograd may have replaced .grad (e.g. after set_to_none elsewhere): re-bind views
        for s in self.slots:
            g = s.param.grad
            if g is None or g.data_ptr() != self.grad_buffer[s.offset :].data_ptr():
                s.param.grad = _slot_view(self.grad_buffer, s.offset, s.param)

    def layout(self) -> List[tuple]:
        """(name, offset, numel, logical shape, transposed) per slot: what an
        optimizer checkpoint needs to map its flat fp32 buffers onto this space."""
        return [(s.name, s.offset, s.numel, tuple(s.param.shape), s.transposed) for s in self.slots]

    def relayout_(self, buf: torch.Tensor, saved: List[tuple]) -> torch.Tensor:
        """Bring a flat fp32 buffer written under ``saved`` (a :meth:`layout`) into
        this space's layout in place: slots stored transposed in one and plainly in
        the other (e.g. GPT-2's fc2 under a different ``CAAMD_FC2_T``) are
        transposed; any other difference is an error."""
        mine = {s.name: s for s in self.slots}
        if len(saved) != len(self.slots):
            raise ValueError(f"optimizer state has {len(saved)} parameter slots, this model {len(self.slots)}")
        with torch.no_grad():
            for name, off, numel, shape, transposed in saved:
                s = mine.get(name)
                if s is None or s.offset != off or s.numel != numel or tuple(s.param.shape) != tuple(shape):
                    raise ValueError(f"optimizer state slot {name!r} (offset {off}, {numel} elements, shape "
                                     f"{tuple(shape)}) does not match this model's parameters")
                if bool(transposed) != s.transposed:
                    seg = buf[off: off + numel]
                    r, c = shape
                    src = seg.view(c, r) if transposed else seg.view(r, c)  # saved physical order
                    seg.copy_(src.t().contiguous().reshape(-1))
        return buf

    def param_index(self) -> Dict[int, ParamSlot]:
        return {id(s.param): s for s in self.slots}

    def sync_params_from_master(self):
        with torch.no_grad():
            self.param_buffer.copy_(self.master.to(self.dtype))
