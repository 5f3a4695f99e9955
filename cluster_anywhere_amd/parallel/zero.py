"""ZeRO-1: bucketed reduce-scatter of gradients, sharded fused AdamW, all-gather of
bf16 weights — same bytes on the xGMI links as an all-reduce, 1/N of the
optimizer HBM traffic and 1/N of the fp32 optimizer state per GPU.

Layout: every bucket ``[start, end)`` of the flat gradient buffer (cut exactly as
in :mod:`.ddp`, each bucket length a multiple of ``8 * world``) is split into
``world`` equal contiguous shards; rank *r* owns shard *r* of every bucket. The
rank's optimizer state is the concatenation of its shards over buckets, so one
fused AdamW launch updates all of it. Reduce-scatters are launched from the
post-accumulate-grad hooks (overlapping backward); all-gathers write straight
into the model's flat bf16 weight buffer.

All-gather overlap: ``step()`` only *issues* the bucket all-gathers (async, on
RCCL's stream) in the order the next forward first touches the buckets, and
returns. A forward pre-hook on every module that owns parameters makes the
compute stream wait (``work.wait()`` — a stream dependency, not a host sync) on
exactly the buckets holding that module's parameters, so layer *l*'s forward
runs while the gathers of layers *l+1..L* are still on the xGMI links. The
first-use order is recorded on the first forward after a step and reused.
Anything that reads the weights outside a forward calls ``wait_params()``.

Reference parity: the ZeRO/FSDP path Ray Train exposes through its DeepSpeed /
FSDP integrations (``python/ray/train/torch/train_loop_utils.py:162``,
``parallel_strategy="fsdp"``).
"""
from __future__ import annotations

from typing import List

import torch
import torch.distributed as dist

from ..ops.optim import FusedAdamW
from .ddp import DEFAULT_BUCKET_MB, _Bucket
from .flat import FlatParamSpace


class _ShardSpace:
    """Duck-types FlatParamSpace for FusedAdamW (master / wd_mask / grad / param)."""

    def __init__(self, master, wd_mask, grad_buffer, param_buffer):
        self.master = master
        self.wd_mask = wd_mask
        self.grad_buffer = grad_buffer
        self.param_buffer = param_buffer


class Zero1Reducer:
    def __init__(
        self,
        flat: FlatParamSpace,
        process_group=None,
        bucket_cap_mb: float = DEFAULT_BUCKET_MB,
        lr: float = 1e-4,
        betas=(0.9, 0.95),
        eps: float = 1e-8,
        weight_decay: float = 0.1,
        max_grad_norm: float = 1.0,
        broadcast_init: bool = True,
        module=None,
    ):
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        W = self.world
        assert flat.align % (8 * W) == 0, "FlatParamSpace align must be a multiple of 8*world"
        assert flat.master is not None
        if broadcast_init:
            dist.broadcast(flat.master, src=self._global_src(), group=process_group)
            dist.broadcast(flat.param_buffer, src=self._global_src(), group=process_group)
        cap = int(bucket_cap_mb * (1 << 20)) // flat.grad_buffer.element_size()
        self.buckets: List[_Bucket] = []
        owner = {}
        cur_end, count = flat.numel, 0
        slots = flat.slots
        for i in range(len(slots) - 1, -1, -1):
            s = slots[i]
            count += 1
            owner[id(s.param)] = len(self.buckets)
            if (cur_end - s.offset) >= cap or i == 0:
                start = 0 if i == 0 else s.offset
                self.buckets.append(_Bucket(len(self.buckets), start, cur_end, count))
                cur_end, count = start, 0
        self._owner = owner
        # shard bookkeeping
        dev = flat.grad_buffer.device
        shard_sizes = [(b.end - b.start) // W for b in self.buckets]
        for b in self.buckets:
            assert (b.end - b.start) % (8 * W) == 0
        n_local = sum(shard_sizes)
        self.shard_offsets = []
        off = 0
        master = torch.empty(n_local, dtype=torch.float32, device=dev)
        mask = torch.empty(n_local // 8, dtype=torch.uint8, device=dev)
        for b, ss in zip(self.buckets, shard_sizes):
            g0 = b.start + self.rank * ss
            master[off : off + ss].copy_(flat.master[g0 : g0 + ss])
            mask[off // 8 : (off + ss) // 8].copy_(flat.wd_mask[g0 // 8 : (g0 + ss) // 8])
            self.shard_offsets.append((off, ss, g0))
            off += ss
        flat.master = None  # the full fp32 copy is no longer needed
        self.grad_shard = torch.zeros(n_local, dtype=flat.grad_buffer.dtype, device=dev)
        self.param_shard = torch.empty(n_local, dtype=flat.param_buffer.dtype, device=dev)
        self.space = _ShardSpace(master, mask, self.grad_shard, self.param_shard)
        self.optimizer = FusedAdamW(
            self.space, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
            max_grad_norm=max_grad_norm,
        )
        self._next = 0
        self._signaled = set()
        self._hooks = [s.param.register_post_accumulate_grad_hook(self._on_grad) for s in slots]
        for s in slots:
            s.param._ca_grad_ready = self._on_grad
        # all-gather overlap with the next forward
        self._ag = {}            # bucket index -> pending all-gather work
        self._ag_order = None    # first-use order of buckets in a forward (recorded)
        self._ag_seen = []
        self._fwd_hooks = []
        if module is not None:
            for mod in module.modules():
                own = [id(p) for p in mod.parameters(recurse=False)]
                bis = sorted({owner[i] for i in own if i in owner}, reverse=True)
                if bis:
                    self._fwd_hooks.append(mod.register_forward_pre_hook(self._make_pre_hook(bis)))

    def _global_src(self):
        return 0 if self.pg is None else dist.get_global_rank(self.pg, 0)

    def _make_pre_hook(self, bucket_ids):
        def hook(_mod, _args):
            if self._ag:
                for bi in bucket_ids:
                    self._wait_bucket(bi)
        return hook

    def _wait_bucket(self, bi):
        h = self._ag.pop(bi, None)
        if h is not None:
            if self._ag_order is None:
                self._ag_seen.append(bi)
            h.wait()

    # -- backward-side -------------------------------------------------------------
    def start(self):
        for b in self.buckets:
            b.pending, b.handle, b.launched = b.nparams, None, False
        self._next = 0
        self._signaled = set()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            b = self.buckets[self._next]
            off, ss, _ = self.shard_offsets[b.index]
            b.handle = dist.reduce_scatter_tensor(
                self.grad_shard[off : off + ss], self.flat.grad_buffer[b.start : b.end],
                op=dist.ReduceOp.SUM, group=self.pg, async_op=True,
            )
            b.launched = True
            self._next += 1

    def _on_grad(self, p):
        bi = self._owner.get(id(p))
        if bi is not None and id(p) not in self._signaled:
            # once per parameter per step (a fused op's direct signal is followed by
            # torch's post-accumulate-grad hook for the same parameter)
            self._signaled.add(id(p))
            self.buckets[bi].pending -= 1
            self._launch_ready()

    def finish(self):
        for b in self.buckets:
            b.pending = 0
        self._launch_ready()
        for b in self.buckets:
            if b.handle is not None:
                b.handle.wait()
                b.handle = None

    # -- optimizer-side ------------------------------------------------------------
    def step(self):
        opt = self.optimizer
        sumsq = None
        if opt.max_grad_norm > 0:
            opt.sumsq.zero_()
            if self.grad_shard.is_cuda:
                from ..ops._lib import kernels

                kernels().grad_sumsq(self.grad_shard, opt.sumsq)
            else:
                opt.sumsq.copy_((self.grad_shard.float() ** 2).sum().reshape(1))
            dist.all_reduce(opt.sumsq, op=dist.ReduceOp.SUM, group=self.pg)
            sumsq = opt.sumsq
        opt.step(inv_world=1.0 / self.world, sumsq=sumsq)
        self.wait_params()  # (no-op unless a forward skipped some module)
        if self._ag_order is None and self._ag_seen:
            seen = list(dict.fromkeys(self._ag_seen))
            self._ag_order = seen + [b.index for b in reversed(self.buckets) if b.index not in seen]
        order = self._ag_order or [b.index for b in reversed(self.buckets)]
        self._ag_seen = []
        for bi in order:
            b = self.buckets[bi]
            off, ss, _ = self.shard_offsets[bi]
            self._ag[bi] = dist.all_gather_into_tensor(
                self.flat.param_buffer[b.start : b.end], self.param_shard[off : off + ss],
                group=self.pg, async_op=True,
            )
        if not self._fwd_hooks:
            self.wait_params()

    def wait_params(self):
        """Make the current stream wait for every outstanding weight all-gather."""
        for bi in list(self._ag):
            self._wait_bucket(bi)

    def remove_hooks(self):
        self.wait_params()
        for h in self._hooks + self._fwd_hooks:
            h.remove()
        self._hooks, self._fwd_hooks = [], []
