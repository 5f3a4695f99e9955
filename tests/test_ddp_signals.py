"""Gradient-readiness accounting of the bucketed reducers: a fused op writes its
parameter's main-grad and signals readiness directly, and torch STILL fires the
parameter's post-accumulate-grad hook afterwards (its Function returned None).
Each parameter must count once per step, or a bucket's collective launches
before the rest of its gradients exist (the bug a world-1 RCCL ZeRO run on the
GPU exposed; tests/test_zero_gpu.py). CPU, gloo world 1, ZeRO path forced."""
import os
import socket

import torch
import torch.distributed as dist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Fused(torch.autograd.Function):
    """y = x W^T with the weight gradient accumulated into W.main_grad and readiness
    signalled directly (the shape of ops.linear._MainGradLinear)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        w.main_grad.add_(dy.t() @ x)
        w._ca_grad_ready(w)
        return dy @ w, None


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.ws = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(64, 64) * 0.1) for _ in range(4)])

    def forward(self, x, y):
        for w in self.ws:
            x = torch.tanh(_Fused.apply(x, w))
        return ((x - y) ** 2).mean()


def test_fused_param_signals_once_and_buckets_see_final_grads():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from cluster_anywhere_amd.train.loop import DataParallelStep

        torch.manual_seed(0)
        st = DataParallelStep(_Net(), lr=1e-3, zero="always", max_grad_norm=0.0,
                              bucket_cap_mb=2 * 64 * 64 * 4 / (1 << 20))  # two weights per bucket
        assert st.zero and len(st.reducer.buckets) >= 2
        snaps = {}
        real = dist.reduce_scatter_tensor

        def spy(out, inp, *a, **k):  # what the collective reads when it launches
            snaps[inp.data_ptr()] = inp.clone()
            return real(out, inp, *a, **k)

        dist.reduce_scatter_tensor = spy
        try:
            x, y = torch.randn(16, 64), torch.randn(16, 64)
            st(x, y)
        finally:
            dist.reduce_scatter_tensor = real
        final = st.flat.grad_buffer
        for b in st.reducer.buckets:
            seen = snaps[final[b.start:b.end].data_ptr()]
            assert torch.equal(seen, final[b.start:b.end]), f"bucket {b.index} launched before its gradients were final"
        assert all(b.pending == 0 for b in st.reducer.buckets)
    finally:
        dist.destroy_process_group()
