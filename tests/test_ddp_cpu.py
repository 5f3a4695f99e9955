"""Bucketed DDP and ZeRO-1 over gloo at world sizes 2, 4 and 8, on CPU: both must
match a single-process run on the concatenated global batch (shard alignment to
8 x world, bucket cuts, all-gather order and the grad-norm all-reduce are all
exercised at the world sizes of a full MI355X node)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make():
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    return GPT2(cfg), cfg


GLOBAL_BATCH = 8


def _worker(rank, world, port, zero, bucket_mb, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cluster_anywhere_amd.train.loop import DataParallelStep

    torch.set_num_threads(1)
    m, cfg = _make()
    st = DataParallelStep(m, lr=1e-2, bucket_cap_mb=bucket_mb, zero=zero, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(42)
    data = torch.randint(0, cfg.vocab_size, (3, GLOBAL_BATCH, 17), generator=g)
    grads = None
    per = GLOBAL_BATCH // world
    for it in range(3):
        x = data[it][rank * per : (rank + 1) * per]
        st(x[:, :-1], x[:, 1:])
        if it == 0:
            if zero:
                full = torch.zeros_like(st.flat.grad_buffer)
                for b in st.reducer.buckets:
                    off, ss, g0 = st.reducer.shard_offsets[b.index]
                    full[g0 : g0 + ss] = st.reducer.grad_shard[off : off + ss]
                dist.all_reduce(full)
                grads = full / world
            else:
                grads = st.flat.grad_buffer.clone() / world
    st.wait_params()  # ZeRO-1 defers the weight all-gather into the next forward
    if rank == 0:
        # numpy arrays pickle by value: torch tensors would go through a shared-memory
        # fd that vanishes if this process exits before the parent has received it
        q.put((st.flat.param_buffer.clone().numpy(), grads.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _single():
    from cluster_anywhere_amd.train.loop import DataParallelStep

    m, cfg = _make()
    st = DataParallelStep(m, lr=1e-2, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(42)
    data = torch.randint(0, cfg.vocab_size, (3, GLOBAL_BATCH, 17), generator=g)
    grads = None
    for it in range(3):
        x = data[it]
        st(x[:, :-1], x[:, 1:])
        if it == 0:
            grads = st.flat.grad_buffer.clone()
    return st.flat.param_buffer.clone(), grads


@pytest.mark.parametrize("world,zero,bucket_mb", [(2, False, 0.01), (2, False, 100.0), (2, True, 0.01),
                                                  (4, False, 0.01), (4, True, 0.01), (4, True, 100.0),
                                                  (8, False, 0.05), (8, True, 0.01)])
def test_dp_matches_single_process(world, zero, bucket_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, zero, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, got_g = (torch.from_numpy(a) for a in q.get(timeout=240))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref, ref_g = _single()
    n = min(got.numel(), ref.numel())
    # the mean of the per-rank losses == full-batch loss (equal token counts)
    assert torch.allclose(got_g[:n], ref_g[:n], atol=1e-6, rtol=1e-4), (got_g[:n] - ref_g[:n]).abs().max()
    # Adam normalises away tiny summation-order noise only approximately; lr = 1e-2
    assert torch.allclose(got[:n], ref[:n], atol=2e-3), (got[:n] - ref[:n]).abs().max()


def test_optimizer_state_survives_transposed_storage_change():
    """An optimizer checkpoint saved with a weight stored transposed (GPT-2's fc2
    under CAAMD_FC2_T=1) resumes into a plainly stored model with the master and
    moments mapped back per element (and vice versa)."""
    from cluster_anywhere_amd.ops.optim import FusedAdamW
    from cluster_anywhere_amd.parallel.flat import FlatParamSpace

    def model(transposed):
        m = torch.nn.Module()
        w = torch.arange(12, dtype=torch.float32).reshape(3, 4) / 7.0
        m.w = torch.nn.Parameter(w.t().contiguous().t() if transposed else w.clone())
        m.b = torch.nn.Parameter(torch.ones(5))
        return m

    torch.manual_seed(0)
    src = model(True)
    fs = FlatParamSpace(src, dtype=torch.float32)
    opt = FusedAdamW(fs, lr=1e-2)
    fs.grad_buffer.normal_()
    opt.step()
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in opt.state_dict().items()}
    assert sd["layout"][0][4] is True

    dst = model(False)
    fd = FlatParamSpace(dst, dtype=torch.float32)
    opt2 = FusedAdamW(fd, lr=1e-2)
    opt2.load_state_dict(sd)
    fd.sync_params_from_master()
    assert torch.equal(dst.w.detach(), src.w.detach())
    # moments: logical element (i, j) must agree
    m_src = fs.slots[0]
    m_dst = fd.slots[0]
    from cluster_anywhere_amd.parallel.flat import _slot_view
    a = _slot_view(opt.exp_avg, m_src.offset, src.w)
    b = _slot_view(opt2.exp_avg, m_dst.offset, dst.w)
    assert torch.equal(a, b)

    bad = dict(sd, layout=[("w", 0, 12, (4, 3), True)] + sd["layout"][1:])
    with pytest.raises(ValueError, match="does not match"):
        FusedAdamW(FlatParamSpace(model(False), dtype=torch.float32)).load_state_dict(bad)
