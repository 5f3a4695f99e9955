"""ZeRO-1 on a world-1 RCCL group on the GPU: DataParallelStep(zero="always")
runs the sharded AdamW, the shard grad-norm, the reduce-scatter / all-gather
buckets and the deferred all-gather pre-hooks, and must land on the same weights
as the plain (zero=False) step after 3 steps (reference role:
python/ray/train/torch/config.py:66 process-group setup)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(port, q):
    import torch.distributed as dist

    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        cfg = GPT2Config.named("gpt2-tiny")
        g = torch.Generator().manual_seed(7)
        data = torch.randint(0, cfg.vocab_size, (3, 8, 129), generator=g).cuda()
        out = {}
        for zero in ("always", False):
            torch.manual_seed(0)
            m = GPT2(cfg).cuda()
            st = DataParallelStep(m, lr=1e-3, zero=zero, max_grad_norm=1.0, bucket_cap_mb=0.5)
            assert st.zero == (zero == "always")
            signals = {}
            if st.zero:  # every parameter must signal "gradient final" exactly once per step
                orig = st.reducer._on_grad
                via = {}

                def counted(p, orig=orig, how="ready"):
                    signals[id(p)] = signals.get(id(p), 0) + 1
                    via.setdefault(id(p), []).append(how)
                    orig(p)

                for sl in st.flat.slots:
                    sl.param._ca_grad_ready = counted
                for h in st.reducer._hooks:
                    h.remove()
                st.reducer._hooks = [sl.param.register_post_accumulate_grad_hook(
                    lambda p: counted(p, how="hook")) for sl in st.flat.slots]
            losses = [float(st(x[:, :-1], x[:, 1:])) for x in data]
            st.wait_params()
            torch.cuda.synchronize()
            names = {id(sl.param): sl.name for sl in st.flat.slots}
            # fused ops signal directly AND torch fires the post-accumulate hook ('rh'):
            # the reducer must count one per step; a parameter never signalled is a bug
            bad = {names[k]: "".join(h[0] for h in via[k]) for k, v in signals.items() if v < len(data)}
            missing = [sl.name for sl in st.flat.slots if id(sl.param) not in signals] if st.zero else []
            slots = [(sl.name, sl.offset, sl.numel) for sl in st.flat.slots]
            out[str(zero)] = (st.flat.param_buffer.float().cpu().numpy(), losses,
                              len(getattr(st.reducer, "buckets", [])), bad, missing, slots)
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_zero1_world1_rccl_matches_plain_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_run, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=300)
    p.join(60)
    assert p.exitcode == 0
    (pz, lz, nb, bad, missing, slots), (pp, lp, *_) = out["always"], out["False"]
    assert nb > 1  # several buckets: the per-bucket reduce-scatter / all-gather order ran
    assert not bad and not missing, (bad, missing)  # every param signalled in every step
    a, b = torch.from_numpy(pz), torch.from_numpy(pp)
    per = sorted(((((a[o:o + n] - b[o:o + n]).norm() / (b[o:o + n].norm() + 1e-12)).item(), nm)
                  for nm, o, n in slots), reverse=True)[:5]
    assert lz[0] == pytest.approx(lp[0], rel=1e-6)
    assert all(abs(a - b) <= 1e-3 * abs(b) for a, b in zip(lz, lp)), (lz, lp)
    assert a.shape == b.shape
    rel = ((a - b).norm() / b.norm()).item()
    assert rel <= 1e-3, (rel, per)
