"""Chunked LM head + cross-entropy (ops/loss.py: logits never materialised, all
three GEMMs on gemm.hip, register-resident softmax kernel) vs a plain fp32
PyTorch reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("rows,V,stride", [(16, 50257, 50432), (9, 1000, 1024), (5, 129, 136), (3, 131000, 131072)])
def test_xent_fused_kernel(rows, V, stride):
    from cluster_anywhere_amd.ops import kernels

    torch.manual_seed(0)
    logits = (3 * torch.randn(rows, stride, device="cuda")).bfloat16()
    tgt = torch.randint(0, V, (rows,), device="cuda")
    tgt[1] = -1  # ignored row
    scale = torch.tensor([0.25], device="cuda")
    lg = logits.clone()
    loss, lse = kernels().xent_fused_(lg, tgt, scale, V)
    lf = logits.float()[:, :V].clone().requires_grad_()
    ref = F.cross_entropy(lf, tgt.clamp(min=0), reduction="none")
    ref = torch.where(tgt >= 0, ref, torch.zeros_like(ref))
    (ref * 0.25).sum().backward()
    assert torch.allclose(loss, ref.detach(), atol=2e-2, rtol=1e-2)
    assert torch.allclose(lse, torch.logsumexp(lf.detach(), dim=1), atol=2e-2, rtol=1e-3)
    assert _rel(lg[:, :V], lf.grad) < 2e-2
    if V < stride:
        assert lg[:, V:].abs().max().item() == 0
    assert lg[1].abs().max().item() == 0


@pytest.mark.parametrize("N,D,V,vocab,chunk", [(1024, 320, 1024, 1000, 512), (2048, 1600, 50432, 50257, 1024),
                                                (768, 640, 2048, 2048, 512)])
@pytest.mark.parametrize("main_grad", [False, True])
def test_linear_cross_entropy(N, D, V, vocab, chunk, main_grad):
    from cluster_anywhere_amd.ops.loss import linear_cross_entropy, linear_cross_entropy_ok

    torch.manual_seed(1)
    h = (torch.randn(N, D, device="cuda") * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(V, D, device="cuda") * 0.05).bfloat16()
    w[vocab:] = 0
    w.requires_grad_()
    if main_grad:
        w.main_grad = torch.full_like(w, 1e-6)  # accumulates into an existing gradient (grad scale)
    tgt = torch.randint(0, vocab, (N,), device="cuda")
    tgt[::7] = -100
    assert linear_cross_entropy_ok(h, w)
    loss = linear_cross_entropy(h, w, tgt, vocab, chunk=chunk)
    (loss * 2.0).backward()  # a non-unit upstream gradient

    hf = h.detach().float().requires_grad_()
    wf = w.detach().float().requires_grad_()
    logits = hf @ wf[:vocab].t()
    ref = F.cross_entropy(logits, tgt, ignore_index=-100)
    (ref * 2.0).backward()
    assert abs(loss.item() - ref.item()) < 2e-2 * max(1.0, abs(ref.item()))
    assert _rel(h.grad, hf.grad) < 3e-2
    gw = (w.main_grad.float() - 1e-6) if main_grad else w.grad
    assert _rel(gw[:vocab], wf.grad[:vocab]) < 3e-2
    if vocab < V:
        assert gw[vocab:].float().abs().max().item() < 1e-3
    if main_grad:
        assert w.grad is None


def test_gpt2_head_matches_unfused(monkeypatch):
    """GPT-2 forward/backward through the chunked head equals the materialised-logits path."""
    import cluster_anywhere_amd.ops.loss as L
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(2)
    cfg = GPT2Config(n_layer=1, n_head=5, n_embd=320, n_positions=256, vocab_size=1000)
    m = GPT2(cfg).cuda().bfloat16()
    x = torch.randint(0, cfg.vocab_size, (4, 257), device="cuda")
    grads = []
    for fused in (True, False):
        monkeypatch.setattr(L, "FUSED_HEAD", fused)
        m.zero_grad(set_to_none=True)
        loss = m(x[:, :-1], x[:, 1:])
        loss.backward()
        grads.append((loss.item(), m.wte.grad.clone(), m.blocks[0].fc_w.grad.clone()))
    (l1, w1, f1), (l0, w0, f0) = grads
    assert abs(l1 - l0) < 2e-2
    assert _rel(w1, w0) < 3e-2
    assert _rel(f1, f0) < 3e-2
