"""Whole-model numerics at GPT-2-XL width through every production default, against
plain fp32 torch autograd (asked for by the round-4 review).

Production path: 2 blocks at d = 1600, 25 heads, T = 1024, B = 16 (16384 tokens: the
smallest batch at which every default engages -- the TN weight-gradient kernel and the
chunked fused LM head need >= 16384 tokens), bf16 flat weights with fp32 master and
main-grad views (DataParallelStep), fused main-grad linears (full-line k64 NT GEMMs
with the split-K tail, TN weight gradients with lockstep split + reduce launch), fused
bias+GELU / dGELU epilogues with the fc bias drained from its fp32 accumulator,
LayerNorm backward writing dgamma / dbeta and the proj / fc2 bias gradients into the
flat buffer, flash attention D = 64, chunked fused LM head + cross-entropy, fc2 stored
transposed.

Reference: the same weights in fp32, a model written from F.embedding / F.layer_norm /
F.linear / math-mode causal softmax attention / F.gelu(tanh) / F.cross_entropy.

Tolerances: every parameter's gradient within 3e-2 relative (Frobenius) of fp32
autograd; loss within 2e-3 relative. Optimizer: 3 DataParallelStep steps (fused
AdamW, clip 1.0) against torch.optim.AdamW on fp32 master weights with
clip_grad_norm_(1.0): losses within 5e-3 relative per step, and each parameter's
total update (p3 - p0) with cosine similarity >= 0.97 to the reference update and a
norm within 10 % (Adam's first steps move each weight by ~lr * sign(g): elements whose
tiny gradients bf16 rounds to the other sign move the other way, so an exact
element-wise match is not the right test). The qkv bias is compared on its q and v
thirds only: the key bias's true gradient is exactly zero (softmax shift invariance),
so both optimizers move it by normalised rounding noise.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

B, T = 16, 1024


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _ref_loss(P, cfg, idx, tgt):
    d, H = cfg.n_embd, cfg.n_head
    dh = d // H
    h = F.embedding(idx, P["wte"]) + P["wpe"][: idx.shape[1]]
    for i in range(cfg.n_layer):
        p = lambda n: P[f"blocks.{i}.{n}"]  # noqa: E731
        a = F.layer_norm(h, (d,), p("ln1_w"), p("ln1_b"), cfg.ln_eps)
        qkv = F.linear(a, p("attn_w"), p("attn_b"))
        Bq, Tq, _ = qkv.shape
        q, k, v = qkv.view(Bq, Tq, 3, H, dh).permute(2, 0, 3, 1, 4).unbind(0)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
        mask = torch.ones(Tq, Tq, dtype=torch.bool, device=s.device).tril()
        y = torch.softmax(s.masked_fill(~mask, float("-inf")), -1) @ v
        y = y.transpose(1, 2).reshape(Bq, Tq, d)
        h = h + F.linear(y, p("proj_w"), p("proj_b"))
        m = F.layer_norm(h, (d,), p("ln2_w"), p("ln2_b"), cfg.ln_eps)
        u = F.gelu(F.linear(m, p("fc_w"), p("fc_b")), approximate="tanh")
        h = h + F.linear(u, p("fc2_w"), p("fc2_b"))
    hf = F.layer_norm(h, (d,), P["lnf_w"], P["lnf_b"], cfg.ln_eps)
    logits = F.linear(hf.reshape(-1, d), P["wte"])[:, : cfg.vocab_size]
    return F.cross_entropy(logits, tgt.reshape(-1))


def _setup(seed=0):
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep

    torch.manual_seed(seed)
    cfg = GPT2Config(n_layer=2, n_head=25, n_embd=1600)
    model = GPT2(cfg).cuda()
    master0 = {n: p.detach().clone().float() for n, p in model.named_parameters()}
    st = DataParallelStep(model, lr=3e-4, max_grad_norm=1.0)
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    idx = torch.randint(0, cfg.vocab_size, (B, T + 1), device="cuda", generator=g)
    return cfg, model, st, master0, idx[:, :-1].contiguous(), idx[:, 1:].contiguous()


def test_gpt2_xl_width_gradients_match_fp32_autograd():
    from cluster_anywhere_amd.ops import gemm as G

    cfg, model, st, _, x, y = _setup(0)
    assert G.tn_plan(6400, 1600, B * T) is not None  # the production wgrad path is what runs
    st.flat.zero_grad()
    st.reducer.start()
    loss = model(x, y)
    loss.backward()
    st.reducer.finish()
    torch.cuda.synchronize()
    # reference on the bf16 weights the production step computed with, in fp32
    P = {n: p.detach().float().clone().requires_grad_() for n, p in model.named_parameters()}
    ref = _ref_loss(P, cfg, x, y)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-3 * abs(ref.item()), (loss.item(), ref.item())
    bad, errs = [], []
    for n, p in model.named_parameters():
        r = _rel(p.main_grad, P[n].grad)
        errs.append((round(r, 5), n))
        if not r < 3e-2:
            bad.append((n, round(r, 4)))
    print("loss", loss.item(), "ref", ref.item(), "worst grad rel errors:", sorted(errs)[-6:])
    assert not bad, bad


def test_gpt2_xl_width_three_steps_match_torch_adamw():
    cfg, model, st, master0, x, y = _setup(1)
    from cluster_anywhere_amd.parallel.flat import _slot_view

    P = {n: t.clone().requires_grad_() for n, t in master0.items()}
    # FlatParamSpace's default rule: decay matrices / embeddings, not biases or gains
    groups = [{"params": [t for t in P.values() if t.dim() >= 2], "weight_decay": 0.1},
              {"params": [t for t in P.values() if t.dim() < 2], "weight_decay": 0.0}]
    opt = torch.optim.AdamW(groups, lr=3e-4, betas=(0.9, 0.95), eps=1e-8)
    losses, ref_losses = [], []
    for _ in range(3):
        losses.append(st(x, y).item())
        opt.zero_grad(set_to_none=True)
        rl = _ref_loss(P, cfg, x, y)
        rl.backward()
        torch.nn.utils.clip_grad_norm_(list(P.values()), 1.0)
        opt.step()
        ref_losses.append(rl.item())
    torch.cuda.synchronize()
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 5e-3 * abs(b), (losses, ref_losses)
    # fp32 master after 3 steps vs the reference weights
    bad = []
    masters = {s.name: _slot_view(st.flat.master, s.offset, s.param) for s in st.flat.slots}
    d = cfg.n_embd
    worst = []
    for n, p in model.named_parameters():
        got = masters[n] - master0[n]
        want = P[n].detach() - master0[n]
        if n.endswith("attn_b"):
            # the KEY bias has an exactly-zero gradient (it adds q . b_k to every score
            # of a query row, which the softmax cancels): both sides update it from
            # rounding noise that Adam normalises to +-lr, so only the q and v thirds
            # can be compared
            got, want = torch.cat([got[:d], got[2 * d:]]), torch.cat([want[:d], want[2 * d:]])
        cos = F.cosine_similarity(got.reshape(1, -1), want.reshape(1, -1)).item()
        nr = (got.norm() / (want.norm() + 1e-12)).item()
        worst.append((round(cos, 4), round(nr, 4), n))
        if not (cos >= 0.97 and 0.9 <= nr <= 1.1):
            bad.append((n, round(cos, 4), round(nr, 4)))
    print("losses", losses, "ref", ref_losses, "lowest update cosines:", sorted(worst)[:6])
    assert not bad, bad
