"""Numerics of every gfx950 HIP kernel vs a plain fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from cluster_anywhere_amd.ops import kernels

    return kernels()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("D", [64, 768, 1600, 2048, 4096])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("variant", [0, 2, 3])
def test_layernorm_fwd_bwd(C, D, with_res, variant):
    """Backward variants: 0 one row per wave, 2 / 3 column-split (4 / 2 rows per
    iteration; D <= 2048, larger D falls back to 0); 148 rows exercise partial row groups."""
    from cluster_anywhere_amd.ops import add_layer_norm, layer_norm

    C.ln_bwd_config(variant, 0)
    try:
        _ln_check(D, with_res)
    finally:
        C.ln_bwd_config(3, 0)


def _ln_check(D, with_res):
    from cluster_anywhere_amd.ops import add_layer_norm, layer_norm

    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(4, 37, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    g = (1 + 0.1 * torch.randn(D, device=dev)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(D, device=dev)).bfloat16().requires_grad_()
    if with_res:
        s, y = add_layer_norm(x, r, g, b)
        dy, ds = torch.randn_like(y), torch.randn_like(s)
        (y * dy).sum().backward(retain_graph=True)
        (s * ds).sum().backward()
    else:
        y = layer_norm(x, g, b)
        dy = torch.randn_like(y)
        (y * dy).sum().backward()
    # fp32 reference
    xf = x.detach().float().requires_grad_()
    rf = r.detach().float().requires_grad_()
    gf = g.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_()
    sf = xf + rf if with_res else xf
    yf = F.layer_norm(sf, (D,), gf, bf, 1e-5)
    loss = (yf * dy.float()).sum()
    if with_res:
        loss = loss + (sf * ds.float()).sum()
    loss.backward()
    assert _rel(y, yf) < 1e-2
    assert _rel(x.grad, xf.grad) < 2e-2
    assert _rel(g.grad, gf.grad) < 2e-2
    assert _rel(b.grad, bf.grad) < 2e-2
    if with_res:
        assert _rel(s, sf) < 1e-2
        assert _rel(r.grad, rf.grad) < 2e-2


@pytest.mark.parametrize("shape", [(8, 64), (256, 6400), (1000, 3072)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_bias_gelu(C, shape, with_bias):
    from cluster_anywhere_amd.ops import bias_gelu

    torch.manual_seed(1)
    h = torch.randn(*shape, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(shape[-1], device="cuda", dtype=torch.bfloat16, requires_grad=True) if with_bias else None
    y = bias_gelu(h, b)
    dy = torch.randn_like(y)
    (y * dy).sum().backward()
    hf = h.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if with_bias else None
    yf = F.gelu(hf + (bf if with_bias else 0), approximate="tanh")
    (yf * dy.float()).sum().backward()
    assert _rel(y, yf) < 1e-2
    assert _rel(h.grad, hf.grad) < 2e-2
    if with_bias:
        assert _rel(b.grad, bf.grad) < 2e-2


@pytest.mark.parametrize("rows,V,stride", [(16, 50257, 50304), (7, 1000, 1000), (33, 129, 136)])
def test_cross_entropy(C, rows, V, stride):
    from cluster_anywhere_amd.ops import cross_entropy

    torch.manual_seed(2)
    logits = (3 * torch.randn(rows, stride, device="cuda")).bfloat16()
    tgt = torch.randint(0, V, (rows,), device="cuda")
    tgt[0] = -100  # ignored row
    lg = logits.clone().requires_grad_()
    loss = cross_entropy(lg, tgt, V)
    w = torch.rand(rows, device="cuda")
    (loss * w).sum().backward()
    lf = logits.float()[:, :V].clone().requires_grad_()
    ref = F.cross_entropy(lf, tgt, reduction="none", ignore_index=-100)
    (ref * w).sum().backward()
    assert torch.allclose(loss, ref, atol=2e-2, rtol=1e-2)
    assert _rel(lg.grad[:, :V], lf.grad) < 2e-2
    if V < stride:
        assert lg.grad[:, V:].abs().max().item() == 0
    assert lg.grad[0].abs().max().item() == 0


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_adamw_matches_reference(C, variant):
    """variant: bit 0 non-temporal loads/stores, bit 1 two vectors per thread."""
    C.adamw_config(variant)
    try:
        _adamw_check()
    finally:
        C.adamw_config(2)  # the default (adamw.hip g_adam_variant)


def _adamw_check():
    from cluster_anywhere_amd.ops.optim import FusedAdamW

    torch.manual_seed(3)

    class Space:
        pass

    n = 4096 + 64
    outs = []
    for dev in ["cuda", "cpu"]:
        sp = Space()
        gen = torch.Generator().manual_seed(5)
        sp.master = torch.randn(n, generator=gen).to(dev)
        sp.grad_buffer = torch.randn(n, generator=gen).to(dev).bfloat16()
        sp.param_buffer = sp.master.bfloat16()
        sp.wd_mask = (torch.arange(n // 8) % 3 == 0).to(torch.uint8).to(dev)
        opt = FusedAdamW(sp, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
        for _ in range(3):
            opt.step(inv_world=0.5)
        outs.append((sp.master.cpu(), sp.param_buffer.float().cpu(), opt.exp_avg_sq.cpu()))
    (pg, bg, vg), (pc, bc, vc) = outs
    assert torch.allclose(pg, pc, atol=1e-5, rtol=1e-4)
    assert torch.allclose(vg, vc, atol=1e-7, rtol=1e-4)
    assert torch.allclose(bg, pc.bfloat16().float(), atol=1e-2)


def test_gae_vtrace(C):
    from cluster_anywhere_amd.ops.rl import gae, gae_ref, vtrace, vtrace_ref

    torch.manual_seed(4)
    T, B = 64, 300
    r = torch.randn(T, B, device="cuda")
    v = torch.randn(T + 1, B, device="cuda")
    nt = (torch.rand(T, B, device="cuda") > 0.05).float()
    a, t = gae(r, v, nt, 0.99, 0.95)
    ar, tr = gae_ref(r.cpu(), v.cpu(), nt.cpu(), 0.99, 0.95)
    assert torch.allclose(a.cpu(), ar, atol=1e-4)
    assert torch.allclose(t.cpu(), tr, atol=1e-4)
    lr = 0.3 * torch.randn(T, B, device="cuda")
    d = 0.99 * nt
    vals = v[:T].contiguous()
    boot = v[T].contiguous()
    vs, pg = vtrace(lr, d, r, vals, boot, 1.0, 1.0)
    vsr, pgr = vtrace_ref(lr.cpu(), d.cpu(), r.cpu(), vals.cpu(), boot.cpu(), 1.0, 1.0)
    assert torch.allclose(vs.cpu(), vsr, atol=1e-4)
    assert torch.allclose(pg.cpu(), pgr, atol=1e-4)


def test_gpt2_train_step_gpu():
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.train.loop import DataParallelStep

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    m = GPT2(cfg).cuda()
    st = DataParallelStep(m, lr=1e-3)
    x = torch.randint(0, cfg.vocab_size, (4, 65), device="cuda")
    first = st(x[:, :-1], x[:, 1:]).item()
    for _ in range(30):
        last = st(x[:, :-1], x[:, 1:]).item()
    assert last < first - 1.0, (first, last)


def test_main_grad_path_matches_autograd():
    """Fused main-grad linears + flat buffer == plain autograd gradients."""
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config
    from cluster_anywhere_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    ref = GPT2(cfg).cuda().bfloat16()
    fused = GPT2(cfg).cuda()
    fused.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    flat = FlatParamSpace(fused, dtype=torch.bfloat16)
    x = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda")
    ref(x[:, :-1], x[:, 1:]).backward()
    flat.zero_grad()
    fused(x[:, :-1], x[:, 1:]).backward()
    for (n, p), (_, q) in zip(ref.named_parameters(), fused.named_parameters()):
        assert _rel(q.main_grad, p.grad) < 3e-2, (n, _rel(q.main_grad, p.grad))


def test_gpt2_gpu_matches_fp32_reference_loss():
    """bf16 model on GPU (HIP kernels) vs fp32 CPU reference: same initial loss."""
    from cluster_anywhere_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    m = GPT2(cfg)
    x = torch.randint(0, cfg.vocab_size, (2, 65))
    ref = m(x[:, :-1], x[:, 1:]).item()
    mg = GPT2(cfg)
    mg.load_state_dict(m.state_dict())
    mg = mg.cuda().bfloat16()
    got = mg(x[:, :-1].cuda(), x[:, 1:].cuda()).item()
    assert abs(got - ref) < 0.05 * abs(ref), (got, ref)


@pytest.mark.parametrize(
    "B,T,H,D,causal",
    [(2, 128, 3, 64, True), (1, 1024, 25, 64, True), (2, 256, 2, 128, True),
     (1, 100, 2, 64, True), (2, 192, 2, 64, False), (1, 77, 1, 128, False)],
)
def test_flash_attention_fwd_bwd(C, B, T, H, D, causal):
    from cluster_anywhere_amd.ops.attention import attention_ref
    from cluster_anywhere_amd.ops.flash import flash_attention_lse, flash_attention_qkv

    torch.manual_seed(7)
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    out = flash_attention_qkv(qkv, H, causal)
    dout = torch.randn_like(out)
    out.backward(dout)
    qf = qkv.detach().float().requires_grad_()
    q, k, v = qf.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    ref = attention_ref(q, k, v, causal)  # [B, H, T, D] fp32
    ref_o = ref.transpose(1, 2).reshape(B, T, H * D)
    ref_o.backward(dout.float())
    assert _rel(out, ref_o) < 2e-2, _rel(out, ref_o)
    g, gr = qkv.grad.view(B, T, 3, H, D), qf.grad.view(B, T, 3, H, D)
    for i, name in enumerate("qkv"):
        assert _rel(g[:, :, i], gr[:, :, i]) < 3e-2, (name, _rel(g[:, :, i], gr[:, :, i]))
    _, lse = flash_attention_lse(qkv.detach(), H, causal)
    s = (q.detach() @ k.detach().transpose(-1, -2)) / D ** 0.5
    if causal:
        s = s.masked_fill(~torch.ones(T, T, dtype=torch.bool, device="cuda").tril(), float("-inf"))
    assert torch.allclose(lse, torch.logsumexp(s, -1), atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("B,T,H,causal,amp,D", [(2, 512, 2, True, 3.0, 64), (1, 320, 3, False, 3.0, 64),
                                                 (1, 1024, 2, True, 6.0, 64), (2, 512, 2, True, 2.0, 128),
                                                 (1, 333, 2, False, 2.0, 128)])
def test_flash_attention_d64_spiky(C, B, T, H, causal, amp, D):
    """Large-magnitude scores, so the second-generation forward's lazy softmax
    rescale (raise the reference max only when it grows by > 8 in log2 units) fires
    on many tiles; keys are scaled up along the sequence so later tiles keep raising
    the max. D = 128 covers the head-dim-128 forward (fwd128_kernel)."""
    from cluster_anywhere_amd.ops.attention import attention_ref
    from cluster_anywhere_amd.ops.flash import flash_attention_qkv

    torch.manual_seed(11)
    x = torch.randn(B, T, 3, H, D, device="cuda")
    ramp = torch.linspace(0.5, 2.0, T, device="cuda").view(1, T, 1, 1)
    x[:, :, 1] = x[:, :, 1] * ramp + 0.5          # keys grow along the sequence
    x[:, :, 0] = x[:, :, 0].abs() * amp / 2 + 0.5  # positive-leaning queries
    qkv = x.reshape(B, T, 3 * H * D).bfloat16().requires_grad_()
    out = flash_attention_qkv(qkv, H, causal)
    dout = torch.randn_like(out)
    out.backward(dout)
    qf = qkv.detach().float().requires_grad_()
    q, k, v = qf.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    ref_o = attention_ref(q, k, v, causal).transpose(1, 2).reshape(B, T, H * D)
    ref_o.backward(dout.float())
    assert _rel(out, ref_o) < 2e-2, _rel(out, ref_o)
    g, gr = qkv.grad.view(B, T, 3, H, D), qf.grad.view(B, T, 3, H, D)
    for i, name in enumerate("qkv"):
        assert _rel(g[:, :, i], gr[:, :, i]) < 4e-2, (name, _rel(g[:, :, i], gr[:, :, i]))


@pytest.mark.parametrize("T,causal", [(1024, True), (200, True), (333, False)])
def test_flash_bwd_qkv_bias_grad(C, T, causal):
    """The D = 64 backward's bias-gradient epilogue equals the column sums of the
    dqkv it writes (fp32 reference: sum of the stored bf16 gradient)."""
    torch.manual_seed(7)
    B, H, D = 2, 5, 64
    qkv = (torch.randn(B, T, 3 * H * D, device="cuda") * 0.5).bfloat16()
    out, lse = C.flash_attn_fwd(qkv, H, causal)
    dout = torch.randn_like(out)
    db = torch.zeros(3 * H * D, device="cuda")
    dqkv = C.flash_attn_bwd(qkv, out, dout, lse, H, causal, db)
    ref = dqkv.float().reshape(-1, 3 * H * D).sum(0)
    assert _rel(db, ref) < 1e-2
    dqkv2 = C.flash_attn_bwd(qkv, out, dout, lse, H, causal)
    assert torch.equal(dqkv, dqkv2)


def test_gpt2_fused_qkv_bias_grad_matches(monkeypatch):
    """GPT-2 block grads in the flat main-grad buffer: qkv bias gradient from the
    attention backward and proj / fc2 bias gradients from the LayerNorm backward ==
    the linears' own column-sum passes."""
    import cluster_anywhere_amd.models.gpt2 as G
    from cluster_anywhere_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(3)
    cfg = G.GPT2Config(n_layer=2, n_head=5, n_embd=320, n_positions=256, vocab_size=1000)
    x = torch.randint(0, cfg.vocab_size, (4, 257), device="cuda")
    grads = []
    for fused in (True, False):
        torch.manual_seed(3)
        m = G.GPT2(cfg).cuda()
        flat = FlatParamSpace(m, dtype=torch.bfloat16)
        monkeypatch.setattr(G, "_FUSED_QKV_BGRAD", True)  # the opt-in qkv path too
        if not fused:
            monkeypatch.setattr(G, "flash_path", lambda *a: False)
            monkeypatch.setattr(G, "ln_bias_fusion_ok", lambda *a: False)
        flat.zero_grad()
        m(x[:, :-1], x[:, 1:]).backward()
        grads.append({n: p.main_grad.float().clone() for n, p in m.named_parameters()})
    for n in grads[0]:
        assert _rel(grads[0][n], grads[1][n]) < 2e-2, n


@pytest.mark.parametrize("d,layers,batch", [(320, 2, 4), (1600, 1, 16)])
def test_gpt2_fc2_transposed_storage(d, layers, batch, monkeypatch):
    """fc2 weight stored transposed (default): same loss and gradients as the plain
    layout; at d = 1600 with 16k tokens its weight gradient runs on gemm.hip's
    split-K kernel (the 6400 x 1600 shape) into the transposed main-grad view."""
    import cluster_anywhere_amd.models.gpt2 as G
    from cluster_anywhere_amd.ops import gemm as _g
    from cluster_anywhere_amd.parallel.flat import FlatParamSpace

    cfg = G.GPT2Config(n_layer=layers, n_head=d // 64, n_embd=d, n_positions=1024, vocab_size=1000)
    torch.manual_seed(5)
    x = torch.randint(0, cfg.vocab_size, (batch, 1025 if d == 1600 else 257), device="cuda")
    state, out = None, []
    for t in (False, True):
        monkeypatch.setattr(G, "_FC2_T", t)
        torch.manual_seed(5)
        m = G.GPT2(cfg).cuda()
        assert m.blocks[0].fc2_w.is_contiguous() != t
        if state is None:
            state = {k: v.detach().clone() for k, v in m.state_dict().items()}
        else:
            m.load_state_dict(state)
        flat = FlatParamSpace(m, dtype=torch.bfloat16)
        flat.zero_grad()
        loss = m(x[:, :-1], x[:, 1:])
        loss.backward()
        out.append((loss.item(), {n: p.main_grad.float().clone() for n, p in m.named_parameters()}))
        if t and d == 1600:
            assert _g.wgrad_runs(4 * d, d, batch * 1024) is not None  # the gemm.hip path ran
    assert abs(out[0][0] - out[1][0]) < 1e-2
    for n in out[0][1]:
        assert _rel(out[0][1][n], out[1][1][n]) < 2e-2, n


@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_bwd_dxsum(C, with_res):
    """The LayerNorm backward's extra output: column sums of dx accumulated into a
    bf16 vector (the residual-branch producer's bias gradient)."""
    torch.manual_seed(8)
    rows, D = 777, 1600
    x = torch.randn(rows, D, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = torch.zeros(D, device="cuda").bfloat16()
    y, mean, rstd, s = C.layernorm_fwd(x, None, g, b, 1e-5)
    dy = torch.randn_like(x)
    dres = torch.randn_like(x) if with_res else None
    assert C.ln_bwd_dxsum_ok(D)
    acc = torch.full((D,), 0.5, device="cuda").bfloat16()
    dx, dg, db = C.layernorm_bwd(dy, x, g, mean, rstd, dres, acc)
    dx2, dg2, db2 = C.layernorm_bwd(dy, x, g, mean, rstd, dres)
    assert torch.equal(dx, dx2) and torch.equal(dg, dg2) and torch.equal(db, db2)
    ref = dx.float().sum(0) + 0.5
    assert _rel(acc, ref) < 1e-2


@pytest.mark.parametrize("with_dxsum", [False, True])
def test_layernorm_bwd_into_main_grads(C, with_dxsum):
    """g_main / b_main: the weight and bias gradients are added into the given bf16
    main-grad vectors in the same launch (and come back as None); the result equals
    the plain backward's dg / db added to the prior contents."""
    torch.manual_seed(9)
    rows, D = 777, 1600
    x = torch.randn(rows, D, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = torch.zeros(D, device="cuda").bfloat16()
    y, mean, rstd, s = C.layernorm_fwd(x, None, g, b, 1e-5)
    dy = torch.randn_like(x)
    gm = torch.full((D,), 0.25, device="cuda").bfloat16()
    bm = torch.full((D,), -0.5, device="cuda").bfloat16()
    acc = torch.zeros(D, device="cuda").bfloat16() if with_dxsum else None
    dx, dg, db = C.layernorm_bwd(dy, x, g, mean, rstd, None, acc, gm, bm)
    assert dg is None and db is None
    dx2, dg2, db2 = C.layernorm_bwd(dy, x, g, mean, rstd, None)
    assert torch.equal(dx, dx2)
    assert _rel(gm, dg2.float() + 0.25) < 1e-2 and _rel(bm, db2.float() - 0.5) < 1e-2
    ref_g = ((x.float() - mean[:, None]) * rstd[:, None] * dy.float()).sum(0)
    assert _rel(gm, ref_g + 0.25) < 2e-2 and _rel(bm, dy.float().sum(0) - 0.5) < 2e-2


def test_drain_f32_into_bf16(C):
    """drain_f32_: bf16 destination += fp32 source, and the source is left zeroed."""
    torch.manual_seed(10)
    src = torch.randn(6400, device="cuda")
    dst = torch.randn(6400, device="cuda").bfloat16()
    ref = dst.float() + src
    C.drain_f32_(src, dst)
    assert _rel(dst, ref) < 1e-2 and int((src != 0).sum()) == 0


@pytest.mark.parametrize("rows,N", [(32768, 1600), (1000, 72), (31, 8)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_bias_grad_rowsum(C, rows, N, accumulate):
    """bias_grad_: column sums of dy (32-row fp32 slab partials + column reduce) vs an
    fp32 torch sum; accumulate adds into the existing bf16 gradient."""
    torch.manual_seed(0)
    dy = torch.randn(rows, N, device="cuda").to(torch.bfloat16)
    out = torch.randn(N, device="cuda").to(torch.bfloat16)
    ref = dy.float().sum(0) + (out.float() if accumulate else 0.0)
    C.bias_grad_(dy, out, accumulate)
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2 * max(1.0, rows ** 0.5 / 10))


@pytest.mark.parametrize("B,T,H", [(2, 1024, 5), (1, 200, 3), (2, 640, 2), (1, 64, 2)])
def test_flash_bwd_paired_dkdv_bit_exact(C, B, T, H):
    """The paired-key-block dK/dV kernel (one workgroup walks key blocks j and
    nkb-1-j as one tile stream) adds every key's contributions in the same tile
    order as the one-block-per-key-block kernel: dqkv bit-identical (odd and even
    key-block counts, partial last blocks, a single block)."""
    torch.manual_seed(11)
    D = 64
    qkv = (torch.randn(B, T, 3 * H * D, device="cuda") * 0.7).bfloat16()
    out, lse = C.flash_attn_fwd(qkv, H, True)
    dout = torch.randn_like(out)
    try:
        C.fa64_set_pair(1)
        paired = C.flash_attn_bwd(qkv, out, dout, lse, H, True)
        C.fa64_set_pair(0)
        single = C.flash_attn_bwd(qkv, out, dout, lse, H, True)
    finally:
        C.fa64_set_pair(1)
    assert torch.equal(paired, single)
