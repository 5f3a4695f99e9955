"""RLlib learner kernels (csrc/kernels/rl_encoder.hip) against fp32 PyTorch references:
the MFMA GEMM in its three layouts and six epilogues, im2col / col2im, the
Nature-CNN encoder forward+backward, the tanh MLP encoder and the fused PPO loss."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too; every test is gpu-marked
    pytest.skip("needs an MI355X", allow_module_level=True)

from cluster_anywhere_amd.ops import kernels  # noqa: E402
from cluster_anywhere_amd.ops import rl_encoder as R  # noqa: E402

DEV = torch.device("cuda")


def _rel(a, b):
    return float((a.detach().float() - b.detach().float()).norm() / (b.detach().float().norm() + 1e-12))


@pytest.mark.parametrize("M,N,K", [(1000, 32, 256), (333, 64, 576), (500, 512, 3136), (64, 40, 96)])
@pytest.mark.parametrize("epi", [R.RE_BF16, R.RE_BIAS_RELU, R.RE_BIAS_TANH])
def test_rl_gemm_forward_layout(M, N, K, epi):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16() / math.sqrt(K)
    bias = torch.randn(N, device=DEV).bfloat16()
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    kernels().rl_gemm(a, b, c, 0, epi, bias, None, M, N, K, K, K, N, 1)
    ref = a.float() @ b.float().t() + bias.float()
    ref = {R.RE_BF16: ref, R.RE_BIAS_RELU: ref.relu(), R.RE_BIAS_TANH: ref.tanh()}[epi]
    assert _rel(c, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(777, 576, 64), (500, 3136, 512), (200, 32, 64)])
@pytest.mark.parametrize("epi", [R.RE_BF16, R.RE_DRELU, R.RE_DTANH])
def test_rl_gemm_dgrad_layout(M, N, K, epi):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16() / math.sqrt(K)
    aux = torch.randn(M, N, device=DEV).tanh().bfloat16()
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    kernels().rl_gemm(a, b, c, 1, epi, None, aux, M, N, K, K, N, N, 1)
    ref = a.float() @ b.float()
    if epi == R.RE_DRELU:
        ref = ref * (aux.float() > 0)
    elif epi == R.RE_DTANH:
        ref = ref * (1 - aux.float() ** 2)
    assert _rel(c, ref) < 1e-2


@pytest.mark.parametrize("rows,n_out,k_in,splits", [(20000, 32, 256, 10), (4050, 64, 512, 2), (500, 512, 3136, 1)])
def test_rl_gemm_wgrad_split_atomic(rows, n_out, k_in, splits):
    torch.manual_seed(2)
    dz = torch.randn(rows, n_out, device=DEV).bfloat16()
    x = torch.randn(rows, k_in, device=DEV).bfloat16()
    dw = torch.full((n_out, k_in), 0.5, device=DEV)  # accumulates on top
    kernels().rl_gemm(dz, x, dw, 2, R.RE_F32_ATOMIC, None, None, n_out, k_in, rows, n_out, k_in, k_in, splits)
    ref = dz.float().t() @ x.float() + 0.5
    assert _rel(dw, ref) < 5e-3


def test_rl_gemm_rejects_bad_shapes():
    a = torch.randn(10, 12, device=DEV).bfloat16()  # K=12 not a multiple of 8
    b = torch.randn(16, 12, device=DEV).bfloat16()
    c = torch.empty(10, 16, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        kernels().rl_gemm(a, b, c, 0, 0, None, None, 10, 16, 12, 12, 12, 16, 1)
    with pytest.raises(RuntimeError):  # operand smaller than M*lda claims
        kernels().rl_gemm(a, b, c, 0, 0, None, None, 20, 16, 8, 8, 8, 16, 1)


@pytest.mark.parametrize("B,H,W,C,k,s", [(3, 84, 84, 4, 8, 4), (2, 20, 20, 32, 4, 2), (2, 9, 9, 64, 3, 1)])
def test_im2col_col2im(B, H, W, C, k, s):
    torch.manual_seed(3)
    if C == 4:
        x = torch.randint(0, 256, (B, H, W, C), device=DEV, dtype=torch.uint8)
        xf = x.float() / 255.0
        scale = 1 / 255.0
    else:
        x = torch.randn(B, H, W, C, device=DEV).bfloat16()
        xf, scale = x.float(), 1.0
    oh, ow = (H - k) // s + 1, (W - k) // s + 1
    col = torch.empty(B * oh * ow, k * k * C, device=DEV, dtype=torch.bfloat16)
    kernels().rl_im2col(x, col, k, k, s, scale)
    # reference: unfold on NCHW gives [B, C*k*k, L] ordered (c, kh, kw); reorder to (kh, kw, c)
    u = F.unfold(xf.permute(0, 3, 1, 2), k, stride=s).view(B, C, k, k, oh * ow)
    ref = u.permute(0, 4, 2, 3, 1).reshape(B * oh * ow, k * k * C)
    assert _rel(col, ref) < 5e-3
    if C % 8:
        return
    dcol = torch.randn_like(col, dtype=torch.float32).bfloat16()
    y = torch.randn(B, H, W, C, device=DEV).bfloat16()
    dz = torch.empty(B, H, W, C, device=DEV, dtype=torch.bfloat16)
    kernels().rl_col2im(dcol, y, dz, k, k, s, 1)
    d = dcol.float().view(B, oh * ow, k, k, C).permute(0, 4, 2, 3, 1).reshape(B, C * k * k, oh * ow)
    ref = F.fold(d, (H, W), k, stride=s).permute(0, 2, 3, 1) * (y.float() > 0)
    assert _rel(dz, ref) < 1e-2


def _nature_params(seed=0, in_ch=4):
    from cluster_anywhere_amd.rllib.core.rl_module import NatureCNN

    torch.manual_seed(seed)
    return NatureCNN(in_ch).to(DEV)


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def _nature_bf16_emulation(x, ps):
    """fp32 torch with bf16 rounding of weights, activations and activation grads."""
    bf = lambda t: t.bfloat16().float()  # noqa: E731
    B = x.shape[0]
    shapes, _ = R.nature_shapes(*x.shape[1:])
    y = bf(x.float() / 255.0).permute(0, 3, 1, 2)
    for li, (h, w, cin, cout, k, s, oh, ow) in enumerate(shapes):
        wgt = bf(ps[2 * li]).view(cout, k, k, cin).permute(0, 3, 1, 2)
        y = _RoundGrad.apply(bf(F.relu(F.conv2d(y, wgt, bf(ps[2 * li + 1]), stride=s))))
    y = y.permute(0, 2, 3, 1).reshape(B, -1)
    return _RoundGrad.apply(bf(F.relu(F.linear(y, bf(ps[6]), bf(ps[7])))))


def test_nature_cnn_forward_backward_vs_fp32_torch():
    enc = _nature_params()
    x = torch.randint(0, 256, (16, 84, 84, 4), device=DEV, dtype=torch.uint8)
    ps = enc.params()
    out = R.nature_cnn(x, ps)
    g = torch.randn_like(out)
    grads = torch.autograd.grad((out * g).sum(), ps)
    ref = R.nature_cnn_ref(x, ps)
    rgrads = torch.autograd.grad((ref * g).sum(), ps)
    assert out.shape == (16, 512)
    assert _rel(out, ref) < 2e-2
    # vs fp32: bf16 activations / gradients cost ~4-9% relative error on this random
    # (heavily cancelling) gradient; the same rounding emulated in fp32 torch shows it
    names = ["w1", "b1", "w2", "b2", "w3", "b3", "wf", "bf"]
    for name, a, b in zip(names, grads, rgrads):
        assert _rel(a, b) < 0.15, name
        assert F.cosine_similarity(a.flatten(), b.flatten(), dim=0) > 0.985, name
    # vs the bf16-rounding emulation (same rounding points as the kernels): tight
    emu = _nature_bf16_emulation(x, ps)
    egrads = torch.autograd.grad((emu * g).sum(), ps)
    assert _rel(out, emu) < 5e-3
    for name, a, b in zip(names, grads, egrads):
        assert _rel(a, b) < 0.05, name
    # accumulate-into-.grad mode (the learner's flat gradient buffer) gives the same result
    for p, a in zip(ps, grads):
        p.grad = torch.full_like(p, 0.25)
    with R.accumulate_into_grad():
        (R.nature_cnn(x, ps) * g).sum().backward()
    for p, a in zip(ps, grads):
        assert torch.allclose(p.grad - 0.25, a, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("M,N", [(200000, 32), (40500, 64), (500, 512), (37, 2048)])
def test_colsum(M, N):
    x = torch.randn(M, N, device=DEV).bfloat16()
    db = torch.full((N,), 1.0, device=DEV)
    kernels().rl_colsum(x, db)
    assert torch.allclose(db, x.float().sum(0) + 1.0, rtol=1e-3, atol=1e-2 * math.sqrt(M / 100 + 1))


def test_mlp_tanh_forward_backward_vs_fp32_torch():
    from cluster_anywhere_amd.rllib.core.rl_module import TanhMLP

    torch.manual_seed(4)
    mlp = TanhMLP([16, 256, 256]).to(DEV)
    assert mlp.kernel_ok
    x = torch.randn(300, 16, device=DEV)
    ps = list(mlp.ws)
    out = R.mlp_tanh(x, ps)
    g = torch.randn_like(out)
    grads = torch.autograd.grad((out * g).sum(), ps)
    ref = R.mlp_tanh_ref(x, ps)
    rgrads = torch.autograd.grad((ref * g).sum(), ps)
    assert _rel(out, ref) < 2e-2
    for a, b in zip(grads, rgrads):
        assert _rel(a, b) < 4e-2


@pytest.mark.parametrize("A", [2, 6, 18])
def test_fused_ppo_loss_matches_autograd(A):
    torch.manual_seed(5)
    B = 500
    logits = torch.randn(B, A, device=DEV, requires_grad=True)
    vf = torch.randn(B, device=DEV, requires_grad=True)
    old_logits = logits.detach() + 0.3 * torch.randn(B, A, device=DEV)
    actions = torch.randint(0, A, (B,), device=DEV)
    old_logp = old_logits.log_softmax(-1).gather(-1, actions[:, None]).squeeze(-1)
    adv = torch.randn(B, device=DEV)
    vt = vf.detach() + torch.randn(B, device=DEV) * 3
    args = (actions, old_logp, adv, vt, old_logits, 0.2, 4.0, 0.5, 0.01, 0.3)
    loss, st = R.ppo_loss_categorical(logits, vf, *args)
    gl, gv = torch.autograd.grad(loss, [logits, vf])
    rloss, rst = R.ppo_loss_categorical_ref(logits, vf, *args)
    rgl, rgv = torch.autograd.grad(rloss, [logits, vf])
    assert abs(float(loss) - float(rloss)) < 1e-4 * max(1.0, abs(float(rloss)))
    assert torch.allclose(st, rst, rtol=1e-4, atol=1e-3)
    assert _rel(gl, rgl) < 1e-4 and _rel(gv, rgv) < 1e-4


def test_ppo_fakeatari_learner_runs_on_kernels():
    from cluster_anywhere_amd import rllib

    cfg = (rllib.PPOConfig().environment("FakeAtari-v0")
           .env_runners(num_envs_per_env_runner=2, rollout_fragment_length=64)
           .learners(num_gpus_per_learner=1)
           .training(train_batch_size=128, minibatch_size=64, num_epochs=2, lr=2.5e-4, entropy_coeff=0.01)
           .debugging(seed=0))
    algo = cfg.build()
    assert algo.learner_group.local.device.type == "cuda"
    r1 = algo.train()
    r2 = algo.train()
    st = r2["learners"]["default_policy"]
    assert all(math.isfinite(v) for v in st.values())
    # weights moved and are synced to the (CPU, reference-path) runner
    w_gpu = algo.learner_group.get_module_state()
    w_cpu = algo.env_runner_group.local.module.get_state()
    for k in w_gpu:
        assert torch.equal(w_gpu[k], w_cpu[k])
    algo.stop()


def test_graphed_learner_step_matches_eager():
    from cluster_anywhere_amd.rllib.algorithms.ppo import PPOConfig, PPOLearner
    from cluster_anywhere_amd.rllib.env import make_env

    env = make_env("FakeAtari-v0")
    cfg = PPOConfig().environment("FakeAtari-v0").training(lr=1e-3, entropy_coeff=0.01).debugging(seed=3)
    fac = cfg.module_factory()
    learners = []
    for graph in (True, False):
        d = dict(cfg.learner_config(), learner_cuda_graph=graph)
        learners.append(PPOLearner(d, fac, env.observation_space, env.action_space, device="cuda"))
    g = torch.Generator().manual_seed(0)
    n = 256
    batch = {"obs": torch.randint(0, 256, (n, 84, 84, 4), generator=g, dtype=torch.uint8),
             "actions": torch.randint(0, env.action_space.n, (n,), generator=g),
             "action_logp": -torch.rand(n, generator=g) * 2,
             "action_dist_inputs": torch.randn(n, env.action_space.n, generator=g),
             "advantages": torch.randn(n, generator=g), "value_targets": torch.randn(n, generator=g)}
    stats = [lrn.update(batch, minibatch_size=64, num_epochs=2, shuffle=False) for lrn in learners]
    assert learners[0]._graphs and not learners[1]._graphs  # the first one really replayed graphs
    for k in stats[1]:
        assert abs(stats[0][k] - stats[1][k]) <= 1e-3 * max(1.0, abs(stats[1][k])), k
    s0, s1 = learners[0].get_module_state(), learners[1].get_module_state()
    for k in s0:
        assert torch.allclose(s0[k], s1[k], rtol=1e-3, atol=1e-5), k
    # the adaptive KL coefficient reaches the captured graph through device memory
    for lrn in learners:
        lrn.update_kl(1.0)
    stats = [lrn.update(batch, minibatch_size=64, num_epochs=1, shuffle=False) for lrn in learners]
    assert abs(stats[0]["total_loss"] - stats[1]["total_loss"]) <= 1e-3 * max(1.0, abs(stats[1]["total_loss"]))
