"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs fp32 torch.matmul: every
layout x tile x pipeline variant, every fused epilogue, and the linear / MLP
autograd paths that use them (rows/cols asymmetric so a transposed store fails)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _mk(shape, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(*shape, device="cuda", generator=g).bfloat16()


@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("tile", [(256, 256), (256, 320), (128, 320)])
@pytest.mark.parametrize("algo", [0, 1, 2, 3, 4])
def test_gemm_layouts(layout, tile, algo):
    from cluster_anywhere_amd.ops.gemm import gemm

    bm, bn = tile
    M, N, K = 2 * bm, 3 * bn, 448  # 7 K-tiles: odd count exercises the pipeline tails
    if layout == 0:
        a, b = _mk((M, K), 1), _mk((N, K), 2)
        ref = a.float() @ b.float().t()
    elif layout == 1:
        a, b = _mk((M, K), 1), _mk((K, N), 2)
        ref = a.float() @ b.float()
    else:
        a, b = _mk((K, M), 1), _mk((K, N), 2)
        ref = a.float().t() @ b.float()
    c = gemm(a, b, layout, algo=algo, tile=tile)
    assert _rel(c, ref) < 5e-3


def test_gemm_short_k():
    from cluster_anywhere_amd.ops.gemm import gemm

    for K in (64, 128, 192):  # fewer K-steps than the prefetch distance
        a, b = _mk((256, K), 3), _mk((320, K), 4)
        for algo in (3, 9):
            assert _rel(gemm(a, b, 0, algo=algo), a.float() @ b.float().t()) < 5e-3


def test_fused_epilogues():
    from cluster_anywhere_amd.ops import gemm as G

    M, K, N = 512, 640, 960
    x, w = _mk((M, K), 5), _mk((N, K), 6) * 0.05
    b = _mk((N,), 7)
    y = G.linear_nt(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    assert _rel(y, ref) < 5e-3
    u, z = G.linear_gelu(x, w, b)
    zr = ref.bfloat16()
    assert _rel(z, ref) < 5e-3
    assert _rel(u, F.gelu(zr.float(), approximate="tanh")) < 1e-2
    # dgrad with GELU' and the bias-gradient column sums
    dy = _mk((M, K), 8)  # gradient w.r.t. an fc2 output of width K, fc2 weight w2 [K, N]
    w2 = _mk((K, N), 9) * 0.05
    db = torch.zeros(N, device="cuda")
    dz = G.dgrad_dgelu(dy, G.transpose(w2), z, db)
    du = dy.float() @ w2.float()
    zf = z.float()
    t = torch.tanh(0.7978845608028654 * (zf + 0.044715 * zf ** 3))
    gp = 0.5 * (1 + t) + 0.5 * zf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * zf * zf)
    dzr = du * gp
    assert _rel(dz, dzr) < 1e-2
    assert _rel(db, dzr.sum(0)) < 1e-2
    assert torch.equal(G.transpose(w2), w2.t().contiguous())


def test_linear_and_mlp_autograd_match_reference():
    from cluster_anywhere_amd.ops.linear import linear, mlp
    from cluster_anywhere_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)

    class M(torch.nn.Module):
        def __init__(s):
            super().__init__()
            s.w1 = torch.nn.Parameter(torch.randn(1280, 640) * 0.03)
            s.b1 = torch.nn.Parameter(torch.randn(1280) * 0.1)
            s.w2 = torch.nn.Parameter(torch.randn(640, 1280) * 0.03)
            s.b2 = torch.nn.Parameter(torch.randn(640) * 0.1)
            s.wq = torch.nn.Parameter(torch.randn(960, 640) * 0.03)
            s.bq = torch.nn.Parameter(torch.randn(960) * 0.1)

    m = M().cuda()
    ref = {k: v.detach().float().clone() for k, v in m.named_parameters()}
    flat = FlatParamSpace(m, dtype=torch.bfloat16)
    x = _mk((2, 256, 640), 11).requires_grad_()
    y = mlp(x, m.w1, m.b1, m.w2, m.b2)
    q = linear(x, m.wq, m.bq)
    dy, dq = _mk(y.shape, 12), _mk(q.shape, 13)
    (y.float() * dy.float()).sum().add((q.float() * dq.float()).sum()).backward()
    # fp32 reference
    xr = x.detach().float().requires_grad_()
    P = {k: v.clone().requires_grad_() for k, v in ref.items()}
    for k in P:  # the bf16 copies the kernels saw
        P[k] = getattr(m, k).detach().float().clone().requires_grad_()
    yr = F.gelu(xr @ P["w1"].t() + P["b1"], approximate="tanh") @ P["w2"].t() + P["b2"]
    qr = xr @ P["wq"].t() + P["bq"]
    ((yr * dy.float()).sum() + (qr * dq.float()).sum()).backward()
    assert _rel(y, yr) < 1e-2 and _rel(q, qr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    for s in flat.slots:
        assert _rel(s.param.main_grad, P[s.name].grad) < 2e-2, s.name


def test_fused_mlp_matches_unfused_reference():
    """GPT-2 MLP on the fused path (fc GEMM with bias+GELU epilogue, fc2 dgrad with
    GELU' + fc bias-grad epilogue, main-grad accumulation) vs an fp32 reference."""
    from cluster_anywhere_amd.ops import linear as L

    torch.manual_seed(3)
    M, d, f = 512, 320, 1280
    x = (torch.randn(M, d, device="cuda") * 0.5).bfloat16().requires_grad_()
    w1 = (torch.randn(f, d, device="cuda") * 0.05).bfloat16().requires_grad_()
    b1 = (torch.randn(f, device="cuda") * 0.1).bfloat16().requires_grad_()
    w2 = (torch.randn(d, f, device="cuda") * 0.05).bfloat16().requires_grad_()
    b2 = (torch.randn(d, device="cuda") * 0.1).bfloat16().requires_grad_()
    for p in (w1, b1, w2, b2):
        p.main_grad = torch.zeros_like(p)
    old = L._FUSED_MLP
    L._FUSED_MLP = True
    try:
        y = L.mlp(x, w1, b1, w2, b2)
    finally:
        L._FUSED_MLP = old
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, w1f, b1f, w2f, b2f = (t.detach().float().requires_grad_() for t in (x, w1, b1, w2, b2))
    yr = torch.nn.functional.gelu(xf @ w1f.t() + b1f, approximate="tanh") @ w2f.t() + b2f
    yr.backward(dy.float())
    assert _rel(y, yr) < 2e-2
    assert _rel(x.grad, xf.grad) < 3e-2
    for p, r in ((w1, w1f), (b1, b1f), (w2, w2f), (b2, b2f)):
        assert _rel(p.main_grad, r.grad) < 3e-2, (p.shape, _rel(p.main_grad, r.grad))
    # a second backward accumulates (the fc bias gradient's fp32 accumulator was drained
    # into b1.main_grad and left zeroed)
    L._FUSED_MLP = True
    try:
        L.mlp(x, w1, b1, w2, b2).backward(dy)
    finally:
        L._FUSED_MLP = old
    assert _rel(b1.main_grad, 2 * b1f.grad) < 3e-2


@pytest.mark.parametrize("algo", [9, 1009, 3009, 4009])
@pytest.mark.parametrize("K", [64, 128, 448, 1600])
def test_gemm_k64_variants(algo, K):
    """Full-line BK=64 kernel (NT only): every DMA-split / phase / L2-prefetch variant,
    K-tile counts 1, 2, 7 (odd: the double-buffer tail) and 25, vs fp32."""
    from cluster_anywhere_amd.ops.gemm import gemm

    M, N = 512, 960
    a, b = _mk((M, K), 21), _mk((N, K), 22)
    c = gemm(a, b, 0, algo=algo, tile=(256, 320))
    assert _rel(c, a.float() @ b.float().t()) < 5e-3


def test_gemm_k64_epilogues_and_dispatch():
    """The dispatcher sends NT GEMMs with max(N, K) >= 1536 to algo 4009; its bias,
    bias+GELU and dGELU+bias-grad epilogues vs fp32, and the result equals an explicit
    algo-4009 launch."""
    from cluster_anywhere_amd.ops import gemm as G
    from cluster_anywhere_amd.ops import kernels

    assert G.k64_ok(0, G.EPI_BF16, 256, 320, 4800, 1600) and G.k64_ok(0, G.EPI_BF16, 256, 320, 1600, 1600)
    assert not G.k64_ok(0, G.EPI_BF16, 256, 320, 1280, 1280)
    M, K, N = 512, 640, 4160  # N = 13 x 320 >= 4096
    x, w = _mk((M, K), 23), _mk((N, K), 24) * 0.05
    b = _mk((N,), 25)
    ref = x.float() @ w.float().t() + b.float()
    y = G.linear_nt(x, w, b)
    assert _rel(y, ref) < 5e-3
    c = torch.empty_like(y)
    kernels().gemm_bf16(x, w, c, 0, G.EPI_BF16, 256, 320, b, None, None, None, 1, None, False, 4009,
                        None, None, 0, 1)
    assert torch.equal(c, y)
    u, z = G.linear_gelu(x, w, b)
    assert _rel(z, ref) < 5e-3
    assert _rel(u, F.gelu(z.float(), approximate="tanh")) < 1e-2
    dy = _mk((M, K), 26)
    w2 = _mk((K, N), 27) * 0.05
    db = torch.zeros(N, device="cuda")
    dz = G.dgrad_dgelu(dy, G.transpose(w2), z, db)
    zf = z.float()
    t = torch.tanh(0.7978845608028654 * (zf + 0.044715 * zf ** 3))
    gp = 0.5 * (1 + t) + 0.5 * zf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * zf * zf)
    dzr = (dy.float() @ w2.float()) * gp
    assert _rel(dz, dzr) < 1e-2 and _rel(db, dzr.sum(0)) < 1e-2


def test_gemm_k64_split_tail():
    """K >= 4096 on algo 4009: the tiles past the last full round of CUs are split
    over K-slices (fp32 slabs + tickets), vs fp32 and vs the unsplit launch."""
    from cluster_anywhere_amd.ops import gemm as G
    from cluster_anywhere_amd.ops import kernels

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    M, N, K = 256 * 16, 320 * 20, 4800  # 320 tiles: one full round + a 64-tile tail on 256 CUs
    full, S = G.tail_plan(M, N, K, 256, 320, torch.device("cuda"), 4009)
    if cus == 256:
        assert S > 1, (full, S)
    a, b = _mk((M, K), 28), _mk((N, K), 29) * 0.05
    c = G.linear_nt(a, b)
    assert _rel(c, a.float() @ b.float().t()) < 5e-3
    c1 = torch.empty_like(c)
    kernels().gemm_bf16(a, b, c1, 0, G.EPI_BF16, 256, 320, None, None, None, None, 1, None, False, 4009,
                        None, None, 0, 1)
    assert _rel(c, c1) < 2e-3


@pytest.mark.parametrize("lockstep,ext", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("MN,runs", [((1600, 1600), 245), ((640, 960), 18), ((1600, 640), 56)])
def test_wgrad_stream_k_and_lockstep(lockstep, ext, MN, runs):
    """Weight-gradient kernel (algo 5, TN layout): dW (+)= dY^T X over 4096 tokens,
    ragged M (1600 = 6.25 x 256), stream-K order and the slice-major lockstep order
    (runs = tiles x slices, slices not dividing the 128 K-steps), overwrite and
    accumulate, vs fp32."""
    from cluster_anywhere_amd.ops import gemm as G

    M, N = MN
    K = 4096
    dy, x = _mk((K, M), 31), _mk((K, N), 32)
    ref = dy.float().t() @ x.float()
    old = G.WGRAD_LOCKSTEP, G.WGRAD_EXT
    G.WGRAD_LOCKSTEP, G.WGRAD_EXT = lockstep, ext
    try:
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        G.run_sk(dy, x, c, 2, False, runs)
        assert _rel(c, ref) < 5e-3
        c0 = _mk((M, N), 33)
        c2 = c0.clone()
        G.run_sk(dy, x, c2, 2, True, runs)
        assert _rel(c2, ref + c0.float()) < 5e-3
        c3 = torch.empty_like(c)
        G.run_sk(dy, x, c3, 2, False, runs)  # tickets were reset by the last arrivers
        assert torch.equal(c, c3)
    finally:
        G.WGRAD_LOCKSTEP, G.WGRAD_EXT = old


def test_wgrad_external_combine_matches_in_kernel_bits():
    """algo 15 (lockstep slabs + separate reduce launch) gives the same bits as the
    in-kernel last-arriver combine, for both the overwrite and accumulate epilogues."""
    from cluster_anywhere_amd.ops import gemm as G

    dy, x = _mk((8192, 1600), 41), _mk((8192, 1600), 42)
    c0 = _mk((1600, 1600), 43)
    out = {}
    old = G.WGRAD_EXT
    try:
        for ext in (True, False):
            G.WGRAD_EXT = ext
            a = torch.empty(1600, 1600, device="cuda", dtype=torch.bfloat16)
            G.run_sk(dy, x, a, 2, False, 245)
            b = c0.clone()
            G.run_sk(dy, x, b, 2, True, 245)
            out[ext] = (a, b)
    finally:
        G.WGRAD_EXT = old
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])


@pytest.mark.parametrize("inkernel", [True, False])
@pytest.mark.parametrize("bm", [256, 192])
@pytest.mark.parametrize("MN,slices", [((1600, 1600), 7), ((640, 960), 1), ((1600, 640), 3), ((960, 320), 2),
                                       ((4800, 1600), 2)])
def test_wgrad_tn64(bm, MN, slices, inkernel):
    """TN full-line weight-gradient kernel (algo 25): dW (+)= dY^T X over 4160 tokens
    (65 K-tiles: odd, and not divisible by the slice counts), ragged M (1600 = 6.25 x 256,
    8.33 x 192), single run per tile and lockstep split-K with the reduce launch,
    overwrite and accumulate, repeatable bits, vs fp32."""
    from cluster_anywhere_amd.ops import gemm as G

    M, N = MN
    K = 4160
    dy, x = _mk((K, M), 51), _mk((K, N), 52)
    ref = dy.float().t() @ x.float()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    G.run_tn(dy, x, c, False, bm, slices, inkernel)
    assert _rel(c, ref) < 5e-3
    c0 = _mk((M, N), 53)
    c2 = c0.clone()
    G.run_tn(dy, x, c2, True, bm, slices, inkernel)
    assert _rel(c2, ref + c0.float()) < 5e-3
    c3 = torch.empty_like(c)
    G.run_tn(dy, x, c3, False, bm, slices, inkernel)  # tickets were reset by the last arrivers
    assert torch.equal(c, c3)
    c4 = torch.empty_like(c)
    G.run_tn(dy, x, c4, False, bm, slices, not inkernel)  # both combines sum the slices in order
    assert torch.equal(c, c4)


def test_wgrad_tn64_strided_views_and_dispatch():
    """The TN kernel on the GPT-2-XL wgrad shapes it is planned for (fewer tokens), and
    through ops.linear._wgrad into a transposed main-grad view (fc2 storage)."""
    from cluster_anywhere_amd.ops import gemm as G

    K = 16384
    for (M, N) in ((6400, 1600), (4800, 1600), (1600, 1600)):
        plan = G.tn_plan(M, N, K)
        assert plan is not None
        dy, x = _mk((K, M), 61), _mk((K, N), 62)
        c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        G.run_tn(dy, x, c, True, *plan)
        assert _rel(c, dy.float().t() @ x.float()) < 5e-3


@pytest.mark.parametrize("M,K,N,bias", [(256, 64, 320, False), (512, 640, 320, True), (256, 4800, 1600, False),
                                        (768, 1600, 640, True)])
def test_gemm_nn64_vs_fp32(M, K, N, bias):
    """NN kernel (TN schedule with a K-major A, gemm.hip algo 27): x [M, K] @ W [K, N]
    (+ bias) with W read as stored, vs fp32; and the dgrad routing through it equals the
    transpose + NT path within bf16 rounding."""
    from cluster_anywhere_amd.ops import gemm as G

    x, w = _mk((M, K), 31), _mk((K, N), 32) * 0.05
    b = _mk((N,), 33) if bias else None
    ref = x.float() @ w.float() + (b.float() if bias else 0.0)
    y = G.linear_nn64(x, w, b)
    assert _rel(y, ref) < 5e-3
    # dgrad: dx = dy @ Wl for an nn.Linear weight Wl [N_out = K, K_in = N]
    y2 = G.dgrad_w(x, w)
    assert _rel(y2, x.float() @ w.float()) < 5e-3
    y3 = G.dgrad(x, G.transpose(w))
    assert _rel(y2, y3.float()) < 5e-3


def test_gemm_nn64_rejects_bad_shapes():
    from cluster_anywhere_amd.ops import kernels

    x, w = _mk((200, 64), 1), _mk((64, 320), 2)
    c = torch.empty(200, 320, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        kernels().gemm_nn64(x, w, c, None)  # M % 256 != 0
