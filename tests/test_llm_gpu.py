"""gfx950 LLM-serving kernels vs fp32 PyTorch references, and the engine on
the GPU (HIP-graph decode == eager decode == dense forward)."""
import math

import pytest
import torch

from cluster_anywhere_amd.ops import llm as L

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.fixture(scope="module")
def C():
    from cluster_anywhere_amd.ops import kernels

    return kernels()


@pytest.mark.parametrize("D", [256, 2048, 4096, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(C, D, with_res):
    torch.manual_seed(0)
    x = torch.randn(3, 37, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x) if with_res else None
    w = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    y, s = C.rmsnorm(x, w, 1e-5, r)
    yr, sr = L.rms_norm_ref(x, w, 1e-5, r)
    assert _rel(y, yr) < 1e-2
    if with_res:
        assert torch.equal(s, sr)


def test_silu_mul(C):
    gu = torch.randn(77, 2 * 14336 // 8, device="cuda", dtype=torch.bfloat16)
    assert _rel(C.silu_mul(gu), L.silu_mul_ref(gu)) < 1e-2


@pytest.mark.parametrize("H,KVH,D", [(32, 8, 128), (8, 2, 64), (4, 4, 128)])
def test_rope_cache(C, H, KVH, D):
    torch.manual_seed(0)
    N, BS, NB = 53, 16, 16
    cs = L.rope_cos_sin(D, 512, 500000.0, {"rope_type": "llama3", "factor": 8.0}, "cuda")
    qkv = torch.randn(N, (H + 2 * KVH) * D, device="cuda", dtype=torch.bfloat16)
    pos = torch.randint(0, 512, (N,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(NB * BS, device="cuda")[:N].int()
    slots[3] = -1
    kc = torch.zeros(NB, KVH, BS, D, device="cuda", dtype=torch.bfloat16)
    vc, kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(kc), torch.zeros_like(kc)
    a = qkv.clone()
    C.rope_cache_(a, cs, pos, slots, kc, vc, H, KVH)
    b = qkv.clone()
    L.rope_cache_ref(b, cs, pos, slots, kc2, vc2, H, KVH)
    assert _rel(a, b) < 1e-2
    assert _rel(kc, kc2) < 1e-2 and torch.equal(vc, vc2)


@pytest.mark.parametrize("H,KVH,D", [(32, 8, 128), (16, 16, 128), (8, 2, 64), (16, 2, 128)])
@pytest.mark.parametrize("lens", [[1, 17, 300], [512, 513, 2000, 4100]])
def test_paged_decode(C, H, KVH, D, lens):
    torch.manual_seed(0)
    BS = 16
    B = len(lens)
    maxb = max(math.ceil(n / BS) for n in lens)
    nblk = B * maxb + 3
    kc = torch.randn(nblk, KVH, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    perm = torch.randperm(nblk, device="cuda").int()
    bt = perm[: B * maxb].view(B, maxb).contiguous()
    ctx = torch.tensor(lens, device="cuda", dtype=torch.int32)
    q = torch.randn(B, (H + 2 * KVH) * D, device="cuda", dtype=torch.bfloat16)  # fused-qkv row stride
    ref = L.paged_decode_ref(q, kc, vc, bt, ctx, H, 1 / math.sqrt(D))
    out = C.paged_decode(q, kc, vc, bt, ctx, max(lens), H, 1 / math.sqrt(D))  # default: MFMA for D=128
    assert _rel(out, ref) < 2e-2
    if D == 128:  # both implementations against the fp32 reference
        for impl in (0, 1):
            o = C.paged_decode(q, kc, vc, bt, ctx, max(lens), H, 1 / math.sqrt(D), impl)
            assert _rel(o, ref) < 2e-2, impl


@pytest.mark.parametrize("lens", [[1, 15, 16, 17, 31, 32, 33], [255, 256, 257, 511, 512, 600, 1500]])
def test_paged_decode_mfma_edges(C, lens):
    torch.manual_seed(1)
    H, KVH, D, BS = 32, 8, 128, 16
    B = len(lens)
    maxb = max(math.ceil(n / BS) for n in lens)
    kc = torch.randn(B * maxb + 2, KVH, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.randperm(B * maxb + 2, device="cuda").int()[: B * maxb].view(B, maxb).contiguous()
    ctx = torch.tensor(lens, device="cuda", dtype=torch.int32)
    q = torch.randn(B, H * D, device="cuda", dtype=torch.bfloat16) * 3  # peaked softmax
    ref = L.paged_decode_ref(q, kc, vc, bt, ctx, H, 1 / math.sqrt(D))
    out = C.paged_decode(q, kc, vc, bt, ctx, max(lens), H, 1 / math.sqrt(D), 1)
    assert _rel(out, ref) < 2e-2
    # max_ctx larger than any sequence (graph replays pass max_model_len)
    out2 = C.paged_decode(q, kc, vc, bt, ctx, maxb * BS, H, 1 / math.sqrt(D), 1)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("H,KVH,D,T", [(32, 8, 128, 300), (8, 2, 64, 1024), (4, 4, 128, 77)])
def test_flash_gqa_prefill(C, H, KVH, D, T):
    torch.manual_seed(0)
    qkv = torch.randn(2, T, (H + 2 * KVH) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[..., : H * D], qkv[..., H * D: (H + KVH) * D], qkv[..., (H + KVH) * D:]
    out, _ = C.flash_attn_gqa(q, k, v, H, KVH, True)
    ref = L.prefill_attention_ref(q, k, v, H, KVH, True)
    assert _rel(out, ref) < 2e-2


def test_llama_engine_gpu():
    from cluster_anywhere_amd.llm import LLMEngine, SamplingParams
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-small")
    m = Llama(cfg).to("cuda", torch.bfloat16).init_weights(std=0.02)
    prompts = [list(range(1, 1 + n)) for n in (5, 64, 300, 17)]
    e1 = LLMEngine(m, max_num_seqs=8, max_model_len=1024, num_blocks=512, use_graphs=True)
    e2 = LLMEngine(m, max_num_seqs=8, max_model_len=1024, num_blocks=512, use_graphs=False)
    o1 = e1.generate(prompts, SamplingParams(max_tokens=24))
    o2 = e2.generate(prompts, SamplingParams(max_tokens=24))
    assert [o.output_token_ids for o in o1] == [o.output_token_ids for o in o2]
    # decode logits (paged cache) agree with a dense forward over prompt + generated tokens
    seq = prompts[1] + o1[1].output_token_ids
    dense = m(torch.tensor([seq], device="cuda"))[0, len(prompts[1]) - 1: -1].float()
    gen = torch.tensor(o1[1].output_token_ids, device="cuda")
    agree = (dense.argmax(-1) == gen).float().mean().item()
    # random-init weights give near-tied logits: where the paged decode (bf16 P in the
    # MFMA P.V) picks another token than the dense forward, it must be a near tie
    top = dense.max(-1).values
    gap = top - dense.gather(1, gen[:, None]).squeeze(1)
    spread = top - dense.median(-1).values
    assert agree > 0.75 and bool((gap <= 0.05 * spread).all()), (agree, (gap / spread).max().item())


def test_llama_engine_one_step_ahead_matches_sync():
    """The one-step-ahead greedy decode (step t + 1 launched before step t's tokens
    are read back) gives the same tokens as the synchronous loop: more prompts than
    sequence slots (draining for admissions), different max_tokens, and stop tokens
    that end sequences while their next step is already in flight."""
    from cluster_anywhere_amd.llm import LLMEngine, SamplingParams
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(3)
    cfg = LlamaConfig.named("llama-small")
    m = Llama(cfg).to("cuda", torch.bfloat16).init_weights(std=0.02)
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(1, cfg.vocab_size, (int(n),), generator=g).tolist()
               for n in torch.randint(3, 90, (11,), generator=g)]

    def run(async_mode, stops):
        e = LLMEngine(m, max_num_seqs=4, max_model_len=512, num_blocks=512, use_graphs=True)
        e._async = async_mode
        ids = [e.add_request(p, SamplingParams(max_tokens=6 + 3 * (i % 4), stop_token_ids=stops.get(i, [])))
               for i, p in enumerate(prompts)]
        final = {}
        while e.has_unfinished():
            for o in e.step():
                if o.finished:
                    final[o.request_id] = o
        assert e._inflight is None
        return [(final[i].output_token_ids, final[i].finish_reason) for i in ids]

    plain = run(False, {})
    stops = {i: [plain[i][0][2]] for i in range(0, len(prompts), 2)}  # every other request stops early
    ref = run(False, stops)
    assert any(r == "stop" for _, r in ref)
    assert run(True, stops) == ref
    assert run(True, {}) == plain

    # every request ends on a stop token (none on max_tokens) -- the step
    # launched ahead for them must be drained at once, not finished inside the next
    # request's first step (which would log a bogus decode time over the idle gap)
    e = LLMEngine(m, max_num_seqs=4, max_model_len=512, num_blocks=512, use_graphs=True)
    e._async = True
    few = prompts[:3]
    outs = e.generate(few, SamplingParams(max_tokens=40, stop_token_ids=[]))
    stop_ids = {i: [o.output_token_ids[3]] for i, o in enumerate(outs)}
    e2 = LLMEngine(m, max_num_seqs=4, max_model_len=512, num_blocks=512, use_graphs=True)
    e2._async = True
    ids = [e2.add_request(p, SamplingParams(max_tokens=40, stop_token_ids=stop_ids[i])) for i, p in enumerate(few)]
    done = {}
    while e2.has_unfinished():
        for o in e2.step():
            if o.finished:
                done[o.request_id] = o
    assert all(done[i].finish_reason == "stop" for i in ids)
    assert e2._inflight is None and e2._last_finish is None
    n_times = len(e2.decode_times)
    import time as _t

    _t.sleep(0.3)
    e2.generate([few[0]], SamplingParams(max_tokens=4))
    assert all(dt < 0.25 for _, dt in e2.decode_times[n_times:]), e2.decode_times[n_times:]


@pytest.mark.parametrize("M", [1, 7, 100, 128])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1024, 2816), (256, 512)])
@pytest.mark.parametrize("packed", [False, True])
def test_decode_gemm_v3_epilogues(M, N, K, packed):
    """decode_gemm.hip vs fp32 torch: plain store, residual add and the SwiGLU
    epilogue (64-row interleaved gate/up weight), plain and prepacked weight
    streams, at the split count the wrapper picks; launched twice (tickets re-arm)."""
    import torch.nn.functional as F

    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    ref = x.float() @ w.float().t()
    wi = L.interleave_gate_up(w)
    wp, wip = (L.pack_decode_weight(w), L.pack_decode_weight(wi)) if packed else (w, wi)
    for _ in range(2):
        assert _rel(L.decode_gemm(x, wp, 0, packed=packed), ref) < 1e-2
        assert _rel(L.decode_gemm(x, wp, 1, residual=r, packed=packed), ref + r.float()) < 1e-2
        g, u = ref[:, : N // 2], ref[:, N // 2:]
        assert _rel(L.decode_gemm(x, wip, 2, packed=packed), F.silu(g) * u) < 1e-2
    assert torch.equal(L.unpack_decode_weight(L.pack_decode_weight(w)), w)


@pytest.mark.parametrize("N,K,splits", [(6144, 4096, 4), (4096, 4096, 8), (4096, 14336, 8), (256, 512, 2),
                                         (6144, 4096, 5), (4096, 14336, 9), (256, 640, 3)])
def test_decode_gemm_reduce_launch_matches(N, K, splits):
    """Split-K combined by the separate reduce launch (decode_gemm_config(1)) gives
    the same bits as the in-kernel last-arriver combine, store and residual epilogues;
    the last three cases have a shorter last split (ragged split-K)."""
    torch.manual_seed(N + K)
    x = torch.randn(128, K, device="cuda", dtype=torch.bfloat16)
    w = L.pack_decode_weight(torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05)
    r = torch.randn(128, N, device="cuda", dtype=torch.bfloat16)
    out = {}
    try:
        for ext in (0, 1):
            L.kernels().decode_gemm_config(ext)
            out[ext] = (L.decode_gemm(x, w, 0, splits=splits, packed=True),
                        L.decode_gemm(x, w, 1, residual=r, splits=splits, packed=True))
    finally:
        L.kernels().decode_gemm_config(1)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    ref = x.float() @ L.unpack_decode_weight(w).float().t()
    assert _rel(out[1][0], ref) < 1e-2 and _rel(out[1][1], ref + r.float()) < 1e-2


@pytest.mark.parametrize("M,H,KVH,K", [(128, 32, 8, 4096), (37, 8, 2, 1024)])
def test_decode_gemm_qkv_rope(M, H, KVH, K):
    """qkv GEMM + RoPE + cache append in the split-K reduce launch vs the fp32 GEMM
    followed by the reference rotation / cache append."""
    torch.manual_seed(M + H)
    D, BS, NB = 128, 16, 64
    N = (H + 2 * KVH) * D
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    cs = L.rope_cos_sin(D, 4096, 500000.0, None, "cuda")
    pos = torch.randint(0, 4096, (M,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(NB * BS, device="cuda")[:M].int()
    slots[min(3, M - 1)] = -1
    kc = torch.zeros(NB, KVH, BS, D, device="cuda", dtype=torch.bfloat16)
    vc, kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(kc), torch.zeros_like(kc)
    y = L.decode_gemm_qkv_rope(x, L.pack_decode_weight(w), cs, pos, slots, kc, vc, H, KVH)
    assert y is not None
    ref = (x.float() @ w.float().t())
    L.rope_cache_ref(ref, cs, pos, slots, kc2.float(), vc2.float(), H, KVH)  # fp32 rotation in place
    kr, vr = torch.zeros_like(kc, dtype=torch.float32), torch.zeros_like(vc, dtype=torch.float32)
    L.rope_cache_ref(ref.clone(), cs, torch.zeros_like(pos), slots, kr, vr, H, KVH)  # cos 1 / sin 0: plain append
    assert _rel(y, ref) < 1e-2
    assert _rel(kc, kr) < 1e-2 and _rel(vc, vr) < 1e-2
    assert int((kc != 0).any(-1).sum()) == (M - 1) * KVH  # slot -1 skipped


def test_llama_decode_gemm_weights(monkeypatch):
    """The model's decode copies (interleaved + packed gate/up, packed qkv / o / down /
    head, RMSNorm weights folded into qkv, gate/up and head) compute the same norm +
    projections as the fp32 math on the original weights."""
    import torch.nn.functional as F

    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(0)
    m = Llama(LlamaConfig.named("llama-small")).to("cuda", torch.bfloat16).init_weights(std=0.02)
    for lay in m.layers:
        for g in (lay.attn_norm, lay.mlp_norm):
            g.data = (1 + 0.2 * torch.randn_like(g.float())).bfloat16()
    m.final_norm.data = (1 + 0.2 * torch.randn_like(m.final_norm.float())).bfloat16()
    monkeypatch.setenv("CAAMD_DECODE_NORM_FUSED", "1")
    assert m.prepare_decode() and m._dec["norm"]
    eps = m.cfg.norm_eps
    lay = m.layers[1]
    gu, dn = m._dec["layers"][1]
    h = torch.randn(64, m.cfg.d_model, device="cuda", dtype=torch.bfloat16)

    def normed(g):
        return L.rms_norm_ref(h, g, eps)[0].float()

    a = L.decode_gemm(h, gu, 2, packed=True, norm_eps=eps)
    gate_up = normed(lay.mlp_norm) @ lay.w_gate_up.float().t()
    f = m.cfg.ffn_dim
    assert _rel(a, F.silu(gate_up[:, :f]) * gate_up[:, f:]) < 1e-2
    r = torch.randn(64, m.cfg.d_model, device="cuda", dtype=torch.bfloat16)
    y = L.decode_gemm(a, dn, 1, residual=r, packed=True)
    assert _rel(y, a.float() @ lay.w_down.float().t() + r.float()) < 1e-2
    logits = L.decode_gemm(h, m._dec["head"], 0, packed=True, norm_eps=eps)
    assert _rel(logits, normed(m.final_norm) @ m.lm_head.float().t()) < 1e-2
    qkv_w, o_w = m._dec["attn"][1]
    assert _rel(L.decode_gemm(h, qkv_w, 0, packed=True, norm_eps=eps),
                normed(lay.attn_norm) @ lay.w_qkv.float().t()) < 1e-2
    o_in = torch.randn(64, o_w.shape[1], device="cuda", dtype=torch.bfloat16)
    assert _rel(L.decode_gemm(o_in, o_w, 0, packed=True), o_in.float() @ lay.w_o.float().t()) < 1e-2


@pytest.mark.parametrize("M", [128, 37])
def test_llama_decode_folded_norms_match(M, monkeypatch):
    """One decode step with the RMSNorms folded into the GEMMs (default) vs the
    unfused decode path (rmsnorm launches, hipBLASLt qkv / o): same logits."""
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(1)
    m = Llama(LlamaConfig.named("llama-small")).to("cuda", torch.bfloat16).init_weights(std=0.02)
    for lay in m.layers:
        for g in (lay.attn_norm, lay.mlp_norm):
            g.data = (1 + 0.2 * torch.randn_like(g.float())).bfloat16()
    cfg, BS = m.cfg, 16
    nb = M * 4 + 4
    kc = [torch.randn(nb, cfg.n_kv_head, BS, cfg.head_dim, device="cuda", dtype=torch.bfloat16)
          for _ in range(cfg.n_layer)]
    vc = [torch.randn_like(t) for t in kc]
    bt = torch.randperm(nb, device="cuda").int()[: M * 4].view(M, 4).contiguous()
    ctx = torch.randint(1, 4 * BS + 1, (M,), device="cuda", dtype=torch.int32)
    pos = (ctx - 1).int()
    slots = (bt.gather(1, (pos // BS).long()[:, None]).squeeze(1) * BS + pos % BS).int()
    tok = torch.randint(0, cfg.vocab_size, (M,), device="cuda")
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CAAMD_DECODE_NORM_FUSED", fused)
        monkeypatch.setenv("CAAMD_DECODE_ATTN_GEMM", fused)
        assert m.prepare_decode()
        k2, v2 = [t.clone() for t in kc], [t.clone() for t in vc]
        out[fused] = (m.decode(tok, pos, slots, k2, v2, bt, ctx, 4 * BS).float(), k2, v2)
    assert m._dec["norm"] is False
    assert _rel(out["1"][0], out["0"][0]) < 2e-2
    assert _rel(torch.stack(out["1"][1]), torch.stack(out["0"][1])) < 1e-2


@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (128, 4096, 14336), (37, 1024, 2816), (5, 512, 1024)])
def test_decode_gemm_norm(M, N, K):
    """o / down projection with split-K combine + residual add + RMSNorm in one launch
    after the GEMM (dg_reduce_norm_kernel) vs the two-launch path (decode GEMM with its
    reduce launch, then rms_norm with the residual) and vs fp32 math."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    wp = L.pack_decode_weight(w)
    g = (1 + 0.2 * torch.randn(N, device="cuda")).bfloat16()
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    res = r.clone()
    h = L.decode_gemm_norm(x, wp, res, g, 1e-5)
    assert h is not None
    h2, res2 = L.rms_norm(L.decode_gemm(x, wp, 0, packed=True), g, 1e-5, r.clone())
    assert _rel(res, res2.float()) < 1e-3 and _rel(h, h2.float()) < 1e-3
    ref_res = x.float() @ w.float().t() + r.float()
    ref_h = ref_res * torch.rsqrt(ref_res.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    assert _rel(res, ref_res) < 1e-2 and _rel(h, ref_h) < 1e-2


@pytest.mark.parametrize("M", [128, 37])
def test_llama_decode_reduce_norm_matches(M, monkeypatch):
    """One decode step with the o / down reduce + residual + RMSNorm launches fused
    (default) vs the reduce launch + rmsnorm launch path: same logits and caches."""
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(2)
    m = Llama(LlamaConfig.named("llama-small")).to("cuda", torch.bfloat16).init_weights(std=0.02)
    for lay in m.layers:
        for g in (lay.attn_norm, lay.mlp_norm):
            g.data = (1 + 0.2 * torch.randn_like(g.float())).bfloat16()
    cfg, BS = m.cfg, 16
    nb = M * 4 + 4
    kc = [torch.randn(nb, cfg.n_kv_head, BS, cfg.head_dim, device="cuda", dtype=torch.bfloat16)
          for _ in range(cfg.n_layer)]
    vc = [torch.randn_like(t) for t in kc]
    bt = torch.randperm(nb, device="cuda").int()[: M * 4].view(M, 4).contiguous()
    ctx = torch.randint(1, 4 * BS + 1, (M,), device="cuda", dtype=torch.int32)
    pos = (ctx - 1).int()
    slots = (bt.gather(1, (pos // BS).long()[:, None]).squeeze(1) * BS + pos % BS).int()
    tok = torch.randint(0, cfg.vocab_size, (M,), device="cuda")
    assert m.prepare_decode() and m._dec["attn"] is not None and not m._dec["norm"]
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CAAMD_DECODE_REDUCE_NORM", fused)
        k2, v2 = [t.clone() for t in kc], [t.clone() for t in vc]
        out[fused] = (m.decode(tok, pos, slots, k2, v2, bt, ctx, 4 * BS).float(), k2, v2)
    assert _rel(out["1"][0], out["0"][0]) < 1e-3
    assert _rel(torch.stack(out["1"][1]), torch.stack(out["0"][1])) < 1e-3


@pytest.mark.parametrize("M,V", [(128, 128256), (3, 1000), (1, 7)])
def test_argmax_rows(M, V):
    """Greedy sampler's HIP row argmax on bf16 logits vs torch.argmax (first maximum
    on ties: bf16 logits tie often); also a strided row view."""
    torch.manual_seed(V)
    x = torch.randn(M, V + 8, device="cuda").bfloat16()
    x[0, 5 % V] = x[0, (V - 1)] = 50.0  # a tie: the first index wins
    for t in (x[:, :V].contiguous(), x[:, :V]):
        got = L.kernels().argmax_rows(t)
        assert torch.equal(got, t.float().argmax(-1)), (got, t.float().argmax(-1))


def _rel2(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(512, 2560, 1024), (2048, 2048, 4096), (256, 5632, 1024)])
def test_prefill_gemm_packed_epilogues(M, N, K):
    """gemm.hip full-line kernel reading B in the decode GEMM's packed order:
    plain store, residual accumulate (o / down) and SwiGLU over the 64-row
    interleaved gate/up weight, vs fp32 (K = 4096 exercises the split-K tail)."""
    import torch.nn.functional as F

    from cluster_anywhere_amd.ops import gemm as G

    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    ref = x.float() @ w.float().t()
    y = G.prefill_linear(x, L.pack_decode_weight(w))
    assert _rel2(y, ref) < 5e-3
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    acc = r.clone()
    G.prefill_linear(x, L.pack_decode_weight(w), out=acc, accumulate=True)
    assert _rel2(acc, ref + r.float()) < 5e-3
    a = G.prefill_linear(x, L.pack_decode_weight(L.interleave_gate_up(w)), epi=G.EPI_SWIGLU)
    g, u = ref[:, : N // 2].bfloat16().float(), ref[:, N // 2:].bfloat16().float()
    assert a.shape == (M, N // 2) and _rel2(a, F.silu(g) * u) < 1e-2


def test_llama_packed_prefill_shares_weights():
    """After prepare_decode the nn.Linear weights are released (one weight copy);
    prefill on gemm.hip from the packed copies matches the dense forward's logits
    at each sequence's last prompt token, and re-preparing restores the originals
    bit-exactly."""
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(3)
    m = Llama(LlamaConfig.named("llama-small")).to("cuda", torch.bfloat16).init_weights(std=0.02)
    orig = {n: p.detach().clone() for n, p in m.named_parameters()}
    B, T = 3, 200  # M = 600: padded to 768 rows inside
    tok = torch.randint(0, m.cfg.vocab_size, (B, T), device="cuda")
    dense = m(tok).float()
    assert m.prepare_decode() and m._shared and m._dec["prefill"]
    assert m.layers[0].w_gate_up.numel() == 0 and m.lm_head.numel() == 0
    pos = torch.arange(T, device="cuda").expand(B, T)
    last = torch.tensor([T - 1, 57, 120], device="cuda")
    logits = m.prefill(tok, pos, None, None, None, last).float()
    ref = dense[torch.arange(B), last]
    assert _rel2(logits, ref) < 3e-2
    assert (logits.argmax(-1) == ref.argmax(-1)).float().mean() >= 2 / 3
    m._restore_originals()
    assert all(torch.equal(p, orig[n]) for n, p in m.named_parameters())
