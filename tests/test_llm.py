"""LLM engine (CPU, fp32 reference ops): paged KV cache + continuous batching
must reproduce greedy decoding of a dense full-recompute forward; preemption
under cache pressure; sampling params (reference: vLLM-style engine tests that
python/ray/llm/tests rely on)."""
import math

import pytest
import torch

from cluster_anywhere_amd.llm import LLMEngine, SamplingParams
from cluster_anywhere_amd.models.llama import Llama, LlamaConfig
from cluster_anywhere_amd.ops import llm as L


def _model(dtype=torch.float32):
    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    return Llama(cfg).init_weights(std=0.05).to(dtype)


def _greedy_ref(model, prompt, n):
    toks = list(prompt)
    for _ in range(n):
        logits = model(torch.tensor([toks]))
        toks.append(int(logits[0, -1].argmax()))
    return toks[len(prompt):]


def test_rope_table_llama3_scaling():
    cs = L.rope_cos_sin(128, 16, 500000.0, LlamaConfig().rope_scaling)
    assert cs.shape == (16, 64, 2)
    assert torch.allclose(cs[0, :, 0], torch.ones(64)) and torch.allclose(cs[0, :, 1], torch.zeros(64))
    plain = L.rope_cos_sin(128, 16, 500000.0, None)
    # high-frequency dims are unscaled, the lowest frequencies are divided by `factor`
    assert torch.allclose(cs[5, 0], plain[5, 0])
    assert not torch.allclose(cs[5, -1], plain[5, -1])


def test_paged_decode_ref_matches_dense():
    torch.manual_seed(0)
    H, KVH, D, BS = 8, 2, 64, 16
    lens = [5, 33, 70]
    nblk = 32
    kc = torch.randn(nblk, KVH, BS, D)
    vc = torch.randn(nblk, KVH, BS, D)
    perm = torch.randperm(nblk)
    bt = torch.zeros(3, 8, dtype=torch.int32)
    k = 0
    for b, n in enumerate(lens):
        nb = math.ceil(n / BS)
        bt[b, :nb] = perm[k:k + nb].int()
        k += nb
    q = torch.randn(3, H * D)
    out = L.paged_decode_ref(q, kc, vc, bt, torch.tensor(lens), H, 1 / math.sqrt(D))
    for b, n in enumerate(lens):
        blocks = bt[b, : math.ceil(n / BS)].long()
        kk = kc[blocks].permute(1, 0, 2, 3).reshape(KVH, -1, D)[:, :n]
        vv = vc[blocks].permute(1, 0, 2, 3).reshape(KVH, -1, D)[:, :n]
        qq = q[b].view(H, D)
        kk = kk.repeat_interleave(H // KVH, 0)
        vv = vv.repeat_interleave(H // KVH, 0)
        p = torch.softmax(torch.einsum("hd,htd->ht", qq, kk) / math.sqrt(D), -1)
        ref = torch.einsum("ht,htd->hd", p, vv).reshape(-1)
        assert torch.allclose(out[b], ref, atol=1e-5)


def test_engine_matches_full_recompute():
    m = _model()
    eng = LLMEngine(m, block_size=16, max_num_seqs=4, max_model_len=256, num_blocks=64, use_graphs=False)
    prompts = [[1, 2, 3], [7] * 20, list(range(40, 75)), [9, 8]]
    outs = eng.generate(prompts, SamplingParams(max_tokens=12))
    for p, o in zip(prompts, outs):
        assert o.finished and o.finish_reason == "length"
        assert o.output_token_ids == _greedy_ref(m, p, 12)
    assert eng.alloc.num_free == 64


def test_engine_preemption_under_cache_pressure():
    m = _model()
    # 10 blocks of 16 tokens: four 30-token sequences cannot all stay resident
    eng = LLMEngine(m, block_size=16, max_num_seqs=4, max_model_len=128, num_blocks=10, use_graphs=False)
    prompts = [list(range(i, i + 20)) for i in range(4)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=20))
    assert eng.stats["preemptions"] > 0
    for p, o in zip(prompts, outs):
        assert o.output_token_ids == _greedy_ref(m, p, 20)


def test_sampling_params():
    m = _model()
    eng = LLMEngine(m, num_blocks=64, max_model_len=128, use_graphs=False)
    a = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=8, temperature=1.0, top_p=0.9, seed=3))[0]
    b = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=8, temperature=1.0, top_p=0.9, seed=3))[0]
    assert a.output_token_ids == b.output_token_ids
    stop = a.output_token_ids[2]
    c = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=8, temperature=1.0, top_p=0.9, seed=3,
                                                 stop_token_ids=[stop]))[0]
    assert c.finish_reason == "stop" and c.output_token_ids[-1] == stop
    assert len(c.output_token_ids) <= 3
    with pytest.raises(ValueError):
        eng.add_request([1] * 120, SamplingParams(max_tokens=20))


def test_hf_checkpoint_roundtrip(tmp_path):
    from cluster_anywhere_amd.llm.weights import load_hf_llama, save_hf_llama

    m = _model()
    save_hf_llama(m, str(tmp_path))
    m2 = load_hf_llama(str(tmp_path), device="cpu", dtype=torch.float32)
    for (n1, p1), (n2, p2) in zip(m.named_parameters(), m2.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2)
    x = torch.tensor([[3, 1, 4, 1, 5]])
    assert torch.equal(m(x), m2(x))
