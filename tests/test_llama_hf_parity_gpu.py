"""The serving path of ``models/llama.py`` at Llama-3-8B width against Hugging Face
``transformers.LlamaForCausalLM`` (fp32, same checkpoint written by
``save_hf_llama``). Two decoder layers, d_model 4096, 32 query / 8 KV heads of 128,
FFN 14336, vocabulary 128256, llama3 rope_scaling, non-trivial norm gains.

What runs on our side is the production path: ``LLMEngine`` (packed prefill GEMMs on
gemm.hip, head-dim-128 flash prefill, paged MFMA decode attention, decode GEMMs,
HIP graphs, one step ahead), and a second engine with the RMSNorms folded into the
GEMMs (``CAAMD_DECODE_NORM_FUSED=1``).

Tolerances (bf16 weights and activations against an fp32 reference):
  * prefill logits of the last prompt token: relative L2 error < 3e-2, and the same
    argmax;
  * 16 greedy decode steps, teacher-forced: HF's logits over prompt + our tokens;
    every token we picked is HF's argmax or within 5 % of the logit spread
    (top - median) of it, and >= 75 % are exact argmax matches (random weights give
    near-tied logits, where bf16 rounding may pick the other of two)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")

PROMPT_LENS = (17, 130, 513, 64)
STEPS = 16


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    from cluster_anywhere_amd.llm.weights import save_hf_llama
    from cluster_anywhere_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(0)
    cfg = LlamaConfig(n_layer=2, max_position=2048)  # Llama-3-8B widths, llama3 rope scaling
    m = Llama(cfg).to("cuda", torch.bfloat16).init_weights(std=0.02)
    with torch.no_grad():
        for ly in m.layers:
            ly.attn_norm.uniform_(0.5, 1.5)
            ly.mlp_norm.uniform_(0.5, 1.5)
        m.final_norm.uniform_(0.5, 1.5)
    d = str(tmp_path_factory.mktemp("hf_llama"))
    save_hf_llama(m, d)
    hf = transformers.LlamaForCausalLM.from_pretrained(d, torch_dtype=torch.float32).to("cuda").eval()
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist() for n in PROMPT_LENS]
    return d, m, hf, prompts


def _hf_logits(hf, ids):
    with torch.no_grad():
        return hf(torch.tensor([ids], device="cuda")).logits[0].float()


def _check_greedy(hf, prompts, outs):
    exact = total = 0
    worst = 0.0
    for p, o in zip(prompts, outs):
        gen = o.output_token_ids
        assert len(gen) == STEPS
        ref = _hf_logits(hf, p + gen[:-1])[len(p) - 1:]
        g = torch.tensor(gen, device="cuda")
        top = ref.max(-1).values
        gap = top - ref.gather(1, g[:, None]).squeeze(1)
        spread = top - ref.median(-1).values
        exact += int((ref.argmax(-1) == g).sum())
        total += len(gen)
        worst = max(worst, float((gap / spread).max()))
    assert worst <= 0.05 and exact >= 0.75 * total, (exact, total, worst)
    return exact / total


def test_prefill_logits_match_transformers(models):
    from cluster_anywhere_amd.llm import LLMEngine

    d, m, hf, prompts = models
    eng = LLMEngine(m, max_num_seqs=8, max_model_len=1024, num_blocks=512, use_graphs=True)
    assert eng.decode_gemm and m._dec.get("prefill"), "the packed production prefill path must be active"
    B, T = len(prompts), max(PROMPT_LENS)
    toks = torch.zeros(B, T, dtype=torch.long, device="cuda")
    for i, p in enumerate(prompts):
        toks[i, :len(p)] = torch.tensor(p, device="cuda")
    pos = torch.arange(T, device="cuda").expand(B, T).contiguous()
    last = torch.tensor([len(p) - 1 for p in prompts], device="cuda")
    with torch.no_grad():
        ours = m.prefill(toks, pos, None, None, None, last).float()
    for i, p in enumerate(prompts):
        ref = _hf_logits(hf, p)[-1]
        rel = ((ours[i] - ref).norm() / ref.norm()).item()
        assert rel < 3e-2, (i, rel)
        assert int(ours[i].argmax()) == int(ref.argmax()), i


def test_engine_greedy_decode_matches_transformers(models):
    from cluster_anywhere_amd.llm import LLMEngine, SamplingParams

    d, m, hf, prompts = models
    eng = LLMEngine(m, max_num_seqs=8, max_model_len=1024, num_blocks=512, use_graphs=True)
    outs = eng.generate(prompts, SamplingParams(max_tokens=STEPS, ignore_eos=True))
    frac = _check_greedy(hf, prompts, outs)
    print(f"greedy tokens equal to HF argmax: {frac:.3f}")


def test_engine_folded_norms_match_transformers(models, monkeypatch):
    from cluster_anywhere_amd.llm import LLMEngine, SamplingParams
    from cluster_anywhere_amd.llm.weights import load_hf_llama

    d, m, hf, prompts = models
    monkeypatch.setenv("CAAMD_DECODE_NORM_FUSED", "1")
    m2 = load_hf_llama(d, device="cuda", dtype=torch.bfloat16)
    eng = LLMEngine(m2, max_num_seqs=8, max_model_len=1024, num_blocks=512, use_graphs=True)
    assert m2._dec is not None and m2._dec["norm"], "norm folding must be active"
    outs = eng.generate(prompts, SamplingParams(max_tokens=STEPS, ignore_eos=True))
    frac = _check_greedy(hf, prompts, outs)
    print(f"folded norms: greedy tokens equal to HF argmax: {frac:.3f}")
    del eng, m2
    os.environ.pop("CAAMD_DECODE_NORM_FUSED", None)
