"""Llama numerics pinned against an independent implementation: Hugging Face
``transformers.LlamaForCausalLM`` loading our ``save_hf_llama`` directory (reference
role: python/ray/llm serves HF Llama checkpoints through vLLM).

CPU, fp32: the dense forward of ``models/llama.py`` (fused w_qkv / w_gate_up,
rotate-half RoPE with llama3 frequency scaling, GQA grouping, RMSNorm) against HF
on a small GQA model. The production GPU path (packed prefill GEMMs, head-dim-128
flash prefill, paged decode, HIP graphs, folded norms) is compared in
``test_llama_hf_parity_gpu.py``."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from cluster_anywhere_amd.llm.weights import load_hf_llama, save_hf_llama  # noqa: E402
from cluster_anywhere_amd.models.llama import Llama, LlamaConfig  # noqa: E402


def _cfg(**kw):
    base = dict(vocab_size=512, d_model=256, n_layer=2, n_head=8, n_kv_head=2, ffn_dim=512, max_position=2048,
                rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                              "high_freq_factor": 4.0, "original_max_position_embeddings": 256})
    base.update(kw)
    return LlamaConfig(**base)


@pytest.mark.parametrize("kw", [{}, {"n_kv_head": 8}, {"rope_scaling": None, "rope_theta": 10000.0},
                                {"tie_embeddings": True}])
def test_dense_forward_matches_transformers(tmp_path, kw):
    torch.manual_seed(0)
    m = Llama(_cfg(**kw)).init_weights(std=0.05)
    with torch.no_grad():  # non-trivial norm weights (all-ones would hide a missing gain)
        for ly in m.layers:
            ly.attn_norm.uniform_(0.5, 1.5)
            ly.mlp_norm.uniform_(0.5, 1.5)
        m.final_norm.uniform_(0.5, 1.5)
    save_hf_llama(m, str(tmp_path))
    hf = transformers.LlamaForCausalLM.from_pretrained(str(tmp_path), torch_dtype=torch.float32).eval()
    x = torch.randint(0, m.cfg.vocab_size, (2, 300))  # positions past original_max_position_embeddings
    with torch.no_grad():
        ref = hf(x).logits
        ours = m(x)
    err = (ours - ref).abs().max().item()
    assert err < 1e-4 * ref.abs().max().item() + 1e-5, err
    # and the checkpoint loads back into the serving layout bit-exactly
    m2 = load_hf_llama(str(tmp_path), device="cpu", dtype=torch.float32)
    with torch.no_grad():
        assert torch.equal(m2(x), ours)
