"""Hugging Face Llama checkpoints (safetensors + config.json, local files only)
<-> the fused serving layout of ``models/llama.py`` (q/k/v rows concatenated
into ``w_qkv``, gate/up into ``w_gate_up``)."""
from __future__ import annotations

import glob
import json
import os
from typing import Dict

import torch

from ..models.llama import Llama, LlamaConfig


def config_from_hf(d: Dict) -> LlamaConfig:
    return LlamaConfig(vocab_size=d["vocab_size"], d_model=d["hidden_size"], n_layer=d["num_hidden_layers"],
                       n_head=d["num_attention_heads"],
                       n_kv_head=d.get("num_key_value_heads", d["num_attention_heads"]),
                       ffn_dim=d["intermediate_size"], rope_theta=d.get("rope_theta", 10000.0),
                       rope_scaling=d.get("rope_scaling"), norm_eps=d.get("rms_norm_eps", 1e-5),
                       max_position=d.get("max_position_embeddings", 8192),
                       tie_embeddings=d.get("tie_word_embeddings", False))


def config_to_hf(c: LlamaConfig) -> Dict:
    return {"architectures": ["LlamaForCausalLM"], "model_type": "llama", "vocab_size": c.vocab_size,
            "hidden_size": c.d_model, "num_hidden_layers": c.n_layer, "num_attention_heads": c.n_head,
            "num_key_value_heads": c.n_kv_head, "intermediate_size": c.ffn_dim, "rope_theta": c.rope_theta,
            "rope_scaling": c.rope_scaling, "rms_norm_eps": c.norm_eps,
            "max_position_embeddings": c.max_position, "tie_word_embeddings": c.tie_embeddings,
            "torch_dtype": "bfloat16"}


def load_hf_llama(path: str, device="cuda", dtype=torch.bfloat16) -> Llama:
    from safetensors import safe_open

    with open(os.path.join(path, "config.json")) as f:
        cfg = config_from_hf(json.load(f))
    with torch.device("meta"):
        model = Llama(cfg)
    model = model.to_empty(device=device).to(dtype)
    tensors = {}
    for fn in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
        with safe_open(fn, framework="pt", device="cpu") as f:
            for k in f.keys():
                tensors[k] = f.get_tensor(k)

    def take(name):
        if name not in tensors:
            raise KeyError(f"checkpoint is missing {name}")
        return tensors.pop(name)

    with torch.no_grad():
        model.embed.copy_(take("model.embed_tokens.weight"))
        for i, ly in enumerate(model.layers):
            p = f"model.layers.{i}."
            ly.attn_norm.copy_(take(p + "input_layernorm.weight"))
            ly.w_qkv.copy_(torch.cat([take(p + "self_attn.q_proj.weight"), take(p + "self_attn.k_proj.weight"),
                                      take(p + "self_attn.v_proj.weight")], 0))
            ly.w_o.copy_(take(p + "self_attn.o_proj.weight"))
            ly.mlp_norm.copy_(take(p + "post_attention_layernorm.weight"))
            ly.w_gate_up.copy_(torch.cat([take(p + "mlp.gate_proj.weight"), take(p + "mlp.up_proj.weight")], 0))
            ly.w_down.copy_(take(p + "mlp.down_proj.weight"))
        model.final_norm.copy_(take("model.norm.weight"))
        if model.lm_head is not None:
            model.lm_head.copy_(take("lm_head.weight") if "lm_head.weight" in tensors else model.embed)
    return model


def save_hf_llama(model: Llama, path: str):
    from safetensors.torch import save_file

    c = model.cfg
    hd = c.head_dim
    os.makedirs(path, exist_ok=True)
    out = {"model.embed_tokens.weight": model.embed, "model.norm.weight": model.final_norm}
    for i, ly in enumerate(model.layers):
        p = f"model.layers.{i}."
        q, k, v = torch.split(ly.w_qkv, [c.n_head * hd, c.n_kv_head * hd, c.n_kv_head * hd], 0)
        g, u = torch.split(ly.w_gate_up, [c.ffn_dim, c.ffn_dim], 0)
        out.update({p + "input_layernorm.weight": ly.attn_norm, p + "self_attn.q_proj.weight": q,
                    p + "self_attn.k_proj.weight": k, p + "self_attn.v_proj.weight": v,
                    p + "self_attn.o_proj.weight": ly.w_o, p + "post_attention_layernorm.weight": ly.mlp_norm,
                    p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u, p + "mlp.down_proj.weight": ly.w_down})
    if model.lm_head is not None:
        out["lm_head.weight"] = model.lm_head
    save_file({k: v.detach().contiguous().cpu() for k, v in out.items()}, os.path.join(path, "model.safetensors"))
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(config_to_hf(c), f, indent=1)
