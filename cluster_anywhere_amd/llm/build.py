"""Engine construction shared by Serve LLM replicas and the batch engine stage:
a Llama model (local HF checkpoint, or a random-init preset — there is no
network for weights), its tokenizer and a :class:`LLMEngine` sized for the
device (HIP graphs + paged cache from the HBM left after weights on MI355X;
a small eager cache on CPU)."""
from __future__ import annotations

from typing import Any, Dict, Optional


def build_engine(model_id: str = "llama-tiny", model_source: Optional[str] = None,
                 tokenizer_source: Optional[str] = None, dtype: str = "bfloat16",
                 engine_kwargs: Optional[Dict[str, Any]] = None, seed: int = 0, device: Optional[str] = None):
    """-> (LLMEngine, tokenizer)."""
    import torch

    from ..models.llama import Llama, LlamaConfig
    from .engine import LLMEngine
    from .tokenizer import load_tokenizer

    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    tdtype = getattr(torch, dtype) if dev != "cpu" else torch.float32
    if model_source:
        from .weights import load_hf_llama

        model = load_hf_llama(model_source, dev, tdtype)
    else:
        lc = LlamaConfig.named(model_id)
        with torch.device(dev):
            model = Llama(lc).to(tdtype)
        torch.manual_seed(seed)
        model.init_weights(std=0.02, seed=seed)
    tok = load_tokenizer(tokenizer_source or model_source, model.cfg.vocab_size)
    kw = dict(engine_kwargs or {})
    kw.setdefault("eos_token_id", getattr(tok, "eos_token_id", None))
    if dev == "cpu":
        kw.setdefault("num_blocks", 256)
        kw.setdefault("use_graphs", False)
    return LLMEngine(model, **kw), tok
