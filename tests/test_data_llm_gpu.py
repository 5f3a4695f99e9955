"""``data.llm`` engine processor on the GPU: a Dataset of chat prompts through
chat-template -> tokenize -> engine (one GPU actor, HIP-graph decode, gfx950
kernels) -> detokenize (reference role: python/ray/llm/tests/batch/gpu/)."""
import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data as rd
from cluster_anywhere_amd.data.llm import EngineProcessorConfig, build_llm_processor

pytestmark = pytest.mark.gpu


def test_engine_processor_generates_on_gpu():
    ray.init(num_cpus=4, num_gpus=1)
    try:
        cfg = EngineProcessorConfig(model="llama-small", batch_size=8, concurrency=1, num_gpus_per_worker=1,
                                    engine_kwargs=dict(num_blocks=512, max_model_len=1024, max_num_seqs=16),
                                    sampling_params=dict(max_tokens=12, ignore_eos=True))
        proc = build_llm_processor(
            cfg, preprocess=lambda r: dict(messages=[{"role": "user", "content": f"question {r['id']}"}]),
            postprocess=lambda r: dict(id=r["id"], n=r["num_generated_tokens"], toks=list(r["generated_tokens"]),
                                       text=r["generated_text"], n_in=r["num_input_tokens"]))
        rows = sorted(proc(rd.range(24)).take_all(), key=lambda r: r["id"])
        assert [r["id"] for r in rows] == list(range(24))
        assert all(r["n"] == 12 and len(r["toks"]) == 12 for r in rows)
        assert all(0 <= int(t) < 4096 for r in rows for t in r["toks"])
        assert all(isinstance(r["text"], str) for r in rows)
        assert all(r["n_in"] > len("question ") for r in rows)
    finally:
        ray.shutdown()
    assert torch.cuda.is_available()
