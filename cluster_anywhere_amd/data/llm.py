"""``ray.data.llm`` (reference: python/ray/data/llm.py:1-79): batch LLM
processors over Datasets.

    from cluster_anywhere_amd.data.llm import EngineProcessorConfig, build_llm_processor
    proc = build_llm_processor(EngineProcessorConfig(model="llama-tiny", concurrency=1,
                                                     sampling_params=dict(max_tokens=16)),
                               preprocess=lambda r: dict(messages=[{"role": "user", "content": r["q"]}]),
                               postprocess=lambda r: dict(answer=r["generated_text"]))
    ds = proc(ds)
"""
from ..llm.batch.processor import EngineProcessorConfig as _EngineProcessorConfig
from ..llm.batch.processor import HttpRequestProcessorConfig as _HttpRequestProcessorConfig
from ..llm.batch.processor import Processor
from ..llm.batch.processor import ProcessorBuilder as _ProcessorBuilder
from ..llm.batch.processor import ProcessorConfig as _ProcessorConfig


class ProcessorConfig(_ProcessorConfig):
    """The processor configuration."""


class HttpRequestProcessorConfig(_HttpRequestProcessorConfig):
    """Send every row as a JSON POST (e.g. to an OpenAI-compatible endpoint such
    as ``serve.llm.build_openai_app``) and merge the response into the row."""


class EngineProcessorConfig(_EngineProcessorConfig):
    """Generate with the in-tree gfx950 engine in GPU actors (the reference's
    vLLM engine processor role)."""


def build_llm_processor(config: ProcessorConfig, **kwargs) -> Processor:
    """Build a processor for ``config`` (kwargs: ``preprocess``, ``postprocess``,
    ``override_stage_config_fn``)."""
    return _ProcessorBuilder.build(config, **kwargs)


__all__ = ["ProcessorConfig", "Processor", "HttpRequestProcessorConfig", "EngineProcessorConfig",
           "build_llm_processor"]
