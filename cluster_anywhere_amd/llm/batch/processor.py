"""Batch-LLM processors: preprocess -> stages -> postprocess over a Dataset.

Reference roles: ``python/ray/llm/_internal/batch/processor/base.py``
(``ProcessorConfig`` :17, ``Processor`` :43, ``ProcessorBuilder`` :157) and
``http_request_proc.py``. The
reference's engine processor wraps vLLM; :class:`EngineProcessorConfig` builds
the same chat-template -> tokenize -> engine -> detokenize pipeline over the
in-tree gfx950 engine, one engine actor per GPU (``concurrency`` actors).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Type

from pydantic import BaseModel, ConfigDict, Field

from .stages import (ChatTemplateStage, DetokenizeStage, EngineStage, HttpRequestStage, PrepareImageStage,
                     StatefulStage, TokenizeStage, wrap_postprocess, wrap_preprocess)


class ProcessorConfig(BaseModel):
    """Processor configuration (reference: processor/base.py:17)."""

    model_config = ConfigDict(arbitrary_types_allowed=True, validate_assignment=True,
                              protected_namespaces=())

    batch_size: int = Field(description="Rows per map_batches call of every stage.")
    accelerator_type: Optional[str] = Field(default=None, description="Accelerator of the LLM stage "
                                            "(None: CPU only, or the engine's default device).")
    concurrency: int = Field(default=1, description="Workers (actors) of the LLM stage.")


class Processor:
    """Dataset -> Dataset pipeline: pack each row into the data column (optionally
    through ``preprocess``), run the stages as ``map_batches`` operators in order,
    unpack (optionally through ``postprocess``). Calling it is lazy: it returns
    the transformed Dataset. Role reference: processor/base.py:43.

    Stages are named after their class; repeats get ``_2``, ``_3`` ... suffixes."""

    data_column: str = "__data"

    def __init__(self, config: ProcessorConfig, stages: List[StatefulStage],
                 preprocess: Optional[Callable] = None, postprocess: Optional[Callable] = None):
        self.config = config
        col = self.data_column
        self.preprocess = wrap_preprocess(preprocess, col) if preprocess is not None else None
        self.postprocess = wrap_postprocess(postprocess, col) if postprocess is not None else None
        self._named: List[tuple] = []
        seen: Dict[str, int] = {}
        for st in stages:
            base = type(st).__name__
            seen[base] = seen.get(base, 0) + 1
            self._named.append((base if seen[base] == 1 else f"{base}_{seen[base]}", st))

    @property
    def stages(self) -> "OrderedDict[str, StatefulStage]":
        return OrderedDict(self._named)

    def __call__(self, dataset):
        col = self.data_column
        dataset = dataset.map(self.preprocess or (lambda row: {col: dict(row)}))
        for _, st in self._named:
            dataset = dataset.map_batches(
                st.fn, **st.get_dataset_map_batches_kwargs(batch_size=self.config.batch_size, data_column=col))
        return dataset.map(self.postprocess or (lambda row: dict(row[col])))

    def list_stage_names(self) -> List[str]:
        return [n for n, _ in self._named]

    def get_stage_by_name(self, name: str) -> StatefulStage:
        for n, st in self._named:
            if n == name:
                return st
        raise ValueError(f"no stage named {name!r}; stages: {self.list_stage_names()}")


class ProcessorBuilder:
    """Maps a config class to the function that builds its Processor. A config
    subclass without its own builder uses the nearest registered base class's.
    Role reference: processor/base.py:157."""

    _builders: Dict[type, Callable] = {}

    @classmethod
    def register(cls, config_type: Type[ProcessorConfig], builder: Callable) -> None:
        if config_type in cls._builders:
            raise ValueError(f"a builder for {config_type.__name__} is already registered")
        cls._builders[config_type] = builder

    @classmethod
    def build(cls, config: ProcessorConfig, override_stage_config_fn: Optional[Callable] = None,
              **kwargs) -> Processor:
        builder = next((cls._builders[k] for k in type(config).__mro__ if k in cls._builders), None)
        if builder is None:
            known = sorted(k.__name__ for k in cls._builders)
            raise ValueError(f"{type(config).__name__} is not registered with ProcessorBuilder "
                             f"(registered configs: {known})")
        proc = builder(config, **kwargs)
        if override_stage_config_fn is not None:
            for name, st in proc._named:
                override_stage_config_fn(name, st)
        return proc


# ------------------------------------------------------------ HTTP processor
class HttpRequestProcessorConfig(ProcessorConfig):
    """Rows -> JSON POST bodies -> merged JSON responses (reference:
    http_request_proc.py:15). ``qps`` paces requests per worker; ``max_concurrent``
    bounds requests in flight per worker."""

    batch_size: int = Field(default=64)
    url: str = Field(description="The URL to query.")
    headers: Optional[Dict[str, Any]] = Field(default=None)
    qps: Optional[float] = Field(default=None)
    max_concurrent: int = Field(default=64)
    max_retries: int = Field(default=3)


def build_http_request_processor(config: HttpRequestProcessorConfig, **kwargs) -> Processor:
    stage = HttpRequestStage(
        fn_constructor_kwargs=dict(url=config.url, additional_header=config.headers, qps=config.qps,
                                   max_concurrent=config.max_concurrent, max_retries=config.max_retries),
        map_batches_kwargs=dict(concurrency=config.concurrency))
    return Processor(config, [stage], **kwargs)


ProcessorBuilder.register(HttpRequestProcessorConfig, build_http_request_processor)


# ------------------------------------------------------------ engine processor
class EngineProcessorConfig(ProcessorConfig):
    """Offline generation with the in-tree engine: [chat template] -> [tokenize]
    -> engine -> [detokenize]. ``model`` is a local HF checkpoint directory or a
    model preset (random init, byte tokenizer). ``sampling_params`` are the
    defaults; a row's ``sampling_params`` column overrides them."""

    batch_size: int = Field(default=64)
    model: str = Field(default="llama-tiny")
    tokenizer: Optional[str] = Field(default=None, description="Tokenizer directory (default: model's).")
    dtype: str = Field(default="bfloat16")
    engine_kwargs: Dict[str, Any] = Field(default_factory=dict)
    sampling_params: Dict[str, Any] = Field(default_factory=dict)
    apply_chat_template: bool = Field(default=True)
    chat_template: Optional[str] = Field(default=None)
    tokenize: bool = Field(default=True)
    detokenize: bool = Field(default=True)
    has_image: bool = Field(default=False)
    num_gpus_per_worker: Optional[float] = Field(default=None, description="Default: 1 when a GPU is visible.")
    seed: int = Field(default=0)


def _source(config: EngineProcessorConfig):
    import os

    src = config.model if os.path.isdir(config.model) else None
    return src, config.tokenizer or src


def build_engine_processor(config: EngineProcessorConfig, **kwargs) -> Processor:
    model_src, tok_src = _source(config)
    stages: List[StatefulStage] = []
    if config.has_image:
        stages.append(PrepareImageStage(map_batches_kwargs=dict(concurrency=config.concurrency)))
    if config.apply_chat_template:
        stages.append(ChatTemplateStage(fn_constructor_kwargs=dict(model=tok_src,
                                                                   chat_template=config.chat_template),
                                        map_batches_kwargs=dict(concurrency=config.concurrency)))
    if config.tokenize:
        stages.append(TokenizeStage(fn_constructor_kwargs=dict(model=tok_src),
                                    map_batches_kwargs=dict(concurrency=config.concurrency)))
    gpus = config.num_gpus_per_worker
    if gpus is None:
        try:
            import torch

            gpus = 1 if torch.cuda.device_count() > 0 else 0
        except Exception:  # noqa: BLE001
            gpus = 0
    mb: Dict[str, Any] = dict(concurrency=config.concurrency, num_cpus=1)
    if gpus:
        mb["num_gpus"] = gpus
    if config.accelerator_type:
        mb["accelerator_type"] = config.accelerator_type
    stages.append(EngineStage(
        fn_constructor_kwargs=dict(model=config.model, model_source=model_src, tokenizer_source=tok_src,
                                   dtype=config.dtype, engine_kwargs=dict(config.engine_kwargs),
                                   sampling_params=dict(config.sampling_params), seed=config.seed),
        map_batches_kwargs=mb))
    if config.detokenize:
        stages.append(DetokenizeStage(fn_constructor_kwargs=dict(model=tok_src),
                                      map_batches_kwargs=dict(concurrency=config.concurrency)))
    return Processor(config, stages, **kwargs)


ProcessorBuilder.register(EngineProcessorConfig, build_engine_processor)
