"""Batch LLM inference over Datasets (reference: python/ray/llm/_internal/batch)."""
from .processor import (EngineProcessorConfig, HttpRequestProcessorConfig, Processor, ProcessorBuilder,
                        ProcessorConfig, build_engine_processor, build_http_request_processor)
from .stages import (ChatTemplateStage, DetokenizeStage, EngineStage, HttpRequestStage, PrepareImageStage,
                     StatefulStage, StatefulStageUDF, TokenizeStage, wrap_postprocess, wrap_preprocess)

__all__ = ["ProcessorConfig", "Processor", "ProcessorBuilder", "HttpRequestProcessorConfig",
           "EngineProcessorConfig", "build_http_request_processor", "build_engine_processor",
           "StatefulStage", "StatefulStageUDF", "ChatTemplateStage", "TokenizeStage", "DetokenizeStage",
           "HttpRequestStage", "PrepareImageStage", "EngineStage", "wrap_preprocess", "wrap_postprocess"]
