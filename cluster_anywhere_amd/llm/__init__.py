"""Native LLM inference: paged-KV continuous-batching engine over the Llama
model and gfx950 kernels (reference: python/ray/llm — which wraps vLLM)."""
from .engine import BlockAllocator, LLMEngine, RequestOutput, SamplingParams

__all__ = ["LLMEngine", "SamplingParams", "RequestOutput", "BlockAllocator"]
