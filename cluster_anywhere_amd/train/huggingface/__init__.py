"""Hugging Face integrations (reference: python/ray/train/huggingface/)."""
from . import transformers  # noqa: F401

__all__ = ["transformers"]
