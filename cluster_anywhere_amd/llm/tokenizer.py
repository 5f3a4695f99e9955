"""Tokenizers: a local HF tokenizer directory when given (no downloads), else
a byte-level fallback (UTF-8 bytes + 3 special ids) so the serving path works
with random-init weights and no network.

Both expose the slice of the HF tokenizer interface the serving and batch
stages use (reference: python/ray/llm/_internal/batch/utils.py:13
``get_cached_tokenizer`` and the chat-template / tokenize / detokenize stages):
``encode`` / ``decode``, batched ``__call__(texts)["input_ids"]``,
``batch_decode`` and ``apply_chat_template``. :func:`load_tokenizer` caches one
instance per source per process (building an HF tokenizer costs ~100 ms).
"""
from __future__ import annotations

import os
import threading
from typing import Any, Dict, List, Optional, Sequence


def _content_text(content: Any) -> str:
    """OpenAI message content: a string or a list of parts (text parts joined,
    image parts dropped — images travel in their own column)."""
    if isinstance(content, str):
        return content
    if content is None:
        return ""
    out = []
    for part in content:
        if isinstance(part, dict):
            if part.get("type", "text") == "text":
                out.append(str(part.get("text", "")))
        else:
            out.append(str(part))
    return "".join(out)


def render_chat(messages: Sequence[Dict[str, Any]], add_generation_prompt: bool = True) -> str:
    """The built-in chat template (used when a tokenizer carries none):
    ``<|role|>content\\n`` per message, then ``<|assistant|>``."""
    text = "".join(f"<|{m['role']}|>{_content_text(m.get('content'))}\n" for m in messages)
    return text + ("<|assistant|>" if add_generation_prompt else "")


class _BatchAPI:
    def __call__(self, texts, add_special_tokens: bool = True):
        if isinstance(texts, str):
            return {"input_ids": self.encode(texts, add_bos=add_special_tokens)}
        return {"input_ids": [self.encode(t, add_bos=add_special_tokens) for t in texts]}

    def batch_decode(self, seqs, skip_special_tokens: bool = True) -> List[str]:
        return [self.decode(list(s)) for s in seqs]

    def apply_chat_template(self, conversations, tokenize: bool = False, add_generation_prompt: bool = True,
                            chat_template: Optional[str] = None):
        single = bool(conversations) and isinstance(conversations[0], dict)
        convs = [conversations] if single else conversations
        texts = [render_chat(c, add_generation_prompt) for c in convs]
        if tokenize:
            texts = [self.encode(t) for t in texts]
        return texts[0] if single else texts


class ByteTokenizer(_BatchAPI):
    bos_token_id, eos_token_id, pad_token_id = 1, 2, 0
    offset = 3

    def __init__(self, vocab_size: int = 259):
        self.vocab_size = max(vocab_size, 259)

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [b + self.offset for b in text.encode("utf-8")]
        return ([self.bos_token_id] if add_bos else []) + ids

    def decode(self, ids: List[int]) -> str:
        bs = bytes(i - self.offset for i in ids if self.offset <= i < 256 + self.offset)
        return bs.decode("utf-8", errors="replace")


class HFTokenizer(_BatchAPI):
    def __init__(self, path: str):
        from transformers import AutoTokenizer

        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.eos_token_id = self.tok.eos_token_id
        self.vocab_size = len(self.tok)

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        return self.tok.encode(text, add_special_tokens=add_bos)

    def decode(self, ids: List[int]) -> str:
        return self.tok.decode(ids, skip_special_tokens=True)

    def __call__(self, texts, add_special_tokens: bool = True):
        return {"input_ids": self.tok(texts, add_special_tokens=add_special_tokens)["input_ids"]}

    def batch_decode(self, seqs, skip_special_tokens: bool = True) -> List[str]:
        return self.tok.batch_decode([list(s) for s in seqs], skip_special_tokens=skip_special_tokens)

    def apply_chat_template(self, conversations, tokenize: bool = False, add_generation_prompt: bool = True,
                            chat_template: Optional[str] = None):
        if chat_template is None and getattr(self.tok, "chat_template", None) is None:
            return super().apply_chat_template(conversations, tokenize, add_generation_prompt)
        return self.tok.apply_chat_template(conversations, tokenize=tokenize,
                                            add_generation_prompt=add_generation_prompt,
                                            chat_template=chat_template)


def get_tokenizer(path: Optional[str] = None, vocab_size: int = 259):
    if path:
        return HFTokenizer(path)
    return ByteTokenizer(vocab_size)


_cache: Dict[Any, Any] = {}
_cache_lock = threading.Lock()


def load_tokenizer(source: Optional[str] = None, vocab_size: int = 259):
    """Tokenizer for ``source``: a local HF tokenizer directory, or (a model preset
    name / ``None`` / ``"byte"``) the byte tokenizer. Cached per process."""
    key = (source if source and os.path.isdir(source) else None, vocab_size)
    with _cache_lock:
        tok = _cache.get(key)
        if tok is None:
            tok = get_tokenizer(key[0], vocab_size)
            _cache[key] = tok
        return tok
