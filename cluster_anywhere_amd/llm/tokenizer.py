"""Tokenizers: a local HF tokenizer directory when given (no downloads), else
a byte-level fallback (UTF-8 bytes + 3 special ids) so the serving path works
with random-init weights and no network."""
from __future__ import annotations

from typing import List, Optional


class ByteTokenizer:
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


class HFTokenizer:
    def __init__(self, path: str):
        from transformers import AutoTokenizer

        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.eos_token_id = self.tok.eos_token_id
        self.vocab_size = len(self.tok)

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        return self.tok.encode(text, add_special_tokens=add_bos)

    def decode(self, ids: List[int]) -> str:
        return self.tok.decode(ids, skip_special_tokens=True)


def get_tokenizer(path: Optional[str] = None, vocab_size: int = 259):
    if path:
        return HFTokenizer(path)
    return ByteTokenizer(vocab_size)
