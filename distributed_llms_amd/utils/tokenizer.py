"""Tokenization for the master's text interface.

The reference tokenizes with an HF ``AutoTokenizer`` downloaded from the hub
(``src/model/loader.py:6``) and then fails to encode the result (D8).  There is no
network here, so a locally available HF tokenizer is used when the checkpoint ships one,
and otherwise a reversible UTF-8 byte tokenizer (ids 3..258) stands in -- enough to drive
the text REPL end to end with random-init models.
"""
from __future__ import annotations

from typing import List


class ByteTokenizer:
    OFFSET = 3

    def __init__(self, vocab_size: int = 259):
        if vocab_size < 259:
            raise ValueError("ByteTokenizer needs vocab_size >= 259")
        self.vocab_size = vocab_size

    def encode(self, text: str) -> List[int]:
        return [b + self.OFFSET for b in text.encode("utf-8")] or [self.OFFSET]

    def decode(self, ids) -> str:
        return bytes((int(i) - self.OFFSET) % 256 for i in ids).decode("utf-8", errors="replace")


class HFTokenizerAdapter:
    def __init__(self, tok):
        self.tok = tok

    def encode(self, text: str) -> List[int]:
        return list(self.tok(text)["input_ids"])

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=True)


def get_tokenizer(hf_tokenizer=None, vocab_size: int = 259):
    if hf_tokenizer is not None:
        return HFTokenizerAdapter(hf_tokenizer)
    return ByteTokenizer(max(vocab_size, 259))
