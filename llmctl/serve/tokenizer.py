"""Tokenizers for serving/eval without network access.

* :class:`ByteTokenizer` — UTF-8 bytes as ids 0..255, ``<eos>`` = 256 (works for any model
  whose vocab ≥ 257; used for random-init models and synthetic benchmarks);
* :func:`load_tokenizer` — a ``tokenizer.json`` (HF ``tokenizers`` format) next to a
  checkpoint is used when present (the reference saved one with ``save_pretrained``,
  ``engine.py:382``), else the byte tokenizer.
"""

from __future__ import annotations

from pathlib import Path
from typing import List, Optional


class ByteTokenizer:
    eos_token_id = 256
    bos_token_id = None
    pad_token_id = 0

    def encode(self, text: str) -> List[int]:
        return list(text.encode("utf-8"))

    def decode(self, ids: List[int]) -> str:
        return bytes(i for i in ids if 0 <= i < 256).decode("utf-8", errors="replace")

    @property
    def vocab_size(self) -> int:
        return 257


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(path)
        self.eos_token_id = None
        for cand in ("</s>", "<|endoftext|>", "<|end_of_text|>", "<eos>"):
            i = self.tok.token_to_id(cand)
            if i is not None:
                self.eos_token_id = i
                break

    def encode(self, text: str) -> List[int]:
        return self.tok.encode(text).ids

    def decode(self, ids: List[int]) -> str:
        return self.tok.decode(ids)

    @property
    def vocab_size(self) -> int:
        return self.tok.get_vocab_size()


def load_tokenizer(model_path: Optional[str]):
    if model_path:
        p = Path(model_path)
        if p.is_dir() and (p / "tokenizer.json").exists():
            try:
                return HFTokenizer(str(p / "tokenizer.json"))
            except Exception:
                pass
    return ByteTokenizer()
