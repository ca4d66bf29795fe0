"""Data-loader throughput (``llmctl bench dataloader``): native C++ mmap loader vs numpy path."""

from __future__ import annotations

import os
import tempfile
import time
from typing import Any, Dict, Optional

import numpy as np


def _make_token_file(path: str, tokens: int, vocab: int = 32000) -> None:
    rng = np.random.default_rng(0)
    rng.integers(0, vocab, size=tokens, dtype=np.uint16).tofile(path)


def run_dataloader_benchmark(io: str = "local", path: Optional[str] = None, seq_len: int = 2048, batch_size: int = 8,
                             batches: int = 200) -> Dict[str, Any]:
    from llmctl.io.dataset import MemmapTokens
    from llmctl.io.synthetic import SyntheticTokens

    res: Dict[str, Any] = {"io": io, "seq_len": seq_len, "batch_size": batch_size, "batches": batches}
    if io == "synthetic":
        ds = SyntheticTokens(32000, seq_len, batch_size)
        t = time.perf_counter()
        for i in range(batches):
            ds.batch(i)
        dt = time.perf_counter() - t
        res["tokens_per_sec"] = batches * batch_size * seq_len / dt
        return res
    tmp = None
    if path is None:
        tmp = tempfile.NamedTemporaryFile(suffix=".bin", delete=False)
        tmp.close()
        path = tmp.name
        _make_token_file(path, max(batches * batch_size * (seq_len + 1) * 2, 1 << 22))
    try:
        for impl in ("native", "numpy"):
            ds = MemmapTokens(path, seq_len, batch_size, dtype="uint16")
            if impl == "numpy":
                ds._native = None
            elif ds._native is None:
                res["native"] = "not built"
                continue
            ds.next_batch()
            t = time.perf_counter()
            for _ in range(batches):
                ds.next_batch()
            dt = time.perf_counter() - t
            res[f"{impl}_tokens_per_sec"] = round(batches * batch_size * seq_len / dt, 1)
    finally:
        if tmp is not None:
            os.unlink(path)
    return res
