"""Checkpoint evaluation (``llmctl eval run``): perplexity, latency, throughput."""

from __future__ import annotations

import math
import time
from typing import Any, Dict, List, Optional

import torch


def _batches(data: Optional[str], vocab: int, seq_len: int, batch_size: int, n: int, device):
    if data:
        from llmctl.io.dataset import MemmapTokens, tokenize_to_bin
        from pathlib import Path

        p = Path(data)
        if p.suffix in (".txt", ".jsonl"):
            dst = p.with_suffix(".bin")
            if not dst.exists():
                tokenize_to_bin(str(p), str(dst))
            p = dst
        ds = MemmapTokens(str(p), seq_len, batch_size, device=device)
        for _ in range(n):
            x, y = ds.next_batch()
            yield x.to(device), y.to(device)
    else:
        from llmctl.io.synthetic import SyntheticTokens

        ds = SyntheticTokens(vocab, seq_len, batch_size, seed=999, device=device)
        for i in range(n):
            yield ds.batch(i)


@torch.no_grad()
def perplexity(model, cfg, data, seq_len, batch_size, batches, device) -> Dict[str, Any]:
    tot, count = 0.0, 0
    for x, y in _batches(data, cfg.vocab_size, seq_len, batch_size, batches, device):
        loss = model(x, y)
        tot += float(loss) * y.numel()
        count += y.numel()
    nll = tot / max(count, 1)
    return {"nll": nll, "perplexity": math.exp(min(nll, 50.0)), "tokens": count,
            "data": data or "synthetic (uniform random tokens: ppl ~ vocab for an untrained model)"}


def evaluate(ckpt: str, tasks: List[str], data: Optional[str] = None, seq_len: int = 512, batches: int = 4,
             batch_size: int = 2, device: str = "auto") -> Dict[str, Any]:
    from llmctl.io.artifact import load_model

    dev = torch.device("cuda" if (device == "auto" and torch.cuda.is_available()) or device == "cuda" else "cpu")
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model, cfg, ck = load_model(ckpt, device=dev, dtype=dtype)
    model.eval()
    out: Dict[str, Any] = {"checkpoint": str(ck or ckpt), "model": cfg.name, "device": str(dev)}
    for t in tasks:
        if t == "perplexity":
            out["perplexity"] = perplexity(model, cfg, data, seq_len, batch_size, batches, dev)
        elif t == "latency":
            from llmctl.benchmarks.serving import single_request_ttft

            out["latency"] = single_request_ttft(str(ck or ckpt), prompt_length=min(seq_len, 2048), repeats=3,
                                                 device=str(dev))
        elif t == "throughput":
            model.train()
            x = torch.randint(0, cfg.vocab_size, (batch_size, seq_len), device=dev)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                loss = model(x, x)
                loss.backward()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            out["throughput"] = {"train_tokens_per_sec_fwd_bwd": batch_size * seq_len / dt}
            model.eval()
        else:
            out[t] = {"error": f"unknown task {t} (perplexity | latency | throughput)"}
    return out
