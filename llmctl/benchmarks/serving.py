"""End-to-end serving benchmark (``llmctl bench e2e``): TTFT / TPOT / throughput through the
paged-KV continuous-batching engine (in-process, no HTTP overhead).

Requests arrive all at once (``qps=None``) or as a Poisson process at ``qps``; prompts are
random token ids of ``prompt_length``; generation is ``gen_length`` tokens with
``ignore_eos`` (fixed work).  Reports p50/p90/p99 TTFT, mean TPOT, output tokens/s.
"""

from __future__ import annotations

import random
import time
from typing import Any, Dict, Optional

import numpy as np


def run_serving_benchmark(model: str = "gpt-7b", prompt_length: int = 2048, gen_length: int = 256,
                          qps: Optional[float] = None, num_requests: int = 16, max_batch_size: int = 16,
                          device: str = "auto", max_batch_tokens: Optional[int] = None, use_graphs: bool = True,
                          seed: int = 0, warmup: bool = True, scheduler: str = "dynamic",
                          kv_cache_dtype: str = "auto", weight_dtype: str = "auto") -> Dict[str, Any]:
    import torch

    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    max_len = prompt_length + gen_length + 16
    eng = InferenceEngine(model, device=device, max_batch_size=max_batch_size,
                          max_batch_tokens=max_batch_tokens or max(prompt_length,
                                                                   4096 if scheduler == "prefill_first" else 8192),
                          max_model_len=max_len,
                          use_graphs=use_graphs, seed=seed, scheduler=scheduler, kv_cache_dtype=kv_cache_dtype,
                          weight_dtype=weight_dtype)
    V = eng.cfg.vocab_size
    rng = random.Random(seed)
    params = SamplingParams(max_tokens=gen_length, temperature=0.0, ignore_eos=True)
    if warmup:  # capture decode graphs, warm the allocator and the GEMM / attention paths of the
        # full-length prefill batches the timed run will form (first-use costs stay out of TTFT)
        eng.generate([[1] * 16 for _ in range(min(max_batch_size, num_requests))],
                     SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
        eng.generate([[2] * prompt_length for _ in range(min(max_batch_size, num_requests))],
                     SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True))
    prompts = [[rng.randrange(V) for _ in range(prompt_length)] for _ in range(num_requests)]
    arrivals = [0.0] * num_requests
    if qps:
        t = 0.0
        for i in range(num_requests):
            t += rng.expovariate(qps)
            arrivals[i] = t
    seqs = []
    start = time.perf_counter()
    pending = list(range(num_requests))
    while pending or any(s.status != "finished" for s in seqs):
        now = time.perf_counter() - start
        while pending and arrivals[pending[0]] <= now:
            i = pending.pop(0)
            s = eng.add_request(prompts[i], params, request_id=str(i))
            s.arrival_time = time.time()
            seqs.append(s)
        if eng.scheduler.has_work():
            eng.step()
        elif pending:
            time.sleep(max(0.0, arrivals[pending[0]] - (time.perf_counter() - start)))
    if eng.device.type == "cuda":
        torch.cuda.synchronize()
    wall = time.perf_counter() - start
    ttft = np.array([s.first_token_time - s.arrival_time for s in seqs])
    tpot = np.array([(s.finish_time - s.first_token_time) / max(len(s.output_ids) - 1, 1) for s in seqs])
    out_tokens = sum(len(s.output_ids) for s in seqs)
    res = {
        "model": eng.cfg.name, "device": str(eng.device), "num_requests": num_requests,
        "prompt_length": prompt_length, "gen_length": gen_length, "qps": qps, "max_batch_size": max_batch_size, "scheduler": scheduler,
        "kv_cache_dtype": str(eng.kv_dtype).replace("torch.", ""), "decode_weight_dtype": eng.weight_dtype,
        "max_batch_tokens": eng.scheduler.max_batch_tokens,
        "ttft_p50_ms": round(float(np.percentile(ttft, 50)) * 1e3, 2),
        "ttft_p90_ms": round(float(np.percentile(ttft, 90)) * 1e3, 2),
        "ttft_p99_ms": round(float(np.percentile(ttft, 99)) * 1e3, 2),
        "tpot_mean_ms": round(float(tpot.mean()) * 1e3, 3),
        "output_tokens_per_sec": round(out_tokens / wall, 1),
        "total_tokens_per_sec": round((out_tokens + num_requests * prompt_length) / wall, 1),
        "wall_s": round(wall, 3), "graph_replays": eng.stats["graph_replays"],
        "kv_blocks": eng.kv.num_blocks, "data": "synthetic prompts, random-init weights",
    }
    eng.close()
    return res


def single_request_ttft(model: str = "gpt-7b", prompt_length: int = 2048, repeats: int = 5, device: str = "auto"
                        ) -> Dict[str, Any]:
    """p50 TTFT of an isolated request (prefill latency + first sample), the BASELINE serve metric."""
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    eng = InferenceEngine(model, device=device, max_batch_size=1, max_model_len=prompt_length + 32)
    p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    eng.generate([[1] * 32], p)  # warm-up
    ts = []
    for r in range(repeats + 1):
        s = eng.add_request([(7 * i + r) % eng.cfg.vocab_size for i in range(prompt_length)], p)
        s.arrival_time = time.time()
        while s.status != "finished":
            eng.step()
        if r > 0:
            ts.append(s.first_token_time - s.arrival_time)
    name = eng.cfg.name
    eng.close()
    return {"model": name, "prompt_length": prompt_length, "ttft_p50_ms": round(float(np.median(ts)) * 1e3, 2),
            "ttft_min_ms": round(min(ts) * 1e3, 2)}
