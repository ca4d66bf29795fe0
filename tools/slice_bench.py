"""Layer-slice training benchmark for models too large for one GPU (BASELINE config #4, Llama-3
70B): the real layer dimensions (hidden 8192, ffn 28672, 64 q / 8 kv heads, vocab 128256) with
only ``--layers`` decoder layers, full fwd + bwd + AdamW on one GPU.  Two depths give the
per-layer step time (slope) and the embedding / LM-head / optimizer overhead (intercept); the
layer stack's MFU is the slope's.  Synthetic tokens, random-init weights, bf16.

    python tools/slice_bench.py --model llama-70b --layers 2 6 --micro-batch 2
"""

import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model, layers, mb, seq, steps, warmup):
    import torch

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = dataclasses.replace(get_model_config(model), layers=layers)
    cfg = TrainingConfig(model_name_or_path=model, batch_size=mb, seq_len=seq, max_steps=steps + warmup,
                         learning_rate=1e-4, device="cuda", log_level="warning")
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, seq, mb, seed=1, rank=0, device=eng.device)
    for i in range(warmup):
        eng.train_step([data.batch(i)])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(steps):
        out = eng.train_step([data.batch(warmup + i)])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    res = {"model": mc.name, "layers": layers, "micro_batch": mb, "seq_len": seq, "ms_per_step": round(dt * 1e3, 2),
           "tokens_per_s": round(mb * seq / dt, 1), "loss": round(float(out["loss"]), 4),
           "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1)}
    eng.shutdown()
    del eng
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    return res, mc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-70b")
    ap.add_argument("--layers", type=int, nargs=2, default=[2, 6])
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    rows = []
    for L in a.layers:
        r, mc = run(a.model, L, a.micro_batch, a.seq_len, a.steps, a.warmup)
        rows.append((r, mc))
        print(json.dumps(r), flush=True)
    (r0, m0), (r1, m1) = rows
    per_layer_ms = (r1["ms_per_step"] - r0["ms_per_step"]) / (r1["layers"] - r0["layers"])
    tokens = a.micro_batch * a.seq_len
    layer_flops = (m1.flops_per_token(a.seq_len) - m0.flops_per_token(a.seq_len)) / (r1["layers"] - r0["layers"])
    print(json.dumps({"model": m0.name, "per_layer_ms": round(per_layer_ms, 3),
                      "overhead_ms": round(r0["ms_per_step"] - per_layer_ms * r0["layers"], 2),
                      "layer_stack_mfu": round(layer_flops * tokens / (per_layer_ms * 1e-3) / 2.5e15, 4),
                      "tokens_per_step": tokens}), flush=True)


if __name__ == "__main__":
    main()
