#!/usr/bin/env python3
"""Serving decode step cost (GPT-7B, 16 x 2048-token prompts, greedy): host wall time per decode
step through ``InferenceEngine.step()`` with the synchronous and the pipelined (knob
``async_decode``) decode paths, against the device time of one decode graph replay (decode +
in-graph sampling, CUDA events, same batch).  The pipelined path launches step N + 1 before reading
step N's tokens, so its host ms/step should sit on the device time.

    python tools/decode_host_breakdown.py [--tokens 96] [--prompt 2048] [--batch 16]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-7b")
    ap.add_argument("--tokens", type=int, default=96)
    ap.add_argument("--prompt", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--kv-cache-dtype", default="auto")
    ap.add_argument("--weight-dtype", default="auto", help="decode projection weights: auto (bf16) | fp8")
    a = ap.parse_args()
    import torch
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    eng = InferenceEngine(a.model, device="cuda", max_batch_size=a.batch, max_model_len=a.prompt + a.tokens + 64,
                          kv_cache_dtype=a.kv_cache_dtype, weight_dtype=a.weight_dtype)
    p = SamplingParams(max_tokens=a.tokens, temperature=0.0, ignore_eos=True)
    base = eng.knobs
    for rnd in range(3):
        for mode in (False, True):
            eng.knobs = dataclasses.replace(base, async_decode=mode)
            seqs = [eng.add_request([(7 * i + r + rnd) % 32000 for i in range(a.prompt)], p) for r in range(a.batch)]
            while any(s.first_token_time is None for s in seqs):  # prefills (+ first tokens)
                eng.step()
            torch.cuda.synchronize()
            start = [len(s.output_ids) for s in seqs]
            t0 = time.perf_counter()
            while any(s.status != "finished" for s in seqs):
                eng.step()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            steps = max(len(s.output_ids) - s0 for s, s0 in zip(seqs, start))
            if rnd > 0:
                print(json.dumps({"async_decode": mode, "decode_steps": steps, "host_ms_per_step": round(wall / steps, 3),
                                  "continued": eng.stats.get("async_continued", 0)}), flush=True)
    # device time of one decode step (graph replay incl. in-graph sampling) for this batch
    g, b = eng._graphs[eng._bucket(a.batch)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        g.replay()
    ev[0].record()
    for _ in range(20):
        g.replay()
    ev[1].record()
    torch.cuda.synchronize()
    print(json.dumps({"gpu_ms_per_step": round(ev[0].elapsed_time(ev[1]) / 20, 3), "batch": a.batch,
                      "context": a.prompt, "kv_cache_dtype": a.kv_cache_dtype,
                      "weight_dtype": a.weight_dtype}), flush=True)


if __name__ == "__main__":
    main()
