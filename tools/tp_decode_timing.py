#!/usr/bin/env python3
"""TP serving decode loop, host vs device time per step (config #5's pipeline): TP = --world
processes on cuda:0 (gloo default group, custom IPC all-reduces, decode hipGraphs with in-graph
sampling), greedy decode of --batch prompts of --prompt tokens, pipelined (knob async_decode on)
then synchronous, on one engine.  Prints one JSON line per run (llmctl.testing.workers.serve_async_gpu).

    python tools/tp_decode_timing.py --world 2 --model gpt-7b --batch 16 --prompt 512 --tokens 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--model", default="gpt-7b")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--kv-blocks", type=int, default=1024)
    a = ap.parse_args()
    from llmctl.testing.harness import run_ranks
    from llmctl.testing.workers import serve_async_gpu

    prompts = [[(7 * i + r) % 32000 + 1 for i in range(a.prompt)] for r in range(a.batch)]
    kw = {"max_batch_size": a.batch, "num_kv_blocks": a.kv_blocks, "max_model_len": a.prompt + a.tokens + 64,
          "max_batch_tokens": 8192}
    env = {"GPU_MAX_HW_QUEUES": "1"} if a.world > 4 else None
    out = run_ranks(serve_async_gpu, a.world, a.model, env, kw, prompts, a.tokens, timeout=900)[0]
    for mode in (1, 0):
        print(json.dumps({"tp": a.world, "model": a.model, "batch": a.batch, "prompt": a.prompt,
                          "async_decode": bool(mode), "continued": out[f"continued_{mode}"],
                          "host_ms_per_step": round(out[f"host_ms_{mode}"], 3),
                          "gpu_ms_per_step": round(out[f"gpu_ms_{mode}"], 3)}), flush=True)
    print(json.dumps({"tokens_equal": out["tokens_1"] == out["tokens_0"]}), flush=True)


if __name__ == "__main__":
    main()
