#!/usr/bin/env python3
"""Burst serving (GPT-7B, 16 x 2048 -> 128, llmctl bench e2e shape) over scheduler policies and
per-step token budgets: one JSON line each (TTFT p50/p90, TPOT).

    python tools/serve_budget_sweep.py [policy:budget ...]   (default: a small sweep)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llmctl.benchmarks.serving import run_serving_benchmark

    arms = sys.argv[1:] or ["prefill_first:4096", "prefill_first:8192", "prefill_first:16384", "dynamic:8192",
                            "dynamic:16384"]
    for arm in arms:
        pol, budget = arm.split(":")
        r = run_serving_benchmark("gpt-7b", prompt_length=2048, gen_length=128, num_requests=16, max_batch_size=16,
                                  scheduler=pol, max_batch_tokens=int(budget))
        print(json.dumps({"arm": arm, "ttft_p50_ms": r["ttft_p50_ms"], "ttft_p90_ms": r["ttft_p90_ms"],
                          "tpot_mean_ms": r["tpot_mean_ms"], "wall_s": r["wall_s"],
                          "output_tokens_per_sec": r["output_tokens_per_sec"]}), flush=True)


if __name__ == "__main__":
    main()
