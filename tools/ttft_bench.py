#!/usr/bin/env python3
"""Single-request serve TTFT (BASELINE serve metric): GPT-7B, 2048-token prompt, p50 over repeats."""
import argparse
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-7b")
    ap.add_argument("--prompt-length", type=int, default=2048)
    ap.add_argument("--repeats", type=int, default=10)
    a = ap.parse_args()
    from llmctl.benchmarks.serving import single_request_ttft

    print(json.dumps(single_request_ttft(a.model, a.prompt_length, a.repeats)), flush=True)


if __name__ == "__main__":
    main()
