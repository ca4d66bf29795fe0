#!/usr/bin/env python3
"""Decode-GEMM streaming bandwidth (M = 16 tokens, GPT-7B projections, bf16): each timed call
reads a different weight copy (8 copies rotate: no L2 / MALL reuse), TB/s of weight bytes per
config of skinny_linear_cfg (0 = automatic) and hipBLASLt.

    python tools/decode_gemm_bw.py [--configs 0 23 25] [--m 16]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008), "lm": (32000, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--configs", type=int, nargs="+", default=[0, 23, 25])
    ap.add_argument("--copies", type=int, default=8)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--knob", action="append", default=[])
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    for kv in a.knob:
        k, v = kv.split("=")
        ops.set_knob(k, int(v))
    for name, (N, K) in SHAPES.items():
        x = torch.randn(a.m, K, device="cuda").to(torch.bfloat16)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(a.copies)]
        row = {"shape": name, "N": N, "K": K, "M": a.m}
        runs = [(f"c{c}", lambda w, c=c: ops.skinny_linear_cfg(x, w, None, c)) for c in a.configs]
        runs.append(("hipblaslt", lambda w: torch.nn.functional.linear(x, w)))
        ref = (x.float() @ ws[0].float().t())
        for tag, fn in runs:
            row[tag + "_err"] = round(((fn(ws[0]).float() - ref).abs().max() / ref.abs().max()).item(), 5)
            # captured: a graph of `iters` back-to-back calls times the kernels, not the host
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for i in range(a.copies):
                    fn(ws[i])
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(a.iters):
                    fn(ws[i % a.copies])
            g.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / a.iters
            row[tag + "_us"] = round(dt * 1e6, 1)
            row[tag + "_tbs"] = round(N * K * 2 / dt / 1e12, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
