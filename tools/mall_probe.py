#!/usr/bin/env python3
"""Does a decode GEMM run faster when (part of) its weights were read just before it?

For each GPT-7B projection (M = 16 tokens, the fused decode path's partials kernel) the GEMM
alone is timed with events after: a 2 GB flush read (cold), the flush plus a read of the first
``frac`` of the weight rows (warm-partial), the flush plus a read of every weight row (warm), and
right after the same GEMM (repeat).  A read that allocates in the Infinity Cache (MALL, 256 MB)
or L2 makes the warm runs faster; the prefetch read's own time is printed alongside.

    python tools/mall_probe.py [--reps 20] [--fracs 0.25 0.5]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fracs", type=float, nargs="+", default=[0.25, 0.5])
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    flush = torch.empty(1 << 30, dtype=torch.bfloat16, device="cuda").fill_(1.0)  # 2 GB
    sink = torch.empty((), device="cuda")
    for name, (N, K) in SHAPES.items():
        x = torch.randn(16, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        gemm = lambda: ops.decode_linear_partials(x, w, None)  # noqa: E731
        gemm()

        def timed(pre):
            ts, tp = [], []
            for _ in range(a.reps):
                torch.sum(flush, dim=0, dtype=torch.float32, out=sink)
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                pre()
                e1.record()
                gemm()
                e2.record()
                torch.cuda.synchronize()
                tp.append(e0.elapsed_time(e1) * 1e3)
                ts.append(e1.elapsed_time(e2) * 1e3)
            ts.sort()
            tp.sort()
            return round(ts[len(ts) // 2], 1), round(tp[len(tp) // 2], 1)

        row = {"shape": name, "MB": round(N * K * 2 / 1e6, 1)}
        row["cold_us"], _ = timed(lambda: None)
        for f in a.fracs + [1.0]:
            n = int(N * f)
            row[f"warm{f}_us"], row[f"pre{f}_us"] = timed(lambda n=n: torch.sum(w[:n], dim=(0, 1), dtype=torch.float32, out=sink))
        row["repeat_us"], _ = timed(gemm)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
