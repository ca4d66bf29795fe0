#!/usr/bin/env python3
"""Which hipBLASLt operand layout is fastest for each GPT-7B projection GEMM on MI355X?

For y = x W^T (x [T, in], W [out, in]) the three products of a training step are
fwd ``x @ W^T``, dgrad ``dy @ W``, wgrad ``dy^T @ x``.  If W is stored transposed
(Wt [in, out]) they become ``x @ Wt``, ``dy @ Wt^T`` and ``x^T @ dy``.  Times both.
"""
import json
import time

import torch

T = 16384
shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
          "lm_head": (32000, 4096)}


def bench(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


res = {}
for name, (out, inn) in shapes.items():
    x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
    Wt = W.t().contiguous()
    g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
    gt = torch.empty(inn, out, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * out * inn / 1e12
    r = {
        "fwd_xWt": bench(lambda: torch.nn.functional.linear(x, W)),
        "dgrad_dyW": bench(lambda: dy.matmul(W)),
        "wgrad_dyT_x": bench(lambda: torch.mm(dy.t(), x, out=g)),
        "fwd_x_Wt": bench(lambda: x.matmul(Wt)),
        "dgrad_dy_WtT": bench(lambda: dy.matmul(Wt.t())),
        "wgrad_xT_dy": bench(lambda: torch.mm(x.t(), dy, out=gt)),
    }
    res[name] = {k: {"ms": round(v, 3), "pflops": round(fl / v, 3)} for k, v in r.items()}
print(json.dumps(res))
