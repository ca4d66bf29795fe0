#!/usr/bin/env python3
"""Timing ablations of the flash-attention backward main kernel (B8 S2048 H32 D128 causal)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

ops = _lib.native()
B, S, H, D = 8, 2048, 32, 128
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k, v, o, do = (torch.randn_like(q) for _ in range(4))
lse = torch.randn(B, H, S, device="cuda") * 0.1 + 5
dq = torch.zeros(B, S, H, D, device="cuda")
dk, dv = torch.empty_like(q), torch.empty_like(q)
fl = 2.5 * 4 * B * H * S * S * D * 0.5
res = {}
for abl in [0, 1, 2, 4, 6]:
    f = lambda: ops.fa_bwd_ablate(do, q, k, v, o, lse, dq, dk, dv, abl)  # noqa: E731
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / 5)
    ms = sorted(ts)[2] * 1e3
    res[abl] = {"ms": round(ms, 3), "tflops_equiv": round(fl / ms / 1e9, 1)}
    print(abl, res[abl], flush=True)
print(json.dumps(res))
