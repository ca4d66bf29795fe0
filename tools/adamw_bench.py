#!/usr/bin/env python3
"""Fused AdamW step over a flat buffer (bf16 params / grads, fp32 master and moments), HBM rate.
    LLMCTL_ADAMW_NT=0|1 python tools/adamw_bench.py [numel]"""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops._lib import native  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(2e9)
dev = "cuda"
p = torch.zeros(n, device=dev, dtype=torch.bfloat16)
g = torch.randn(n, device=dev).to(torch.bfloat16)
w, m, v = (torch.zeros(n, device=dev) for _ in range(3))
ops = native()
f = lambda: ops.adamw_step_(p, w, g, m, v, 1e-4, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.5, None)  # noqa: E731
f()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    f()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 10
print(json.dumps({"nt": os.environ.get("LLMCTL_ADAMW_NT", "1"), "numel": n, "ms": round(ms, 3),
                  "TBps": round(28.0 * n / ms / 1e9, 2)}))
