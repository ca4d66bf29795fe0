#!/usr/bin/env python3
"""Run one gemm64 configuration (or hipBLASLt) on a GPT-7B shape a few times, for rocprofv3
--pmc passes.  Usage: gemm64_one.py {fwd|dgrad|wgrad} {config|torch} [iters] [shape]
(shape: qkv | o | up | down; 32768 tokens)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.exec.gemm_tuning import enable_tuned_gemms  # noqa: E402
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}
kind = sys.argv[1]
cfg = sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
out, inn = SHAPES[sys.argv[4] if len(sys.argv) > 4 else "up"]
assert _lib.load(), _lib._error
enable_tuned_gemms()
ops = torch.ops.llmctl
T = 32768
x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
Wt = W.t().contiguous()
y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    if cfg == "torch":
        if kind == "fwd":
            torch.nn.functional.linear(x, W)
        elif kind == "dgrad":
            torch.nn.functional.linear(dy, Wt)
        else:
            torch.mm(dy.t(), x, out=g)
    else:
        c = int(cfg)
        if kind == "fwd":
            ops.gemm64_ex(x, W, y, False, False, False, c)
        elif kind == "dgrad":
            ops.gemm64_ex(dy, W, dx, False, True, False, c)
        else:
            ops.gemm64_ex(dy, x, g, True, True, False, c)
torch.cuda.synchronize()
print("ok", kind, cfg)
