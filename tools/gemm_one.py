#!/usr/bin/env python3
"""Run one gemm_ex configuration a few times (for rocprofv3 --pmc runs).
Usage: gemm_one.py {fwd|dgrad|wgrad} [variant] [iters]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "wgrad"
v = int(sys.argv[2]) if len(sys.argv) > 2 else -1
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
assert _lib.load(), _lib._error
ops = torch.ops.llmctl
T, out, inn = 16384, 22016, 4096
x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    if kind == "fwd":
        ops.gemm_ex(x, W, y, False, False, False, v)
    elif kind == "dgrad":
        ops.gemm_ex(dy, W, dx, False, True, False, v)
    elif kind == "torch_wgrad":
        torch.mm(dy.t(), x, out=g)
    elif kind == "torch_fwd":
        torch.nn.functional.linear(x, W)
    else:
        ops.gemm_ex(dy, x, g, True, True, False, v)
torch.cuda.synchronize()
print("ok", kind, v)
