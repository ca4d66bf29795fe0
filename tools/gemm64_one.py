#!/usr/bin/env python3
"""Run one GEMM configuration a few times (for rocprofv3 --pmc runs), GPT-7B QKV shape at
24576 tokens.  Usage: gemm64_one.py {fwd|dgrad|wgrad|w4_*|torch_*} [config] [iters]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 104
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
assert _lib.load(), _lib._error
ops = torch.ops.llmctl
T, out, inn = 24576, 12288, 4096
x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
fns = {
    "fwd": lambda: ops.gemm64_ex(x, W, y, False, False, False, cfg),
    "dgrad": lambda: ops.gemm64_ex(dy, W, dx, False, True, False, cfg),
    "wgrad": lambda: ops.gemm64_ex(dy, x, g, True, True, False, cfg),
    "w4_fwd": lambda: ops.gemm_w4_ex(x, W, y, False, False, False, cfg),
    "w4_dgrad": lambda: ops.gemm_w4_ex(dy, W, dx, False, True, False, cfg),
    "w4_wgrad": lambda: ops.gemm_w4_ex(dy, x, g, True, True, False, cfg),
    "torch_fwd": lambda: torch.nn.functional.linear(x, W),
    "torch_dgrad": lambda: dy.matmul(W),
    "torch_wgrad": lambda: torch.mm(dy.t(), x, out=g),
}
for _ in range(iters):
    fns[kind]()
torch.cuda.synchronize()
print("ok", kind, cfg)
