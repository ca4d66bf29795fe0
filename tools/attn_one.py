#!/usr/bin/env python3
"""Run ONE flash-attention kernel repeatedly (for rocprofv3 --pmc passes):
    attn_one.py {fwd|dkv|dq|dkv_old|dkv_pipe} [iters] [B S H D]
Env ATTN_KNOBS="name=value,..." sets native knobs first (e.g. fa_w64=3)."""
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

kind = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, S, H, D = (int(x) for x in (sys.argv[3:7] if len(sys.argv) > 6 else (8, 2048, 32, 128)))
ops = _lib.native()
for kv in filter(None, os.environ.get("ATTN_KNOBS", "").split(",")):
    name, val = kv.split("=")
    ops.set_knob(name, int(val))
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k, v, do = (torch.randn_like(q) for _ in range(3))
scale = D ** -0.5
o, lse = ops.flash_attn_fwd(q, k, v, scale, True)
delta = (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(iters):
    if kind == "fwd":
        ops.flash_attn_fwd(q, k, v, scale, True)
    else:
        ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, {"dkv": 1, "dq": 2, "dkv_old": 3, "dkv_pipe": 4}[kind])
torch.cuda.synchronize()
print("ok", kind)
