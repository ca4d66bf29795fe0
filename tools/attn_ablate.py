#!/usr/bin/env python3
"""Timing of the flash-attention backward kernels (B8 S2048 H32 D128 causal, random data):
abl 0 = dQ + dK/dV kernels, 1 = dK/dV kernel only, 2 = dQ kernel only, 3 / 4 / 6 = dK/dV through the
unpipelined / software-pipelined / persistent kernel; plus the whole
``flash_attn_bwd`` op (delta pre-kernel included) and the forward for reference."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

ops = _lib.native()
B, S, H, D = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (8, 2048, 32, 128)))
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k, v, do = (torch.randn_like(q) for _ in range(3))
scale = D ** -0.5
o, lse = ops.flash_attn_fwd(q, k, v, scale, True)
delta = (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
fl_fwd = 4 * B * H * S * S * D * 0.5
fl = 2.5 * fl_fwd  # the 5 bwd products of the fused formulation (the split form does 7)


def timeit(f):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / 5)
    return sorted(ts)[2] * 1e3


res = {"shape": [B, S, H, D]}
for abl, name in [(0, "dq+dkv"), (1, "dkv"), (2, "dq"), (3, "dkv_unpipelined"), (4, "dkv_pipelined"),
                  (6, "dkv_persistent"), (3, "dkv_unpipelined_again"), (4, "dkv_pipelined_again"),
                  (6, "dkv_persistent_again")]:
    ms = timeit(lambda: ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, abl))
    res[name] = {"ms": round(ms, 3), "tflops_equiv_5prod": round(fl / ms / 1e9, 1)}
    print(name, res[name], flush=True)
ms = timeit(lambda: ops.flash_attn_bwd(do, q, k, v, o, lse, scale, True))
res["flash_attn_bwd_op"] = {"ms": round(ms, 3), "tflops_equiv_5prod": round(fl / ms / 1e9, 1)}
ms = timeit(lambda: ops.flash_attn_fwd(q, k, v, scale, True))
res["flash_attn_fwd_op"] = {"ms": round(ms, 3), "tflops": round(fl_fwd / ms / 1e9, 1)}
print(json.dumps(res), flush=True)
