#!/usr/bin/env python3
"""Which dK/dV kernel differs from the unpipelined one, and where (rows / heads)."""
import sys
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

ops = _lib.native()
for (B, S, Hq, Hkv) in [(1, 512, 4, 4), (2, 320, 8, 2), (1, 2048, 2, 2), (3, 256, 24, 8), (12, 2048, 32, 32)]:
    D = 128
    g = torch.Generator(device="cuda")
    def bf(*sh, seed):
        g.manual_seed(seed)
        return torch.randn(*sh, generator=g, device="cuda").to(torch.bfloat16)
    q, k, v, do = bf(B, S, Hq, D, seed=61), bf(B, S, Hkv, D, seed=62), bf(B, S, Hkv, D, seed=63), bf(B, S, Hq, D, seed=64)
    o, lse = ops.flash_attn_fwd(q, k, v, D ** -0.5, True)
    delta = (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()
    outs = {}
    for impl in (3, 4, 6, 6):
        dq, dk, dv = torch.zeros_like(q), torch.zeros_like(k), torch.zeros_like(v)
        ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, impl)
        torch.cuda.synchronize()
        key = impl if impl not in outs else impl + 100
        outs[key] = (dk, dv)
    for key in (4, 6, 106):
        dk, dv = outs[key]
        bk = (dk != outs[3][0]).any(-1)  # [B, S, Hkv]
        bv = (dv != outs[3][1]).any(-1)
        rows = bk.nonzero()[:8].tolist()
        mx = (dk.float() - outs[3][0].float()).abs().max().item()
        print(f"B{B} S{S} Hq{Hq} Hkv{Hkv} impl {key}: dk rows differ {int(bk.sum())}/{bk.numel()} dv {int(bv.sum())} maxdiff {mx:.3g} first {rows}", flush=True)
