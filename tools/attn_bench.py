#!/usr/bin/env python3
"""Attention kernel throughput: llmctl HIP flash-attn fwd/bwd vs torch SDPA on MI355X."""
import argparse, json, time
import torch
import torch.nn.functional as F
from llmctl.ops import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=8); ap.add_argument("--S", type=int, default=2048)
ap.add_argument("--H", type=int, default=32); ap.add_argument("--Hkv", type=int, default=32)
ap.add_argument("--D", type=int, default=128); ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--no-causal", action="store_true")
a = ap.parse_args()
causal = not a.no_causal
ops = _lib.native()
dev = "cuda"
q = torch.randn(a.B, a.S, a.H, a.D, device=dev, dtype=torch.bfloat16)
k = torch.randn(a.B, a.S, a.Hkv, a.D, device=dev, dtype=torch.bfloat16)
v = torch.randn(a.B, a.S, a.Hkv, a.D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(q)
scale = a.D ** -0.5
flops_fwd = 4 * a.B * a.H * a.S * a.S * a.D * (0.5 if causal else 1.0)

def timeit(fn, n):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n

o, lse = ops.flash_attn_fwd(q, k, v, scale, causal)
tf = timeit(lambda: ops.flash_attn_fwd(q, k, v, scale, causal), a.iters)
tb = timeit(lambda: ops.flash_attn_bwd(do, q, k, v, o, lse, scale, causal), a.iters)
res = {"shape": [a.B, a.S, a.H, a.Hkv, a.D], "causal": causal,
       "llmctl_fwd_ms": tf * 1e3, "llmctl_fwd_tflops": flops_fwd / tf / 1e12,
       "llmctl_bwd_ms": tb * 1e3, "llmctl_bwd_tflops": 2.5 * flops_fwd / tb / 1e12}
try:
    qt, kt, vt = [t.transpose(1, 2).contiguous().requires_grad_(True) for t in (q, k, v)]
    gq = a.H // a.Hkv
    kt2 = kt.repeat_interleave(gq, 1) if gq > 1 else kt
    vt2 = vt.repeat_interleave(gq, 1) if gq > 1 else vt
    ts = timeit(lambda: F.scaled_dot_product_attention(qt, kt2, vt2, is_causal=causal), a.iters)
    out = F.scaled_dot_product_attention(qt, kt2, vt2, is_causal=causal)
    dot = do.transpose(1, 2).contiguous()
    tsb = timeit(lambda: torch.autograd.grad(out, (qt, kt, vt), dot, retain_graph=True), a.iters)
    res.update({"sdpa_fwd_ms": ts * 1e3, "sdpa_fwd_tflops": flops_fwd / ts / 1e12, "sdpa_bwd_ms": tsb * 1e3,
                "sdpa_bwd_tflops": 2.5 * flops_fwd / tsb / 1e12})
except Exception as e:
    res["sdpa_error"] = str(e)[:200]
print(json.dumps(res))
