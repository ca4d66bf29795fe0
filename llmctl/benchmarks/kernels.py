"""Kernel benchmarks (``llmctl bench kernels``): llmctl HIP kernels vs PyTorch counterparts."""

from __future__ import annotations

import time
from typing import Any, Dict

import torch


def _t(fn, iters: int = 10) -> float:
    fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def run_kernel_benchmarks(attention=True, matmul=True, kv_cache=False, flash=False, rope=False,
                          device: str = "auto") -> Dict[str, Any]:
    dev = torch.device("cuda" if (device == "auto" and torch.cuda.is_available()) or device == "cuda" else "cpu")
    out: Dict[str, Any] = {"device": str(dev)}
    if dev.type != "cuda":
        out["note"] = "HIP kernels need a GPU; CPU runs the fp32 oracle only"
    from llmctl import ops
    from llmctl.ops import _lib

    nat = _lib.native() if dev.type == "cuda" else None
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    if matmul:
        n = 8192 if dev.type == "cuda" else 512
        a = torch.randn(n, n, device=dev, dtype=dt)
        b = torch.randn(n, n, device=dev, dtype=dt)
        fl = 2 * n ** 3
        r = {"shape": [n, n, n], "torch_tflops": fl / _t(lambda: a @ b.t()) / 1e12}
        if nat is not None:
            r["llmctl_mfma_tflops"] = fl / _t(lambda: nat.gemm_bf16(a, b)) / 1e12
        out["matmul"] = r
    if attention or flash:
        B, S, H, D = (8, 2048, 32, 128) if dev.type == "cuda" else (1, 256, 4, 64)
        q = torch.randn(B, S, H, D, device=dev, dtype=dt)
        k, v = torch.randn_like(q), torch.randn_like(q)
        fl = 4 * B * H * S * S * D / 2
        r = {"shape": [B, S, H, D], "causal": True}
        if nat is not None:
            o, lse = nat.flash_attn_fwd(q, k, v, D ** -0.5, True)
            r["llmctl_fwd_tflops"] = fl / _t(lambda: nat.flash_attn_fwd(q, k, v, D ** -0.5, True)) / 1e12
            if flash:
                do = torch.randn_like(q)
                r["llmctl_bwd_tflops"] = 2.5 * fl / _t(lambda: nat.flash_attn_bwd(do, q, k, v, o, lse, D ** -0.5, True)) / 1e12
        qt, kt, vt = (x.transpose(1, 2) for x in (q, k, v))
        r["sdpa_fwd_tflops"] = fl / _t(lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True)) / 1e12
        out["attention"] = r
    if rope:
        T, nq, nkv, D = (16384, 32, 32, 128) if dev.type == "cuda" else (256, 4, 4, 64)
        qkv = torch.randn(T, (nq + 2 * nkv) * D, device=dev, dtype=dt)
        cos, sin = ops.ref.rope_tables(T, D, device=dev)
        s = _t(lambda: ops.rope_qkv(qkv, cos, sin, nq, nkv, T))
        out["rope"] = {"tokens": T, "ms": s * 1e3, "gbps": 2 * qkv.numel() * qkv.element_size() / s / 1e9}
    if kv_cache:
        N, Hq, Hkv, D, L, bs = (64, 32, 32, 128, 2048, 16) if dev.type == "cuda" else (4, 4, 4, 64, 128, 16)
        nb = N * L // bs
        kc = torch.randn(nb, bs, Hkv, D, device=dev, dtype=dt)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, device=dev, dtype=torch.int32).view(N, L // bs)
        lens = torch.full((N,), L, device=dev, dtype=torch.int32)
        q = torch.randn(N, Hq, D, device=dev, dtype=dt)
        s = _t(lambda: ops.paged_attention_decode(q, kc, vc, bt, lens))
        out["paged_decode"] = {"seqs": N, "context": L, "ms": s * 1e3,
                               "kv_gbps": 2 * kc.numel() * kc.element_size() / s / 1e9}
    return out
