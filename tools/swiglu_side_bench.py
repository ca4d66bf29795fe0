#!/usr/bin/env python3
"""Down-projection backward of the GPT-7B MLP, three ways (one MI355X, bf16, T x H x F):

  epilogue : wgrad (gemm64) + data gradient with the SwiGLU backward in its store epilogue
  side     : data gradient (hipBLASLt through W^T, or gemm64) + wgrad carrying the SwiGLU
             backward as a side job (gemm64_wgrad_swiglu)
  plain    : wgrad + data gradient + separate swiglu_bwd kernel

    python tools/swiglu_side_bench.py [--tokens 24576] [--hidden 4096] [--ffn 11008] [--iters 20]

Prints one JSON line per variant (ms per backward, and each part alone)."""
import argparse
import json

import torch


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=11008)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from llmctl.ops._lib import load, native

    assert load()
    T, H, F = a.tokens, a.hidden, a.ffn
    dev = "cuda"
    dy = torch.randn(T, H, device=dev).to(torch.bfloat16)
    act = torch.randn(T, F, device=dev).to(torch.bfloat16)
    gu = torch.randn(T, 2 * F, device=dev).to(torch.bfloat16)
    w = (torch.randn(H, F, device=dev) * 0.02).to(torch.bfloat16)
    wt = w.t().contiguous()
    gw = torch.empty(H, F, device=dev, dtype=torch.bfloat16)
    lib = native()
    cfg = 104
    dact = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
    flop = 2.0 * T * H * F

    def wgrad():
        lib.gemm64_ex(dy, act, gw, True, True, False, cfg)

    def dgrad_fused():
        return lib.gemm64_swiglu_dgrad(dy, w, gu, cfg)

    def dgrad_blas():
        return torch.nn.functional.linear(dy, wt)

    def dgrad_g64():
        lib.gemm64_ex(dy, w, dact, False, True, False, cfg)

    def wgrad_side():
        return lib.gemm64_wgrad_swiglu(dy, act, gw, False, dact, gu, cfg)

    def swb():
        return lib.swiglu_bwd(dact, gu)

    res = {k: timeit(f, a.iters) for k, f in
           [("wgrad", wgrad), ("dgrad_fused", dgrad_fused), ("dgrad_blas", dgrad_blas), ("dgrad_g64", dgrad_g64),
            ("wgrad_side", wgrad_side), ("swiglu_bwd", swb)]}
    res["epilogue_total"] = timeit(lambda: (wgrad(), dgrad_fused()), a.iters)
    res["side_blas_total"] = timeit(lambda: (dgrad_blas(), wgrad_side()), a.iters)
    res["side_g64_total"] = timeit(lambda: (dgrad_g64(), wgrad_side()), a.iters)
    res["plain_total"] = timeit(lambda: (wgrad(), dgrad_blas(), swb()), a.iters)
    tf = {k + "_tf": round(flop / (v * 1e-3) / 1e12, 1) for k, v in res.items() if k in
          ("wgrad", "dgrad_fused", "dgrad_blas", "dgrad_g64", "wgrad_side")}
    # side job correctness spot check against the separate kernel
    ref = lib.swiglu_bwd(dact, gu)
    got = wgrad_side()
    err = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    import os

    print(json.dumps({"diag": os.environ.get("LLMCTL_SIDE_DIAG", ""), "T": T, "H": H, "F": F, "ms": {k: round(v, 4) for k, v in res.items()}, "tf": tf,
                      "side_vs_kernel_err": err}))


if __name__ == "__main__":
    main()
