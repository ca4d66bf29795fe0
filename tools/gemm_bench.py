#!/usr/bin/env python3
"""llmctl gemm_ex (hand-written MFMA, llmctl/ops/csrc/gemm_bf16.hip) vs torch/hipBLASLt on the
GPT-7B projection GEMMs at 16384 tokens, for the three products of a training step:

  fwd   y  = x W^T        (torch: F.linear)            llmctl: gemm_ex(x, W, at=0, bt=0)
  dgrad dx = dy W         (torch: dy @ W)              llmctl: gemm_ex(dy, W, at=0, bt=1)
  wgrad dW = dy^T x       (torch: mm(dy.t(), x, out=)) llmctl: gemm_ex(dy, x, at=1, bt=1)

Random operands (DVFS: zero data reads ~20% high), interleaved rounds in one process,
median of rounds.  Prints one JSON object.
"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

T = 16384
SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008), "lm_head": (32000, 4096)}


def timeit(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    res = {}
    for name, (out, inn) in SHAPES.items():
        x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
        g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * out * inn / 1e12
        cases = {
            "fwd_torch": lambda: torch.nn.functional.linear(x, W),
            "fwd_llmctl": lambda: ops.gemm_ex(x, W, y, False, False, False),
            "dgrad_torch": lambda: dy.matmul(W),
            "dgrad_llmctl": lambda: ops.gemm_ex(dy, W, dx, False, True, False),
            "wgrad_torch": lambda: torch.mm(dy.t(), x, out=g),
            "wgrad_llmctl": lambda: ops.gemm_ex(dy, x, g, True, True, False),
            "wgrad_acc_torch": lambda: g.addmm_(dy.t(), x),
            "wgrad_acc_llmctl": lambda: ops.gemm_ex(dy, x, g, True, True, True),
        }
        # correctness spot check (fp32 reference on a slice)
        ops.gemm_ex(dy, x, g, True, True, False)
        ref = dy[:, :256].float().t() @ x[:, :256].float()
        err = ((g[:256, :256].float() - ref).norm() / ref.norm()).item()
        ops.gemm_ex(dy, W, dx, False, True, False)
        ref2 = dy[:256].float() @ W[:, :256].float()
        err2 = ((dx[:256, :256].float() - ref2).norm() / ref2.norm()).item()
        times = {k: [] for k in cases}
        for k, f in cases.items():
            f()
        for _ in range(rounds):
            for k, f in cases.items():
                times[k].append(timeit(f, 5))
        r = {"wgrad_rel_err": err, "dgrad_rel_err": err2}
        for k, v in times.items():
            ms = statistics.median(v)
            r[k] = {"ms": round(ms, 4), "tflops": round(fl / ms * 1e3, 1)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
    tot = {}
    for kind in ("fwd", "dgrad", "wgrad", "wgrad_acc"):
        for impl in ("torch", "llmctl"):
            tot[f"{kind}_{impl}_ms"] = round(sum(res[n][f"{kind}_{impl}"]["ms"] for n in SHAPES if n != "lm_head")
                                             + 0.0, 3)
    res["per_layer_total"] = tot
    print(json.dumps(res))


if __name__ == "__main__":
    main()
