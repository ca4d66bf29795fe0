#!/usr/bin/env python3
"""gemm64_ex (64-deep K-tile MFMA GEMM, llmctl/ops/csrc/gemm64.hip) vs gemm_ex (32-deep,
gemm_bf16.hip) vs torch/hipBLASLt on the GPT-7B projection GEMMs, for the three products of a
training step:

  fwd   y  = x W^T      torch: F.linear           llmctl: (x, W, at=0, bt=0)
  dgrad dx = dy W       torch: dy @ W             llmctl: (dy, W, at=0, bt=1)
  wgrad dW = dy^T x     torch: mm(dy.t(), x)      llmctl: (dy, x, at=1, bt=1)

Correctness first (every output element vs the torch result, per-row max error), then timing:
random operands (DVFS: zero data reads ~20% high), interleaved rounds in one process, median.
Prints one JSON line per shape and a summary line.

    python tools/gemm64_bench.py [--tokens 24576] [--rounds 5] [--groups 4 8]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008), "lm_head": (32000, 4096)}


def timeit(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def max_row_err(got, ref):
    """max over rows of (max |got-ref| in the row) / (max |ref| in the row)"""
    d = (got.float() - ref.float()).abs().amax(dim=1)
    s = ref.float().abs().amax(dim=1).clamp_min(1e-6)
    return (d / s).max().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--groups", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--no-old", action="store_true")
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    T = a.tokens
    res = {}
    worst = 0.0
    for name in a.shapes:
        out, inn = SHAPES[name]
        torch.manual_seed(0)
        x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
        g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * out * inn / 1e12
        N_ok = out % 256 == 0
        # ---- correctness of gemm64 vs torch (both bf16 outputs of fp32 accumulations)
        errs = {}
        if N_ok:
            ref = torch.nn.functional.linear(x, W)
            ops.gemm64_ex(x, W, y, False, False, False, 4)
            errs["fwd"] = max_row_err(y, ref)
            ref = dy.matmul(W)
            ops.gemm64_ex(dy, W, dx, False, True, False, 4)
            errs["dgrad"] = max_row_err(dx, ref)
            ref = torch.mm(dy.t(), x)
            ops.gemm64_ex(dy, x, g, True, True, False, 4)
            errs["wgrad"] = max_row_err(g, ref)
            g2 = g.clone()
            ops.gemm64_ex(dy, x, g2, True, True, True, 4)
            errs["wgrad_acc"] = max_row_err(g2, (ref.float() * 2).to(torch.bfloat16))
            del ref, g2
            worst = max(worst, max(errs.values()))
        cases = {
            "fwd_torch": lambda: torch.nn.functional.linear(x, W),
            "dgrad_torch": lambda: dy.matmul(W),
            "wgrad_torch": lambda: torch.mm(dy.t(), x, out=g),
        }
        if N_ok:
            if not a.no_old:
                cases["fwd_old"] = lambda: ops.gemm_ex(x, W, y, False, False, False)
                cases["dgrad_old"] = lambda: ops.gemm_ex(dy, W, dx, False, True, False)
                cases["wgrad_old"] = lambda: ops.gemm_ex(dy, x, g, True, True, False)
            for grp in a.groups:
                cases[f"fwd_g{grp}"] = lambda grp=grp: ops.gemm64_ex(x, W, y, False, False, False, grp)
                cases[f"dgrad_g{grp}"] = lambda grp=grp: ops.gemm64_ex(dy, W, dx, False, True, False, grp)
                cases[f"wgrad_g{grp}"] = lambda grp=grp: ops.gemm64_ex(dy, x, g, True, True, False, grp)
        times = {k: [] for k in cases}
        for f in cases.values():
            f()
        for _ in range(a.rounds):
            for k, f in cases.items():
                times[k].append(timeit(f, 5))
        r = {"err": {k: round(v, 5) for k, v in errs.items()}}
        for k, v in times.items():
            ms = statistics.median(v)
            r[k] = {"ms": round(ms, 4), "tf": round(fl / ms * 1e3, 1)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
        del x, dy, W, y, dx, g
        torch.cuda.empty_cache()
    print(json.dumps({"tokens": T, "worst_row_err": worst, "shapes": res}))


if __name__ == "__main__":
    main()
