#!/usr/bin/env python3
"""A/B the gemm_ex schedule variants (V bits, llmctl/ops/csrc/gemm_bf16.hip) in one process,
interleaved rounds, random operands.  Usage: gemm_variants.py [rounds] [variants...]"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

T = 16384


def timeit(fn, n=5):
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
    variants = [int(v) for v in sys.argv[2:]] or list(range(8))
    out, inn = 22016, 4096
    x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
    dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
    W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
    dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
    g = torch.empty(out, inn, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * out * inn / 1e12
    kinds = {
        "fwd": lambda v: ops.gemm_ex(x, W, y, False, False, False, v),
        "dgrad": lambda v: ops.gemm_ex(dy, W, dx, False, True, False, v),
        "wgrad": lambda v: ops.gemm_ex(dy, x, g, True, True, False, v),
    }
    ref = {}
    for k, f in kinds.items():
        f(0)
        ref[k] = {"fwd": y, "dgrad": dx, "wgrad": g}[k].clone()
    res = {}
    for k, f in kinds.items():
        tgt = {"fwd": y, "dgrad": dx, "wgrad": g}[k]
        for v in variants:
            f(v)
            same = torch.equal(tgt, ref[k])
            res.setdefault(k, {})[v] = {"bitwise_equal_v0": same, "ms": []}
        for _ in range(rounds):
            for v in variants:
                res[k][v]["ms"].append(timeit(lambda: f(v)))
        for v in variants:
            ms = statistics.median(res[k][v]["ms"])
            res[k][v] = {"eq": res[k][v]["bitwise_equal_v0"], "ms": round(ms, 4), "tflops": round(fl / ms * 1e3, 1)}
        print(k, json.dumps(res[k]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
