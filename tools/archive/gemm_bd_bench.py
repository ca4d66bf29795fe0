#!/usr/bin/env python3
"""B-direct GEMM experiment (csrc/gemm_bd.hip) vs the persistent gemm64 kernel (config 304) vs
hipBLASLt (tuned solutions) on the GPT-7B forward and W^T-copy data-gradient shapes (both NT:
C = A B^T, K-contiguous operands), random data, TF/s (median of interleaved rounds), with a row
error vs fp32 for every kernel.

    python tools/gemm_bd_bench.py [--tokens 32768] [--rounds 5] [--group 8]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.exec.gemm_tuning import enable_tuned_gemms  # noqa: E402
from llmctl.ops import _lib  # noqa: E402
from llmctl.testing.numerics import row_err  # noqa: E402

# name: (N, K) of C [T, N] = A [T, K] . B [N, K]^T
SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008),
          "qkv_dg": (4096, 12288), "up_dg": (4096, 22016), "down_dg": (11008, 4096)}


def timeit(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--no-g304", action="store_true")
    ap.add_argument("--exps", type=int, nargs="*", default=[], help="timing ablations of the kernel (knob bd_exp)")
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    print("tuned hipBLASLt solutions:", enable_tuned_gemms(), flush=True)
    ops = torch.ops.llmctl
    T = a.tokens
    for name in a.shapes:
        N, K = SHAPES[name]
        fl = 2 * T * N * K / 1e12
        torch.manual_seed(0)
        A = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        C = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        want = (A.float() @ B.float().t())
        cases = {"hipblaslt": lambda: torch.nn.functional.linear(A, B),
                 "bd": lambda: ops.gemm_bd(A, B, a.group)}
        if not a.no_g304:
            cases["g304"] = lambda: ops.gemm64_ex(A, B, C, False, False, False, 304)

        def exp_case(e):
            def run():
                ops.set_knob("bd_exp", e)
                try:
                    return ops.gemm_bd(A, B, a.group)
                finally:
                    ops.set_knob("bd_exp", 0)
            return run
        exps = {f"bd_exp{e}": exp_case(e) for e in a.exps}
        r = {"shape": name, "T": T, "N": N, "K": K}
        for k, fn in cases.items():
            out = fn()
            out = C if out is None else out
            r["err_" + k] = round(row_err(out.float(), want), 5)
        del want
        cases.update(exps)
        n = max(3, int(20 / fl))
        ts = {k: [] for k in cases}
        for _ in range(a.rounds):
            for k, fn in cases.items():
                ts[k].append(timeit(fn, n))
        for k in cases:
            r[k] = round(fl / (statistics.median(ts[k]) / 1e3), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
