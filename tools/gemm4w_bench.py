#!/usr/bin/env python3
"""4-wave GEMM (gemm64 config variant 9) vs the 8-wave kernel (104) vs hipBLASLt (TunableOp
solutions) on the GPT-7B training shapes: forward / dgrad / wgrad layouts, random data, TF/s
(median of interleaved rounds), plus a row-error check of every variant against fp32.

    python tools/gemm4w_bench.py [--tokens 32768] [--configs 104 904]
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

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}


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
    ap.add_argument("--configs", type=int, nargs="+", default=[104, 904])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--layouts", nargs="+", default=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--knob", action="append", default=[], help="native knob name=value (repeatable)")
    ap.add_argument("--knob-sets", nargs="+", default=[],
                    help="extra cases per config: 'name=value,name=value' native knob sets, timed interleaved "
                         "with the base case (e.g. gemm_stagger=400)")
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    print("tuned hipBLASLt solutions:", enable_tuned_gemms(), flush=True)
    ops = torch.ops.llmctl
    for kv in a.knob:
        k, v = kv.split("=")
        ops.set_knob(k, int(v))
    T = a.tokens
    for name in a.shapes:
        out, inn = SHAPES[name]
        fl = 2 * T * out * inn / 1e12
        torch.manual_seed(0)
        x = (torch.rand(T, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(out, inn, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(T, out, device="cuda") * 2 - 1).to(torch.bfloat16)
        Wt = W.t().contiguous()
        y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
        gw = torch.empty(out, inn, device="cuda", dtype=torch.float32)
        for lay in a.layouts:
            if lay == "fwd":
                ref = lambda: torch.nn.functional.linear(x, W)  # noqa: E731
                run = lambda c: ops.gemm64_ex(x, W, y, False, False, False, c)  # noqa: E731
                res, want = y, None
            elif lay == "dgrad":
                ref = lambda: torch.nn.functional.linear(dy, Wt)  # noqa: E731
                run = lambda c: ops.gemm64_ex(dy, W, dx, False, True, False, c)  # noqa: E731
                res = dx
            else:
                ref = lambda: torch.mm(dy.t(), x)  # noqa: E731
                run = lambda c: ops.gemm64_ex(dy, x, gw, True, True, False, c)  # noqa: E731
                res = gw
            want = ref().float()
            r = {"shape": name, "layout": lay, "tokens": T}
            cases = {"hipblaslt": ref}
            base = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.knob}

            def with_knobs(ks, c):
                def f():
                    for k, v in ks.items():
                        ops.set_knob(k, v)
                    run(c)
                    for k in ks:
                        ops.set_knob(k, base.get(k, 0))
                return f

            for c in a.configs:
                run(c)
                torch.cuda.synchronize()
                r[f"err{c}"] = round(row_err(res, want), 5)
                cases[f"g{c}"] = lambda c=c: run(c)
                for ksv in a.knob_sets:
                    ks = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in ksv.split(",")}
                    f = with_knobs(ks, c)
                    f()
                    torch.cuda.synchronize()
                    r[f"err{c}[{ksv}]"] = round(row_err(res, want), 5)
                    cases[f"g{c}[{ksv}]"] = f
            times = {k: [] for k in cases}
            for _ in range(a.rounds):
                for k, f in cases.items():
                    times[k].append(timeit(f, 5))
            for k, v in times.items():
                r[k] = round(fl / statistics.median(v) * 1e3, 1)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
