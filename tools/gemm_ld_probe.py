#!/usr/bin/env python3
"""Leading-dimension probe for the forward-layout GEMM (y = x W^T, both operands K-contiguous).

Hypothesis: at K = 4096 every operand row starts 8 KiB after the previous one, so the 256 rows
a 256x256 tile streams per K-tile share their low 13 address bits and may camp on a subset of
HBM channels; the K = 11008 shape (22,016-B rows) is the fastest forward.  Padding the row
stride (ld = K + pad) breaks the power-of-two stride without changing the math.

Prints one JSON line per (shape, pad): gemm64 fwd (config 104) and hipBLASLt (TunableOp
solutions loaded, as in the training step) on the same operands, random data, median of
interleaved rounds.
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402
from llmctl.exec.gemm_tuning import enable_tuned_gemms  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008), "lm_head": (32000, 4096)}


def timeit(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def padded(rows, cols, pad):
    base = (torch.rand(rows, cols + pad, device="cuda") * 2 - 1).to(torch.bfloat16)
    return base[:, :cols]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pads", type=int, nargs="+", default=[0, 64, 128])
    ap.add_argument("--configs", type=int, nargs="+", default=[104])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    print("tuned hipBLASLt solutions:", enable_tuned_gemms(), flush=True)
    ops = torch.ops.llmctl
    T = a.tokens
    for name in a.shapes:
        out, inn = SHAPES[name]
        fl = 2 * T * out * inn / 1e12
        for pad in a.pads:
            torch.manual_seed(0)
            x = padded(T, inn, pad)
            W = padded(out, inn, pad)
            dy = padded(T, out, pad)
            y = torch.empty(T, out, device="cuda", dtype=torch.bfloat16)
            dx = torch.empty(T, inn, device="cuda", dtype=torch.bfloat16)
            ref = torch.nn.functional.linear(x, W)
            ops.gemm64_ex(x, W, y, False, False, False, a.configs[0])
            err = ((y.float() - ref.float()).abs().amax() / ref.float().abs().amax()).item()
            cases = {"torch_fwd": lambda: torch.nn.functional.linear(x, W)}
            for c in a.configs:
                cases[f"g{c}_fwd"] = lambda c=c: ops.gemm64_ex(x, W, y, False, False, False, c)
                cases[f"g{c}_dgrad"] = lambda c=c: ops.gemm64_ex(dy, W, dx, False, True, False, c)
            times = {k: [] for k in cases}
            for f in cases.values():
                f()
            for _ in range(a.rounds):
                for k, f in cases.items():
                    times[k].append(timeit(f, 5))
            r = {"shape": name, "pad": pad, "err": round(err, 5)}
            for k, v in times.items():
                ms = statistics.median(v)
                r[k] = round(fl / ms * 1e3, 1)
            print(json.dumps(r), flush=True)
            del x, W, dy, y, dx, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
