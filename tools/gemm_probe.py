#!/usr/bin/env python3
"""Bottleneck probes of the one-shot 4-wave GEMM (gemm64 config variants 6-9; native knob
gemm_probe): 1 = operand loads out of range (the same instruction stream without memory
traffic), 2 = no workgroup barriers, 4 = no epilogue; sums combine.  Results are garbage under a
probe; only the time means anything.  Prints TF/s per probe next to hipBLASLt.

    python tools/gemm_probe.py [--config 904] [--shape up] [--layout fwd]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

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
    ap.add_argument("--config", type=int, default=904)
    ap.add_argument("--shapes", nargs="+", default=["up", "o"])
    ap.add_argument("--probes", type=int, nargs="+", default=[0, 1, 2, 4, 3, 5, 6, 7])
    # 8: one tile's operands for every tile (L2-resident), 16: K-tile 0 for every K-tile
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    lib = torch.ops.llmctl
    for sh in a.shapes:
        N, K = SHAPES[sh]
        M = a.tokens
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16) * K ** -0.5
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * M * N * K
        res = {p: [] for p in a.probes}
        res["hipblaslt"] = []
        for _ in range(a.rounds):
            for p in a.probes:
                lib.set_knob("gemm_probe", p)
                lib.gemm64_ex(x, w, out, False, False, False, a.config)
                res[p].append(flop / timeit(lambda: lib.gemm64_ex(x, w, out, False, False, False, a.config), 10) / 1e9)
            lib.set_knob("gemm_probe", 0)
            res["hipblaslt"].append(flop / timeit(lambda: torch.nn.functional.linear(x, w), 10) / 1e9)
        lib.set_knob("gemm_probe", 0)
        print(json.dumps({"shape": sh, "config": a.config, **{str(k): round(statistics.median(v), 1) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
