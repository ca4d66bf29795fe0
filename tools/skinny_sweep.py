#!/usr/bin/env python3
"""Decode GEMM sweep: skinny_linear_cfg configs vs hipBLASLt (F.linear) on the GPT-7B decode
projections, weights cycled through a pool larger than the caches (uncached stream, as in a
real decode step).  Prints one JSON line per (shape, M)."""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008), "lm_head": (32000, 4096)}


def main():
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    cfgs = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,2,3,4,5,6,7,8".split(","))]
    for name, (N, K) in SHAPES.items():
        pool = max(2, int(2.5e9 // (N * K * 2)))  # > 2 GB of distinct weights: no cache reuse
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(pool)]
        for M in (1, 16, 32):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            ref = torch.nn.functional.linear(x, ws[0]).float()
            cases = {"torch": lambda w: torch.nn.functional.linear(x, w)}
            for c in cfgs:
                try:
                    y = ops.skinny_linear_cfg(x, ws[0], None, c).float()
                except RuntimeError:
                    continue
                err = ((y - ref).abs().max() / ref.abs().max()).item()
                assert err < 2e-2, (name, M, c, err)
                cases[f"c{c}"] = lambda w, c=c: ops.skinny_linear_cfg(x, w, None, c)
            res = {}
            for k, f in cases.items():
                ts = []
                for _ in range(5):
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    for i in range(20):
                        f(ws[i % pool])
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t) / 20 * 1e6)
                us = statistics.median(ts)
                res[k] = {"us": round(us, 2), "TBps": round(N * K * 2 / us / 1e6, 2)}
            best = min(res, key=lambda k: res[k]["us"])
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "best": best, **res}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
