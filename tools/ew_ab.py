#!/usr/bin/env python3
"""A/B of memory-bound kernel variants (native knob sets) at the GPT-7B mb-16 training shapes
(T = 32768): add + RMSNorm forward and SwiGLU forward, TB/s of the bytes each must move, median of
interleaved rounds.

    python tools/ew_ab.py --sets "norm_fwd_v=0" "norm_fwd_v=1" "swiglu_v=0" "swiglu_v=4"
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def timeit(f, reps=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    T, H, F = 32768, 4096, 11008
    x, r = torch.randn(T, H, device="cuda").bfloat16(), torch.randn(T, H, device="cuda").bfloat16()
    w = torch.randn(H, device="cuda").bfloat16()
    gu = torch.randn(T, 2 * F, device="cuda").bfloat16()
    sets = [{kv.split("=")[0]: int(kv.split("=")[1]) for kv in s.split(",")} for s in a.sets]
    ref_n = ops.add_rmsnorm_fwd(x, r, w, 1e-5)
    ref_s = ops.swiglu_fwd(gu)
    cases = {"add_rmsnorm_fwd": (lambda: ops.add_rmsnorm_fwd(x, r, w, 1e-5), 4 * T * H * 2),
             "swiglu_fwd": (lambda: ops.swiglu_fwd(gu), 3 * T * F * 2)}
    ts = {(i, k): [] for i in range(len(sets)) for k in cases}
    for i, ks in enumerate(sets):  # correctness of every variant vs the first set
        for k, v in ks.items():
            ops.set_knob(k, v)
        n = ops.add_rmsnorm_fwd(x, r, w, 1e-5)
        assert all(torch.equal(p, q) for p, q in zip(n, ref_n)), ("norm", ks)
        assert torch.equal(ops.swiglu_fwd(gu), ref_s), ("swiglu", ks)
    for _ in range(a.rounds):
        for i, ks in enumerate(sets):
            for k, v in ks.items():
                ops.set_knob(k, v)
            for name, (fn, nbytes) in cases.items():
                ts[(i, name)].append(timeit(fn))
    for i, s in enumerate(a.sets):
        row = {"set": s}
        for name, (fn, nbytes) in cases.items():
            ms = statistics.median(ts[(i, name)])
            row[name] = {"us": round(ms * 1e3, 1), "TBps": round(nbytes / ms / 1e9, 2)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
