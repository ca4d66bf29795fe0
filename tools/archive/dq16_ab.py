#!/usr/bin/env python3
"""dQ kernel A/B: MFMA 32x32x16 (knob dq16 = 0) vs 16x16x32 (dq16 = 1), B16 S2048 H32 D128 causal,
random data, interleaved rounds after a 2 s warm-up (steady clock): the dQ kernel alone
(fa_bwd_ablate abl 2) and the whole backward op.

    python tools/dq16_ab.py [--rounds 6]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--shape", type=int, nargs=4, default=[16, 2048, 32, 128])
    a = ap.parse_args()
    ops = _lib.native()
    B, S, H, D = a.shape
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k, v, do = (torch.randn_like(q) for _ in range(3))
    scale = D ** -0.5
    o, lse = ops.flash_attn_fwd(q, k, v, scale, True)
    delta = (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    fl3 = 3 * 2 * B * H * S * S * D * 0.5  # the dQ kernel's 3 products (S, dP, dQ)

    def run_dq():
        ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, 2)

    def run_bwd():
        ops.flash_attn_bwd(do, q, k, v, o, lse, scale, True)

    def timeit(f, n=10):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    t_end = time.perf_counter() + 2.0
    while time.perf_counter() < t_end:
        run_bwd()
    res = {m: {"dq": [], "bwd": []} for m in (0, 1)}
    for _ in range(a.rounds):
        for m in (0, 1):
            ops.set_knob("dq16", m)
            res[m]["dq"].append(timeit(run_dq))
            res[m]["bwd"].append(timeit(run_bwd))
    ops.set_knob("dq16", 0)
    for m in (0, 1):
        dqm = statistics.median(res[m]["dq"])
        print(json.dumps({"dq16": m, "shape": a.shape, "dq_ms": round(dqm, 4), "dq_min_ms": round(min(res[m]["dq"]), 4),
                          "dq_tflops": round(fl3 / dqm / 1e9, 1),
                          "bwd_ms": round(statistics.median(res[m]["bwd"]), 4)}), flush=True)


if __name__ == "__main__":
    main()
