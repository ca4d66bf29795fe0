#!/usr/bin/env python3
"""Single-prompt prefill attention (B 1, S 2048, 32 heads, HD 128, causal: the K/V-split path +
combine kernel), graph-replayed x20, alternating native knob settings (--knob name --values a b)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="fa_split")
    ap.add_argument("--values", type=int, nargs="+", default=[1, 0])
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    B, S, H, D = 1, a.S, 32, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
    res = {}
    for _ in range(a.rounds):
        for val in a.values:
            ops.set_knob(a.knob, val)
            for _ in range(3):
                ops.flash_attn_fwd(q, k, v, D ** -0.5, True)
            gr = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                ops.flash_attn_fwd(q, k, v, D ** -0.5, True)
                with torch.cuda.graph(gr, stream=st):
                    for _ in range(20):
                        ops.flash_attn_fwd(q, k, v, D ** -0.5, True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(val, []).append(round(e0.elapsed_time(e1) * 1e3 / 20, 2))
    ops.set_knob(a.knob, a.values[0])
    print(json.dumps({"B": B, "S": S, "H": H, "knob": a.knob, "us_per_call": res}))


if __name__ == "__main__":
    main()
