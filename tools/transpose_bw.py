#!/usr/bin/env python3
"""Solo bandwidth of the W^T refresh kernel (llmctl transpose_) on the GPT-7B weight shapes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmctl.ops._lib import native  # noqa: E402


def main():
    ops = native()
    for name, (r, c) in {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}.items():
        w = torch.randn(r, c, device="cuda", dtype=torch.bfloat16)
        wt = torch.empty(c, r, device="cuda", dtype=torch.bfloat16)
        ops.transpose_(w, wt)
        assert torch.equal(wt, w.t())
        for _ in range(3):
            ops.transpose_(w, wt)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            ops.transpose_(w, wt)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        print(json.dumps({"shape": name, "rows": r, "cols": c, "us": round(us, 1),
                          "TB_per_s": round(2 * w.numel() * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
