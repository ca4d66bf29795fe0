#!/usr/bin/env python3
"""Persistent 4-wave GEMM race hunt: repeated runs of a BT (B stored [K, N]) product, per-probe
failure counts (probe 8: drain at item boundaries, 16: drain before epilogues)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

assert _lib.load(), _lib._error
ops = torch.ops.llmctl
M, N, K = 32768, 11008, 4096  # down-projection dgrad: dx = dy W, W [4096, 11008] read as [K, N]
g = torch.Generator(device="cuda")
g.manual_seed(1)
A = torch.randn(M, K, generator=g, device="cuda").to(torch.bfloat16)
B = (torch.randn(K, N, generator=g, device="cuda") * K ** -0.5).to(torch.bfloat16)
want = (A.float() @ B.float()).to(torch.bfloat16).float()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for cfg in (304, 904):
    for probe in (0, 1):
        ops.set_knob("gemm_p3_drain", probe)
        fails = []
        for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
            ops.gemm64_ex(A, B, out, False, True, False, cfg)
            torch.cuda.synchronize()
            err = (out.float() - want).abs()
            badrows = (err.amax(dim=1) > 0.25).nonzero().flatten()
            if len(badrows):
                r0 = int(badrows[0])
                badcols = (err[r0] > 0.25).nonzero().flatten()
                fails.append((len(badrows), r0, r0 // 256, int(badcols[0]) // 256 if len(badcols) else -1, len(badcols)))
        print(f"cfg={cfg} probe={probe} fails={len(fails)} {fails[:6]}", flush=True)
ops.set_knob("gemm_p3_drain", 1)
