#!/usr/bin/env python3
"""Persistent 4-wave GEMM debug: per-tile error map of one config / layout over a few runs."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

assert _lib.load(), _lib._error
ops = torch.ops.llmctl
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
tiles = n_cu * 3 + n_cu // 3
M, N, K = 256 * (tiles // 4 + 1), 256 * 4, 512
g = torch.Generator(device="cuda")
g.manual_seed(11)
A = torch.randn(M, K, generator=g, device="cuda").to(torch.bfloat16)
g.manual_seed(12)
B = torch.randn(N, K, generator=g, device="cuda").to(torch.bfloat16)
want = A.float() @ B.float().t()
for at, bt in ((False, False), (False, True), (True, True)):
    a = A.t().contiguous() if at else A
    b = B.t().contiguous() if bt else B
    for cfg in [int(c) for c in sys.argv[1:]] or [308, 304]:
        for rep in range(3):
            out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            ops.gemm64_ex(a, b, out, at, bt, False, cfg)
            torch.cuda.synchronize()
            err = (out.float() - want).abs().view(M // 256, 256, N // 256, 256).amax(dim=(1, 3))
            bad = (err > 0.5).nonzero().tolist()
            nan = torch.isnan(out.float()).view(M // 256, 256, N // 256, 256).any(dim=3).any(dim=1).nonzero().tolist()
            rows = []
            if bad:
                tm, tn = bad[0]
                blk = (out.float() - want).abs()[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256]
                rows = (blk.amax(dim=1) > 0.5).nonzero().flatten().tolist()
                cols = (blk.amax(dim=0) > 0.5).nonzero().flatten().tolist()
                rows = [rows[:8], len(rows), cols[:8], len(cols)]
            print(f"at={at} bt={bt} cfg={cfg} rep={rep} bad_tiles={len(bad)} {bad[:10]} nan_tiles={len(nan)} first_bad_rows/cols={rows}",
                  flush=True)
