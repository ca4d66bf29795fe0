#!/usr/bin/env python3
"""gemm64 config matrix on small shapes: per-config row error and the 256x256 output tiles that
are wrong (debugging aid for schedule / work-item changes)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def main():
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    for (M, N, K) in [(768, 512, 1024), (2304, 1280, 256), (256 * 40, 1024, 512)]:
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
        want = A.float() @ B.float().t()
        for at, bt in [(False, False), (True, True)]:
            a = A.t().contiguous() if at else A
            b = B.t().contiguous() if bt else B
            for cfg in (104, 1104, 2104, 4104, 504, 1504, 2504, 4504):
                out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
                try:
                    ops.gemm64_ex(a, b, out, at, bt, False, cfg)
                except RuntimeError as e:
                    print(M, N, K, at, bt, cfg, "ERR", str(e)[:80], flush=True)
                    continue
                torch.cuda.synchronize()
                d = (out.float() - want).abs()
                d = torch.nan_to_num(d, nan=1e30)
                rel = (d.amax(1) / want.abs().amax(1)).max().item()
                bad = []
                if rel > 0.02:
                    t = d.view(M // 256, 256, N // 256, 256).amax(dim=(1, 3))
                    bad = (t > 0.05 * want.abs().max()).nonzero().tolist()
                print(M, N, K, "at" if at else "fw", cfg, "rowerr %.3g" % rel, "bad tiles", bad[:12], flush=True)


if __name__ == "__main__":
    main()
