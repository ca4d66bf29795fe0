#!/usr/bin/env python3
"""Gate/up + SwiGLU GEMM (gemm64_swiglu_fwd, GPT-7B F 11008, K 4096) with / without the tail split
(native knob swiglu_fwd_split), CUDA-event timed, interleaved passes, at several token counts."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def main():
    import torch

    from llmctl.ops import _lib

    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    F, K = 11008, 4096
    w = (torch.randn(2 * F, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    for M in (2048, 4096, 8192):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        r = (0.5 + torch.rand(M, device="cuda")).float()
        res = {0: [], 1: []}
        for _ in range(4):
            for sw in (1, 0):
                ops.set_knob("swiglu_fwd_split", sw)
                for _ in range(3):
                    ops.gemm64_swiglu_fwd(x, w, 304, r)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                torch.cuda.synchronize()
                ev[0].record()
                for _ in range(20):
                    ops.gemm64_swiglu_fwd(x, w, 304, r)
                ev[1].record()
                torch.cuda.synchronize()
                res[sw].append(ev[0].elapsed_time(ev[1]) / 20 * 1e3)
        ops.set_knob("swiglu_fwd_split", 1)
        print(json.dumps({"M": M, "split_us": [round(v, 1) for v in res[1]], "whole_us": [round(v, 1) for v in res[0]],
                          "tflops_split": round(2 * M * 2 * F * K / min(res[1]) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
