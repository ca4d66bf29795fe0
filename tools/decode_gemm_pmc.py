#!/usr/bin/env python3
"""Decode GEMM (16 tokens) on uncached weights for rocprofv3 counter passes: the fused-path v3
kernel (decode_linear_partials) on the GPT-7B QKV / o / up / down shapes, rotating over enough
weight copies (> 256 MB Infinity Cache) that every call streams its weights from HBM."""
import sys

import torch


def main():
    from llmctl.ops._lib import native

    lib = native()
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    x = {k: torch.randn(16, K, device="cuda").to(torch.bfloat16) for k, (N, K) in shapes.items()}
    for name, (N, K) in shapes.items():
        copies = max(2, int(1.2e9 // (N * K * 2)))
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for i in range(reps):
            lib.decode_linear_partials(x[name], ws[i % copies])
        torch.cuda.synchronize()
        del ws
    print("done", flush=True)


if __name__ == "__main__":
    main()
