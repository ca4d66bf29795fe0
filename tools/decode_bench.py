"""Paged-attention decode bandwidth sweep (GPT-7B heads: 32 x 128, bf16 KV, block 16):
batch N in {1, 4, 16, 64} at 2k context over a shuffled block table, with the automatic
context split and with LLMCTL_DECODE_SPLITS=1 (one workgroup per sequence x kv-head).

    python tools/decode_bench.py [--ctx 2048] [--hkv 32] [--json-out f]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=32)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    import torch

    from llmctl.ops import _lib

    assert _lib.load(), _lib._error
    nat = _lib.native()
    D, bs = 128, 16
    rows = []
    for N in (1, 4, 16, 64):
        nbs = a.ctx // bs
        nb = N * nbs
        kc = torch.randn(nb, bs, a.hkv, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.randperm(nb, device="cuda").to(torch.int32).view(N, nbs).contiguous()
        lens = torch.full((N,), a.ctx, device="cuda", dtype=torch.int32)
        q = torch.randn(N, a.hq, D, device="cuda", dtype=torch.bfloat16)
        for mode in ("1", "auto"):
            if mode == "auto":
                os.environ.pop("LLMCTL_DECODE_SPLITS", None)
            else:
                os.environ["LLMCTL_DECODE_SPLITS"] = mode
            fn = lambda: nat.paged_attention_decode(q, kc, vc, bt, lens, D ** -0.5)  # noqa: E731
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 50
            e0.record()
            for _ in range(it):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / it
            byts = 2 * kc.numel() * kc.element_size()
            row = {"seqs": N, "context": a.ctx, "hkv": a.hkv, "splits": mode, "us": round(ms * 1e3, 1),
                   "kv_tbps": round(byts / (ms * 1e-3) / 1e12, 2)}
            rows.append(row)
            print(json.dumps(row), flush=True)
        del kc, vc
    os.environ.pop("LLMCTL_DECODE_SPLITS", None)
    # decode-shaped projection GEMMs (GPT-7B): weight-streaming MFMA kernel vs hipBLASLt
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008),
              "lm_head": (32000, 4096)}
    for M in (1, 8, 16, 32):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            # cycle through > 256 MB of weight copies so the MALL does not serve repeats
            nw = max(2, -(-768 * 2**20 // (N * K * 2)))
            ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(nw)]
            it = iter(range(1 << 30))
            row = {"gemm": name, "M": M, "N": N, "K": K}
            for impl, fn in (("skinny", lambda: nat.skinny_linear(x, ws[next(it) % nw], None)),
                             ("hipblaslt", lambda: torch.nn.functional.linear(x, ws[next(it) % nw]))):
                for _ in range(5):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 50 * 1e3
                row[f"{impl}_us"] = round(us, 1)
                row[f"{impl}_tbps"] = round(N * K * 2 / (us * 1e-6) / 1e12, 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del ws
    if a.json_out:
        with open(a.json_out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
