#!/usr/bin/env python3
"""Flash-attention forward A/B: the 2-waves-per-SIMD kernel (knob fa_w64 = 0) against the
one-wave-per-SIMD 64-row kernel (fa_w64 = 1 compiler-scheduled, 2 sched_group_barrier
interleave).  Per variant: max |O - O_ref| / max |O_ref| and max |LSE - LSE_ref| against the
fa_w64 = 0 output (itself checked against the fp32 oracle in tests/kernels), and the mean time of
--iters launches after a warm-up, as causal TFLOP/s.

    python tools/attn_fwd_ab.py [--B 16] [--S 2048] [--H 32] [--variants 0 1 2]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, nargs="+", default=[2048])
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="fa_w64 = 3 diagnostic build: cycles per section")
    ap.add_argument("--qscale", type=float, default=1.0, help="scale q (score spread: softmax max growth)")
    ap.add_argument("--packed", action="store_true", help="q / k / v as views of one [B, S, 3, H, D] QKV tensor (the training step's layout)")
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    causal = not a.no_causal
    D = 128
    for S in a.S:
        g = torch.Generator(device="cuda").manual_seed(S)
        hkv = a.Hkv or a.H
        if a.packed:
            qkv = torch.randn(a.B, S, a.H + 2 * hkv, D, device="cuda", generator=g).to(torch.bfloat16)
            q, k, v = qkv[:, :, :a.H], qkv[:, :, a.H:a.H + hkv], qkv[:, :, a.H + hkv:]
        else:
            q = torch.randn(a.B, S, a.H, D, device="cuda", generator=g).to(torch.bfloat16)
            k = torch.randn(a.B, S, hkv, D, device="cuda", generator=g).to(torch.bfloat16)
            v = torch.randn(a.B, S, hkv, D, device="cuda", generator=g).to(torch.bfloat16)
        if a.qscale != 1.0:
            q = (q.float() * a.qscale).to(torch.bfloat16)
        scale = D ** -0.5
        flops = 4 * a.B * a.H * S * S * D * (0.5 if causal else 1.0)
        ref = None
        for var in a.variants:
            ops.set_knob("fa_w64", var)
            o, lse = ops.flash_attn_fwd(q, k, v, scale, causal)
            torch.cuda.synchronize()
            if ref is None:
                ref = (o.float(), lse)
            err_o = ((o.float() - ref[0]).abs().max() / ref[0].abs().max()).item()
            err_l = (lse - ref[1]).abs().max().item()
            for _ in range(3):
                ops.flash_attn_fwd(q, k, v, scale, causal)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.iters):
                ops.flash_attn_fwd(q, k, v, scale, causal)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / a.iters * 1e3
            print(json.dumps({"B": a.B, "S": S, "H": a.H, "Hkv": hkv, "causal": causal, "packed": a.packed, "qscale": a.qscale, "fa_w64": var,
                              "ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                              "err_o_vs_w0": round(err_o, 5), "err_lse_vs_w0": round(err_l, 5)}), flush=True)
        if a.stamps:
            for mode, name in ((1, "full"), (2, "no softmax"), (3, "no fragment reads"), (4, "no DMA")):
                ops.set_knob("fa_w64_mode", mode)
                stamps(ops, q, k, v, scale, causal, S, name)
            ops.set_knob("fa_w64_mode", 1)
        ops.set_knob("fa_w64", 0)


SECTIONS = ["prologue", "phase1", "sync", "phase2", "rescale+loop", "last", "tail", "drain", "epilogue"]


def stamps(ops, q, k, v, scale, causal, S, name=""):
    """Per-wave cycle totals of the asm program's sections (workgroups 0..1023), per loop tile."""
    import numpy as np
    buf = torch.zeros(1024 * 4 * 16, dtype=torch.int32, device="cuda")
    ops.set_knob("fa_w64", 3)
    ops.set_knob("fa_stamp_ptr", buf.data_ptr())
    ops.flash_attn_fwd(q, k, v, scale, causal)
    torch.cuda.synchronize()
    ops.set_knob("fa_stamp_ptr", 0)
    x = buf.view(1024, 4, 16)[:, :, :9].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    nqb = (S + 255) // 256
    # workgroup i -> q-block (heaviest first, XCD order) is not needed: per wave, loop tiles = tw
    live = x.sum(-1) > 0
    tot = x[live].sum(0)
    loops = x[live][:, 1].size
    res = {sec: int(v_) for sec, v_ in zip(SECTIONS, tot)}
    per_wave = {sec: round(float(v_) / loops, 1) for sec, v_ in zip(SECTIONS, tot)}
    share = {sec: round(float(v_) / float(tot.sum()), 4) for sec, v_ in zip(SECTIONS, tot)}
    tiles = 0  # loop iterations (tiles before each wave's last one): causal tw = 4 qblk + wave
    for i in range(1024):
        j = i >> 3
        qblk = nqb - 1 - (j % nqb)
        for w in range(4):
            if live[i, w]:
                tiles += 4 * qblk + w if causal else (S + 63) // 64 - 1
    per_tile = {sec: round(float(tot[k]) / max(tiles, 1), 1) for k, sec in enumerate(SECTIONS) if 1 <= k <= 4}
    print(json.dumps({"build": name, "stamps_waves": int(loops), "loop_tiles": tiles, "cycles_per_loop_tile": per_tile,
                      "cycles_per_wave": per_wave, "share": share}), flush=True)


if __name__ == "__main__":
    main()
