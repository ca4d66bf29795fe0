#!/usr/bin/env python3
"""Per-phase cycle timeline of the persistent 4-wave GEMM (gemm64 config 304) from its STAMP
diagnostic build: s_memtime at the start of every phase (4 per 64-deep K-tile), before and after
the epilogue, for every wave of workgroups 0-31 over their first 4 items.  Prints, per shape and
ablation (--exps: 0 full kernel, 1 no DMA pieces, 2 no barriers, 3 no fragment reads; results are
garbage under 1-3), the median cycles of each phase slot (P0-P3), the item's loop and epilogue
cycles and the ideal MFMA cycles of a phase (32 x v_mfma_f32_16x16x32_bf16 = 512).

    LLMCTL_BUILD_DEFINES="LLMCTL_STAMP LLMCTL_STAMP_EXP=<n>" python -m llmctl.ops.build --force
    python tools/gemm_stamps.py [--shapes o up] [--layouts fwd dgrad]

The stamps and the ablations (EXP) exist only in a library built with those defines (one
ablation per build); rebuild without them afterwards.
"""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008)}
STAMPS = 272


def analyse(s, K):
    KT = K // 64
    nph = 4 * KT
    whole = nph + 3 <= STAMPS  # the epilogue stamps fit
    n = nph if whole else STAMPS - 1
    d = np.diff(s[..., : (nph + 3 if whole else STAMPS)], axis=-1) % (1 << 32)
    ph = d[..., 0:n]  # stamp i -> i + 1: phase i's body and its closing wait / barrier
    res = {"phase_median": {f"P{j}": float(np.median(ph[..., j::4])) for j in range(4)},
           "phase_mean": round(float(ph.mean()), 1), "phase_p90": float(np.percentile(ph, 90)),
           "first_phase_median": float(np.median(ph[..., 0])),
           "mfma_share_of_phases": round(512.0 / float(ph[..., 1:].mean()), 3),
           "wave_skew_median": float(np.median(s[..., 1:n].max(1) - s[..., 1:n].min(1)))}
    if whole:
        loop = ph.sum(-1)
        res.update({"loop_cycles_median": float(np.median(loop)), "ideal_loop": 512 * nph,
                    "epilogue_median": float(np.median(d[..., nph + 1]))})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--shapes", nargs="+", default=["o", "up"])
    ap.add_argument("--layouts", nargs="+", default=["fwd", "dgrad"])
    ap.add_argument("--exps", type=int, nargs="+", default=[0])
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    T = a.tokens
    buf = torch.zeros(32 * 4 * 4 * STAMPS, dtype=torch.int32, device="cuda")
    for name in a.shapes:
        out_f, in_f = SHAPES[name]
        x = (torch.rand(T, in_f, device="cuda") * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(out_f, in_f, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(T, out_f, device="cuda") * 2 - 1).to(torch.bfloat16)
        for lay in a.layouts:
            if lay == "fwd":
                A, B, at, bt, K = x, W, False, False, in_f
                C = torch.empty(T, out_f, device="cuda", dtype=torch.bfloat16)
            else:
                A, B, at, bt, K = dy, W, False, True, out_f
                C = torch.empty(T, in_f, device="cuda", dtype=torch.bfloat16)
            for ex in a.exps:
                for _ in range(3):  # warm clocks
                    ops.gemm64_ex(A, B, C, at, bt, False, 304)
                buf.zero_()
                ops.set_knob("gemm_exp", ex)
                ops.set_knob("gemm_stamp_ptr", buf.data_ptr())
                ops.gemm64_ex(A, B, C, at, bt, False, 304)
                torch.cuda.synchronize()
                ops.set_knob("gemm_stamp_ptr", 0)
                s = buf.view(32, 4, 4, STAMPS).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
                print(json.dumps({"shape": name, "layout": lay, "exp": ex, "K": K, **analyse(s, K)}), flush=True)


if __name__ == "__main__":
    main()
