#!/usr/bin/env python3
"""HBM-bound kernels at the GPT-7B mb-12 shapes (T = 24576 tokens): time and effective
bandwidth (bytes each kernel must move / time).  MI355X HBM3E: ~8 TB/s peak, ~6.3 achievable."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

ops = _lib.native()
T, H, F, NQ, NKV, D = 24576, 4096, 11008, 32, 32, 128
dev = "cuda"


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / reps)
    return sorted(ts)[2] * 1e3


def bf(*s):
    return torch.randn(*s, device=dev).bfloat16()


res = {}


def rec(name, ms, nbytes):
    res[name] = {"ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}
    print(name, res[name], flush=True)


x, r, dy, dres = bf(T, H), bf(T, H), bf(T, H), bf(T, H)
w = bf(H)
y, ro, rstd = ops.add_rmsnorm_fwd(x, r, w, 1e-5)
E = T * H * 2
rec("add_rmsnorm_fwd", timeit(lambda: ops.add_rmsnorm_fwd(x, r, w, 1e-5)), 4 * E)
rec("rmsnorm_bwd+dres", timeit(lambda: ops.rmsnorm_bwd(dy, ro, w, rstd, dres)), 4 * E)
rec("rmsnorm_bwd", timeit(lambda: ops.rmsnorm_bwd(dy, ro, w, rstd, None)), 3 * E)
gu = bf(T, 2 * F)
da = bf(T, F)
rec("swiglu_fwd", timeit(lambda: ops.swiglu_fwd(gu)), 3 * T * F * 2)
rec("swiglu_bwd", timeit(lambda: ops.swiglu_bwd(da, gu)), 5 * T * F * 2)
S = 2048
qkv = bf(T, (NQ + 2 * NKV) * D)
pos = torch.arange(8192, device=dev, dtype=torch.float32)
inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=dev, dtype=torch.float32) / D))
ang = torch.outer(pos, inv)
cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
rec("rope_qkv_fwd", timeit(lambda: ops.rope_qkv_fwd(qkv, cos, sin, NQ, NKV, S, None)), 2 * qkv.numel() * 2)
q, k, v = ops.rope_qkv_fwd(qkv, cos, sin, NQ, NKV, S, None)
rec("rope_qkv_bwd", timeit(lambda: ops.rope_qkv_bwd(q, k, v, cos, sin, S, None)), 2 * qkv.numel() * 2)
n = 1 << 28
p, g = bf(n), bf(n)
master = p.float()
m, vv = torch.zeros_like(master), torch.zeros_like(master)
sc = torch.ones(1, device=dev)
rec("adamw_step (per 2^28 params)",
    timeit(lambda: ops.adamw_step_(p, master, g, m, vv, 1e-4, 0.9, 0.95, 1e-8, 0.1, 0.9, 0.95, sc), reps=5),
    n * (4 + 8 + 8 + 8 + 2))
print(json.dumps(res))
