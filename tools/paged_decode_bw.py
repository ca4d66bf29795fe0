#!/usr/bin/env python3
"""Paged decode attention bandwidth: time `paged_attention_decode` on the serving decode shape
(GPT-7B: 32 kv heads x 128, 16 sequences x 2k context, 16-token blocks in shuffled order) and
report the cache bytes read per second.  Context splits (`--splits`, knob decode_splits; 0 = the
auto heuristic) and kernel variants under A/B (`--vars`, knob decode_var, when one is built) are
timed alternately on the same caches.  tools/paged_decode_sweep.sh runs the serving shapes.

    python tools/paged_decode_bw.py [--N 16] [--ctx 2048] [--dtypes bf16 fp8] [--splits 0 1 2] [--contig]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--dtypes", nargs="+", default=["bf16", "fp8"])
    ap.add_argument("--vars", type=int, nargs="+", default=[0])
    ap.add_argument("--splits", type=int, nargs="+", default=[0])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--contig", action="store_true", help="blocks in allocation order (a fresh engine's) instead of shuffled")
    a = ap.parse_args()
    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    nb_seq = (a.ctx + a.bs - 1) // a.bs
    nblocks = a.N * nb_seq + 8
    if a.contig:
        perm = torch.arange(1, a.N * nb_seq + 1, device=dev, dtype=torch.int32)
    else:
        perm = torch.randperm(nblocks - 1, device=dev, generator=g)[: a.N * nb_seq].to(torch.int32) + 1
    bt = perm.view(a.N, nb_seq).contiguous()
    lens = torch.full((a.N,), a.ctx, dtype=torch.int32, device=dev)
    q = torch.randn(a.N, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16)
    scale = a.D ** -0.5
    caches = {}
    for dt in a.dtypes:
        k = torch.randn(nblocks, a.bs, a.Hkv, a.D, device=dev, generator=g)
        v = torch.randn(nblocks, a.bs, a.Hkv, a.D, device=dev, generator=g)
        tdt = torch.float8_e4m3fn if dt == "fp8" else torch.bfloat16
        caches[dt] = (k.to(tdt), v.to(tdt))
        del k, v
    res = {}
    ref = {}
    for r in range(a.rounds):
        for dt, (kc, vc) in caches.items():
            nbytes = 2 * a.N * a.ctx * a.Hkv * a.D * kc.element_size()
            for var in a.vars:
                for sp in a.splits:
                    ops.set_knob("decode_var", var)
                    ops.set_knob("decode_splits", sp)
                    out = ops.paged_attention_decode(q, kc, vc, bt, lens, scale)
                    key = (dt, var, sp)
                    if dt not in ref:
                        ref[dt] = out.float()
                    err = (out.float() - ref[dt]).abs().max().item()
                    gr = torch.cuda.CUDAGraph()
                    s = torch.cuda.Stream()
                    with torch.cuda.stream(s):
                        ops.paged_attention_decode(q, kc, vc, bt, lens, scale)
                        with torch.cuda.graph(gr, stream=s):
                            for _ in range(10):
                                ops.paged_attention_decode(q, kc, vc, bt, lens, scale)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    gr.replay()
                    e0.record()
                    for _ in range(a.iters // 10):
                        gr.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / (a.iters // 10 * 10)
                    res.setdefault(key, []).append(us)
                    if r == a.rounds - 1:
                        best = min(res[key])
                        print(json.dumps({"contig": a.contig, "dtype": dt, "decode_var": var, "decode_splits": sp, "N": a.N, "ctx": a.ctx,
                                          "Hkv": a.Hkv, "us": round(best, 2), "us_all": [round(x, 2) for x in res[key]],
                                          "TBps": round(nbytes / best / 1e6, 3), "max_diff_vs_first": round(err, 5)}),
                              flush=True)
    ops.set_knob("decode_var", 0)
    ops.set_knob("decode_splits", 0)


if __name__ == "__main__":
    main()
