#!/usr/bin/env python3
"""GEMM library-selection study for the GPT-7B projection shapes (T tokens per step).

For each shape it times, on the same random data (activations ~N(0,1), weights ~N(0,0.02)):
  fwd   y  = x @ w^T        (F.linear)
  dgrad dx = dy @ w
  wgrad dw = dy^T @ x       (hipBLASLt vs the llmctl MFMA kernel)
under (a) hipBLASLt default heuristics, (b) rocBLAS, (c) PyTorch TunableOp (exhaustive
hipBLASLt + rocBLAS solution search per shape; results written to a CSV that the engine can
load with tuning off).

    python tools/gemm_tunable.py --tokens 24576 --csv profiles/tunableop_gpt7b.csv --json gpurun_out/gemm_tunable.json
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "up": (22016, 4096), "down": (4096, 11008),
          "lm_head": (32000, 4096)}


def timeit(f, reps=10, rounds=5):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        t = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / reps)
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--csv", default="gpurun_out/tunableop.csv")
    ap.add_argument("--json", default=None)
    ap.add_argument("--skip-rocblas", action="store_true")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad", help="subset to time/tune")
    ap.add_argument("--append", action="store_true", help="load --csv first and add to it")
    args = ap.parse_args()
    want = set(args.ops.split(","))
    from llmctl.ops._lib import native

    ops = native()
    T = args.tokens
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    data = {}
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        dy = (torch.randn(T, N, device=dev, generator=g) * 1e-2).bfloat16()
        data[name] = (x, w, dy, torch.empty(N, K, device=dev, dtype=torch.bfloat16))
        if "wgradT" in want:  # K(=tokens)-contiguous copies: the wgrad as an NT GEMM
            data[name] += (dy.t().contiguous(), x.t().contiguous())
        if "dgradT" in want:  # a transposed weight copy: the dgrad in the forward's (TN) layout
            data[name] += (None, None, w.t().contiguous())

    def ops_for(name):
        x, w, dy, dw = data[name][:4]
        dyT, xT = data[name][4:6] if len(data[name]) > 4 else (None, None)
        wT = data[name][6] if len(data[name]) > 6 else None
        return {k: f for k, f in {
            "fwd": lambda: F.linear(x, w),
            "dgrad": lambda: dy @ w,
            "wgrad": lambda: torch.mm(dy.t(), x, out=dw),
            "wgradT": lambda: torch.mm(dyT, xT.t(), out=dw),
            "dgradT": lambda: F.linear(dy, wT),
            "transpose": lambda: (dy.t().contiguous(), x.t().contiguous()),
        }.items() if k in want}

    res = {}

    def run(tag):
        for name in SHAPES:
            N, K = SHAPES[name]
            fl = 2.0 * T * N * K
            for op, f in ops_for(name).items():
                ms = timeit(f)
                res.setdefault(name, {})[f"{op}_{tag}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
                print(name, op, tag, res[name][f"{op}_{tag}"], flush=True)

    run("hipblaslt")
    for name in (SHAPES if "wgrad" in want else []):  # the llmctl MFMA wgrad kernel
        N, K = SHAPES[name]
        x, w, dy, dw = data[name][:4]
        ms = timeit(lambda: ops.gemm_ex(dy, x, dw, True, True, False))
        res[name]["wgrad_llmctl"] = {"ms": round(ms, 4), "tflops": round(2.0 * T * N * K / ms / 1e9, 1)}
        print(name, "wgrad llmctl", res[name]["wgrad_llmctl"], flush=True)
    if not args.skip_rocblas:
        torch.backends.cuda.preferred_blas_library("cublas")  # = rocBLAS on ROCm
        run("rocblas")
        torch.backends.cuda.preferred_blas_library("cublaslt")
    tun = torch.cuda.tunable
    os.makedirs(os.path.dirname(os.path.abspath(args.csv)), exist_ok=True)
    tun.set_filename(args.csv, insert_device_ordinal=False)
    tun.enable(True)
    if args.append and os.path.exists(args.csv):
        tun.read_file(args.csv)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(40)
    tun.set_max_tuning_iterations(30)
    t0 = time.time()
    for name in SHAPES:  # tune every op once
        for op, f in ops_for(name).items():
            f()
            torch.cuda.synchronize()
            print("tuned", name, op, f"{time.time() - t0:.0f}s", flush=True)
    tun.tuning_enable(False)
    run("tunableop")
    tun.enable(False)
    summary = {}
    for tag in ("hipblaslt", "rocblas", "tunableop"):
        tot = 0.0
        ok = True
        for name in SHAPES:
            for op in sorted(want):
                k = f"{op}_{tag}"
                if k not in res[name]:
                    ok = False
                    continue
                tot += res[name][k]["ms"]
        if ok:
            summary[tag] = round(tot, 3)
    if want == {"fwd", "dgrad", "wgrad"}:
        summary["hipblaslt_with_llmctl_wgrad"] = round(sum(
            res[n]["fwd_hipblaslt"]["ms"] + res[n]["dgrad_hipblaslt"]["ms"] + res[n]["wgrad_llmctl"]["ms"]
            for n in SHAPES), 3)
    res["summary_ms_one_layer_each"] = summary
    print(json.dumps(summary), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
