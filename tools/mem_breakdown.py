#!/usr/bin/env python3
"""Training-state memory by component after one step of a model slice (one GPU, ZeRO-0):
parameters, flat data / grad buffers, optimizer masters and moments, W^T copies, and the rest
of torch.cuda.memory_allocated.  Bytes per parameter show what a per-GPU planner must assume.

    python tools/mem_breakdown.py --model llama3-70b --layers 1 2
"""
import argparse
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GiB = 2**30


def nbytes(t):
    return 0 if t is None else t.numel() * t.element_size()


def one(model, layers, mb, seq):
    import torch

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = dataclasses.replace(get_model_config(model), layers=layers)
    cfg = TrainingConfig(model_name_or_path=model, batch_size=mb, seq_len=seq, max_steps=4, learning_rate=1e-4,
                         device="cuda", log_level="warning", activation_checkpoint="selective")
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, seq, mb, seed=1, rank=0, device=eng.device)
    eng.train_step([data.batch(0)])
    torch.cuda.synchronize()
    params = sum(p.numel() for p in eng.model.parameters())
    opt = eng.optimizer
    comp = {
        "param_storage": nbytes(eng.flat.data),
        "flat_grad": nbytes(eng.flat.grad),
        "opt_master": nbytes(getattr(opt, "master", None)),
        "opt_exp_avg": nbytes(getattr(opt, "exp_avg", None)),
        "opt_exp_avg_sq": nbytes(getattr(opt, "exp_avg_sq", None)),
        "weight_t_copies": sum(nbytes(getattr(p, "_llmctl_wt", None)) for p in eng.model.parameters()),
        "param_dot_grad_outside_flat": sum(nbytes(p.grad) for p in eng.model.parameters()
                                           if p.grad is not None and p.grad.data_ptr() not in
                                           range(eng.flat.grad.data_ptr(), eng.flat.grad.data_ptr() + nbytes(eng.flat.grad)))
        if eng.flat.grad is not None else 0,
    }
    alloc = torch.cuda.memory_allocated()
    comp["other"] = alloc - sum(comp.values())
    out = {"layers": layers, "params": params, "allocated_gb": round(alloc / GiB, 2)}
    out.update({k: round(v / GiB, 3) for k, v in comp.items()})
    out["bytes_per_param"] = {k: round(v / params, 2) for k, v in comp.items()}
    eng.shutdown()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=2048)
    a = ap.parse_args()
    import torch

    for L in a.layers:
        print(json.dumps(one(a.model, L, a.micro_batch, a.seq_len)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
