"""Locate device copies / fills in one GPT-7B-shaped training step (fewer layers): torch.profiler
with Python stacks, printing the llmctl call sites of ``aten::copy_`` / ``clone`` / ``fill_`` /
``zero_`` ops that launched device work, by device time.

    python tools/find_copies.py [--layers 4] [--micro-batch 12]
"""

import argparse
import collections
import dataclasses
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--micro-batch", type=int, default=12)
    ap.add_argument("--seq-len", type=int, default=2048)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = dataclasses.replace(get_model_config("gpt-7b"), layers=a.layers)
    cfg = TrainingConfig(model_name_or_path="gpt-7b", batch_size=a.micro_batch, seq_len=a.seq_len,
                         max_steps=10, device="cuda", log_level="warning")
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, a.seq_len, a.micro_batch, seed=1, rank=0, device=eng.device)
    for i in range(2):
        eng.train_step([data.batch(i)])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        eng.train_step([data.batch(3)])
        torch.cuda.synchronize()
    names = ("aten::copy_", "aten::clone", "aten::fill_", "aten::zero_", "aten::contiguous", "aten::zeros",
             "aten::cat", "aten::index_select")
    n = collections.Counter()
    us = collections.defaultdict(float)
    for ev in prof.events():
        if ev.name not in names:
            continue
        dev = sum(k.duration for k in ev.kernels) if getattr(ev, "kernels", None) else 0.0
        if dev <= 0:
            continue
        stack = [s for s in (ev.stack or []) if "llmctl" in s or "torch/autograd" in s][:5]
        key = (ev.name, str(ev.input_shapes[:2]) if ev.input_shapes else "", " <- ".join(stack))
        n[key] += 1
        us[key] += dev
    print(f"{'device us':>10} {'n':>4}  op shapes / site")
    for key, t in sorted(us.items(), key=lambda kv: -kv[1])[:30]:
        print(f"{t:10.1f} {n[key]:4d}  {key[0]} {key[1]}\n{'':16}{key[2]}")
    print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=25))


if __name__ == "__main__":
    main()
