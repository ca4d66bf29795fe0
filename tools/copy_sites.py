#!/usr/bin/env python3
"""Where do the per-step device copies / fills of the GPT-7B training step come from?  One
profiled step under torch.profiler (CPU op stacks), aggregated by the Python frame that issued
aten::copy_ / aten::fill_ / aten::zero_ / aten::contiguous."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from torch.profiler import ProfilerActivity, profile

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = get_model_config("gpt-7b")
    cfg = TrainingConfig(model_name_or_path="gpt-7b", batch_size=12, seq_len=2048, learning_rate=3e-4,
                         max_steps=10, mixed_precision="bf16", device="cuda", log_level="warning")
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, 2048, 12, seed=1, device=eng.device)
    for i in range(2):
        eng.train_step([data.batch(i)])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        eng.train_step([data.batch(2)])
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::contiguous", "aten::zeros", "aten::to",
                       "aten::_to_copy", "aten::clone"):
            st = [f for f in (ev.stack or []) if "llmctl" in f or "bench" in f]
            key = (ev.name, str(ev.input_shapes)[:80], st[0] if st else "?")
            sites[key] += 1
    for (name, shp, site), n in sites.most_common(30):
        print(f"{n:5d}  {name:18s} {shp:80s} {site}")


if __name__ == "__main__":
    main()
