#!/usr/bin/env python3
"""Host-side phase timing of serving decode steps (GPT-7B, 16 x 2048-token prompts): schedule,
decode plan, graph replay (incl. input staging), sampling + token readback, bookkeeping."""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    eng = InferenceEngine("gpt-7b", device="cuda", max_batch_size=16, max_model_len=2048 + 160)
    p = SamplingParams(max_tokens=96, temperature=0.0, ignore_eos=True)
    seqs = [eng.add_request([(7 * i + r) % 32000 for i in range(2048)], p) for r in range(16)]
    while any(s.first_token_time is None for s in seqs):  # prefills
        eng.step()
    t = collections.defaultdict(float)
    n = 0
    torch.cuda.synchronize()
    t_all = time.perf_counter()
    while any(s.status != "finished" for s in seqs):
        a = time.perf_counter()
        out = eng.scheduler.schedule()
        b = time.perf_counter()
        plan = eng.decode_plan(out.decode)
        c = time.perf_counter()
        logits = eng.decode_exec(plan)
        d = time.perf_counter()
        toks = eng.sample(logits, out.decode)
        e = time.perf_counter()
        for seq, tok in zip(out.decode, toks):
            eng.scheduler.computed(seq, 1)
            eng._append(seq, tok)
        f = time.perf_counter()
        for k, v in (("schedule", b - a), ("plan", c - b), ("exec_replay", d - c), ("sample_sync", e - d), ("append", f - e)):
            t[k] += v * 1e3
        n += 1
    wall = (time.perf_counter() - t_all) * 1e3
    print(json.dumps({"steps": n, "ms_per_step": round(wall / n, 3), **{k: round(v / n, 3) for k, v in t.items()}}))


if __name__ == "__main__":
    main()
