#!/usr/bin/env python3
"""Host-side phase timing of the prefill steps of a 16 x 2048-token burst (GPT-7B,
prefill_first): schedule, prefill plan, prefill launch, sampling + token readback (GPU wait),
bookkeeping; per prefill token budget given on the command line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    budgets = [int(b) for b in sys.argv[1:]] or [8192]
    eng = InferenceEngine("gpt-7b", device="cuda", max_batch_size=16, max_model_len=2048 + 160,
                          scheduler="prefill_first", max_batch_tokens=max(budgets))
    p = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    for budget in budgets + budgets:  # first pass per budget warms up
        eng.scheduler.max_batch_tokens = budget
        seqs = [eng.add_request([(7 * i + r + budget) % 32000 for i in range(2048)], p) for r in range(16)]
        torch.cuda.synchronize()
        t = {"schedule": 0.0, "plan": 0.0, "launch": 0.0, "sample_sync": 0.0, "append": 0.0}
        steps = 0
        t0 = time.perf_counter()
        firsts = []
        while any(s.first_token_time is None for s in seqs):
            a = time.perf_counter()
            out = eng.scheduler.schedule()
            b = time.perf_counter()
            plan = eng.prefill_plan(out.prefill)
            c = time.perf_counter()
            logits = eng.prefill_exec(plan)
            d = time.perf_counter()
            final = [ch.seq for ch in out.prefill if ch.final]
            toks = eng.sample(logits, final) if final else []
            e = time.perf_counter()
            for ch in out.prefill:
                eng.scheduler.computed(ch.seq, ch.count)
            for s, tok in zip(final, toks):
                eng._append(s, tok)
                firsts.append((time.perf_counter() - t0) * 1e3)
            f = time.perf_counter()
            for k, v in (("schedule", b - a), ("plan", c - b), ("launch", d - c), ("sample_sync", e - d),
                         ("append", f - e)):
                t[k] += v * 1e3
            steps += 1
        while any(s.status != "finished" for s in seqs):
            eng.step()
        firsts.sort()
        print(json.dumps({"budget": budget, "prefill_steps": steps, "ttft_p50_ms": round((firsts[7] + firsts[8]) / 2, 2),
                          **{k: round(v / steps, 3) for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
