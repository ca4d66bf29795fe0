#!/usr/bin/env python3
"""Where a single-request TTFT goes (GPT-7B, 2048-token prompt): host time in the scheduler,
the plan build, the launch of the prefill forward, the wait for the GPU, and sampling, by
wrapping the engine's methods (one request at a time, after warm-up); plus the GPU time of the
same prefill forward alone (CUDA events around prefill_exec on an idle stream).

    python tools/ttft_breakdown.py [--repeats 10]
"""
import argparse
import json
import statistics
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-7b")
    ap.add_argument("--prompt-length", type=int, default=2048)
    ap.add_argument("--repeats", type=int, default=10)
    a = ap.parse_args()
    import torch

    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    eng = InferenceEngine(a.model, device="cuda", max_batch_size=1, max_model_len=a.prompt_length + 32)
    p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    V = eng.cfg.vocab_size
    eng.generate([[1] * 32], p)
    acc = {}

    def wrap(name, fn):
        def w(*args, **kw):
            t = time.perf_counter()
            out = fn(*args, **kw)
            acc[name] = acc.get(name, 0.0) + (time.perf_counter() - t) * 1e3
            return out
        return w

    eng.scheduler.schedule = wrap("schedule", eng.scheduler.schedule)
    eng.prefill_plan = wrap("plan", eng.prefill_plan)
    eng.prefill_exec = wrap("exec_launch", eng.prefill_exec)
    eng.sample = wrap("sample_incl_gpu_wait", eng.sample)
    rows = []
    for r in range(a.repeats + 2):
        acc.clear()
        s = eng.add_request([(7 * i + r) % V for i in range(a.prompt_length)], p)
        torch.cuda.synchronize()
        t = time.perf_counter()
        while s.status != "finished":
            eng.step()
        ttft = (time.perf_counter() - t) * 1e3
        if r >= 2:
            rows.append(dict(acc, ttft=ttft))
    out = {k: round(statistics.median([x[k] for x in rows]), 3) for k in rows[0]}
    # GPU time of the prefill forward alone
    seq = eng.add_request([(5 * i) % V for i in range(a.prompt_length)], p)
    from llmctl.serve.scheduler import PrefillChunk

    assert eng.kv.add_sequence(seq.seq_id, seq.num_tokens)
    plan = eng.prefill_plan([PrefillChunk(seq, 0, seq.num_tokens)])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    gpu = []
    for _ in range(5):
        torch.cuda.synchronize()
        ev[0].record()
        eng.prefill_exec(plan)
        ev[1].record()
        torch.cuda.synchronize()
        gpu.append(ev[0].elapsed_time(ev[1]))
    out["prefill_gpu_ms"] = round(statistics.median(gpu), 3)
    out["model"], out["prompt_length"] = a.model, a.prompt_length
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
