#!/usr/bin/env python3
"""Host cost of one captured decode step (GPT-7B, 16 x 2048-token prompts): input staging
(pinned host buffers -> device), hipGraph replay call, and the GPU time behind it."""
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
    p = SamplingParams(max_tokens=64, temperature=0.0, ignore_eos=True)
    seqs = [eng.add_request([(7 * i + r) % 32000 for i in range(2048)], p) for r in range(16)]
    while any(s.first_token_time is None for s in seqs):
        eng.step()
    out = eng.scheduler.schedule()
    plan = eng.decode_plan(out.decode)
    eng.decode_exec(plan)  # capture
    torch.cuda.synchronize()
    g, b = eng._graphs[eng._bucket(len(out.decode))]
    stage, replay, gpu = [], [], []
    with torch.inference_mode():
        for _ in range(40):
            t0 = time.perf_counter()
            for k in ("ids", "positions", "slots", "block_tables", "ctx_lens"):
                b[k].copy_(b["host_" + k], non_blocking=True)
            t1 = time.perf_counter()
            g.replay()
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            stage.append(t1 - t0)
            replay.append(t2 - t1)
            gpu.append(t3 - t2)
    med = lambda v: round(sorted(v)[len(v) // 2] * 1e3, 3)  # noqa: E731
    print(json.dumps({"staging_ms": med(stage), "replay_call_ms": med(replay), "after_replay_ms": med(gpu)}))


if __name__ == "__main__":
    main()
