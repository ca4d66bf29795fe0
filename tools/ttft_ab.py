#!/usr/bin/env python3
"""Single-request TTFT A/B (GPT-7B, 2048-token prompt): one engine, knob sets timed in interleaved
rounds (same process, same box: CDNA guide §5.4 rule 24); p50 / min TTFT per set.  A knob that is
a PerfKnobs field is set on the engine's own knobs, any other name is a native knob.

    python tools/ttft_ab.py --knob-sets gemm_fused_split=0 gemm_fused_split=1 [--rounds 5 --repeats 4]
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
    ap.add_argument("--knob-sets", nargs="+", required=True, help="'name=value,name=value' native knob sets")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=4)
    ap.add_argument("--init-knobs", default="", help="'name=value,...' PerfKnobs given to the engine at construction")
    a = ap.parse_args()
    import torch

    from llmctl.ops import _lib
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    assert _lib.load(), _lib._error
    ops = torch.ops.llmctl
    sets = [{kv.split("=")[0]: int(kv.split("=")[1]) for kv in ks.split(",")} for ks in a.knob_sets]
    init = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.init_knobs.split(",") if kv}
    eng = InferenceEngine(a.model, device="cuda", max_batch_size=1, max_model_len=a.prompt_length + 32,
                          perf_knobs=init or None)
    p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    V = eng.cfg.vocab_size
    eng.generate([[1] * 32], p)
    times = {i: [] for i in range(len(sets))}
    n = 0
    import dataclasses

    base = eng.knobs
    for rnd in range(a.rounds + 1):
        for i, ks in enumerate(sets):
            eng.knobs = base
            for k, v in ks.items():
                if hasattr(base, k):
                    eng.knobs = dataclasses.replace(eng.knobs, **{k: type(getattr(base, k))(v)})
                else:
                    ops.set_knob(k, v)
            for _ in range(a.repeats):
                n += 1
                s = eng.add_request([(7 * j + n) % V for j in range(a.prompt_length)], p)
                torch.cuda.synchronize()
                t = time.perf_counter()
                while s.status != "finished":
                    eng.step()
                if rnd > 0:  # round 0 warms every set
                    times[i].append((time.perf_counter() - t) * 1e3)
    for i, ks in enumerate(a.knob_sets):
        print(json.dumps({"knobs": ks, "ttft_p50_ms": round(statistics.median(times[i]), 3),
                          "ttft_min_ms": round(min(times[i]), 3), "n": len(times[i]),
                          "prompt_length": a.prompt_length, "model": a.model}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
