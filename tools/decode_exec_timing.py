#!/usr/bin/env python3
"""Where the host time of InferenceEngine.decode_exec goes (graph path), step by step:
pinned-buffer fills, H2D copies, replay call; plus sample() and the bookkeeping."""
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
    p = SamplingParams(max_tokens=64, temperature=0.0, ignore_eos=True)
    seqs = [eng.add_request([(7 * i + r) % 32000 for i in range(2048)], p) for r in range(16)]
    while any(s.first_token_time is None for s in seqs):
        eng.step()
    t = collections.defaultdict(float)
    n = 0
    with torch.inference_mode():
        while any(s.status != "finished" for s in seqs):
            c0 = time.perf_counter()
            out = eng.scheduler.schedule()
            plan = eng.decode_plan(out.decode)
            c1 = time.perf_counter()
            ids, positions, slots, ctx, bt = plan["ids"], plan["positions"], plan["slots"], plan["ctx"], plan["bt"]
            nn = len(ids)
            nb = eng._bucket(nn)
            if nb not in eng._graphs:
                eng._capture(nb)
            g, b = eng._graphs[nb]
            f0 = time.perf_counter()
            h = {k: b["host_" + k].numpy() for k in ("ids", "positions", "slots", "block_tables", "ctx_lens")}
            f1 = time.perf_counter()
            h["ids"][:nn] = ids
            h["positions"][:nn] = positions
            h["slots"][:] = -1
            h["slots"][:nn] = slots
            f2 = time.perf_counter()
            h["block_tables"][:nn] = bt
            f3 = time.perf_counter()
            h["ctx_lens"][:] = 1
            h["ctx_lens"][:nn] = ctx
            c2 = time.perf_counter()
            t["f_numpy"] += (f1 - f0) * 1e3
            t["f_small"] += (f2 - f1) * 1e3
            t["f_bt"] += (f3 - f2) * 1e3
            t["f_ctx"] += (c2 - f3) * 1e3
            t["bt_shape_dtype"] = 0
            info = (bt.shape, str(bt.dtype), str(h["block_tables"].dtype), h["block_tables"].shape)
            for k in ("ids", "positions", "slots", "block_tables", "ctx_lens"):
                b[k].copy_(b["host_" + k], non_blocking=True)
            c3 = time.perf_counter()
            g.replay()
            c4 = time.perf_counter()
            toks = eng.sample(b["logits"][:nn], out.decode)
            c5 = time.perf_counter()
            for seq, tok in zip(out.decode, toks):
                eng.scheduler.computed(seq, 1)
                eng._append(seq, tok)
            c6 = time.perf_counter()
            for k, v in (("sched_plan", c1 - c0), ("fill", c2 - c1), ("copies", c3 - c2), ("replay", c4 - c3),
                         ("sample_sync", c5 - c4), ("append", c6 - c5)):
                t[k] += v * 1e3
            n += 1
    print(json.dumps({"steps": n, **{k: round(v / n, 3) for k, v in t.items()}, "info": str(info)}))


if __name__ == "__main__":
    main()
