#!/usr/bin/env python3
"""Per-GPU memory of BASELINE config #4 (Llama-3-70B, PP4 x DP2, ZeRO-3) from a 1-GPU slice,
against the planner's estimate (llmctl/partition/planner.py ``compute_memory_requirement``).

Two slices of the real 70B layer (hidden 8192, ffn 28672, 64 q / 8 kv heads, vocab 128256) with
L0 and L1 decoder layers train one step each on one MI355X (ZeRO-0, one rank).  Their difference
gives, per decoder layer:
  * state bytes (bf16 param + grad, fp32 master + Adam m / v): allocated after a step;
  * saved activation bytes per micro-batch: allocated at the end of the forward (before the
    backward frees anything) minus the state -- differenced over the two slices;
The intercept is the embedding / LM head / logits share.  The PP4 x DP2 ZeRO-3 layout's stage
(20 layers; stage 0 holds the embedding, stage 3 the LM head) then needs
  state / dp  (ZeRO-3 shards params, grads and optimizer state over the DP pair)
  + 2 gathered layers of bf16 parameters (current + prefetched)
  + activations x layers x in-flight micro-batches (1F1B: min(pp, microbatches) on stage 0)
  + the edge (embedding or LM head + logits) share,
which is printed next to the planner's number for the same micro-batch / recompute setting.

    python tools/memory_check_70b.py --layers 1 2 --micro-batch 1 --ac selective
"""

import argparse
import dataclasses
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GiB = 2**30


def measure(model, layers, mb, seq, ac):
    import torch

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = dataclasses.replace(get_model_config(model), layers=layers)
    cfg = TrainingConfig(model_name_or_path=model, batch_size=mb, seq_len=seq, max_steps=4, learning_rate=1e-4,
                         device="cuda", log_level="warning", activation_checkpoint=ac)
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, seq, mb, seed=1, rank=0, device=eng.device)
    eng.train_step([data.batch(0)])  # allocates everything lazy (grads, optimizer state)
    torch.cuda.synchronize()
    state = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    # the forward's saved activations: allocated bytes at the end of the forward (loss computed,
    # before backward frees anything) minus the resident state
    fwd_end = {}
    inner = eng._forward_backward

    def fb(input_ids, labels, denom, before_backward=None):
        def hook():
            fwd_end["bytes"] = torch.cuda.memory_allocated()
            if before_backward is not None:
                before_backward()
        return inner(input_ids, labels, denom, before_backward=hook)

    eng._forward_backward = fb
    eng.train_step([data.batch(1)])
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated()
    wt = sum(getattr(p, "_llmctl_wt").numel() * 2 for p in eng.model.parameters()
             if getattr(p, "_llmctl_wt", None) is not None)
    res = {"layers": layers, "state_gb": round(state / GiB, 2), "peak_gb": round(peak / GiB, 2),
           "fwd_end_gb": round(fwd_end["bytes"] / GiB, 3),
           "weight_t_gb": round(wt / GiB, 2), "params": sum(p.numel() for p in eng.model.parameters())}
    eng.shutdown()
    del eng
    torch.cuda.empty_cache()
    return res, mc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, nargs=2, default=[1, 2])
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--ac", default="selective")
    ap.add_argument("--pp", type=int, default=4)
    ap.add_argument("--dp", type=int, default=2)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--one", type=int, default=0, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.one:  # child: one slice, one JSON line
        r, _ = measure(a.model, a.one, a.micro_batch, a.seq_len, a.ac)
        print("SLICE " + json.dumps(r), flush=True)
        return
    import subprocess

    rows = []
    for L in a.layers:
        # every slice in a fresh process: a second engine in the same process found ~15 GB of the
        # first still allocated
        cp = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", str(L), "--model", a.model,
                             "--micro-batch", str(a.micro_batch), "--seq-len", str(a.seq_len), "--ac", a.ac],
                            capture_output=True, text=True, check=True)
        r = json.loads([ln for ln in cp.stdout.splitlines() if ln.startswith("SLICE ")][-1][6:])
        print(json.dumps(r), flush=True)
        rows.append(r)
    (r0, r1) = rows
    dl = r1["layers"] - r0["layers"]
    # the slices (ZeRO-0, one rank) keep W^T copies for the data gradients (the grad-sink path);
    # ZeRO-3 installs no grad sink, so the projection leaves them out
    wt_layer = (r1["weight_t_gb"] - r0["weight_t_gb"]) / dl
    state_layer = (r1["state_gb"] - r0["state_gb"]) / dl - wt_layer
    # saved activations per layer per micro-batch: the forward-end allocation minus the state,
    # differenced over the slices (the step's PEAK is set at the LM head / optimizer, not by the
    # layer stack: round 4's peak difference read 0.0 per layer)
    act_layer = ((r1["fwd_end_gb"] - r1["state_gb"]) - (r0["fwd_end_gb"] - r0["state_gb"])) / dl
    edge_state = r0["state_gb"] - r0["weight_t_gb"] - state_layer * r0["layers"]
    # the last stage's edge: LM head / logits / loss transients above the layer activations
    edge_act = (r0["peak_gb"] - r0["state_gb"]) - act_layer * r0["layers"]
    from llmctl.models import get_model_config
    from llmctl.partition.planner import ParallelismPlanner

    full = get_model_config(a.model)
    layers_stage = math.ceil(full.layers / a.pp)
    inflight = min(a.pp, a.microbatches)
    layer_bf16_gb = 2.0 * (full.num_parameters(include_embedding=False) / full.layers) / GiB
    # stage 0: embedding (+ its optimizer state) is about half the measured edge state (embedding +
    # LM head in the slice); stage 3 holds the LM head and the logits
    stage0 = (state_layer * layers_stage + edge_state / 2) / a.dp + 2 * layer_bf16_gb + act_layer * layers_stage * inflight
    stage_last = (state_layer * layers_stage + edge_state / 2) / a.dp + 2 * layer_bf16_gb + \
        act_layer * layers_stage * 1 + edge_act
    planner = ParallelismPlanner(full.to_dict(), {"gpu": {"count": a.pp * a.dp}}, seq_len=a.seq_len)
    est = planner.compute_memory_requirement(1, a.pp, a.dp, 3, a.micro_batch, sp=False, ac=a.ac,
                                             num_microbatches=a.microbatches)
    print(json.dumps({"model": full.name, "layout": f"pp{a.pp}-dp{a.dp}-zero3", "micro_batch": a.micro_batch,
                      "seq_len": a.seq_len, "ac": a.ac, "state_gb_per_layer": round(state_layer, 3),
                      "weight_t_gb_per_layer_zero0": round(wt_layer, 3),
                      "act_gb_per_layer_per_microbatch": round(act_layer, 3), "edge_state_gb": round(edge_state, 2),
                      "edge_act_gb": round(edge_act, 2), "stage0_gb_from_slice": round(stage0, 1),
                      "last_stage_gb_from_slice": round(stage_last, 1), "planner_gb": round(est, 1)}), flush=True)


if __name__ == "__main__":
    main()
