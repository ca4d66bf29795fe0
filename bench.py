#!/usr/bin/env python3
"""Flagship benchmark: GPT-7B pre-training step throughput (tokens/s per node).

Metric/config from BASELINE.json: ``tokens/sec (node) GPT-7B train at 1/2/4/8 MI355X`` on
the reference's ``gpt-7b`` template (32 layers, hidden 4096, ffn 11008, 32 heads, vocab
32000 — ``llmctl/cli/commands/init.py:18-27``) at seq 2048, bf16, synthetic tokens,
random-init weights.  Each step = forward + backward + DP gradient sync + grad-norm clip +
fused AdamW update of ALL parameters (nothing skipped in the timed region).

Usage (driver contract):
    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

Scaling is *weak*: each GPU processes ``--micro-batch`` sequences per step, so the global
batch grows with N.  Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Measured reference-equivalent stack on one MI355X (HF LlamaForCausalLM eager + torch
# AdamW, same GPT-7B config/seq/bf16) — see BASELINE.md §3.  None until measured.
REFERENCE_STACK_TOKENS_PER_SEC_PER_GPU = 17348.3  # best of mb 4/8/12/16 (mb=16), profiles/reference_stack_hf_sdpa_mb_sweep.jsonl


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt-7b")
    ap.add_argument("--seq-len", type=int, default=2048)
    # micro-batch 16 (round 3): 30.44k vs 29.97k tok/s at mb 12 on one box (the per-step optimizer
    # pass and the GEMM tails amortise over 33 % more tokens), 244 vs 212 GB of the 288 GB HBM3E
    # (profiles/bench_r3_mb16.txt); round 1 had measured mb 12-16 flat within noise
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--virtual-stages", type=int, default=1, help="interleaved pipeline chunks per rank")
    ap.add_argument("--microbatches", type=int, default=0, help="pipeline micro-batches (0: 2*pp)")
    ap.add_argument("--zero", type=int, default=-1, help="ZeRO stage (-1: the planner's choice)")
    ap.add_argument("--layout", default="auto", choices=["auto", "manual"],
                    help="auto: TP/PP/ZeRO/SP/recompute/virtual stages from llmctl.partition's planner at the "
                         "fixed micro-batch when no layout flag is given; manual: the flags as given")
    ap.add_argument("--sequence-parallel", action="store_true")
    ap.add_argument("--cp", type=int, default=1, help="context-parallel degree")
    ap.add_argument("--cp-mode", default="ulysses", choices=["ulysses", "ring"])
    ap.add_argument("--ep", type=int, default=1, help="expert-parallel degree (MoE models)")
    ap.add_argument("--activation-checkpoint", default="none")
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--backend", default="auto", help="auto (RCCL on GPU, gloo on CPU) | nccl | gloo")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    mc = get_model_config(args.model)
    plan = None
    if args.layout == "auto" and args.tp == 1 and args.pp == 1 and args.zero < 0 and args.cp == 1 and args.ep == 1 \
            and not args.sequence_parallel and args.activation_checkpoint == "none":
        # run what `llmctl plan --strategy auto` picks for this node size (the micro-batch is
        # part of the metric's config, so it is fixed)
        import dataclasses

        from llmctl.partition.planner import HardwareModel, ParallelismPlanner

        planner = ParallelismPlanner(dataclasses.asdict(mc), {}, args.seq_len, hw=HardwareModel(gpus=world))
        plan = planner.search_optimal_plan(fixed={"mb": args.micro_batch})
        args.tp, args.pp = plan["tensor_parallel"], plan["pipeline_parallel"]
        args.zero = plan["zero_stage"]
        args.sequence_parallel = plan["sequence_parallel"]
        args.activation_checkpoint = plan["activation_checkpoint"]
        args.virtual_stages = plan["virtual_stages"]
        if args.pp > 1:
            args.microbatches = plan["num_microbatches"]
    zero = args.zero if args.zero >= 0 else (1 if world > 1 else 0)
    cfg = TrainingConfig(
        model_name_or_path=args.model, batch_size=args.micro_batch, seq_len=args.seq_len,
        gradient_accumulation_steps=args.grad_accum, learning_rate=3e-4, weight_decay=0.1, scheduler="cosine",
        warmup_steps=10, max_steps=args.warmup + args.steps, gradient_clipping=1.0, mixed_precision="bf16",
        tensor_parallel=args.tp, pipeline_parallel=args.pp, zero_stage=zero,
        virtual_stages=args.virtual_stages, num_microbatches=args.microbatches,
        sequence_parallel=args.sequence_parallel, activation_checkpoint=args.activation_checkpoint,
        context_parallel=args.cp, context_parallel_mode=args.cp_mode, expert_parallel=args.ep,
        bucket_mb=args.bucket_mb, device=args.device, distributed_backend=args.backend, seed=1234,
        log_level="warning")
    eng = TrainingEngine(cfg, mc)
    dev = eng.device
    data = SyntheticTokens(mc.vocab_size, args.seq_len, args.micro_batch, seed=1234, rank=eng.pg.dp_rank, device=dev)
    accum = args.grad_accum if args.pp == 1 else eng.pipeline.num_microbatches

    def step(i):
        batches = [data.batch(i * accum + j) for j in range(accum)]
        return eng.train_step(batches)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    out = None
    for i in range(args.warmup):
        out = step(i)
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step(args.warmup + i)
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if eng.backend == "nccl" else "cpu")
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t)
    loss = float(out["loss"]) if out is not None else float("nan")
    if eng.pipeline is not None:
        loss = eng.pipeline.broadcast_loss(out["loss"])
    dp = eng.pg.layout.dp
    global_batch = args.micro_batch * accum * dp
    tokens = global_batch * args.seq_len * args.steps
    tps = tokens / elapsed
    ms = 1000.0 * elapsed / args.steps
    fpt = mc.flops_per_token(args.seq_len)
    mfu = tps * fpt / (2.5e15 * world) if dev.type == "cuda" else None
    par = f"dp{dp}" + (f"-tp{args.tp}" if args.tp > 1 else "") + (f"-pp{args.pp}" if args.pp > 1 else "") + \
        (f"v{args.virtual_stages}" if args.pp > 1 and args.virtual_stages > 1 else "") + \
        (f"-zero{zero}" if zero else "") + ("-sp" if args.sequence_parallel else "") + \
        (f"-cp{args.cp}{'ring' if args.cp_mode == 'ring' else ''}" if args.cp > 1 else "") + \
        (f"-ep{args.ep}" if args.ep > 1 else "")
    vs = None
    if REFERENCE_STACK_TOKENS_PER_SEC_PER_GPU and mc.name == "gpt-7b" and args.seq_len == 2048 and dev.type == "cuda":
        vs = tps / (REFERENCE_STACK_TOKENS_PER_SEC_PER_GPU * world)
    res = {
        "metric": "tokens/sec (node) GPT-7B train",
        "value": round(tps, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(vs, 4) if vs else None,
        "dtype": "bf16",
        "data": "synthetic (random tokens, random-init weights)",
        "config": {"model": mc.name, "global_batch": global_batch, "seq_len": args.seq_len,
                   "parallelism": par, "micro_batch": args.micro_batch, "grad_accum": accum,
                   "activation_checkpoint": args.activation_checkpoint,
                   "layout": "planner" if plan is not None else "flags",
                   "planner_estimate_tokens_per_sec": plan["estimated_tokens_per_sec"] if plan else None},
        "mfu": round(mfu, 4) if mfu is not None else None,
        "max_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if dev.type == "cuda" else None,
        "final_loss": round(loss, 4),
    }
    if eng.is_main:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    eng.shutdown()


if __name__ == "__main__":
    main()
