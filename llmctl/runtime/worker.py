"""Per-rank training worker (``python -m llmctl.runtime.worker`` under torchrun / srun / mpirun).

Reference: ``llmctl/runtime/train_script.py`` — same argparse flags (``train_script.py:18-89``),
plus plan/parallelism flags.  Fixes: the ``--config`` file may be TOML
*or* JSON, ``--plan`` and ``--dataset-path`` are actually consumed, and only flags the user
set override the config file (precedence: defaults < --config < --plan < explicit flags).
MPI launches are mapped from ``OMPI_COMM_WORLD_*`` to the torch env here, in the worker.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import sys
from pathlib import Path
from typing import Any, Dict, List, Optional

DEFAULTS: Dict[str, Any] = dict(
    learning_rate=5e-5, batch_size=8, gradient_accumulation_steps=1, num_epochs=3, max_steps=-1, warmup_steps=0,
    weight_decay=0.01, optimizer="adamw", scheduler="linear", gradient_clipping=1.0, mixed_precision="bf16",
    distributed_backend="auto", deepspeed_config=None, save_steps=500, eval_steps=500, save_total_limit=3,
    resume_from_checkpoint=None, logging_steps=10, log_level="info", seed=42, deterministic=False, config=None,
    plan=None, seq_len=2048, tensor_parallel=1, pipeline_parallel=1, context_parallel=1, context_parallel_mode="ulysses", expert_parallel=1, sequence_parallel=False, zero_stage=0,
    activation_checkpoint="none", num_microbatches=0, device="auto", metrics_jsonl=None, prometheus_port=0,
)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="llmctl distributed LLM training worker")
    S = argparse.SUPPRESS  # unset flags stay absent so config files can supply them
    p.add_argument("--model-name-or-path", type=str, required=True)
    p.add_argument("--dataset-path", type=str, required=True)
    p.add_argument("--output-dir", type=str, required=True)
    p.add_argument("--learning-rate", type=float, default=S)
    p.add_argument("--batch-size", type=int, default=S)
    p.add_argument("--gradient-accumulation-steps", type=int, default=S)
    p.add_argument("--num-epochs", type=int, default=S)
    p.add_argument("--max-steps", type=int, default=S)
    p.add_argument("--warmup-steps", type=int, default=S)
    p.add_argument("--weight-decay", type=float, default=S)
    p.add_argument("--optimizer", type=str, choices=["adamw"], default=S)
    p.add_argument("--scheduler", type=str, choices=["linear", "cosine", "constant"], default=S)
    p.add_argument("--gradient-clipping", type=float, default=S)
    p.add_argument("--mixed-precision", type=str, choices=["no", "fp16", "bf16", "fp32"], default=S)
    p.add_argument("--distributed-backend", type=str, choices=["nccl", "gloo", "auto"], default=S)
    p.add_argument("--deepspeed-config", type=str, default=S, help="accepted for compatibility (ZeRO is native)")
    p.add_argument("--save-steps", type=int, default=S)
    p.add_argument("--eval-steps", type=int, default=S)
    p.add_argument("--save-total-limit", type=int, default=S)
    p.add_argument("--resume-from-checkpoint", type=str, default=S)
    p.add_argument("--logging-steps", type=int, default=S)
    p.add_argument("--log-level", type=str, choices=["debug", "info", "warning", "error"], default=S)
    p.add_argument("--seed", type=int, default=S)
    p.add_argument("--deterministic", action="store_true", default=S)
    p.add_argument("--config", type=str, default=S, help="training config (TOML or JSON)")
    # MI355X / plan additions
    p.add_argument("--plan", type=str, default=S, help="plan TOML from `llmctl plan`")
    p.add_argument("--seq-len", type=int, default=S)
    p.add_argument("--tensor-parallel", type=int, default=S)
    p.add_argument("--pipeline-parallel", type=int, default=S)
    p.add_argument("--sequence-parallel", action="store_true", default=S)
    p.add_argument("--context-parallel", type=int, default=S, help="context-parallel degree")
    p.add_argument("--context-parallel-mode", type=str, choices=["ulysses", "ring"], default=S,
                   help="ulysses (all-to-all around attention) or ring attention")
    p.add_argument("--expert-parallel", type=int, default=S, help="MoE: experts sharded over this many DP ranks")
    p.add_argument("--zero-stage", type=int, default=S)
    p.add_argument("--activation-checkpoint", type=str, choices=["none", "selective", "full"], default=S)
    p.add_argument("--num-microbatches", type=int, default=S)
    p.add_argument("--device", type=str, default=S)
    p.add_argument("--metrics-jsonl", type=str, default=S)
    p.add_argument("--prometheus-port", type=int, default=S)
    p.add_argument("--pack-sequences", action="store_true", default=S, help="document-masked packed sequences")
    p.add_argument("--profile-dir", type=str, default=S, help="torch.profiler Chrome traces per rank")
    p.add_argument("--profile-schedule", type=str, default=S, help="wait=a,warmup=b,active=c | step(N)")
    p.add_argument("--collective-timeout-s", type=float, default=S)
    return p


def map_mpi_env() -> None:
    if "OMPI_COMM_WORLD_RANK" in os.environ and "RANK" not in os.environ:
        os.environ["RANK"] = os.environ["OMPI_COMM_WORLD_RANK"]
        os.environ["WORLD_SIZE"] = os.environ["OMPI_COMM_WORLD_SIZE"]
        os.environ["LOCAL_RANK"] = os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")
    if "PMI_RANK" in os.environ and "RANK" not in os.environ:
        os.environ["RANK"] = os.environ["PMI_RANK"]
        os.environ["WORLD_SIZE"] = os.environ.get("PMI_SIZE", "1")


def resolve(args: argparse.Namespace) -> Dict[str, Any]:
    from llmctl.config.schemas import resolve_training_config
    from llmctl.config.toml_io import load_any

    explicit = vars(args).copy()
    file_cfg = None
    if explicit.get("config"):
        raw = load_any(explicit["config"])
        if any(k in raw for k in ("optimizer", "parallel", "checkpoint", "training")):
            file_cfg = raw
        else:  # flat JSON in TrainingConfig field names (reference train_script.py:91-103)
            file_cfg = None
            for k, v in raw.items():
                explicit.setdefault(k, v)
    plan = load_any(explicit["plan"]) if explicit.get("plan") else None
    cli = {}
    for k, v in explicit.items():
        if k in ("config", "plan", "metrics_jsonl", "prometheus_port", "model_name_or_path"):
            continue
        cli[k] = v
    merged = resolve_training_config(file_cfg, plan, cli)
    out = dict(DEFAULTS)
    out.update(merged)
    if explicit.get("plan"):
        out["plan_file"] = explicit["plan"]
    out["dataset_path"] = explicit.get("dataset_path", "synthetic")
    out["output_dir"] = explicit["output_dir"]
    # the CLI always passes a model (default "gpt2"); a config/plan-specified model wins over that default
    cli_model = explicit.get("model_name_or_path")
    if cli_model and not ("model_name_or_path" in merged and cli_model == "gpt2"):
        out["model_name_or_path"] = cli_model
    elif plan and plan.get("model", {}).get("layers") and cli_model == "gpt2":
        out["model_name_or_path"] = plan.get("metadata", {}).get("model_file", cli_model)
    out["metrics_jsonl"] = explicit.get("metrics_jsonl")
    out["prometheus_port"] = explicit.get("prometheus_port", 0)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    map_mpi_env()
    from llmctl.utils.env import install_hang_dump

    install_hang_dump()
    args = build_parser().parse_args(argv)
    opts = resolve(args)
    from llmctl.runtime.engine import TrainingEngine, create_training_config

    metrics_jsonl = opts.pop("metrics_jsonl", None)
    prom_port = opts.pop("prometheus_port", 0)
    opts.pop("config", None)
    opts.pop("plan", None)
    cfg = create_training_config(**opts)
    eng = TrainingEngine(cfg)
    from llmctl.metrics.observability import attach_training_metrics

    attach_training_metrics(eng, jsonl_path=metrics_jsonl or os.path.join(cfg.output_dir, "logs",
                                                                         f"metrics_rank{eng.rank}.jsonl"),
                            prometheus_port=prom_port if eng.is_main else 0)
    try:
        result = eng.train()
    finally:
        eng.shutdown()
    if eng.is_main:
        print(json.dumps({"final_loss": result["final_loss"], "steps": result["steps"]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
