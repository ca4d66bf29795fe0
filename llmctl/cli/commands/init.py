"""``llmctl init`` — scaffold a project (reference: ``llmctl/cli/commands/init.py:53-264``).

Same directory tree, model JSON, ``configs/default.toml`` (same keys/defaults),
``configs/data/example.toml``, ``scripts/train.sh`` and README; additionally writes the
MI355X hardware preset and accepts more templates (gpt/125m, llama/13b/30b/70b).  Bare
``llmctl init`` scaffolds with the defaults (the reference crashed).
"""

from __future__ import annotations

import json
import sys
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Initialize project and create configs")


def default_train_config(template: str, size: str) -> dict:
    return {
        "model": {"name": f"{template}-{size}", "arch": "decoder-only",
                  "config_file": f"configs/models/{template}-{size}.json"},
        "optimizer": {"type": "adamw", "lr": 2e-4, "betas": [0.9, 0.95], "weight_decay": 0.1,
                      "scheduler": {"type": "cosine", "warmup_steps": 2000}},
        "data": {"train": "data/train", "val": "data/val", "tokenizer": "tokenizers/gpt-bpe.json",
                 "pack_sequences": True, "num_workers": 8},
        "hardware": {"gpus_per_node": 1, "gpu": "auto-detect", "memory_gb": "auto-detect",
                     "intra_node_interconnect": "auto-detect", "inter_node_interconnect": "auto-detect",
                     "cpu_pinning": "numa-aware"},
        "parallel": {"strategy": "auto", "tensor_parallel": 1, "pipeline_parallel": 1, "sequence_parallel": False,
                     "zero_stage": 1, "activation_checkpoint": "selective", "micro_batch_size": 1,
                     "global_batch_size": 64},
        "limits": {"target_flops": 1.0e12, "max_memory_gb": 16, "max_comm_bw_gbps": 100},
        "checkpoint": {"path": "checkpoints", "interval_steps": 1000, "sharded": True, "async": True},
        "telemetry": {"otlp_endpoint": None,
                      "metrics": ["flops", "mem_bw", "comm_bw", "latency", "throughput", "loss"], "traces": True},
    }


DATASET_CONFIG = {
    "name": "example-dataset", "format": "json",
    "sources": [{"path": "data/train.jsonl", "split": "train"}, {"path": "data/val.jsonl", "split": "validation"}],
    "preprocessing": {"tokenizer": "gpt2", "max_length": 2048, "padding": "max_length", "truncation": True},
}


@app.command()
def scaffold(
    template: str = typer.Option("gpt", help="Model template (gpt, gpt2, llama)"),
    size: str = typer.Option("7b", help="Model size (125m, 7b, 13b, 30b, 70b)"),
    name: Optional[str] = typer.Option(None, help="Project name"),
    output_dir: Path = typer.Option(Path("."), help="Output directory"),
    force: bool = typer.Option(False, "--force", help="Overwrite existing files"),
) -> None:
    """Scaffold a new LLM project with configs and directory structure."""
    from llmctl.config.toml_io import dump_toml
    from llmctl.models.config import MODEL_TEMPLATES

    if name is None:
        name = f"{template}-{size}-project"
    project_dir = output_dir / name
    if project_dir.exists() and not force and sys.stdin.isatty():
        from rich.prompt import Confirm

        if not Confirm.ask(f"Directory {project_dir} exists. Continue?"):
            raise typer.Abort()
    console.print(f"[bold green]Creating project: {name}[/bold green]")
    console.print(f"[blue]Location: {project_dir}[/blue]")
    for d in ["configs/presets", "configs/hw", "configs/data", "configs/models", "plans", "checkpoints",
              "artifacts", "logs", "data", "scripts"]:
        (project_dir / d).mkdir(parents=True, exist_ok=True)
        console.print(f"[dim]Created: {d}[/dim]")
    if template in MODEL_TEMPLATES and size in MODEL_TEMPLATES[template]:
        model_file = project_dir / "configs" / "models" / f"{template}-{size}.json"
        model_file.write_text(json.dumps(MODEL_TEMPLATES[template][size], indent=2))
        console.print(f"[green]Created model config: {model_file}[/green]")
    else:
        console.print(f"[yellow]No template {template}/{size}; skipping model config[/yellow]")
    cfg_file = project_dir / "configs" / "default.toml"
    dump_toml(default_train_config(template, size), cfg_file)
    console.print(f"[green]Created default config: {cfg_file}[/green]")
    data_file = project_dir / "configs" / "data" / "example.toml"
    dump_toml(DATASET_CONFIG, data_file)
    console.print(f"[green]Created dataset config: {data_file}[/green]")
    from llmctl.cli.commands.hw import mi355x_preset

    dump_toml(mi355x_preset(8), project_dir / "configs" / "presets" / "mi355x8.toml")
    script = f"""#!/bin/bash
# Example training script for {name}

# Basic single-node training
llmctl train \\
    --config configs/default.toml \\
    --data configs/data/example.toml \\
    --launcher local \\
    --gpus-per-node 1

# Multi-node training (uncomment for distributed setup)
# llmctl train \\
#     --config configs/default.toml \\
#     --data configs/data/example.toml \\
#     --launcher slurm \\
#     --nodes 4 \\
#     --gpus-per-node 8
"""
    sf = project_dir / "scripts" / "train.sh"
    sf.write_text(script)
    sf.chmod(0o755)
    console.print(f"[green]Created training script: {sf}[/green]")
    readme = f"""# {name}

This project was scaffolded using llmctl with template: {template}-{size}

## Quick Start

1. Probe hardware:
   ```bash
   llmctl hw probe --emit configs/hw/local.toml
   ```

2. Compute parallelism plan:
   ```bash
   llmctl plan --model configs/models/{template}-{size}.json --hardware configs/hw/local.toml --out plans/local.toml
   ```

3. Launch training:
   ```bash
   llmctl train --config configs/default.toml --plan plans/local.toml
   ```

## Directory Structure

- `configs/` - Configuration files (models, hardware profiles, data, presets)
- `plans/` - Parallelism plans
- `checkpoints/` - Model checkpoints
- `artifacts/` - Exported model artifacts
- `logs/` - Training logs
- `data/` - Training data
- `scripts/` - Helper scripts
"""
    (project_dir / "README.md").write_text(readme)
    console.print(f"[green]Created README: {project_dir / 'README.md'}[/green]")
    console.print(f"\n[bold green]✅ Project {name} initialized successfully![/bold green]")
    console.print("\n[yellow]Next steps:[/yellow]")
    console.print(f"1. cd {project_dir}")
    console.print("2. llmctl hw probe --emit configs/hw/local.toml")
    console.print(f"3. llmctl plan --model configs/models/{template}-{size}.json --hardware configs/hw/local.toml")
    console.print("4. ./scripts/train.sh")


@app.callback(invoke_without_command=True)
def main(
    ctx: typer.Context,
    template: str = typer.Option("gpt", help="Model template"),
    size: str = typer.Option("7b", help="Model size"),
    name: Optional[str] = typer.Option(None, help="Project name"),
    output_dir: Path = typer.Option(Path("."), help="Output directory"),
    force: bool = typer.Option(False, "--force", help="Overwrite existing files"),
) -> None:
    """Initialize project and create configs (bare ``llmctl init`` == ``init scaffold``)."""
    if ctx.invoked_subcommand is None:
        scaffold(template=template, size=size, name=name, output_dir=output_dir, force=force)
