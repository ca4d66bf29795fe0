"""``llmctl`` command line (Typer).

Same surface as the reference (``llmctl/cli/main.py:19-150``): 13 sub-apps and the global
options.  Differences that fix reference defects:
* heavy modules (torch, the engine, FastAPI) are imported lazily inside commands, so
  ``llmctl --help`` / ``init`` / ``plan`` start instantly and never touch the GPU;
* global options are parsed into a shared :class:`RunContext` that subcommands consume
  (seed, determinism, log level, OTLP endpoint, launcher defaults) instead of being ignored;
* every group works bare (``llmctl init``) and the README short forms work
  (``llmctl plan --model … --hardware …``, ``llmctl train --plan …``, ``llmctl serve --artifact …``).
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()

app = typer.Typer(
    name="llmctl",
    help="Distributed LLM Training and Inference System",
    rich_markup_mode="rich",
    no_args_is_help=True,
)


@dataclass
class RunContext:
    config: Optional[Path] = None
    profile: Optional[str] = None
    backend: str = "torch"
    launcher: str = "local"
    nodes: int = 1
    gpus_per_node: Optional[int] = None
    cpus_per_task: Optional[int] = None
    mixed_precision: str = "bf16"
    seed: int = 42
    deterministic: bool = False
    log_level: str = "info"
    otlp_endpoint: Optional[str] = None
    verbose: bool = False


def get_run_context(ctx: Optional[typer.Context] = None) -> RunContext:
    c = ctx
    while c is not None:
        if isinstance(c.obj, RunContext):
            return c.obj
        c = c.parent
    return RunContext()


from .commands import admin, bench, eval as eval_cmd, export, health, hw, init, plan, replay, serve, trace, train, tune  # noqa: E402

app.add_typer(init.app, name="init", help="Initialize project and create configs")
app.add_typer(hw.app, name="hw", help="Hardware probing and profiling")
app.add_typer(plan.app, name="plan", help="Compute parallelism plans")
app.add_typer(train.app, name="train", help="Launch distributed training")
app.add_typer(eval_cmd.app, name="eval", help="Evaluate checkpoints")
app.add_typer(export.app, name="export", help="Export models to deployment formats")
app.add_typer(serve.app, name="serve", help="Start inference server")
app.add_typer(bench.app, name="bench", help="Run benchmarks")
app.add_typer(trace.app, name="trace", help="Capture and visualize traces")
app.add_typer(replay.app, name="replay", help="Replay runs for debugging")
app.add_typer(tune.app, name="tune", help="Auto-tune kernels and communication")
app.add_typer(health.app, name="health", help="Cluster health checks")
app.add_typer(admin.app, name="admin", help="Administrative operations")


@app.callback()
def main(
    ctx: typer.Context,
    config: Optional[Path] = typer.Option(None, "--config", "-c", help="Configuration file path (TOML/YAML)",
                                          exists=True, file_okay=True, dir_okay=False),
    profile: Optional[str] = typer.Option(None, "--profile", "-p", help="Hardware/cluster profile name"),
    backend: Optional[str] = typer.Option("torch", "--backend", "-b", help="Backend to use"),
    launcher: Optional[str] = typer.Option("local", "--launcher", "-l", help="Launcher to use"),
    nodes: Optional[int] = typer.Option(1, "--nodes", "-n", help="Number of nodes", min=1),
    gpus_per_node: Optional[int] = typer.Option(None, "--gpus-per-node", "-g", help="GPUs per node", min=1),
    cpus_per_task: Optional[int] = typer.Option(None, "--cpus-per-task", help="CPUs per task", min=1),
    mixed_precision: Optional[str] = typer.Option("bf16", "--mixed-precision", help="Mixed precision mode"),
    seed: Optional[int] = typer.Option(42, "--seed", "-s", help="Random seed for reproducibility"),
    deterministic: bool = typer.Option(False, "--deterministic", help="Enable deterministic mode"),
    log_level: str = typer.Option("info", "--log-level", help="Log level"),
    otlp_endpoint: Optional[str] = typer.Option(None, "--otlp-endpoint", help="OpenTelemetry endpoint URL"),
    verbose: bool = typer.Option(False, "--verbose", "-v", help="Enable verbose output"),
) -> None:
    """
    Distributed LLM Training and Inference System

    A comprehensive CLI tool for orchestrating data preparation, model partitioning,
    distributed training, checkpointing, evaluation, and low-latency inference —
    MI355X-native (HIP kernels on CDNA4, RCCL over xGMI).
    """
    rc = RunContext(config=config, profile=profile, backend=backend or "torch", launcher=launcher or "local",
                    nodes=nodes or 1, gpus_per_node=gpus_per_node, cpus_per_task=cpus_per_task,
                    mixed_precision=mixed_precision or "bf16", seed=42 if seed is None else seed,
                    deterministic=deterministic, log_level=log_level, otlp_endpoint=otlp_endpoint, verbose=verbose)
    ctx.obj = rc
    os.environ.setdefault("LLMCTL_LOG_LEVEL", log_level)
    if otlp_endpoint:
        os.environ["LLMCTL_OTLP_ENDPOINT"] = otlp_endpoint
    if verbose:
        console.print(f"[dim]Global options: backend={rc.backend}, launcher={rc.launcher}, nodes={rc.nodes}, "
                      f"seed={rc.seed}, precision={rc.mixed_precision}[/dim]")


def run() -> None:  # console-script entry point
    app()


if __name__ == "__main__":
    app()
