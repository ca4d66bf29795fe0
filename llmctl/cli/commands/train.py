"""``llmctl train`` — launch plan-driven distributed training (reference: ``train.py:15-113``).

Same flags; fixes: ``--plan``/``--config``/``--data`` reach the
worker (TOML or JSON), ``k8s`` is a real launcher, bare ``llmctl train --plan …`` works.
New flags: ``--max-steps``, ``--seq-len``, ``--max-restarts`` (auto-resume from
``<output_dir>/latest``), ``--device``.
"""

from __future__ import annotations

from pathlib import Path
from typing import List, Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Launch distributed training")


def build_worker_args(model: str, data: Optional[Path], output_dir: str, batch_size: int, learning_rate: float,
                      num_epochs: int, mixed_precision: str, grad_accum: int, clip_grad: float,
                      config: Optional[Path], plan: Optional[Path], checkpoint: Optional[str], max_steps: Optional[int],
                      seq_len: Optional[int], seed: int, deterministic: bool, log_level: str,
                      device: Optional[str]) -> List[str]:
    a = ["--model-name-or-path", model, "--dataset-path", str(data) if data else "synthetic",
         "--output-dir", output_dir, "--batch-size", str(batch_size), "--learning-rate", str(learning_rate),
         "--num-epochs", str(num_epochs), "--mixed-precision", mixed_precision,
         "--gradient-accumulation-steps", str(grad_accum), "--gradient-clipping", str(clip_grad),
         "--seed", str(seed), "--log-level", log_level]
    if config:
        a += ["--config", str(config)]
    if plan:
        a += ["--plan", str(plan)]
    if checkpoint:
        a += ["--resume-from-checkpoint", checkpoint]
    if max_steps:
        a += ["--max-steps", str(max_steps)]
    if seq_len:
        a += ["--seq-len", str(seq_len)]
    if deterministic:
        a += ["--deterministic"]
    if device:
        a += ["--device", device]
    return a


@app.command()
def launch(
    ctx: typer.Context,
    plan: Optional[Path] = typer.Option(None, help="Parallelism plan file"),
    config: Optional[Path] = typer.Option(None, help="Training configuration file"),
    data: Optional[Path] = typer.Option(None, help="Data configuration file / token file"),
    model: str = typer.Option("gpt2", help="Model name or path"),
    output_dir: str = typer.Option("./outputs", help="Output directory"),
    checkpoint: Optional[str] = typer.Option(None, help="Checkpoint path for resuming"),
    launcher: str = typer.Option("local", help="Launcher (local, slurm, mpi, k8s)"),
    nodes: int = typer.Option(1, help="Number of nodes"),
    gpus_per_node: int = typer.Option(1, help="GPUs per node"),
    batch_size: int = typer.Option(8, help="Batch size per device"),
    learning_rate: float = typer.Option(5e-5, help="Learning rate"),
    num_epochs: int = typer.Option(3, help="Number of epochs"),
    mixed_precision: str = typer.Option("bf16", help="Mixed precision mode"),
    grad_accum: int = typer.Option(1, help="Gradient accumulation steps"),
    clip_grad: float = typer.Option(1.0, help="Gradient clipping norm"),
    max_steps: Optional[int] = typer.Option(None, help="Stop after N optimizer steps"),
    seq_len: Optional[int] = typer.Option(None, help="Sequence length"),
    max_restarts: int = typer.Option(0, help="Elastic restarts (auto-resume from the latest checkpoint)"),
    save_steps: Optional[int] = typer.Option(None, help="Checkpoint every N steps"),
    device: Optional[str] = typer.Option(None, help="auto | cuda | cpu"),
    dry_run: bool = typer.Option(False, help="Dry run - show command without executing"),
) -> None:
    """Launch distributed training with the computed plan."""
    from llmctl.cli.main import get_run_context
    from llmctl.runtime.launcher import LaunchConfig, ProcessOrchestrator

    rc = get_run_context(ctx)
    console.print("[blue]Preparing distributed training...[/blue]")
    for label, v in (("plan", plan), ("config", config), ("data config", data)):
        if v:
            console.print(f"[green]✓[/green] Using {label}: {v}")
    console.print(f"[yellow]Model: {model}[/yellow]")
    console.print(f"[yellow]Output directory: {output_dir}[/yellow]")
    console.print(f"[yellow]Launcher: {launcher}[/yellow]")
    console.print(f"[yellow]Resources: {nodes} nodes × {gpus_per_node} GPUs[/yellow]")
    console.print(f"[yellow]Batch size: {batch_size}, Learning rate: {learning_rate}[/yellow]")
    args = build_worker_args(model, data, output_dir, batch_size, learning_rate, num_epochs, mixed_precision,
                             grad_accum, clip_grad, config, plan, checkpoint, max_steps, seq_len, rc.seed,
                             rc.deterministic, rc.log_level, device)
    if save_steps:
        args += ["--save-steps", str(save_steps)]
    if max_restarts and not checkpoint:
        args += ["--resume-from-checkpoint", "auto"]  # each (re)start resumes from <output_dir>/latest if present
    lc = LaunchConfig(nodes=nodes, gpus_per_node=gpus_per_node, launcher=launcher, mixed_precision=mixed_precision,
                      config_path=str(config) if config else None, data_path=str(data) if data else None,
                      plan_path=str(plan) if plan else None, checkpoint_path=checkpoint,
                      gradient_accumulation_steps=grad_accum, gradient_clipping=clip_grad, seed=rc.seed,
                      deterministic=rc.deterministic, log_level=rc.log_level, max_restarts=max_restarts,
                      cpus_per_task=rc.cpus_per_task)
    orch = ProcessOrchestrator(lc, echo=lambda s: console.print(s, markup=False, highlight=False))
    if dry_run:
        cmd = orch.launcher.build_command("llmctl.runtime.worker", args) if launcher == "local" else None
        console.print("[yellow]Dry run - would launch training with above configuration[/yellow]")
        if cmd:
            console.print(" ".join(cmd), markup=False)
        return
    try:
        rcode = orch.start_training("llmctl.runtime.worker", args, auto_resume_dir=output_dir, restarts=max_restarts)
    except KeyboardInterrupt:
        console.print("\n[yellow]Training interrupted by user[/yellow]")
        orch.stop_training()
        raise typer.Exit(130)
    if rcode == 0:
        console.print("[green]✓ Training completed successfully![/green]")
    else:
        console.print(f"[red]Training failed (exit code {rcode})![/red]")
        raise typer.Exit(1)


@app.callback(invoke_without_command=True)
def main(
    ctx: typer.Context,
    plan: Optional[Path] = typer.Option(None, help="Parallelism plan file"),
    config: Optional[Path] = typer.Option(None, help="Training configuration file"),
    data: Optional[Path] = typer.Option(None, help="Data configuration file"),
    model: str = typer.Option("gpt2", help="Model name or path"),
    launcher: str = typer.Option("local", help="Launcher (local, slurm, mpi, k8s)"),
    nodes: int = typer.Option(1, help="Number of nodes"),
    gpus_per_node: int = typer.Option(1, help="GPUs per node"),
    max_steps: Optional[int] = typer.Option(None, help="Stop after N optimizer steps"),
    output_dir: str = typer.Option("./outputs", help="Output directory"),
    dry_run: bool = typer.Option(False, help="Dry run"),
) -> None:
    """Launch distributed training (``llmctl train --plan P`` == ``train launch --plan P``)."""
    if ctx.invoked_subcommand is None:
        launch(ctx, plan=plan, config=config, data=data, model=model, output_dir=output_dir, checkpoint=None,
               launcher=launcher, nodes=nodes, gpus_per_node=gpus_per_node, batch_size=8, learning_rate=5e-5,
               num_epochs=3, mixed_precision="bf16", grad_accum=1, clip_grad=1.0, max_steps=max_steps, seq_len=None,
               max_restarts=0, device=None, dry_run=dry_run)
