"""``llmctl eval run`` — evaluate a checkpoint (reference: ``eval.py:13-36``, a stub there).

Tasks: ``perplexity`` (token-level NLL over a token file or synthetic stream),
``latency`` (prefill + decode timing with the serving engine), ``throughput`` (training
step tokens/s of the checkpoint's architecture).  Results are written as JSON to ``--out``.
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Evaluate checkpoints")


@app.command()
def run(
    ckpt: str = typer.Option(..., help="Checkpoint directory (or model template for random init)"),
    suite: Optional[str] = typer.Option(None, help="Evaluation suite name (default: tasks)"),
    tasks: str = typer.Option("perplexity", help="Comma-separated: perplexity, latency, throughput"),
    out: Optional[Path] = typer.Option(None, help="Output JSON file"),
    data: Optional[str] = typer.Option(None, help="Token file (.bin) or text/jsonl for perplexity"),
    seq_len: int = typer.Option(512, help="Evaluation sequence length"),
    batches: int = typer.Option(4, help="Number of evaluation batches"),
    batch_size: int = typer.Option(2, help="Sequences per batch"),
    device: str = typer.Option("auto", help="auto | cuda | cpu"),
) -> None:
    """Evaluate a model checkpoint."""
    from llmctl.benchmarks.evaluate import evaluate

    task_list = [t.strip() for t in (suite or tasks).split(",") if t.strip()]
    console.print(f"[blue]Evaluating {ckpt} on {task_list}[/blue]")
    res = evaluate(ckpt, task_list, data=data, seq_len=seq_len, batches=batches, batch_size=batch_size,
                   device=device)
    console.print_json(json.dumps(res))
    if out:
        out.parent.mkdir(parents=True, exist_ok=True)
        out.write_text(json.dumps(res, indent=2))
        console.print(f"[green]✓ Results saved to {out}[/green]")


@app.callback(invoke_without_command=True)
def main(ctx: typer.Context, ckpt: Optional[str] = typer.Option(None, help="Checkpoint directory")) -> None:
    """Evaluate checkpoints (``llmctl eval --ckpt C`` == ``eval run --ckpt C``)."""
    if ctx.invoked_subcommand is None:
        if ckpt is None:
            console.print("Use 'llmctl eval run --ckpt <checkpoint>'")
            raise typer.Exit(1)
        run(ckpt=ckpt, suite=None, tasks="perplexity", out=None, data=None, seq_len=512, batches=4, batch_size=2,
            device="auto")
