"""``llmctl replay run`` — deterministic replay of a recorded run (reference: ``replay.py``, a stub).

Every ``llmctl train`` run directory holds ``run_manifest.json`` (resolved config, seed,
world layout, data position, git revision, loss trace) written by the engine.  ``replay``
re-executes it from the recorded checkpoint (or from scratch) with the same seed and data
order, in deterministic mode, and compares the loss trace step by step.
"""

from __future__ import annotations

import json
from pathlib import Path

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Replay runs for debugging")


@app.command()
def run(run_id: str = typer.Option(..., help="Run directory (output_dir) or manifest path"),
        steps: int = typer.Option(0, help="Steps to replay (0 = all recorded)"),
        tolerance: float = typer.Option(1e-3, help="Max |loss difference| to count as identical")) -> None:
    """Replay a run and diff its loss trace against the recording."""
    from llmctl.runtime.replay import replay_run

    res = replay_run(run_id, steps=steps, tolerance=tolerance)
    console.print_json(json.dumps(res))
    if not res.get("match", False):
        raise typer.Exit(1)
