"""``llmctl trace`` — capture and visualise traces (reference: ``trace.py:9-18``, stubs there).

``capture`` runs a short training job under ``torch.profiler`` (ROCm activities via
roctracer/Kineto) and writes a Chrome/Perfetto JSON trace plus a kernel summary table; with
``--rocprof`` it instead wraps the job in ``rocprofv3 --kernel-trace --stats`` (kernel-level
proof that the MFMA kernels run).  ``visualize`` summarises a trace file (top kernels by
time, by category: GEMM / attention / norm / comm / optimizer).
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console
from rich.table import Table

console = Console()
app = typer.Typer(help="Capture and visualize traces")


@app.command()
def capture(
    run: str = typer.Option("latest", help="Run id / output dir to capture (latest = new short run)"),
    model: str = typer.Option("tiny", help="Model template for the traced run"),
    steps: int = typer.Option(3, help="Profiled steps"),
    micro_batch: int = typer.Option(2, help="Micro-batch"),
    seq_len: int = typer.Option(256, help="Sequence length"),
    out_dir: Path = typer.Option(Path("./traces"), help="Output directory"),
    rocprof: bool = typer.Option(False, "--rocprof", help="Use rocprofv3 --kernel-trace --stats instead"),
) -> None:
    """Capture a trace of a short training run."""
    from llmctl.benchmarks.tracing import capture_trace

    res = capture_trace(model=model, steps=steps, micro_batch=micro_batch, seq_len=seq_len, out_dir=out_dir,
                        rocprof=rocprof, run=run)
    console.print_json(json.dumps(res))


@app.command()
def visualize(trace_file: Path = typer.Option(..., help="Trace file (Chrome JSON or rocprof kernel_stats.csv)"),
              top: int = typer.Option(20, help="Rows to show")) -> None:
    """Summarise a trace: top kernels and per-category time."""
    from llmctl.benchmarks.tracing import summarize_trace

    s = summarize_trace(trace_file)
    t = Table(title=f"Top kernels — {trace_file.name}")
    for c in ("kernel", "calls", "total ms", "%"):
        t.add_column(c)
    for row in s["kernels"][:top]:
        t.add_row(row["name"][:90], str(row["calls"]), f"{row['total_ms']:.2f}", f"{row['pct']:.1f}")
    console.print(t)
    console.print_json(json.dumps(s["categories"]))
