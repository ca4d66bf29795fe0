"""``llmctl tune`` — kernel / communication auto-tuning (reference: ``tune.py:13-209``).

Same subcommands, flags and output files (``full_tuning_results.json``,
``tuning_cache.json``); the knobs are real (see :mod:`llmctl.plugins.autotuning`).
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Auto-tune kernels and communication")

DTYPES = {"float32": "float32", "float16": "float16", "bfloat16": "bfloat16", "fp32": "float32", "bf16": "bfloat16",
          "fp16": "float16"}


@app.command()
def kernels(
    kernel_type: str = typer.Option("matmul", help="Kernel type to tune (matmul, attention, all)"),
    matrix_size: str = typer.Option("1024x1024x1024", help="Matrix size for matmul (MxKxN)"),
    seq_len: int = typer.Option(512, help="Sequence length for attention"),
    batch_size: int = typer.Option(8, help="Batch size for attention"),
    num_heads: int = typer.Option(8, help="Number of attention heads"),
    head_dim: int = typer.Option(64, help="Head dimension for attention"),
    device: str = typer.Option("auto", help="Device to use (auto, cuda, cpu)"),
    max_iterations: int = typer.Option(50, help="Maximum tuning iterations"),
    timeout: float = typer.Option(300.0, help="Tuning timeout in seconds"),
    save_results: Optional[Path] = typer.Option(None, help="Save results to file"),
    load_cache: Optional[Path] = typer.Option(None, help="Load cached results from file"),
) -> None:
    """Auto-tune kernel performance."""
    from llmctl.plugins.autotuning import TuningConfig, create_auto_tuner

    console.print("[blue]Auto-tuning kernels...[/blue]")
    tuner = create_auto_tuner(TuningConfig(max_iterations=max_iterations, timeout=timeout))
    if load_cache and load_cache.exists():
        tuner.load_results(str(load_cache))
    if kernel_type in ("matmul", "all"):
        try:
            m, k, n = map(int, matrix_size.lower().split("x"))
        except ValueError:
            console.print(f"[red]Invalid matrix size format: {matrix_size}. Use MxKxN format.[/red]")
            raise typer.Exit(2)
        r = tuner.tune_matmul((m, k, n), device)
        console.print(f"[green]MatMul tuning completed: best {r.best_config} "
                      f"{r.best_performance * 1e3:.3f} ms ({r.improvement:.1f}% vs first config)[/green]")
    if kernel_type in ("attention", "all"):
        r = tuner.tune_attention(seq_len, head_dim, batch_size, num_heads, device)
        console.print(f"[green]Attention tuning completed: best {r.best_config} "
                      f"{r.best_performance * 1e3:.3f} ms ({r.improvement:.1f}%)[/green]")
    if save_results:
        tuner.save_results(str(save_results))
    console.print("[green]✓ Kernel tuning completed successfully![/green]")


@app.command()
def comms(
    tensor_size: str = typer.Option("1024x1024", help="Tensor size (e.g. 1024x1024)"),
    dtype: str = typer.Option("float32", help="Data type"),
    max_iterations: int = typer.Option(50, help="Maximum tuning iterations"),
    timeout: float = typer.Option(300.0, help="Tuning timeout in seconds"),
    save_results: Optional[Path] = typer.Option(None, help="Save results to file"),
    load_cache: Optional[Path] = typer.Option(None, help="Load cached results from file"),
) -> None:
    """Auto-tune communication (bucket size, collective algorithm)."""
    import torch

    from llmctl.plugins.autotuning import TuningConfig, create_auto_tuner

    try:
        shape = tuple(int(x) for x in tensor_size.lower().split("x"))
    except ValueError:
        console.print(f"[red]Invalid tensor size: {tensor_size}[/red]")
        raise typer.Exit(2)
    dt = getattr(torch, DTYPES.get(dtype, dtype))
    tuner = create_auto_tuner(TuningConfig(max_iterations=max_iterations, timeout=timeout))
    if load_cache and load_cache.exists():
        tuner.load_results(str(load_cache))
    r = tuner.tune_communication(shape, dt)
    console.print(f"[green]Communication tuning completed: best {r.best_config} "
                  f"{r.best_performance * 1e3:.3f} ms ({r.improvement:.1f}%)[/green]")
    if save_results:
        tuner.save_results(str(save_results))


@app.command()
def full(
    device: str = typer.Option("auto", help="Device to use (auto, cuda, cpu)"),
    max_iterations: int = typer.Option(25, help="Maximum iterations per component"),
    timeout: float = typer.Option(600.0, help="Total tuning timeout in seconds"),
    output_dir: Path = typer.Option(Path("./tuning_results"), help="Output directory for results"),
) -> None:
    """Run comprehensive auto-tuning for all components."""
    from llmctl.plugins.autotuning import TuningConfig, create_auto_tuner

    output_dir.mkdir(parents=True, exist_ok=True)
    tuner = create_auto_tuner(TuningConfig(max_iterations=max_iterations, timeout=timeout / 3))
    summary = {}
    console.print("[blue]1/3 Tuning matrix multiplication...[/blue]")
    r = tuner.tune_matmul((1024, 1024, 1024), device)
    summary["matmul"] = {"improvement": r.improvement, "best_config": r.best_config, "time": r.total_time}
    console.print("[blue]2/3 Tuning attention kernels...[/blue]")
    r = tuner.tune_attention(512, 64, 8, 8, device)
    summary["attention"] = {"improvement": r.improvement, "best_config": r.best_config, "time": r.total_time}
    console.print("[blue]3/3 Tuning communication...[/blue]")
    r = tuner.tune_communication((1024, 1024))
    summary["communication"] = {"improvement": r.improvement, "best_config": r.best_config, "time": r.total_time}
    (output_dir / "full_tuning_results.json").write_text(json.dumps(summary, indent=2))
    tuner.save_results(str(output_dir / "tuning_cache.json"))
    console.print("\n[green]✓ Comprehensive auto-tuning completed![/green]")
    for comp, res in summary.items():
        console.print(f"  {comp}: {res['improvement']:.1f}% improvement in {res['time']:.1f}s")
    console.print(f"[green]Results saved to: {output_dir}[/green]")
