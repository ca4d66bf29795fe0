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
    kernel_type: str = typer.Option("matmul", help="Kernel type to tune (matmul, attention, all; GPU HIP knobs: "
                                    "gemm64, decode-splits, fa-split, skinny, hip = all four)"),
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
    _tune_hip_knobs(tuner, kernel_type, matrix_size, seq_len, batch_size, num_heads, head_dim, device)
    if save_results:
        tuner.save_results(str(save_results))
    console.print("[green]✓ Kernel tuning completed successfully![/green]")


def _tune_hip_knobs(tuner, kind: str, matrix_size: str, seq_len: int, batch_size: int, num_heads: int, head_dim: int,
                    device: str) -> dict:
    """HIP kernel knobs (GPU only) whose winners TrainingEngine / InferenceEngine dispatch when
    given the saved tuning cache (``llmctl.plugins.tuning_cache``)."""
    import torch

    out = {}
    if kind not in ("gemm64", "decode-splits", "fa-split", "skinny", "hip"):
        return out
    if not torch.cuda.is_available() or device == "cpu":
        console.print("[yellow]HIP kernel knobs need a GPU: skipped[/yellow]")
        return out
    m, k, n = map(int, matrix_size.lower().split("x"))
    if kind in ("gemm64", "hip"):
        for layout in ("dgrad", "wgrad"):
            r = tuner.tune_gemm64(m, n, k, layout, device)
            out[f"gemm64_{layout}"] = r.best_config
            console.print(f"[green]gemm64 {layout} {m}x{n}x{k}: best {r.best_config} "
                          f"{r.best_performance * 1e3:.3f} ms[/green]")
    if kind in ("decode-splits", "hip"):
        r = tuner.tune_decode_splits(batch_size, seq_len, num_heads, num_heads, head_dim, device)
        out["decode_splits"] = r.best_config
        console.print(f"[green]decode splits {batch_size}x{seq_len}: best {r.best_config}[/green]")
    if kind in ("fa-split", "hip"):
        r = tuner.tune_fa_split(batch_size, seq_len, num_heads, head_dim, device)
        out["fa_split"] = r.best_config
        console.print(f"[green]flash-attn split {batch_size}x{seq_len}: best {r.best_config}[/green]")
    if kind in ("skinny", "hip"):
        r = tuner.tune_skinny(batch_size, n, k, device)
        out["skinny"] = r.best_config
        console.print(f"[green]decode GEMM {batch_size}x{n}x{k}: best {r.best_config}[/green]")
    return out


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
    # GPU: the HIP kernel knobs on GPT-7B shapes (consumed via the saved tuning cache)
    summary.update(_tune_hip_knobs(tuner, "hip", "24576x4096x12288", 2048, 16, 32, 128, device))
    (output_dir / "full_tuning_results.json").write_text(json.dumps(summary, indent=2, default=str))
    tuner.save_results(str(output_dir / "tuning_cache.json"))
    console.print("\n[green]✓ Comprehensive auto-tuning completed![/green]")
    for comp, res in summary.items():
        console.print(f"  {comp}: {res['improvement']:.1f}% improvement in {res['time']:.1f}s")
    console.print(f"[green]Results saved to: {output_dir}[/green]")
