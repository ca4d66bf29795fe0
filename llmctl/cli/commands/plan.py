"""``llmctl plan`` — parallelism plan + shard map (reference: ``plan.py:204-386``).

Flags and the plan TOML keys (``[metadata]``, ``[parallelism]``, ``[model]``,
``[hardware]``) are the reference's; ``[parallelism]`` gains ``sequence_parallel``,
``activation_checkpoint``, ``grad_accum``, ``num_microbatches``, step-time/throughput
estimates, and a ``[shard_map]`` section (per-rank layer ranges, TP shard ids, ZeRO
partition, process-group rank lists) that ``train`` consumes.  ``--compat-reference`` runs
the reference's exact cost model.  ``llmctl plan --model … --hardware …`` (README short
form) works as well as ``llmctl plan compute …``.
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Dict, Optional

import typer
from rich.console import Console
from rich.table import Table

console = Console()
app = typer.Typer(help="Compute parallelism plans")


def _load(path: Path) -> Dict[str, Any]:
    from llmctl.config.toml_io import load_any

    return load_any(path)


def compute_plan(model: Path, hardware: Path, target_flops: Optional[float] = 1e14, max_memory_gb: Optional[float] = 40,
                 max_comm_bw_gbps: Optional[float] = 100, strategy: str = "auto", tensor_parallel: Optional[int] = None,
                 pipeline_parallel: Optional[int] = None, zero_stage: Optional[int] = None,
                 sequence_parallel: Optional[bool] = None, activation_checkpoint: Optional[str] = None,
                 micro_batch_size: Optional[int] = None, global_batch_size: Optional[int] = None,
                 seq_len: int = 2048, compat_reference: bool = False, max_memory_explicit: bool = False,
                 virtual_stages: Optional[int] = None) -> Dict[str, Any]:
    from llmctl.partition.planner import ParallelismPlanner, ReferenceCompatPlanner
    from llmctl.partition.shard_map import build_shard_map

    model_config = _load(model)
    if "layers" not in model_config and "model" in model_config:
        model_config = model_config["model"]
    hw_profile = _load(hardware)
    if compat_reference:
        planner = ReferenceCompatPlanner(model_config, hw_profile)
        if strategy == "auto":
            plan = planner.search_optimal_plan(target_flops, max_memory_gb, max_comm_bw_gbps)
        else:
            plan = planner.manual_plan(tensor_parallel or 1, pipeline_parallel or 1, zero_stage or 1)
        params = planner.estimate_parameters()
        model_mem = planner.estimate_model_memory()
    else:
        planner = ParallelismPlanner(model_config, hw_profile, seq_len=seq_len)
        mem_limit = max_memory_gb if max_memory_explicit else None
        if strategy == "auto":
            fixed = {"tp": tensor_parallel, "pp": pipeline_parallel, "zs": zero_stage, "sp": sequence_parallel,
                     "ac": activation_checkpoint, "mb": micro_batch_size, "vs": virtual_stages}
            plan = planner.search_optimal_plan(max_memory=mem_limit, global_batch=global_batch_size,
                                               fixed={k: v for k, v in fixed.items() if v is not None} or None)
        else:
            plan = planner.manual_plan(tensor_parallel or 1, pipeline_parallel or 1, 1 if zero_stage is None else zero_stage,
                                       sp=bool(sequence_parallel), ac=activation_checkpoint or "selective",
                                       mb=micro_batch_size or 1, global_batch=global_batch_size,
                                       vs=virtual_stages or 1)
        params = planner.estimate_parameters()
        model_mem = planner.estimate_model_memory()
    sm = None
    if plan.get("data_parallel", 0) >= 1:
        sm = build_shard_map(model_config, plan["tensor_parallel"], plan["pipeline_parallel"], plan["data_parallel"],
                             plan["zero_stage"], plan.get("virtual_stages", 1))
    return {"plan": plan, "params": params, "model_memory_gb": model_mem, "model": model_config,
            "hardware": hw_profile, "shard_map": sm}


def _display(plan: Dict[str, Any], params: int, model_mem: float, target_flops, max_memory_gb, max_comm_bw_gbps):
    console.print("\n[bold blue]Parallelism Plan[/bold blue]")
    t = Table()
    t.add_column("Parameter", style="cyan")
    t.add_column("Value", style="green")
    t.add_column("Description", style="dim")
    rows = [("Tensor Parallel", "tensor_parallel", "Degree of tensor parallelism"),
            ("Pipeline Parallel", "pipeline_parallel", "Degree of pipeline parallelism"),
            ("Virtual Stages", "virtual_stages", "Model chunks per pipeline rank (interleaved 1F1B)"),
            ("Data Parallel", "data_parallel", "Degree of data parallelism"),
            ("ZeRO Stage", "zero_stage", "ZeRO optimizer sharding stage"),
            ("Sequence Parallel", "sequence_parallel", "Megatron-SP inside the TP group"),
            ("Activation Checkpoint", "activation_checkpoint", "Recompute policy"),
            ("Micro Batch Size", "micro_batch_size", "Micro-batch size per GPU"),
            ("Global Batch Size", "global_batch_size", "Global batch size across all GPUs"),
            ("Grad Accumulation", "grad_accum", "Micro-steps per optimizer step")]
    for label, k, desc in rows:
        if k in plan:
            t.add_row(label, str(plan[k]), desc)
    console.print(t)
    console.print("\n[bold blue]Resource Estimates[/bold blue]")
    r = Table()
    for c in ("Resource", "Estimate", "Limit", "Status"):
        r.add_column(c)
    ok = lambda b: "[green]✓[/green]" if b else "[red]✗[/red]"  # noqa: E731
    r.add_row("Memory per GPU", f"{plan['estimated_memory_gb']:.2f} GB", f"{max_memory_gb:.2f} GB",
              ok(plan["estimated_memory_gb"] <= max_memory_gb))
    r.add_row("Communication", f"{plan['estimated_comm_gb']:.2f} GB/s", f"{max_comm_bw_gbps:.2f} GB/s",
              ok(plan["estimated_comm_gb"] <= max_comm_bw_gbps))
    r.add_row("FLOPs per step", f"{plan['estimated_flops']:.2e}", f"{target_flops:.2e}",
              ok(plan["estimated_flops"] <= target_flops))
    if "estimated_tokens_per_sec" in plan:
        r.add_row("Throughput", f"{plan['estimated_tokens_per_sec']:.0f} tok/s", "-", "")
        r.add_row("Step time", f"{plan['estimated_step_time_s']:.3f} s", "-", "")
    console.print(r)
    console.print(f"\n[dim]Model parameters: {params:,}[/dim]")
    console.print(f"[dim]Model memory: {model_mem:.2f} GB[/dim]")


@app.command()
def compute(
    model: Path = typer.Option(..., help="Model configuration file"),
    hardware: Path = typer.Option(..., help="Hardware profile file"),
    target_flops: Optional[float] = typer.Option(1e14, help="Target FLOPs ceiling"),
    max_memory_gb: Optional[float] = typer.Option(None, help="Max memory per GPU in GB (default: 40 in "
                                                   "--compat-reference mode, 90% of HBM otherwise)"),
    max_comm_bw_gbps: Optional[float] = typer.Option(100, help="Max communication bandwidth in GB/s"),
    strategy: str = typer.Option("auto", help="Strategy (auto, manual)"),
    tensor_parallel: Optional[int] = typer.Option(None, help="Manual tensor parallel degree"),
    pipeline_parallel: Optional[int] = typer.Option(None, help="Manual pipeline parallel degree"),
    virtual_stages: Optional[int] = typer.Option(None, "--virtual-stages",
                                                 help="Interleaved pipeline: model chunks per pipeline rank"),
    zero_stage: Optional[int] = typer.Option(None, help="Manual ZeRO stage"),
    sequence_parallel: Optional[bool] = typer.Option(None, "--sequence-parallel/--no-sequence-parallel",
                                                     help="Megatron sequence parallelism"),
    activation_checkpoint: Optional[str] = typer.Option(None, help="none | selective | full"),
    micro_batch_size: Optional[int] = typer.Option(None, help="Micro-batch size per GPU"),
    global_batch_size: Optional[int] = typer.Option(None, help="Global batch size (sets grad accumulation)"),
    seq_len: int = typer.Option(2048, help="Sequence length"),
    compat_reference: bool = typer.Option(False, "--compat-reference", help="Use the reference's cost model"),
    output: Optional[Path] = typer.Option(None, "--out", help="Output plan file"),
    dry_run: bool = typer.Option(False, help="Dry run - don't save plan"),
) -> None:
    """Compute parallelism and sharding plan."""
    console.print("[blue]Loading configurations...[/blue]")
    explicit = max_memory_gb is not None
    mm = max_memory_gb if explicit else (40.0 if compat_reference else None)
    res = compute_plan(model, hardware, target_flops, mm if mm is not None else 40.0, max_comm_bw_gbps, strategy,
                       tensor_parallel, pipeline_parallel, zero_stage, sequence_parallel, activation_checkpoint,
                       micro_batch_size, global_batch_size, seq_len, compat_reference,
                       max_memory_explicit=explicit, virtual_stages=virtual_stages)
    plan = res["plan"]
    hw_count = res["hardware"].get("gpu", {}).get("count", 0)
    console.print(f"[green]✓[/green] Model: {res['model'].get('name', 'Unknown')}")
    console.print(f"[green]✓[/green] Hardware: {hw_count} GPUs")
    shown_mem = mm if mm is not None else 0.9 * (res["hardware"].get("gpu", {}).get("devices", [{}]) or [{}])[0].get(
        "memory_gb", 288.0) or 259.2
    _display(plan, res["params"], res["model_memory_gb"], target_flops, shown_mem, max_comm_bw_gbps)
    if output and not dry_run:
        from llmctl.config.toml_io import dump_toml

        output.parent.mkdir(parents=True, exist_ok=True)
        full = {
            "metadata": {"model_file": str(model), "hardware_file": str(hardware), "strategy": strategy,
                         "cost_model": "reference" if compat_reference else "mi355x", "seq_len": seq_len,
                         "constraints": {"target_flops": target_flops, "max_memory_gb": shown_mem,
                                         "max_comm_bw_gbps": max_comm_bw_gbps}},
            "parallelism": plan,
            "model": res["model"],
            "hardware": res["hardware"],
        }
        if res["shard_map"] is not None:
            full["shard_map"] = res["shard_map"]
        dump_toml(full, output)
        console.print(f"\n[green]✅ Plan saved to: {output}[/green]")
    elif dry_run:
        console.print("\n[yellow]Dry run - plan not saved[/yellow]")
    if plan["estimated_memory_gb"] > shown_mem:
        console.print("\n[red]⚠ Memory requirement exceeds limit![/red]")
        console.print("[yellow]Suggestions:[/yellow]\n  • Increase tensor parallelism\n  • Use higher ZeRO stage\n"
                      "  • Reduce micro-batch size / enable activation checkpointing")


@app.callback(invoke_without_command=True)
def main(
    ctx: typer.Context,
    model: Optional[Path] = typer.Option(None, help="Model configuration file"),
    hardware: Optional[Path] = typer.Option(None, help="Hardware profile file"),
    strategy: str = typer.Option("auto", help="Strategy (auto, manual)"),
    tensor_parallel: Optional[int] = typer.Option(None, help="Manual tensor parallel degree"),
    pipeline_parallel: Optional[int] = typer.Option(None, help="Manual pipeline parallel degree"),
    zero_stage: Optional[int] = typer.Option(None, help="Manual ZeRO stage"),
    sequence_parallel: Optional[bool] = typer.Option(None, "--sequence-parallel/--no-sequence-parallel"),
    compat_reference: bool = typer.Option(False, "--compat-reference"),
    output: Optional[Path] = typer.Option(None, "--out", help="Output plan file"),
) -> None:
    """Compute parallelism plans (``llmctl plan --model M --hardware H`` == ``plan compute``)."""
    if ctx.invoked_subcommand is not None:
        return
    if model is None or hardware is None:
        console.print("Use 'llmctl plan compute' (or 'llmctl plan') with --model and --hardware options")
        raise typer.Exit(1)
    compute(model=model, hardware=hardware, target_flops=1e14, max_memory_gb=None, max_comm_bw_gbps=100,
            strategy=strategy, tensor_parallel=tensor_parallel, pipeline_parallel=pipeline_parallel,
            zero_stage=zero_stage, sequence_parallel=sequence_parallel, activation_checkpoint=None,
            micro_batch_size=None, global_batch_size=None, seq_len=2048, compat_reference=compat_reference,
            output=output, dry_run=False)
