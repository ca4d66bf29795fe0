"""``llmctl serve`` — paged-KV continuous-batching inference server (reference: ``serve.py:16-69``).

Same flags (``--artifact --port --host --scheduler --max-batch-size --max-batch-tokens
--max-concurrent --device``), now all forwarded (the reference dropped ``--scheduler`` and
``--device``).  ``--artifact`` is a checkpoint directory written by ``llmctl train``
(``config.json`` + safetensors) or a model template name (random init, for benchmarking).
"""

from __future__ import annotations

from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Start inference server")


@app.command()
def start(
    artifact: str = typer.Option(..., help="Checkpoint directory or model template name"),
    port: int = typer.Option(8080, help="Server port"),
    host: str = typer.Option("0.0.0.0", help="Server host"),
    scheduler: str = typer.Option("dynamic", help="Scheduler (dynamic = continuous batching, prefill_first = TTFT-oriented continuous batching, static)"),
    max_batch_size: int = typer.Option(8, help="Maximum sequences per decode step"),
    max_batch_tokens: int = typer.Option(8192, help="Maximum tokens per engine step"),
    max_concurrent: int = typer.Option(128, help="Maximum concurrent requests"),
    device: str = typer.Option("auto", help="Device (auto, cuda, cpu)"),
    kv_cache_fraction: float = typer.Option(0.85, help="Fraction of free HBM for the paged KV cache"),
    block_size: int = typer.Option(16, help="KV cache block size (tokens)"),
    cuda_graphs: bool = typer.Option(True, "--hip-graphs/--no-hip-graphs", help="Capture decode steps in hipGraphs"),
    tensor_parallel: int = typer.Option(1, help="TP degree (run under torchrun for >1)"),
    kv_cache_dtype: str = typer.Option("auto", help="KV cache element: auto (the model dtype) or fp8 (OCP e4m3fn)"),
    weight_dtype: str = typer.Option("auto", help="Decode projection weights: auto (the model dtype) or fp8 (OCP "
                                                  "e4m3fn, per-row scales; prefill keeps the model dtype)"),
) -> None:
    """Start the inference server."""
    from llmctl.serve.server import create_inference_server

    p = Path(artifact)
    from llmctl.models.config import ALIASES

    if not p.exists() and artifact.lower() not in ALIASES:
        console.print(f"[red]Artifact not found: {artifact}[/red]")
        raise typer.Exit(1)
    console.print("[blue]Starting inference server...[/blue]")
    console.print(f"[yellow]Artifact: {artifact}[/yellow]  [yellow]Endpoint: http://{host}:{port}[/yellow]")
    console.print(f"[yellow]Scheduler: {scheduler}, max batch {max_batch_size}, max tokens {max_batch_tokens}, "
                  f"max concurrent {max_concurrent}, device {device}[/yellow]")
    if tensor_parallel > 1:
        # one process per GPU: torchrun -> llmctl.serve.tp (rank 0 serves HTTP, the rest run
        # the TP worker loop); started as a child process, never exec'd
        import os
        import subprocess
        import sys

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tensor_parallel}",
               "--master-addr=127.0.0.1", f"--master-port={os.environ.get('MASTER_PORT', '29512')}",
               "-m", "llmctl.serve.tp", "--artifact", artifact, "--host", host, "--port", str(port),
               "--max-batch-size", str(max_batch_size), "--max-batch-tokens", str(max_batch_tokens),
               "--max-concurrent", str(max_concurrent), "--kv-cache-fraction", str(kv_cache_fraction),
               "--block-size", str(block_size), "--scheduler", scheduler,
               "--kv-cache-dtype", kv_cache_dtype, "--weight-dtype", weight_dtype] + ([] if cuda_graphs else ["--no-graphs"])
        console.print(f"[yellow]Tensor parallel: {tensor_parallel} ranks (RCCL)[/yellow]")
        raise typer.Exit(subprocess.call(cmd))
    server = create_inference_server(model_path=artifact, host=host, port=port, max_batch_size=max_batch_size,
                                     max_batch_tokens=max_batch_tokens, max_concurrent=max_concurrent,
                                     scheduler=scheduler, device=device, kv_cache_fraction=kv_cache_fraction,
                                     block_size=block_size, use_graphs=cuda_graphs, tensor_parallel=tensor_parallel,
                                     kv_cache_dtype=kv_cache_dtype, weight_dtype=weight_dtype)
    try:
        server.run()
    except KeyboardInterrupt:
        console.print("\n[yellow]Server stopped[/yellow]")


@app.callback(invoke_without_command=True)
def main(
    ctx: typer.Context,
    artifact: Optional[str] = typer.Option(None, help="Checkpoint directory or model template name"),
    port: int = typer.Option(8080, help="Server port"),
    host: str = typer.Option("0.0.0.0", help="Server host"),
    device: str = typer.Option("auto", help="Device"),
) -> None:
    """Start inference server (``llmctl serve --artifact A`` == ``serve start --artifact A``)."""
    if ctx.invoked_subcommand is not None:
        return
    if artifact is None:
        console.print("Use 'llmctl serve start --artifact <checkpoint-dir|template>'")
        raise typer.Exit(1)
    start(artifact=artifact, port=port, host=host, scheduler="dynamic", max_batch_size=8, max_batch_tokens=8192,
          max_concurrent=128, device=device, kv_cache_fraction=0.85, block_size=16, cuda_graphs=True,
          tensor_parallel=1, kv_cache_dtype="auto", weight_dtype="auto")
