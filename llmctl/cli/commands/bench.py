"""``llmctl bench`` — kernels / e2e serving / comms / dataloader (reference: ``bench.py``, stubs there).

* ``kernels``: llmctl HIP kernels vs their PyTorch counterparts (``--attention --matmul
  --kv-cache --flash --rope``), TFLOP/s and GB/s;
* ``e2e``: serving TTFT / TPOT / throughput through the paged-KV engine
  (``--prompt-length 2048 --gen-length 256 --qps``);
* ``comms``: RCCL bus bandwidth, nccl-tests style (``--pattern allreduce --size 1GB
  --ranks N``; spawns N local ranks, or use under torchrun);
* ``dataloader``: token-loader throughput (``--io local``).
"""

from __future__ import annotations

import json
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Run benchmarks")


@app.command()
def kernels(
    attention: bool = typer.Option(True, "--attention/--no-attention", help="Benchmark attention"),
    matmul: bool = typer.Option(True, "--matmul/--no-matmul", help="Benchmark matmul"),
    kv_cache: bool = typer.Option(False, "--kv-cache", help="Benchmark KV-cache write + paged decode"),
    flash: bool = typer.Option(False, "--flash", help="Flash-attention fwd+bwd"),
    rope: bool = typer.Option(False, "--rope", help="RoPE kernel"),
    device: str = typer.Option("auto", help="auto | cuda | cpu"),
) -> None:
    """Benchmark the HIP kernel library."""
    from llmctl.benchmarks.kernels import run_kernel_benchmarks

    res = run_kernel_benchmarks(attention=attention or flash, matmul=matmul, kv_cache=kv_cache, flash=flash,
                                rope=rope, device=device)
    console.print_json(json.dumps(res))


@app.command()
def e2e(
    prompt_length: int = typer.Option(2048, help="Prompt length"),
    gen_length: int = typer.Option(256, help="Generation length"),
    qps: Optional[float] = typer.Option(None, help="Request rate (None = all at once)"),
    num_requests: int = typer.Option(16, help="Number of requests"),
    model: str = typer.Option("gpt-7b", help="Checkpoint dir or template"),
    max_batch_size: int = typer.Option(16, help="Max decode batch"),
    device: str = typer.Option("auto", help="auto | cuda | cpu"),
    scheduler: str = typer.Option("prefill_first", help="prefill_first | dynamic | static"),
    max_batch_tokens: Optional[int] = typer.Option(None, help="Prefill token budget per step (default: 4096 "
                                                                 "for prefill_first, 8192 otherwise)"),
    kv_cache_dtype: str = typer.Option("auto", help="KV cache element: auto (model dtype) | fp8 (e4m3fn)"),
    weight_dtype: str = typer.Option("auto", help="Decode projection weights: auto (model dtype) | fp8 (e4m3fn, row scales)"),
) -> None:
    """End-to-end serving benchmark (TTFT p50/p99, TPOT, tokens/s).

    Defaults to the ``prefill_first`` policy with a 4096-token prefill budget: on a burst of
    2048-token prompts it gave the lowest TTFT p50 and TPOT of the measured policies/budgets
    (``profiles/serve_r2_session6.txt``: p50 213 ms at 4096 vs 222 ms at 8192 tokens;
    ``dynamic`` 300 ms)."""
    from llmctl.benchmarks.serving import run_serving_benchmark

    res = run_serving_benchmark(model=model, prompt_length=prompt_length, gen_length=gen_length, qps=qps,
                                num_requests=num_requests, max_batch_size=max_batch_size, device=device,
                                scheduler=scheduler, max_batch_tokens=max_batch_tokens, kv_cache_dtype=kv_cache_dtype,
                                weight_dtype=weight_dtype)
    console.print_json(json.dumps(res))


@app.command()
def comms(
    pattern: str = typer.Option("allreduce", help="allreduce | reduce_scatter | all_gather | alltoall | p2p"),
    size: str = typer.Option("1GB", help="Message size (e.g. 64MB, 1GB)"),
    ranks: int = typer.Option(2, help="Ranks to spawn when not already under torchrun"),
    iters: int = typer.Option(20, help="Timed iterations"),
    backend: str = typer.Option("auto", help="auto | nccl | gloo"),
) -> None:
    """Collective bandwidth (algbw / busbw) over RCCL (xGMI) or gloo."""
    from llmctl.benchmarks.comms import parse_size, run_comms_benchmark

    res = run_comms_benchmark(pattern, parse_size(size), ranks, iters, backend)
    console.print_json(json.dumps(res))


@app.command()
def dataloader(
    io: str = typer.Option("local", help="local | synthetic"),
    throughput: bool = typer.Option(True, "--throughput/--no-throughput", help="Report tokens/s"),
    path: Optional[str] = typer.Option(None, help="Token file (.bin); generated if absent"),
    seq_len: int = typer.Option(2048, help="Sequence length"),
    batch_size: int = typer.Option(8, help="Batch size"),
    batches: int = typer.Option(200, help="Batches to read"),
) -> None:
    """Data-loader throughput (native C++ memmap loader vs numpy)."""
    from llmctl.benchmarks.dataloader import run_dataloader_benchmark

    res = run_dataloader_benchmark(io=io, path=path, seq_len=seq_len, batch_size=batch_size, batches=batches)
    console.print_json(json.dumps(res))
