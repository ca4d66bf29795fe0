"""``llmctl export convert`` — export a checkpoint (reference: ``export.py:13-35``, a stub there).

Formats: ``safetensors`` (consolidated, layout-independent llmctl names), ``hf``
(HF-Llama tensor names + ``config.json``, loadable by ``transformers``).  ``onnx`` /
``tensorrt`` / ``gguf`` are reported as unsupported on this platform (exit code 2).
Quantizers (plugin group ``quantizers``): ``int8`` (per-output-channel absmax RTN) and
``fp8`` (OCP e4m3, per-channel scale — the gfx950 MFMA fp8 format); the reference's names
``int8-awq`` / ``int4-gptq`` map to RTN int8 / int4 with a warning (no calibration data).
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console

console = Console()
app = typer.Typer(help="Export models to deployment formats")


@app.command()
def convert(
    ckpt: str = typer.Option(..., help="Checkpoint directory"),
    format: str = typer.Option("safetensors", help="safetensors | hf | onnx | tensorrt | gguf"),
    quant: Optional[str] = typer.Option(None, help="int8 | fp8 | int4 | int8-awq | int4-gptq"),
    out: Path = typer.Option(..., help="Output directory"),
) -> None:
    """Convert a checkpoint to a deployment format."""
    from llmctl.plugins.exporters import export_checkpoint

    try:
        info = export_checkpoint(ckpt, format, str(out), quant)
    except NotImplementedError as e:
        console.print(f"[red]{e}[/red]")
        raise typer.Exit(2)
    console.print_json(json.dumps(info))
    console.print(f"[green]✓ Exported to {out}[/green]")


@app.callback(invoke_without_command=True)
def main(ctx: typer.Context, ckpt: Optional[str] = typer.Option(None), out: Optional[Path] = typer.Option(None),
         format: str = typer.Option("safetensors")) -> None:
    """Export models (``llmctl export --ckpt C --out O`` == ``export convert …``)."""
    if ctx.invoked_subcommand is None:
        if ckpt is None or out is None:
            console.print("Use 'llmctl export convert --ckpt <dir> --out <dir>'")
            raise typer.Exit(1)
        convert(ckpt=ckpt, format=format, quant=None, out=out)
