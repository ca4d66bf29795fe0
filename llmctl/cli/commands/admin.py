"""``llmctl admin`` — checkpoint GC, tensor inspection, dataset indexing (reference: ``admin.py``, stubs).

* ``gc``: keep the newest ``--keep`` ``checkpoint-*`` directories under ``--root`` (the
  config's ``checkpoint.keep_latest``); never deletes ``final/`` or the ``latest`` target;
* ``inspect``: per-tensor shape/dtype/norm of a checkpoint (+ training_state summary);
* ``index``: tokenize a text/jsonl corpus into a memory-mappable ``.bin`` token file with a
  document index (``.idx``) via the native C++ indexer (numpy fallback).
"""

from __future__ import annotations

import json
import shutil
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console
from rich.table import Table

console = Console()
app = typer.Typer(help="Administrative operations")


@app.command()
def gc(root: Path = typer.Option(Path("./outputs"), help="Training output directory"),
       keep: int = typer.Option(3, help="Checkpoints to keep"),
       dry_run: bool = typer.Option(False, help="Only list what would be removed")) -> None:
    """Garbage-collect old checkpoints."""
    ckpts = sorted((p for p in root.glob("checkpoint-*") if p.is_dir()), key=lambda p: int(p.name.split("-")[-1]))
    latest = (root / "latest").read_text().strip() if (root / "latest").exists() else None
    victims = [p for p in ckpts[:-keep] if p.name != latest] if keep > 0 else [p for p in ckpts if p.name != latest]
    for p in victims:
        console.print(f"{'would remove' if dry_run else 'removing'} {p}")
        if not dry_run:
            shutil.rmtree(p, ignore_errors=True)
    console.print(f"[green]✓ {len(victims)} checkpoint(s) {'eligible' if dry_run else 'removed'}; "
                  f"kept {min(keep, len(ckpts))}[/green]")


@app.command()
def inspect(checkpoint: Path = typer.Option(..., help="Checkpoint directory")) -> None:
    """Inspect a checkpoint's tensors and training state."""
    from llmctl.io.checkpoint import load_full_state_dict
    from llmctl.models.config import ModelConfig

    cfg = ModelConfig.from_file(checkpoint / "config.json")
    sd = load_full_state_dict(checkpoint, cfg)
    t = Table(title=str(checkpoint))
    for c in ("tensor", "shape", "dtype", "rms"):
        t.add_column(c)
    total = 0
    for k in sorted(sd):
        v = sd[k]
        total += v.numel()
        t.add_row(k, str(tuple(v.shape)), str(v.dtype).replace("torch.", ""),
                  f"{v.float().pow(2).mean().sqrt().item():.4g}")
    console.print(t)
    console.print(f"parameters: {total:,}")
    st = checkpoint / "training_state.json"
    if st.exists():
        s = json.loads(st.read_text())
        console.print_json(json.dumps({k: s.get(k) for k in ("global_step", "epoch", "consumed_samples",
                                                             "world_size", "layout", "zero_stage")}))


@app.command()
def index(dataset: Path = typer.Option(..., help="Text / jsonl corpus (or directory of them)"),
          out: Optional[Path] = typer.Option(None, help="Output .bin (default: alongside input)")) -> None:
    """Tokenize + index a dataset into a memory-mapped token file."""
    from llmctl.io.indexer import index_dataset

    res = index_dataset(str(dataset), str(out) if out else None)
    console.print_json(json.dumps(res))
