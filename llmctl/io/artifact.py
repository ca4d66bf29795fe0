"""Load a model for inference / eval / export from a checkpoint directory or a template.

A checkpoint directory is what ``TrainingEngine`` writes (``config.json`` + ``model.safetensors``
or TP/PP shards + index); shards are consolidated and the model is rebuilt at TP=1 (or
re-sharded for the serving TP degree).  A template name (``gpt-7b``) builds a random-init
model of that architecture (benchmarks; no Hub access on the GPU box).
"""

from __future__ import annotations

from pathlib import Path
from typing import Optional, Tuple

import torch

from llmctl.models import DecoderLM, ModelConfig, ParallelContext, build_model, get_model_config


def resolve_checkpoint_dir(path: str) -> Optional[Path]:
    p = Path(path)
    if not p.exists():
        return None
    if (p / "config.json").exists():
        return p
    if (p / "latest").exists():
        q = p / (p / "latest").read_text().strip()
        if (q / "config.json").exists():
            return q
    if (p / "final" / "config.json").exists():
        return p / "final"
    return None


def load_model(path: str, device=None, dtype=torch.bfloat16, pc: Optional[ParallelContext] = None,
               seed: int = 0) -> Tuple[DecoderLM, ModelConfig, Optional[Path]]:
    ck = resolve_checkpoint_dir(path)
    if ck is None:
        cfg = get_model_config(path)
        model = build_model(cfg, device=device, dtype=dtype, pc=pc, seed=seed)
        return model, cfg, None
    cfg = ModelConfig.from_file(ck / "config.json")
    from llmctl.io.checkpoint import _global_name, load_full_state_dict, shard_tp

    full = load_full_state_dict(ck, cfg)
    with torch.device("meta"):
        pass
    model = build_model(cfg, device=device, dtype=dtype, pc=pc, seed=seed)
    tp = pc.tp_size if pc else 1
    tpr = pc.tp_rank if pc else 0
    start = pc.layer_index if pc else 0
    with torch.no_grad():
        for n, p in model.named_parameters():
            g = _global_name(n, start)
            if g not in full:
                raise KeyError(f"{ck}: missing tensor {g}")
            p.copy_(shard_tp(g, full[g], tp, tpr, cfg).to(p.dtype))
    return model, cfg, ck
