"""Run manifests and deterministic replay (``llmctl replay run``).

The reference's ``replay.py`` is an echo stub.  Here every ``TrainingEngine.train`` writes
``<output_dir>/run_manifest.json``: the resolved ``TrainingConfig``, the model config, the
world layout (tp/pp/dp), the git revision, torch/ROCm versions and the logged loss trace.
``replay_run`` re-executes the recorded config (same seed, same data order, deterministic
mode, scratch output dir) — in-process for single-rank runs, via ``torch.distributed.run``
with the worker entry point for multi-rank runs — and diffs the loss trace step by step.
"""

from __future__ import annotations

import dataclasses
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Any, Dict, List, Optional

MANIFEST = "run_manifest.json"


def _git_rev() -> Optional[str]:
    try:
        root = Path(__file__).resolve().parents[2]
        return subprocess.run(["git", "-C", str(root), "rev-parse", "HEAD"], capture_output=True, text=True,
                              timeout=5).stdout.strip() or None
    except Exception:
        return None


def write_manifest(engine, history: List[Dict[str, Any]], status: str = "running") -> Optional[Path]:
    if not engine.is_main:
        return None
    import torch

    c = engine.config
    out = Path(c.output_dir)
    out.mkdir(parents=True, exist_ok=True)
    lay = engine.pg.layout
    man = {
        "version": 1,
        "status": status,
        "created": time.strftime("%Y-%m-%dT%H:%M:%S"),
        "git_rev": _git_rev(),
        "torch": torch.__version__,
        "hip": getattr(torch.version, "hip", None),
        "world": {"world_size": lay.world_size, "tp": lay.tp, "pp": lay.pp, "dp": lay.dp},
        "training_config": {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(c).items()},
        "model_config": engine.model_config.to_dict(),
        # the resolved performance knobs (config + tuning cache + LLMCTL_KNOBS): replay runs with these
        "perf_knobs": _active_knobs(),
        "global_step": engine.global_step,
        "history": [{k: float(v) if isinstance(v, (int, float)) else v for k, v in r.items()} for r in history],
    }
    p = out / MANIFEST
    tmp = p.with_suffix(".tmp")
    tmp.write_text(json.dumps(man, indent=1))
    os.replace(tmp, p)
    return p


def _active_knobs() -> Dict[str, Any]:
    from llmctl.config.knobs import knobs

    return knobs().as_dict()


def load_manifest(path: str) -> Dict[str, Any]:
    p = Path(path)
    if p.is_dir():
        p = p / MANIFEST
    if not p.exists():
        raise FileNotFoundError(f"no {MANIFEST} at {path}")
    return json.loads(p.read_text())


def _replay_inprocess(tc: Dict[str, Any], mc: Dict[str, Any]) -> List[Dict[str, Any]]:
    from llmctl.models.config import ModelConfig
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    fields = {f.name for f in dataclasses.fields(TrainingConfig)}
    cfg = TrainingConfig(**{k: (tuple(v) if k == "betas" else v) for k, v in tc.items() if k in fields})
    eng = TrainingEngine(cfg, ModelConfig.from_dict(mc))
    try:
        return eng.train()["history"]
    finally:
        eng.shutdown()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _replay_distributed(tc: Dict[str, Any], world: int, scratch: Path) -> List[Dict[str, Any]]:
    cfg_path = scratch / "replay_config.json"
    cfg_path.write_text(json.dumps(tc))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           "-m", "llmctl.runtime.worker", "--config", str(cfg_path), "--model-name-or-path",
           str(tc["model_name_or_path"]), "--dataset-path", str(tc["dataset_path"]), "--output-dir",
           str(tc["output_dir"])]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"replay workers failed ({r.returncode}): {r.stderr[-2000:]}")
    return load_manifest(tc["output_dir"])["history"]


def replay_run(run: str, steps: int = 0, tolerance: float = 1e-3) -> Dict[str, Any]:
    man = load_manifest(run)
    rec = man.get("history", [])
    tc = dict(man["training_config"])
    if man.get("perf_knobs"):
        tc["perf_knobs"] = dict(man["perf_knobs"])  # the knobs the recorded run resolved to
    if steps > 0:
        tc["max_steps"] = steps
    elif man.get("global_step"):
        tc["max_steps"] = int(man["global_step"])
    scratch = Path(tempfile.mkdtemp(prefix="llmctl-replay-"))
    tc.update(output_dir=str(scratch / "out"), deterministic=True, save_steps=0, eval_steps=0,
              resume_from_checkpoint=None)
    world = int(man["world"]["world_size"])
    got = _replay_inprocess(tc, man["model_config"]) if world == 1 else _replay_distributed(tc, world, scratch)
    by_step = {int(r["step"]): r for r in got}
    diffs = []
    for r in rec:
        s = int(r["step"])
        if s > tc["max_steps"] or s not in by_step:
            continue
        d = abs(float(by_step[s]["loss"]) - float(r["loss"]))
        diffs.append({"step": s, "recorded": r["loss"], "replayed": by_step[s]["loss"], "abs_diff": d})
    first_div = next((d["step"] for d in diffs if d["abs_diff"] > tolerance), None)
    return {"run": str(run), "git_rev_recorded": man.get("git_rev"), "git_rev_now": _git_rev(),
            "world_size": world, "steps_compared": len(diffs), "max_abs_diff": max((d["abs_diff"] for d in diffs),
                                                                                    default=None),
            "first_divergence": first_div, "match": bool(diffs) and first_div is None, "diffs": diffs}
