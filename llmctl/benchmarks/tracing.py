"""Trace capture / summary (``llmctl trace``).

``capture_trace``: a short training run under ``torch.profiler`` (CPU + ROCm GPU
activities through Kineto/roctracer), exported as Chrome/Perfetto JSON plus a kernel
table; or, with ``rocprof=True``, the same run under ``rocprofv3 --kernel-trace --stats``
(launched as a child process — the profiled program must be the direct child of rocprofv3).
``summarize_trace``: top kernels and per-category time from either output.
"""

from __future__ import annotations

import csv
import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path
from typing import Any, Dict, List

CATEGORIES = [
    ("gemm", ("Cijk", "gemm", "Gemm", "matmul", "hipblaslt")),
    ("attention", ("fa_fwd", "fa_bwd", "flash", "paged_decode", "attention", "delta_kernel")),
    ("norm", ("norm_fwd", "norm_bwd", "col_reduce", "layer_norm", "rms")),
    ("elementwise", ("rope", "swiglu", "gelu", "elementwise", "Functor", "copy")),
    ("loss", ("ce_fwd", "ce_bwd", "cross_entropy")),
    ("optimizer", ("adamw", "sumsq", "l2norm")),
    ("communication", ("nccl", "rccl", "AllReduce", "ReduceScatter", "AllGather", "SendRecv")),
]


def _category(name: str) -> str:
    for cat, keys in CATEGORIES:
        if any(k in name for k in keys):
            return cat
    return "other"


def capture_trace(model: str = "tiny", steps: int = 3, micro_batch: int = 2, seq_len: int = 256,
                  out_dir: Path = Path("./traces"), rocprof: bool = False, run: str = "latest") -> Dict[str, Any]:
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    stamp = time.strftime("%Y%m%d-%H%M%S")
    if rocprof:
        exe = shutil.which("rocprofv3")
        if exe is None:
            return {"error": "rocprofv3 not found"}
        d = out_dir / f"rocprof-{stamp}"
        cmd = [exe, "--kernel-trace", "--stats", "-d", str(d), "-o", "run", "--output-format", "csv", "--",
               sys.executable, str(Path(__file__).resolve().parents[2] / "bench.py"), "--model", model,
               "--micro-batch", str(micro_batch), "--seq-len", str(seq_len), "--steps", str(steps), "--warmup", "1"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        stats = list(d.rglob("*kernel_stats.csv"))
        return {"mode": "rocprofv3", "returncode": r.returncode, "dir": str(d),
                "kernel_stats": str(stats[0]) if stats else None}
    import torch
    from torch.profiler import ProfilerActivity, profile

    from llmctl.io.synthetic import SyntheticTokens
    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    mc = get_model_config(model)
    cfg = TrainingConfig(model_name_or_path=model, batch_size=micro_batch, seq_len=seq_len, log_level="warning",
                         max_steps=steps + 1)
    eng = TrainingEngine(cfg, mc)
    data = SyntheticTokens(mc.vocab_size, seq_len, micro_batch, device=eng.device)
    eng.train_step([data.batch(0)])  # warm-up
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts, record_shapes=False) as prof:
        for i in range(steps):
            eng.train_step([data.batch(i + 1)])
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    trace = out_dir / f"trace-{stamp}.json"
    prof.export_chrome_trace(str(trace))
    (out_dir / "latest").write_text(trace.name)
    table = prof.key_averages().table(sort_by="cuda_time_total" if torch.cuda.is_available() else "cpu_time_total",
                                      row_limit=25)
    (out_dir / f"summary-{stamp}.txt").write_text(table)
    return {"mode": "torch.profiler", "trace": str(trace), "summary": str(out_dir / f"summary-{stamp}.txt"),
            "steps": steps, "model": model}


def summarize_trace(path: Path) -> Dict[str, Any]:
    path = Path(path)
    rows: List[Dict[str, Any]] = []
    if path.suffix == ".csv":
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append({"name": r["Name"], "calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6})
    else:
        data = json.loads(path.read_text())
        events = data["traceEvents"] if isinstance(data, dict) else data
        agg: Dict[str, Dict[str, float]] = {}
        for e in events:
            if e.get("ph") != "X" or e.get("cat") not in ("kernel", "gpu_memcpy", "gpu_memset"):
                continue
            a = agg.setdefault(e["name"], {"calls": 0, "total_ms": 0.0})
            a["calls"] += 1
            a["total_ms"] += float(e.get("dur", 0)) / 1e3
        rows = [{"name": k, "calls": int(v["calls"]), "total_ms": v["total_ms"]} for k, v in agg.items()]
    tot = sum(r["total_ms"] for r in rows) or 1.0
    for r in rows:
        r["pct"] = 100.0 * r["total_ms"] / tot
    rows.sort(key=lambda r: -r["total_ms"])
    cats: Dict[str, float] = {}
    for r in rows:
        c = _category(r["name"])
        cats[c] = cats.get(c, 0.0) + r["total_ms"]
    return {"kernels": rows, "categories": {k: {"ms": round(v, 3), "pct": round(100 * v / tot, 2)}
                                            for k, v in sorted(cats.items(), key=lambda kv: -kv[1])},
            "total_ms": tot}
