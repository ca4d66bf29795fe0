"""Consumer of the autotuner's ``tuning_cache.json`` (``llmctl tune ... --save-results`` /
``tune full``): turns the measured best configurations back into dispatch decisions.

Keys (written by :class:`llmctl.plugins.autotuning.AutoTuner`):

* ``gemm64_<layout>_<M>x<N>x<K>`` -> ``{"config": c}``: gemm64_ex tile-order group / schedule
  variant for that GEMM (``layout`` dgrad | wgrad | fwd); the most frequent winner per layout
  becomes the layout default, exact shapes keep their own.
* ``comm_<shape>_<dtype>`` -> ``{"bucket_mb": b, ...}``: DP gradient bucket size (training).
* ``fa_split_<B>x<S>x<H>x<D>`` -> ``{"split": 0|1}``: flash-attention forward K/V split.
* ``decode_splits_<N>x<ctx>x<Hkv>`` -> ``{"splits": s}``: paged-decode context splits.
* ``skinny_<M>x<N>x<K>`` -> ``{"config": c}``: decode GEMM (0 = hipBLASLt).

The reference's ``AutoTuner.load_results`` filled an in-memory dict nothing read
(``llmctl/plugins/autotuning.py:64-201``).  Here ``TrainingEngine(tuning_cache=...)`` and
``InferenceEngine(tuning_cache=...)`` (or ``LLMCTL_TUNING_CACHE``) apply the knobs at start-up
and report what they applied.
"""

from __future__ import annotations

import json
import logging
import os
import re
from collections import Counter
from pathlib import Path
from typing import Any, Dict, Optional

log = logging.getLogger("llmctl.tuning_cache")

_SHAPE = re.compile(r"(\d+)x(\d+)x(\d+)")


def resolve(path: Optional[str] = None) -> Optional[Path]:
    p = path or os.environ.get("LLMCTL_TUNING_CACHE")
    if not p:
        return None
    p = Path(p)
    return p if p.exists() else None


def load(path) -> Dict[str, Dict[str, Any]]:
    with open(path) as f:
        data = json.load(f)
    return {k: dict(v.get("best_config") or {}) for k, v in data.items()}


def knobs(cache: Dict[str, Dict[str, Any]]) -> Dict[str, Any]:
    """Group the cache entries by knob."""
    out: Dict[str, Any] = {"gemm64": {}, "gemm64_shapes": {}, "skinny": {}, "bucket_mb": None, "fa_split": None,
                           "decode_splits": None}
    per_layout: Dict[str, Counter] = {}
    scalar: Dict[str, set] = {}
    for k, cfg in cache.items():
        if k.startswith("gemm64_") and "config" in cfg:
            layout = k.split("_")[1]
            m = _SHAPE.search(k)
            if m:
                out["gemm64_shapes"][(layout,) + tuple(int(x) for x in m.groups())] = int(cfg["config"])
            per_layout.setdefault(layout, Counter())[int(cfg["config"])] += 1
        elif k.startswith("skinny_") and "config" in cfg:
            m = _SHAPE.search(k)
            if m:
                out["skinny"][tuple(int(x) for x in m.groups())] = int(cfg["config"])
        elif k.startswith("comm_") and cfg.get("bucket_mb"):
            scalar.setdefault("bucket_mb", set()).add(float(cfg["bucket_mb"]))
        elif k.startswith("fa_split_") and "split" in cfg:
            scalar.setdefault("fa_split", set()).add(int(cfg["split"]))
        elif k.startswith("decode_splits_") and "splits" in cfg:
            scalar.setdefault("decode_splits", set()).add(int(cfg["splits"]))
    out["gemm64"] = {lay: c.most_common(1)[0][0] for lay, c in per_layout.items()}
    # process-wide overrides (bucket size, attention / decode splits) only when every tuned shape
    # agrees: a split tuned for one (N, ctx, Hkv) or (B, S, H, D) must not replace the adaptive
    # per-grid rule for all the others
    for name, vals in scalar.items():
        if len(vals) == 1:
            out[name] = next(iter(vals))
        else:
            log.info("tuning cache: %s differs across shapes %s; keeping the built-in per-shape rule",
                     name, sorted(vals))
    return out


def apply_training(path, config) -> Dict[str, Any]:
    """Apply the training-side knobs (``config`` is the TrainingConfig, edited in place)."""
    k = knobs(load(path))
    applied: Dict[str, Any] = {}
    import importlib

    linear = importlib.import_module("llmctl.exec.linear")  # the package re-exports a function named linear

    for layout, c in k["gemm64"].items():
        linear.GEMM64_CONFIGS[layout] = c
        applied[f"gemm64_{layout}"] = c
    linear.GEMM64_SHAPE_CONFIGS.update(k["gemm64_shapes"])
    if k["bucket_mb"] and config is not None:
        config.bucket_mb = k["bucket_mb"]
        applied["bucket_mb"] = k["bucket_mb"]
    if k["fa_split"] is not None:
        _set_knobs(fa_split=k["fa_split"])
        applied["fa_split"] = k["fa_split"]
    return applied


def _set_knobs(**kw) -> None:
    """Tuned values become the active performance knobs (llmctl.config.knobs; recorded in the
    run manifest like every other knob)."""
    import dataclasses

    from llmctl.config import knobs as K

    # LLMCTL_KNOBS stays highest in precedence: re-applied over the tuned values
    K.apply(K.with_env(dataclasses.replace(K.knobs(), **kw)))


def apply_serving(path) -> Dict[str, Any]:
    k = knobs(load(path))
    applied: Dict[str, Any] = {}
    from llmctl.ops import functional

    functional.SKINNY_CONFIGS.update(k["skinny"])
    if k["skinny"]:
        applied["skinny_shapes"] = len(k["skinny"])
    if k["decode_splits"] is not None:
        _set_knobs(decode_splits=k["decode_splits"])
        applied["decode_splits"] = k["decode_splits"]
    if k["fa_split"] is not None:
        _set_knobs(fa_split=k["fa_split"])
        applied["fa_split"] = k["fa_split"]
    return applied
