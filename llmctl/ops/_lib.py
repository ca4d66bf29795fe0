"""Loader for the in-tree HIP kernel library ``llmctl/ops/_llmctl_hip.so``.

The library registers its kernels as ``torch.ops.llmctl.*`` (TORCH_LIBRARY, CUDA dispatch
key = HIP on ROCm), so no pybind / Python headers are needed and every op is usable from
autograd Functions and hipGraph capture alike.

Policy (no silent fallback on a GPU box): any op called on a GPU tensor goes to the HIP
kernel; if the library is missing or failed to load, :func:`native` raises.  CPU tensors use
the fp32 oracle in :mod:`llmctl.ops.ref` (that is the gloo/CPU path, not a fallback).
"""

from __future__ import annotations

import os
from pathlib import Path

import torch

LIB_PATH = Path(os.environ.get("LLMCTL_HIP_LIB") or Path(__file__).resolve().parent / "_llmctl_hip.so")  # override: A/B of two builds
_loaded = False
_error: str | None = None


def load(force: bool = False) -> bool:
    global _loaded, _error
    if _loaded and not force:
        return True
    if not LIB_PATH.exists():
        _error = f"{LIB_PATH} not built (run `python -m llmctl.ops.build`)"
        return False
    try:
        torch.ops.load_library(str(LIB_PATH))
        _loaded = True
        _error = None
    except Exception as e:  # pragma: no cover - depends on the box
        _error = f"failed to load {LIB_PATH}: {e}"
    if _loaded:
        from llmctl.config.knobs import push_native

        push_native()  # the launchers' knob table starts from the active PerfKnobs
    return _loaded


def loaded() -> bool:
    """True once the library is loaded (no load attempt)."""
    return _loaded


def available() -> bool:
    return load()


def native():
    """Return the ``torch.ops.llmctl`` namespace, raising loudly if the HIP library is absent."""
    if not load():
        raise RuntimeError(
            "llmctl HIP kernels are required for GPU tensors but are unavailable: " + str(_error)
        )
    return torch.ops.llmctl


def use_native(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    # debugging aid only (kernel tests assert it is unset; one oracle test toggles it at run time)
    return os.environ.get("LLMCTL_FORCE_REF") != "1"
