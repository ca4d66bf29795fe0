"""Error metrics for the kernel-vs-oracle tests.

``row_err`` is the one the kernel tests gate on: the worst row's max abs error relative to
that row's max magnitude.  Tiled kernels fail tile by tile, and a wrong 16x16 or 32-row tile
moves a tensor-wide Frobenius ratio by well under 1 % on realistic shapes, so the norm ratio
(``rel_frob``) is only used for reductions over rows (weight / bias gradients)."""

from __future__ import annotations

import torch


def rel_frob(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float(), b.float()
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


def row_err(got: torch.Tensor, want: torch.Tensor, floor: float = 0.0) -> float:
    """``floor`` > 0 scales rows by at least ``floor`` x the median row magnitude: for outputs
    with rows whose exact value cancels to ~0 (causal dQ of the first query: P = 1 and
    dP - rowsum(dO*O) = 0), where any rounding residue is an infinite relative error."""
    g = got.float().reshape(-1, got.shape[-1])
    w = want.float().reshape(-1, want.shape[-1])
    scale = w.abs().amax(1)
    if floor > 0:
        scale = scale.clamp_min(floor * scale.median().item())
    return ((g - w).abs().amax(1) / scale.clamp_min(1e-6)).max().item()
