"""Sequence-parallel linears with the token collective overlapped with the GEMM ("async TP").

Megatron-SP (``tensor_parallel.py``) brackets every TP region with an all-gather of the token
shards before the column-parallel GEMM (QKV, gate/up) and a reduce-scatter after the
row-parallel one (o, down), each a synchronous collective on the critical path.  Here both are
decomposed into ``tp`` ring steps fused with per-chunk GEMMs:

* **AG-GEMM** (column-parallel forward; row-parallel backward):
  ``y = gather(x_shard) @ W^T`` — at step s the rank multiplies the token chunk it holds
  while the next chunk is on the wire (batched isend/irecv to the ring neighbours, RCCL's
  stream running beside the GEMM); the chunks are kept, so the full input is available for
  the weight gradient.
* **GEMM-RS** (row-parallel forward; column-parallel backward):
  ``y_shard = reduce_scatter(x_full @ W^T)`` — at step s the rank computes the partial product
  of the chunk that is one hop further from its owner, adds the partial received from the
  previous rank and passes it on; after ``tp`` steps each rank holds its own chunk's sum.

Bytes on the wire are those of the collectives they replace; each ring step's transfer hides
under a 1/tp-size GEMM.  The reference only modelled this communication (TP term of
``llmctl/cli/commands/plan.py:110-113``).  ``LLMCTL_ASYNC_TP=0`` restores the plain collectives.
"""

from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from llmctl.exec.linear import data_grad, weight_grad


def enabled() -> bool:
    return os.environ.get("LLMCTL_ASYNC_TP", "1") != "0"


def _peers(group):
    ws, r = dist.get_world_size(group), dist.get_rank(group)
    return ws, r, dist.get_global_rank(group, (r + 1) % ws), dist.get_global_rank(group, (r - 1) % ws)


def _shift(send: torch.Tensor, nxt: int, prv: int, group):
    """send -> next rank, receive the previous rank's tensor; returns (recv, works, send) —
    the send buffer is kept referenced until the works are waited for."""
    recv = torch.empty_like(send)
    works = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, nxt, group),
                                    dist.P2POp(dist.irecv, recv, prv, group)])
    return recv, works, send


def _ag_matmul(x: torch.Tensor, group, mm) -> (torch.Tensor, torch.Tensor):
    """gather(x) (token chunks in rank order) fed chunk by chunk to ``mm``; returns
    (cat of mm outputs in rank order, gathered x)."""
    ws, r, nxt, prv = _peers(group)
    chunks: List[Optional[torch.Tensor]] = [None] * ws
    outs: List[Optional[torch.Tensor]] = [None] * ws
    cur = x.contiguous()
    for s in range(ws):
        c = (r - s) % ws
        chunks[c] = cur
        pending = _shift(cur, nxt, prv, group) if s < ws - 1 else None  # next chunk on the wire
        outs[c] = mm(cur)
        if pending is not None:
            for w in pending[1]:
                w.wait()
            cur = pending[0]
    return torch.cat(outs, 0), torch.cat(chunks, 0)


def _matmul_rs(x_full: torch.Tensor, group, mm) -> torch.Tensor:
    """reduce_scatter over token chunks of mm(x_full), chunk-wise: the partial sum of chunk
    (r - s - 1) % ws is computed at step s, added to the one received and passed on."""
    ws, r, nxt, prv = _peers(group)
    if x_full.shape[0] % ws:
        raise ValueError(f"token dim {x_full.shape[0]} not divisible by tp={ws}")
    xs = x_full.chunk(ws, 0)
    acc = None
    pending = None
    for s in range(ws):
        c = (r - s - 1) % ws
        part = mm(xs[c].contiguous())
        if pending is not None:  # the partial of chunk c from the previous rank
            for w in pending[1]:
                w.wait()
            part = part + pending[0]
        if s < ws - 1:
            pending = _shift(part.contiguous(), nxt, prv, group)
        else:
            acc = part
    return acc


class _ColumnSP(torch.autograd.Function):
    """y = gather(x_shard) @ W^T (+ b) with the gather overlapped; W column-parallel."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        y, x_full = _ag_matmul(x, group, lambda xc: F.linear(xc, w, b))
        ctx.save_for_backward(x_full, w)
        ctx.wparam, ctx.group, ctx.has_b = w, group, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x_full, w = ctx.saved_tensors
        dy = dy.contiguous()
        dw = None
        if ctx.needs_input_grad[1]:
            dw = weight_grad(ctx.wparam, dy, x_full)  # through the grad sink when present
        dx = _matmul_rs(dy, ctx.group, lambda g: data_grad(g, ctx.wparam)) if ctx.needs_input_grad[0] else None
        db = dy.sum(0) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None


class _RowSP(torch.autograd.Function):
    """y_shard = reduce_scatter(x_full @ W^T) with the reduce-scatter overlapped; W row-parallel."""

    @staticmethod
    def forward(ctx, x, w, group):
        ctx.save_for_backward(x, w)
        ctx.wparam, ctx.group = w, group
        return _matmul_rs(x.contiguous(), group, lambda xc: F.linear(xc, w))

    @staticmethod
    def backward(ctx, dy):
        x_full, w = ctx.saved_tensors
        dx, dy_full = _ag_matmul(dy.contiguous(), ctx.group, lambda g: data_grad(g, ctx.wparam))
        dw = None
        if ctx.needs_input_grad[1]:
            dw = weight_grad(ctx.wparam, dy_full, x_full.reshape(-1, x_full.shape[-1]))
        return (dx if ctx.needs_input_grad[0] else None), dw, None


def column_parallel_sp(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], group) -> torch.Tensor:
    """``linear(gather_from_sp(x), w, b)`` with the token all-gather overlapped."""
    return _ColumnSP.apply(x, w, b, group)


def row_parallel_sp(x: torch.Tensor, w: torch.Tensor, group) -> torch.Tensor:
    """``reduce_scatter_to_sp(linear(x, w))`` with the token reduce-scatter overlapped."""
    return _RowSP.apply(x, w, group)
