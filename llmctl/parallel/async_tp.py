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
``llmctl/cli/commands/plan.py:110-113``).  Knob ``async_tp`` off restores the plain collectives.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from llmctl.config.knobs import knobs
from llmctl.exec.linear import data_grad, weight_grad


def enabled() -> bool:
    return knobs().async_tp


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


def _ag_matmul(x: torch.Tensor, group, mm, n_out: int, keep_full: bool = True):
    """gather(x) (token chunks in rank order) fed chunk by chunk to ``mm(chunk, out_view)``,
    which writes its product straight into the rows of one preallocated output (no torch.cat
    pass); received chunks land directly in the rows of one preallocated gathered-input buffer
    (returned when ``keep_full``, else None)."""
    ws, r, nxt, prv = _peers(group)
    x = x.contiguous()
    T = x.shape[0]
    y = torch.empty(ws * T, n_out, dtype=x.dtype, device=x.device)
    full = torch.empty(ws * T, *x.shape[1:], dtype=x.dtype, device=x.device) if keep_full or ws > 2 else None
    cur = x
    for s in range(ws):
        c = (r - s) % ws
        pending = None
        if s < ws - 1:  # the next chunk on the wire while this one multiplies
            cp = (c - 1) % ws
            dst = full[cp * T:(cp + 1) * T] if full is not None else torch.empty_like(x)
            pending = (dst, dist.batch_isend_irecv([dist.P2POp(dist.isend, cur, nxt, group),
                                                     dist.P2POp(dist.irecv, dst, prv, group)]))
        mm(cur, y[c * T:(c + 1) * T])
        if pending is not None:
            for w in pending[1]:
                w.wait()
            cur = pending[0]
    if full is not None and keep_full:
        full[r * T:(r + 1) * T].copy_(x)
        return y, full
    return y, None


def _matmul_rs(x_full: torch.Tensor, group, mm) -> torch.Tensor:
    """reduce_scatter over token chunks of mm(x_full), chunk-wise: the partial sum of chunk
    (r - s - 1) % ws is computed at step s, added (in place) to the one received and passed on."""
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
            part.add_(pending[0])
        if s < ws - 1:
            pending = _shift(part, nxt, prv, group)
        else:
            acc = part
    return acc


def _save_full() -> bool:
    """Keep the gathered input of a column-parallel SP linear for its weight gradient (tp x the
    shard's activation memory per QKV / up projection) instead of re-gathering it in backward."""
    return knobs().async_tp_save_full


def _fwd_into(w, b):
    """Chunk GEMM writing into a row slice of the preallocated output: gemm64 straight into the
    slice where forward_linear would pick it, else forward_linear (hipBLASLt) + one copy."""
    from llmctl.exec.linear import forward_linear

    def mm(xc, out):
        if _direct(xc, w, out):
            _gemm_into(xc, w, b, out)
        elif out.is_contiguous():
            torch.mm(xc, w.t(), out=out)
            if b is not None:
                out += b
        else:
            out.copy_(forward_linear(xc, w, b))
    return mm


def _direct(xc, w, out) -> bool:
    from llmctl.exec.linear import fwd64_pick, _gemm64_ok

    M, K = xc.shape
    N = w.shape[0]
    return fwd64_pick(M, N, K) and _gemm64_ok(M, N, K, xc, w, out)


def _gemm_into(xc, w, b, out):
    from llmctl.exec.linear import gemm64_config
    from llmctl.ops._lib import native

    M, K = xc.shape
    native().gemm64_ex(xc, w, out, False, False, False, gemm64_config("fwd", M, w.shape[0], K))
    if b is not None:
        out += b


class _ColumnSP(torch.autograd.Function):
    """y = gather(x_shard) @ W^T (+ b) with the gather overlapped; W column-parallel.  Saves only
    the local token shard: backward re-gathers it (an async all-gather running beside the
    data-gradient ring) for the weight gradient, as Megatron does — keeping the gathered input
    would cost tp x the shard's memory per projection, undoing SP's activation saving."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        keep = _save_full()
        y, x_full = _ag_matmul(x, group, _fwd_into(w, b), w.shape[0], keep_full=keep)
        ctx.save_for_backward(x_full if keep else x.contiguous(), w)
        ctx.wparam, ctx.group, ctx.has_b, ctx.keep = w, group, b is not None, keep
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, w = ctx.saved_tensors
        dy = dy.contiguous()
        gather = None
        if ctx.needs_input_grad[1] and not ctx.keep:
            ws = dist.get_world_size(ctx.group)
            x_full = torch.empty(ws * xs.shape[0], *xs.shape[1:], dtype=xs.dtype, device=xs.device)
            gather = dist.all_gather_into_tensor(x_full, xs, group=ctx.group, async_op=True)
        else:
            x_full = xs
        dx = _matmul_rs(dy, ctx.group, lambda g: data_grad(g, ctx.wparam)) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if gather is not None:
                gather.wait()
            dw = weight_grad(ctx.wparam, dy, x_full)  # through the grad sink when present
        db = dy.sum(0) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None


class _RowSP(torch.autograd.Function):
    """y_shard = reduce_scatter(x_full @ W^T) with the reduce-scatter overlapped; W row-parallel."""

    @staticmethod
    def forward(ctx, x, w, group):
        from llmctl.exec.linear import forward_linear

        ctx.save_for_backward(x, w)
        ctx.wparam, ctx.group = w, group
        return _matmul_rs(x.contiguous(), group, lambda xc: forward_linear(xc, w))

    @staticmethod
    def backward(ctx, dy):
        x_full, w = ctx.saved_tensors

        def dgrad_into(g, out):
            from llmctl.exec.linear import data_grad_into

            data_grad_into(g, ctx.wparam, out)

        dx, dy_full = _ag_matmul(dy.contiguous(), ctx.group, dgrad_into, w.shape[1])
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
