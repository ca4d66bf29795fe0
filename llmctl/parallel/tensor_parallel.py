"""Tensor / sequence parallelism primitives (Megatron-style), built on torch.distributed.

The reference only *declares* TP/SP (config keys ``tensor_parallel``/``sequence_parallel``,
``init.py:134-136``; planner degrees ``plan.py:136``) — nothing executes.
Here they run for real:

* column-parallel linear: weight rows split over the TP group, input replicated;
* row-parallel linear: weight columns split, partial outputs summed (all-reduce, or
  reduce-scatter along tokens when sequence parallelism is on);
* sequence parallelism: the token dimension of the residual stream is sharded across the TP
  group between the attention/MLP blocks; all-gather before the column-parallel GEMMs and
  reduce-scatter after the row-parallel GEMMs replace the TP all-reduce (same bytes on the
  wire, but the norms/residual adds work on 1/tp of the tokens);
* vocab-parallel embedding and vocab-parallel cross-entropy.

On MI355X the TP group should stay inside one node's xGMI mesh (7 links/GPU): the planner
(``llmctl.partition``) never places a TP group across nodes.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def _ws(group) -> int:
    return 1 if group is None else dist.get_world_size(group)


def _rank(group) -> int:
    return 0 if group is None else dist.get_rank(group)


# ----------------------------------------------------------------------------- raw collectives
def _all_reduce(x: torch.Tensor, group) -> torch.Tensor:
    if _ws(group) == 1:
        return x
    x = x.contiguous()
    dist.all_reduce(x, group=group)
    return x


def _all_gather_tokens(x: torch.Tensor, group) -> torch.Tensor:
    """[T/tp, ...] -> [T, ...] (concatenated along dim 0 in rank order)."""
    ws = _ws(group)
    if ws == 1:
        return x
    x = x.contiguous()
    out = torch.empty((x.shape[0] * ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


def _reduce_scatter_tokens(x: torch.Tensor, group) -> torch.Tensor:
    """[T, ...] (partial sums) -> [T/tp, ...] (summed shard)."""
    ws = _ws(group)
    if ws == 1:
        return x
    x = x.contiguous()
    if x.shape[0] % ws:
        raise ValueError(f"token dim {x.shape[0]} not divisible by tp={ws}")
    out = torch.empty((x.shape[0] // ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=group)
    return out


def _split_tokens(x: torch.Tensor, group) -> torch.Tensor:
    ws = _ws(group)
    if ws == 1:
        return x
    n = x.shape[0] // ws
    return x[_rank(group) * n:(_rank(group) + 1) * n].contiguous()


# ----------------------------------------------------------------------------- autograd wrappers
class _CopyToTP(torch.autograd.Function):
    """identity fwd, all-reduce bwd (input of a column-parallel linear without SP)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        return _all_reduce(g.clone() if _ws(ctx.group) > 1 else g, ctx.group), None


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce fwd, identity bwd (output of a row-parallel linear without SP)."""

    @staticmethod
    def forward(ctx, x, group):
        return _all_reduce(x, group)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromSP(torch.autograd.Function):
    """all-gather tokens fwd, reduce-scatter bwd (input of column-parallel linear with SP)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _all_gather_tokens(x, group)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter_tokens(g, ctx.group), None


class _ReduceScatterToSP(torch.autograd.Function):
    """reduce-scatter tokens fwd, all-gather bwd (output of row-parallel linear with SP)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_tokens(x, group)

    @staticmethod
    def backward(ctx, g):
        return _all_gather_tokens(g, ctx.group), None


class _ScatterToSP(torch.autograd.Function):
    """split tokens fwd (no comm), all-gather bwd."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_tokens(x, group)

    @staticmethod
    def backward(ctx, g):
        return _all_gather_tokens(g, ctx.group), None


class _GatherFromSPNoReduce(torch.autograd.Function):
    """all-gather tokens fwd, split bwd (for the final norm -> replicated lm_head input)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _all_gather_tokens(x, group)

    @staticmethod
    def backward(ctx, g):
        return _split_tokens(g, ctx.group), None


def copy_to_tp(x, group):
    return x if _ws(group) == 1 else _CopyToTP.apply(x, group)


def reduce_from_tp(x, group):
    return x if _ws(group) == 1 else _ReduceFromTP.apply(x, group)


def gather_from_sp(x, group):
    return x if _ws(group) == 1 else _GatherFromSP.apply(x, group)


def reduce_scatter_to_sp(x, group):
    return x if _ws(group) == 1 else _ReduceScatterToSP.apply(x, group)


def scatter_to_sp(x, group):
    return x if _ws(group) == 1 else _ScatterToSP.apply(x, group)


def gather_from_sp_replicated(x, group):
    return x if _ws(group) == 1 else _GatherFromSPNoReduce.apply(x, group)


# ----------------------------------------------------------------------------- vocab parallel
class _VocabParallelEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, vocab_start, group, sequence_parallel):
        vocab_local = weight.shape[0]
        local = ids - vocab_start
        mask = (local < 0) | (local >= vocab_local)
        local = local.masked_fill(mask, 0)
        out = weight.index_select(0, local.reshape(-1))
        out = out.masked_fill(mask.reshape(-1, 1), 0)
        ctx.save_for_backward(local.reshape(-1), mask.reshape(-1))
        ctx.vshape = weight.shape
        ctx.group, ctx.sp = group, sequence_parallel
        if _ws(group) > 1:
            out = _reduce_scatter_tokens(out, group) if sequence_parallel else _all_reduce(out, group)
        return out

    @staticmethod
    def backward(ctx, g):
        local, mask = ctx.saved_tensors
        if _ws(ctx.group) > 1 and ctx.sp:
            g = _all_gather_tokens(g, ctx.group)
        g = g.masked_fill(mask.reshape(-1, 1), 0)
        dw = torch.zeros(ctx.vshape, dtype=torch.float32, device=g.device)
        dw.index_add_(0, local, g.float())
        return None, dw.to(g.dtype), None, None, None


def vocab_parallel_embedding(ids, weight, vocab_start: int, group, sequence_parallel: bool = False):
    """ids [T] -> [T, h] (or [T/tp, h] under SP).  weight holds rows [vocab_start, +V/tp)."""
    return _VocabParallelEmbed.apply(ids, weight, vocab_start, group, sequence_parallel)


class _VocabParallelCE(torch.autograd.Function):
    """Cross-entropy over vocab-sharded logits [T, V/tp]: distributed logsumexp with three
    tiny all-reduces (max, sum-exp, target-logit), no gather of the [T, V] logits."""

    @staticmethod
    def forward(ctx, logits, labels, vocab_start, group, denom, ignore_index):
        lf = logits.float()
        lmax = lf.max(dim=-1).values
        dist.all_reduce(lmax, op=dist.ReduceOp.MAX, group=group)
        ex = torch.exp(lf - lmax.unsqueeze(-1))
        sumexp = ex.sum(-1)
        V = logits.shape[-1]
        valid = labels != ignore_index
        local = labels - vocab_start
        inside = (local >= 0) & (local < V) & valid
        tgt = torch.where(inside, lf.gather(-1, local.clamp(0, V - 1).unsqueeze(-1)).squeeze(-1),
                          torch.zeros_like(lmax))
        stats = torch.stack([sumexp, tgt])
        dist.all_reduce(stats, group=group)
        sumexp, tgt = stats[0], stats[1]
        lse = torch.log(sumexp) + lmax
        loss = torch.where(valid, lse - tgt, torch.zeros_like(lse))
        ctx.save_for_backward(logits, lse, local, inside, valid)
        ctx.denom = denom
        return loss.sum() / denom

    @staticmethod
    def backward(ctx, g):
        logits, lse, local, inside, valid = ctx.saved_tensors
        p = torch.exp(logits.float() - lse.unsqueeze(-1))
        V = logits.shape[-1]
        onehot = torch.zeros_like(p)
        onehot.scatter_(-1, local.clamp(0, V - 1).unsqueeze(-1), inside.float().unsqueeze(-1))
        scale = (g / ctx.denom) * valid.float()
        return ((p - onehot) * scale.unsqueeze(-1)).to(logits.dtype), None, None, None, None, None


def vocab_parallel_cross_entropy(logits, labels, vocab_start: int, group, denom: float, ignore_index: int = -100):
    return _VocabParallelCE.apply(logits, labels, vocab_start, group, denom, ignore_index)
