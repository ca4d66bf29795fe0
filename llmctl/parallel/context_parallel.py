"""Context parallelism (DeepSpeed-Ulysses style) for long sequences.

Not in the reference (SURVEY §2.3 "A" rows: CP / ring attention / Ulysses).  Each rank of a
CP group holds a contiguous ``S / cp`` chunk of every sequence for the whole layer stack
(embedding, norms, projections, MLP, loss are per-token); around attention two all-to-alls
re-shard Q/K/V from *sequence-split, all heads* to *all tokens, heads / cp*:

    [B, S/cp, H, D] --all-to-all--> [B, S, H/cp, D] --flash attention (causal)--> ...
    ... [B, S, H/cp, D] --all-to-all--> [B, S/cp, H, D]

so the attention kernel sees full causal rows.  On one MI355X node the all-to-alls run on
RCCL over the xGMI mesh (each rank exchanges ``(cp-1)/cp`` of its Q/K/V/O tiles — 4×
``B·S·H·D·2/cp`` bytes per layer, independent of sequence length per rank).  RoPE uses the
tokens' global positions.  Gradients are reduced over DP×CP (``ProcessGroups.dpcp_group``).
Requirement: (kv_heads / tp) divisible by cp.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def _a2a(x: torch.Tensor, group, scatter_dim: int, gather_dim: int) -> torch.Tensor:
    cp = dist.get_world_size(group)
    send = torch.stack(list(x.chunk(cp, dim=scatter_dim)), 0).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return torch.cat(list(recv.unbind(0)), dim=gather_dim)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _a2a(x, group, scatter_dim=2, gather_dim=1)

    @staticmethod
    def backward(ctx, g):
        return _a2a(g.contiguous(), ctx.group, scatter_dim=1, gather_dim=2), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _a2a(x, group, scatter_dim=1, gather_dim=2)

    @staticmethod
    def backward(ctx, g):
        return _a2a(g.contiguous(), ctx.group, scatter_dim=2, gather_dim=1), None


def seq_to_head(x: torch.Tensor, group) -> torch.Tensor:
    """[B, S/cp, H, D] (sequence chunk) -> [B, S, H/cp, D] (head chunk)."""
    return _SeqToHead.apply(x, group)


def head_to_seq(x: torch.Tensor, group) -> torch.Tensor:
    """[B, S, H/cp, D] -> [B, S/cp, H, D]."""
    return _HeadToSeq.apply(x, group)


def local_positions(B: int, S_local: int, cp_rank: int, device) -> torch.Tensor:
    """Global token positions of this rank's chunk, flattened [B * S_local] (int32)."""
    pos = torch.arange(cp_rank * S_local, (cp_rank + 1) * S_local, device=device, dtype=torch.int32)
    return pos.repeat(B)


def split_sequence(t: torch.Tensor, cp: int, cp_rank: int) -> torch.Tensor:
    """This rank's contiguous chunk of a [B, S, ...] batch tensor."""
    S = t.shape[1]
    if S % cp:
        raise ValueError(f"sequence length {S} not divisible by context_parallel={cp}")
    n = S // cp
    return t[:, cp_rank * n:(cp_rank + 1) * n].contiguous()
