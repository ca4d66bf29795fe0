"""Context parallelism for long sequences: Ulysses all-to-all or ring attention.

Not in the reference (SURVEY §2.3 "A" rows: CP / ring attention / Ulysses).  Each rank of a
CP group holds a contiguous ``S / cp`` chunk of every sequence for the whole layer stack
(embedding, norms, projections, MLP, loss are per-token).  Two ways to run attention over it:

**ring** (``ring_attention``): K/V chunks travel around the CP ring (batched isend/irecv to the
next rank, overlapped with the flash kernel on the chunk in hand); each rank attends its
query chunk to every earlier chunk (full) and its own (causal) and merges the partial outputs
by their log-sum-exp.  Backward runs the ring again with the chunk's dK/dV travelling along
and one extra hop returning them to the owner; the per-chunk backward uses the *global*
output and LSE, so every partial gradient is exact.  No head-count constraint; per-rank
attention memory is O(S/cp).  (Contiguous chunks: rank r computes r+1 chunk pairs — a zigzag
split would balance the causal work; the layer stack's per-token ops are balanced either way.)

**ulysses** (``seq_to_head`` / ``head_to_seq``): around attention two all-to-alls
re-shard Q/K/V from *sequence-split, all heads* to *all tokens, heads / cp*:

    [B, S/cp, H, D] --all-to-all--> [B, S, H/cp, D] --flash attention (causal)--> ...
    ... [B, S, H/cp, D] --all-to-all--> [B, S/cp, H, D]

so the attention kernel sees full causal rows.  On one MI355X node the all-to-alls run on
RCCL over the xGMI mesh (each rank exchanges ``(cp-1)/cp`` of its Q/K/V/O tiles — 4×
``B·S·H·D·2/cp`` bytes per layer, independent of sequence length per rank).  RoPE uses the
tokens' global positions.  Gradients are reduced over DP×CP (``ProcessGroups.dpcp_group``).
Requirement (ulysses only): (kv_heads / tp) divisible by cp.
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


# ============================================================================ ring attention
def _ring_peers(group):
    cp = dist.get_world_size(group)
    r = dist.get_rank(group)
    nxt = dist.get_global_rank(group, (r + 1) % cp)
    prv = dist.get_global_rank(group, (r - 1) % cp)
    return cp, r, nxt, prv


def _ring_shift(tensors, nxt: int, prv: int, group):
    """Send ``tensors`` to the next rank, receive the previous rank's; returns (recv, wait)."""
    recv = [torch.empty_like(t) for t in tensors]
    ops = [dist.P2POp(dist.isend, t, nxt, group) for t in tensors] + \
          [dist.P2POp(dist.irecv, t, prv, group) for t in recv]
    reqs = dist.batch_isend_irecv(ops)

    def wait():
        for q in reqs:
            q.wait()
        return recv
    return wait


def _attn_fwd(q, k, v, scale, causal):
    from llmctl.ops import ref
    from llmctl.ops._lib import native, use_native

    if use_native(q):
        return native().flash_attn_fwd(q, k, v, scale, causal, None)
    return ref.attention_fwd(q, k, v, scale, causal)


def _attn_bwd(do, q, k, v, o, lse, scale, causal):
    from llmctl.ops import ref
    from llmctl.ops._lib import native, use_native

    if use_native(q):
        return native().flash_attn_bwd(do, q, k, v, o, lse, scale, causal, None)
    return ref.attention_bwd(do, q, k, v, o, lse, scale, causal)


class _RingAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, group):
        cp, r, nxt, prv = _ring_peers(group)
        kc, vc = k.contiguous(), v.contiguous()
        o_acc = lse_acc = None
        for j in range(cp):
            src = (r - j) % cp
            wait = _ring_shift([kc, vc], nxt, prv, group) if j < cp - 1 else None
            if src <= r:  # chunks after this rank's are entirely in the causal future
                o_j, lse_j = _attn_fwd(q, kc, vc, scale, src == r)
                o_j = o_j.float()
                if o_acc is None:
                    o_acc, lse_acc = o_j, lse_j
                else:
                    lse_new = torch.logaddexp(lse_acc, lse_j)
                    a = torch.exp(lse_acc - lse_new).transpose(1, 2).unsqueeze(-1)  # [B,S,H,1]
                    b = torch.exp(lse_j - lse_new).transpose(1, 2).unsqueeze(-1)
                    o_acc = o_acc * a + o_j * b
                    lse_acc = lse_new
            if wait is not None:
                kc, vc = wait()
        o = o_acc.to(q.dtype)
        ctx.save_for_backward(q, k, v, o, lse_acc)
        ctx.scale, ctx.group = scale, group
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, scale = ctx.group, ctx.scale
        cp, r, nxt, prv = _ring_peers(group)
        do = do.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        kc, vc = k.contiguous(), v.contiguous()
        dkc = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
        dvc = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
        for j in range(cp):
            src = (r - j) % cp
            if src <= r:
                dq_j, dk_j, dv_j = _attn_bwd(do, q, kc, vc, o, lse, scale, src == r)
                dq += dq_j.float()
                dkc += dk_j.float()
                dvc += dv_j.float()
            # every chunk (with its dK/dV) moves one hop; after cp hops dK/dV are home again
            if j < cp - 1:
                kc, vc, dkc, dvc = _ring_shift([kc, vc, dkc, dvc], nxt, prv, group)()
            else:
                dkc, dvc = _ring_shift([dkc, dvc], nxt, prv, group)()
        return dq.to(q.dtype), dkc.to(k.dtype), dvc.to(v.dtype), None, None


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group,
                   softmax_scale: float = None) -> torch.Tensor:
    """Causal attention of this rank's query chunk over the whole sequence, held as contiguous
    chunks across the CP ``group`` (rank i holds tokens [i*S/cp, (i+1)*S/cp)).  q ``[B,S/cp,Hq,D]``,
    k/v ``[B,S/cp,Hkv,D]`` -> o ``[B,S/cp,Hq,D]``."""
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    return _RingAttn.apply(q, k, v, scale, group)
