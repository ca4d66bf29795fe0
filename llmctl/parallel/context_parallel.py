"""Context parallelism for long sequences: Ulysses all-to-all or ring attention.

Not in the reference (SURVEY §2.3 "A" rows: CP / ring attention / Ulysses).  Each rank of a
CP group holds a contiguous ``S / cp`` chunk of every sequence for the whole layer stack
(embedding, norms, projections, MLP, loss are per-token).  Two ways to run attention over it:

**ring** (``ring_attention``): K/V chunks travel around the CP ring (batched isend/irecv to the
next rank, overlapped with the flash kernel on the chunk in hand); each rank attends its
queries to every visible key chunk and merges the partial outputs by their log-sum-exp
(``ops.attn_merge_``, one HIP pass per partial).  Load balance (round 2): the sequence is cut
into 2*cp pieces and rank r holds pieces r and 2cp-1-r ("zigzag"), so every rank does the
same causal work at every ring step (two piece-pairs); with contiguous chunks rank r did r+1
chunk pairs and rank cp-1 set the pace.  Backward: the K/V ring shift of the next step is
issued before this step's kernels; each rank's bf16 dK/dV contribution to a remote chunk goes
straight back to the chunk's owner (one point-to-point hop, posted asynchronously and waited
for only at the end) and is accumulated there in fp32 — no fp32 dK/dV travelling the ring.
The per-piece backward uses the *global* output and LSE, so every partial gradient is exact.
No head-count constraint; per-rank attention memory is O(S/cp).  Knob ``cp_zigzag`` off
restores contiguous chunks (A/B).

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


def zigzag_enabled() -> bool:
    import os

    from llmctl.config.knobs import knobs

    return knobs().cp_zigzag


def local_positions(B: int, S_local: int, cp_rank: int, device, cp: int = 1, zigzag: bool = False) -> torch.Tensor:
    """Global token positions of this rank's part of the sequence, flattened [B * S_local]
    (int32): one contiguous chunk, or (zigzag) pieces cp_rank and 2cp-1-cp_rank of 2cp."""
    if zigzag:
        c = S_local // 2
        a = torch.arange(cp_rank * c, (cp_rank + 1) * c, device=device, dtype=torch.int32)
        b = torch.arange((2 * cp - 1 - cp_rank) * c, (2 * cp - cp_rank) * c, device=device, dtype=torch.int32)
        pos = torch.cat([a, b])
    else:
        pos = torch.arange(cp_rank * S_local, (cp_rank + 1) * S_local, device=device, dtype=torch.int32)
    return pos.repeat(B)


def split_sequence(t: torch.Tensor, cp: int, cp_rank: int, zigzag: bool = False) -> torch.Tensor:
    """This rank's part of a [B, S, ...] batch tensor: the contiguous chunk cp_rank of cp, or
    (zigzag, load-balanced ring attention) pieces cp_rank and 2cp-1-cp_rank of 2cp."""
    S = t.shape[1]
    if zigzag:
        if S % (2 * cp):
            raise ValueError(f"sequence length {S} not divisible by 2 * context_parallel = {2 * cp} (zigzag)")
        c = S // (2 * cp)
        return torch.cat([t[:, cp_rank * c:(cp_rank + 1) * c], t[:, (2 * cp - 1 - cp_rank) * c:(2 * cp - cp_rank) * c]],
                         dim=1).contiguous()
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


def _pieces(src: int, r: int, zigzag: bool):
    """(query part, key part, causal) products of this rank's queries with rank ``src``'s K/V:
    parts "all" (contiguous chunks) or "a" / "b" (zigzag pieces r | 2cp-1-r and src | 2cp-1-src)."""
    if not zigzag:
        return [("all", "all", True)] if src == r else ([("all", "all", False)] if src < r else [])
    if src == r:
        return [("a", "a", True), ("b", "a", False), ("b", "b", True)]
    if src < r:  # piece src precedes both query pieces; piece 2cp-1-src follows both
        return [("a", "a", False), ("b", "a", False)]
    return [("b", "a", False), ("b", "b", False)]  # src > r: only the late query piece sees it


def _part(x: torch.Tensor, which: str, dim: int = 1) -> torch.Tensor:
    if which == "all":
        return x
    c = x.shape[dim] // 2
    return x.narrow(dim, 0, c) if which == "a" else x.narrow(dim, c, c)


class _RingAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, group, zigzag):
        from llmctl import ops

        cp, r, nxt, prv = _ring_peers(group)
        kc, vc = k.contiguous(), v.contiguous()
        qparts = ("a", "b") if zigzag else ("all",)
        o_acc = {p: torch.zeros(_part(q, p).shape, dtype=torch.float32, device=q.device) for p in qparts}
        lse_acc = {p: torch.full((q.shape[0], q.shape[2], _part(q, p).shape[1]), float("-inf"), dtype=torch.float32,
                                 device=q.device) for p in qparts}
        for j in range(cp):
            src = (r - j) % cp
            wait = _ring_shift([kc, vc], nxt, prv, group) if j < cp - 1 else None
            for qp, kp, causal in _pieces(src, r, zigzag):
                o_j, lse_j = _attn_fwd(_part(q, qp), _part(kc, kp), _part(vc, kp), scale, causal)
                ops.attn_merge_(o_acc[qp], lse_acc[qp], o_j, lse_j)
            if wait is not None:
                kc, vc = wait()
        o = torch.cat([o_acc[p] for p in qparts], dim=1).to(q.dtype)
        lse = torch.cat([lse_acc[p] for p in qparts], dim=2)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale, ctx.group, ctx.zigzag = scale, group, zigzag
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, scale, zigzag = ctx.group, ctx.scale, ctx.zigzag
        cp, r, nxt, prv = _ring_peers(group)
        do = do.contiguous()
        qparts = ("a", "b") if zigzag else ("all",)
        dq = {p: torch.zeros(_part(q, p).shape, dtype=torch.float32, device=q.device) for p in qparts}
        lse_p = {p: _part(lse, p, dim=2).contiguous() for p in qparts}
        dk_home = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
        dv_home = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
        kc, vc = k.contiguous(), v.contiguous()
        pending = []  # (works, [recv dk, recv dv], [kept send buffers])
        for j in range(cp):
            src = (r - j) % cp
            # the next step's K/V are on the wire while this step's kernels run
            kv_wait = _ring_shift([kc, vc], nxt, prv, group) if j < cp - 1 else None
            dk_j = dk_home if j == 0 else torch.zeros(k.shape, dtype=torch.float32, device=k.device)
            dv_j = dv_home if j == 0 else torch.zeros(v.shape, dtype=torch.float32, device=v.device)
            for qp, kp, causal in _pieces(src, r, zigzag):
                dq_p, dk_p, dv_p = _attn_bwd(_part(do, qp), _part(q, qp), _part(kc, kp), _part(vc, kp), _part(o, qp),
                                             lse_p[qp], scale, causal)
                dq[qp] += dq_p.float()
                _part(dk_j, kp).add_(dk_p.float())
                _part(dv_j, kp).add_(dv_p.float())
            if j > 0:  # this rank's contribution to chunk src goes home in bf16; src's owner
                # receives from the rank j hops ahead of it
                send = [dk_j.to(k.dtype), dv_j.to(v.dtype)]
                recv = [torch.empty_like(send[0]), torch.empty_like(send[1])]
                to, frm = dist.get_global_rank(group, src), dist.get_global_rank(group, (r + j) % cp)
                ops_ = [dist.P2POp(dist.isend, t, to, group) for t in send] + \
                       [dist.P2POp(dist.irecv, t, frm, group) for t in recv]
                pending.append((dist.batch_isend_irecv(ops_), recv, send))
            if kv_wait is not None:
                kc, vc = kv_wait()
        for works, recv, _ in pending:  # accumulate the returned contributions in fp32 at home
            for w in works:
                w.wait()
            dk_home += recv[0].float()
            dv_home += recv[1].float()
        dq_all = torch.cat([dq[p] for p in qparts], dim=1)
        return dq_all.to(q.dtype), dk_home.to(k.dtype), dv_home.to(v.dtype), None, None, None


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group,
                   softmax_scale: float = None, zigzag: bool = False) -> torch.Tensor:
    """Causal attention of this rank's queries over the whole sequence, spread over the CP
    ``group`` as contiguous chunks (rank i holds tokens [i*S/cp, (i+1)*S/cp)) or, with
    ``zigzag``, as pieces i and 2cp-1-i of 2cp (see ``split_sequence``).  q ``[B,S/cp,Hq,D]``,
    k/v ``[B,S/cp,Hkv,D]`` -> o ``[B,S/cp,Hq,D]``."""
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    return _RingAttn.apply(q, k, v, scale, group, zigzag)
