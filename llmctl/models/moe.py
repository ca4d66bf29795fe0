"""Mixture-of-experts MLP with expert parallelism (Mixtral-style top-k SwiGLU experts).

Not in the reference (SURVEY §2.3 "EP (expert parallel / MoE)": absent, all reference
templates are dense); added as a model family (``mixtral-8x7b``, ``tiny-moe``) with the EP
dimension the MI355X plan carries.

Per layer, on token-major activations ``x [T, h]``:

1. router: ``softmax(x W_r^T)`` in fp32, top-k experts per token, weights renormalised over
   the k picks; Switch/GShard load-balancing loss ``E * sum_e f_e * P_e`` (``f_e`` share of
   routed slots, ``P_e`` mean router probability) is kept on the module for the model loss;
2. dispatch: token copies are sorted by expert (one stable argsort) into contiguous
   per-expert segments;
3. expert parallel (``ep > 1``): experts are sharded rank-major over the EP group (rank j owns
   experts ``[j*E/ep, (j+1)*E/ep)``); per-expert counts go through one small all-to-all, then
   the token rows through a variable-split ``all_to_all_single`` (RCCL over the xGMI mesh: on
   a K8 node every pair of GPUs has its own link, so the all-to-all uses all 7 links at once);
   received rows are regrouped by local expert.  The only host sync per layer is the split
   sizes (dropless routing: no capacity factor, no dropped tokens);
4. experts: per local expert ``down(swiglu(up(x_e)))`` on its contiguous segment (hipBLASLt
   GEMMs + the SwiGLU HIP kernel on GPU);
5. the reverse all-to-all and a weighted ``index_add`` back to token order.

Gradients flow through the same path (the all-to-all's backward is the reverse all-to-all).
Expert parameters carry ``p.expert = True``: the engine reduces their gradients over the
expert-DP group instead of the full DP group (``llmctl.parallel.groups``).
"""

from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from llmctl import ops
from llmctl.exec.linear import linear


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, send_splits: List[int], recv_splits: List[int], group):
        ctx.group, ctx.send, ctx.recv = group, send_splits, recv_splits
        out = x.new_empty((sum(recv_splits),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), recv_splits, send_splits, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        out = g.new_empty((sum(ctx.send),) + tuple(g.shape[1:]))
        dist.all_to_all_single(out, g.contiguous(), ctx.send, ctx.recv, group=ctx.group)
        return out, None, None, None


class MoEMLP(nn.Module):
    def __init__(self, cfg, num_layers: int, ep_group=None, ep_size: int = 1, ep_rank: int = 0, device=None,
                 dtype=None):
        super().__init__()
        E, k = cfg.num_experts, cfg.experts_per_token
        if E % ep_size:
            raise ValueError(f"num_experts={E} not divisible by expert_parallel={ep_size}")
        self.E, self.k, self.ep, self.ep_group = E, k, ep_size, ep_group
        self.El = E // ep_size
        self.e0 = ep_rank * self.El  # global index of this rank's first expert
        h, f = cfg.hidden, cfg.moe_ffn
        kw = dict(device=device, dtype=dtype)
        self.w_router = nn.Parameter(torch.empty(E, h, **kw))
        self.experts_up = nn.ParameterList([nn.Parameter(torch.empty(2 * f, h, **kw)) for _ in range(self.El)])
        self.experts_down = nn.ParameterList([nn.Parameter(torch.empty(h, f, **kw)) for _ in range(self.El)])
        with torch.no_grad():
            self.w_router.normal_(0.0, 0.02)
            # every rank draws all E experts in order and keeps its own: the initial weights do
            # not depend on the EP layout (equivalence tests, resharding)
            for e in range(E):
                up = torch.empty(2 * f, h, **kw).normal_(0.0, 0.02)
                down = torch.empty(h, f, **kw).normal_(0.0, 0.02 / math.sqrt(2 * num_layers))
                if self.e0 <= e < self.e0 + self.El:
                    self.experts_up[e - self.e0].copy_(up)
                    self.experts_down[e - self.e0].copy_(down)
        for p in list(self.experts_up) + list(self.experts_down):
            p.expert = True
        self.aux_loss: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ names (global expert ids)
    def global_expert_index(self, local: int) -> int:
        return self.e0 + local

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        T, h = x.shape
        E, k = self.E, self.k
        probs = linear(x, self.w_router).float().softmax(-1)  # [T, E]
        topw, topi = probs.topk(k, dim=-1)
        topw = topw / topw.sum(-1, keepdim=True)
        flat = topi.reshape(-1)  # [T*k] expert of each token copy
        counts = torch.bincount(flat, minlength=E)
        self.aux_loss = E * (counts.float() / float(T * k) * probs.mean(0)).sum()
        order = torch.argsort(flat, stable=True)
        tok = torch.div(order, k, rounding_mode="floor")
        xs = x.index_select(0, tok)  # token copies grouped by expert
        if self.ep > 1:
            g = self.ep_group
            cnt_recv = torch.empty_like(counts)
            dist.all_to_all_single(cnt_recv, counts, group=g)  # [src rank, local expert]
            host = torch.cat([counts, cnt_recv]).tolist()  # the layer's one host sync
            c_send = [sum(host[r * self.El:(r + 1) * self.El]) for r in range(self.ep)]
            c_recv2 = [host[E + r * self.El:E + (r + 1) * self.El] for r in range(self.ep)]
            c_recv = [sum(c) for c in c_recv2]
            xr = _AllToAll.apply(xs, c_send, c_recv, g)  # src-major, expert-minor
            # regroup the received rows by local expert (expert-major, src-minor)
            starts, o = [], 0
            for r in range(self.ep):
                row = []
                for e in range(self.El):
                    row.append(o)
                    o += c_recv2[r][e]
                starts.append(row)
            perm = [i for e in range(self.El) for r in range(self.ep)
                    for i in range(starts[r][e], starts[r][e] + c_recv2[r][e])]
            perm_t = torch.tensor(perm, dtype=torch.long, device=x.device)
            xe = xr.index_select(0, perm_t)
            local_counts = [sum(c_recv2[r][e] for r in range(self.ep)) for e in range(self.El)]
        else:
            xe = xs
            local_counts = counts.tolist()
        pad = self._pad_rows(xe, local_counts)
        if pad is not None:
            # every expert's rows padded with zero rows to a multiple of 256: all expert GEMMs -- the
            # token-deep weight gradients included -- then take gemm64's shapes (hipBLASLt's
            # weight-gradient layout runs ~1.0 PF); zero rows contribute zero outputs and gradients
            dst, padded = pad
            xp = xe.new_zeros((sum(padded), h)).index_copy(0, dst, xe)
            outs, o = [], 0
            for e, n in enumerate(padded):
                if n:
                    outs.append(linear(ops.swiglu(linear(xp[o:o + n], self.experts_up[e])), self.experts_down[e]))
                    o += n
            ye = torch.cat(outs, 0).index_select(0, dst) if outs else xe.new_zeros((0, h))
        else:
            outs = []
            o = 0
            for e, n in enumerate(local_counts):
                if n == 0:
                    continue
                seg = xe[o:o + n]
                o += n
                outs.append(linear(ops.swiglu(linear(seg, self.experts_up[e])), self.experts_down[e]))
            ye = torch.cat(outs, 0) if outs else xe.new_zeros((0, h))
        if self.ep > 1:
            inv = torch.empty_like(perm_t)
            inv[perm_t] = torch.arange(perm_t.numel(), device=x.device)
            ys = _AllToAll.apply(ye.index_select(0, inv), c_recv, c_send, self.ep_group)
        else:
            ys = ye
        w = topw.reshape(-1).index_select(0, order).to(ys.dtype).unsqueeze(-1)
        return torch.zeros_like(x).index_add(0, tok, ys * w)


    def _pad_rows(self, xe: torch.Tensor, counts: List[int]):
        """(destination row of every expert row in the padded buffer, padded count per expert), or
        None: GPU only (gemm64 shapes), knob ``moe_pad``."""
        from llmctl.config.knobs import knobs

        if not (knobs().moe_pad and xe.is_cuda and xe.dtype == torch.bfloat16 and xe.shape[1] % 128 == 0
                and self.experts_up[0].shape[0] % 256 == 0 and self.experts_down[0].shape[0] % 256 == 0
                and self.experts_down[0].shape[1] % 128 == 0):
            return None
        padded = [(n + 255) // 256 * 256 for n in counts]
        idx, o = [], 0
        for n, npad in zip(counts, padded):
            idx.append(torch.arange(o, o + n))
            o += npad
        dst = torch.cat(idx).to(xe.device, non_blocking=True) if idx else torch.zeros(0, dtype=torch.long,
                                                                                       device=xe.device)
        return dst, padded


def expert_param_global_name(name: str, module_e0: int) -> str:
    """``...experts_up.<local>`` -> ``...experts_up.<global>`` (and the inverse with -e0)."""
    parts = name.split(".")
    for i, p in enumerate(parts[:-1]):
        if p in ("experts_up", "experts_down"):
            parts[i + 1] = str(int(parts[i + 1]) + module_e0)
            return ".".join(parts)
    return name
