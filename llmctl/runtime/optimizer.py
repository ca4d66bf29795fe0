"""Flat-buffer AdamW with ZeRO-1/2 sharding, device-side clipping and LR schedules.

Reference: ``torch.optim.AdamW(betas=(0.9, 0.95), eps=1e-8)`` + linear warmup
(``llmctl/runtime/engine.py:217-256``) over *fp16* params with no master copy
(SURVEY App. C #4).  Here: bf16 params, fp32 master weights, fp32 moments, one fused HIP
kernel launch per flat region (``llmctl.ops.adamw_step_``), gradient clipping whose
coefficient stays on the device (no host sync per step), and optional ZeRO sharding of
the master/moment state across the DP group.

ZeRO layout: each bucket ``b`` of the flat buffer is split into ``dp`` equal chunks; rank
``r`` owns chunk ``r`` of every bucket.  The owned chunks are concatenated into the rank's
fp32 master / m / v shards, so a bucket's reduce-scatter output and all-gather input are
contiguous slices of those shards.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from llmctl import ops
from llmctl.runtime.flat import Bucket, FlatParameters


def forward_order(buckets):
    """Buckets in the order the next forward needs them: the small 1-D regions (norm weights /
    biases of EVERY layer, incl. layer 0's) first, then the matrices in flat order (embedding,
    layer 0, ..., LM head).  Flat-offset order would put the norm buckets last, and layer 0's
    pre-hook would then wait for the whole gather / update."""
    return sorted(buckets, key=lambda b: (b.region == "decay", b.start))


class _StreamEvent:
    """A pending side-stream update: ``wait()`` orders the current stream after it."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class LRSchedule:
    """``constant`` | ``linear`` (reference default, engine.py:246-253) | ``cosine``
    (declared by reference configs but unsupported there).

    ``step`` is the 0-based index of the optimizer step being applied, as in HF's
    ``get_linear_schedule_with_warmup`` (which the reference uses): warmup ramps
    ``step / warmup`` (0 on the very first step when warmup > 0), the first post-warmup step
    runs at the base LR, and the last step of a ``total``-step linear schedule runs at
    ``base / (total - warmup)`` — never 0."""

    def __init__(self, base_lr: float, kind: str = "cosine", warmup_steps: int = 0, total_steps: int = 0,
                 min_lr_ratio: float = 0.1):
        self.base_lr, self.kind = base_lr, kind
        self.warmup, self.total, self.min_ratio = warmup_steps, max(total_steps, 1), min_lr_ratio

    def __call__(self, step: int) -> float:  # step: 0-based index of the step being applied
        if self.warmup and step < self.warmup:
            return self.base_lr * step / self.warmup
        if self.kind == "constant":
            return self.base_lr
        prog = min(max(step - self.warmup, 0) / max(self.total - self.warmup, 1), 1.0)
        if self.kind == "linear":
            return self.base_lr * (1.0 - prog)
        if self.kind == "cosine":
            lo = self.base_lr * self.min_ratio
            return lo + 0.5 * (self.base_lr - lo) * (1 + math.cos(math.pi * prog))
        raise ValueError(f"unknown schedule {self.kind}")

    def state_dict(self):
        return dict(base_lr=self.base_lr, kind=self.kind, warmup=self.warmup, total=self.total,
                    min_ratio=self.min_ratio)


class FlatAdamW:
    def __init__(self, flat: FlatParameters, *, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: float = 1.0, dp_group=None, zero_stage: int = 0,
                 tp_group=None, norm_group=None):
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps, self.weight_decay, self.max_grad_norm = eps, weight_decay, max_grad_norm
        self.dp_group = dp_group
        # convention: a None group is the trivial size-1 group
        self.dp = dist.get_world_size(dp_group) if dp_group is not None else 1
        self.dp_rank = dist.get_rank(dp_group) if dp_group is not None else 0
        self.zero_stage = zero_stage if self.dp > 1 else 0
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.tp_rank = dist.get_rank(tp_group) if self.tp > 1 else 0
        self.norm_group = norm_group  # extra group (e.g. pipeline) for the global norm
        self.dp_sharded = False  # set by ZeRO-3: every rank holds a disjoint parameter shard
        self.step_count = 0
        dev = flat.device
        self.skipped_steps = torch.zeros((), dtype=torch.int32, device=dev)  # non-finite-norm steps (device)
        if self.zero_stage == 0:
            self.master = flat.data.float().clone()
            self.exp_avg = torch.zeros_like(self.master)
            self.exp_avg_sq = torch.zeros_like(self.master)
            self.grad_shard = None
            self.shard_offsets = None
        else:
            n = flat.numel // self.dp
            self.shard_offsets: Dict[int, Tuple[int, int]] = {}
            off = 0
            chunks = []
            for b in sorted(flat.buckets, key=lambda b: b.start):
                c = b.numel // self.dp
                self.shard_offsets[b.index] = (off, c)
                s = b.start + self.dp_rank * c
                chunks.append(flat.data[s:s + c])
                off += c
            assert off == n
            self.master = torch.cat(chunks).float()
            self.exp_avg = torch.zeros_like(self.master)
            self.exp_avg_sq = torch.zeros_like(self.master)
            self.grad_shard = torch.zeros(n, dtype=flat.grad_dtype, device=dev)
        self._norm_buf = torch.zeros(1, dtype=torch.float32, device=dev)
        self.norm_exclude: List = []  # callables -> (this rank's part of) a grad the clip norm skips
        self._pending = {}  # bucket index -> (all-gather work, input buffer)
        self.overlap_param_gather = False  # engines with forward pre-hooks turn this on
        self.overlap_update = False  # ZeRO-0: per-bucket update on a side stream, waited per layer
        self._update_stream = None
        self.last_grad_norm: Optional[torch.Tensor] = None
        self.last_coef: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ ZeRO helpers
    def shard_view(self, b: Bucket) -> torch.Tensor:
        off, c = self.shard_offsets[b.index]
        return self.grad_shard[off:off + c]

    def _segments(self):
        """(param-view, master, grad, m, v, decay, region) tuples the kernel runs over."""
        f = self.flat
        if self.zero_stage == 0:
            for region, s, e in f.regions:
                yield (f.data[s:e], self.master[s:e], f.grad[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e],
                       region == "decay", region)
        else:
            # param shard chunks are non-contiguous in flat.data: update the fp32 master in
            # one launch per region run, then all-gather bf16 chunks bucket by bucket.
            for b in sorted(f.buckets, key=lambda b: b.start):
                off, c = self.shard_offsets[b.index]
                s = b.start + self.dp_rank * c
                yield (f.data[s:s + c], self.master[off:off + c], self.grad_shard[off:off + c],
                       self.exp_avg[off:off + c], self.exp_avg_sq[off:off + c], b.decay, b.region)

    # ------------------------------------------------------------------ norm / clip
    def grad_norm_sq(self) -> torch.Tensor:
        buf = self._norm_buf
        buf.zero_()
        for pv, ms, g, m, v, decay, region in self._segments():
            if region == "replicated" and self.tp > 1 and self.tp_rank != 0:
                continue  # counted once per TP group
            ops.l2norm_sq(g, buf)
        for get in self.norm_exclude:  # a second copy of a tied matrix counts once
            g = get()
            if g is not None:
                buf.sub_(g.float().square().sum())
        if self.zero_stage > 0 or self.dp_sharded:
            dist.all_reduce(buf, group=self.dp_group)
        if self.tp > 1:
            dist.all_reduce(buf, group=self.tp_group)
        if self.norm_group is not None:
            dist.all_reduce(buf, group=self.norm_group)
        return buf

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, lr: Optional[float] = None, grad_divisor: float = 1.0,
             extra_norm_sq: Optional[torch.Tensor] = None, coef: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One update.  ``grad_divisor`` = DP world size × accumulation micro-steps when the
        gradients are still sums; returns the (pre-clip, averaged) global grad norm as a
        device tensor.  ``extra_norm_sq``: squared norm of parameters stepped by another
        optimizer (MoE expert shards) that belongs in the same clip norm; ``coef``: apply a
        scale computed by that other optimizer instead of computing one."""
        self.step_count += 1
        self.wait_params()  # defensive: never update a bucket whose previous gather is in flight
        lr = self.lr if lr is None else lr
        if coef is None:
            nsq = self.grad_norm_sq()
            if extra_norm_sq is not None:
                nsq = nsq + extra_norm_sq
            norm = torch.sqrt(nsq) / grad_divisor
            if self.max_grad_norm and self.max_grad_norm > 0:
                coef = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0) / grad_divisor
            else:
                coef = torch.ones_like(norm) / grad_divisor
            # skip-step policy: a non-finite global norm (identical on every rank) turns the scale
            # into NaN, which the fused kernel treats as "leave everything untouched"
            finite = torch.isfinite(norm)
            coef = torch.where(finite, coef, torch.full_like(coef, float("nan")))
            self.skipped_steps = self.skipped_steps + (~finite).to(torch.int32)
        else:
            norm = self.last_grad_norm if self.last_grad_norm is not None else torch.zeros_like(coef)
        self.last_coef = coef
        if self.zero_stage == 0 and self.overlap_update:
            # bucket by bucket, in forward order, on a side stream: the HBM-bound update of
            # bucket i+1.. runs under the next forward's (MFMA-bound) GEMMs of the layers in
            # bucket i; each layer's forward pre-hook waits only for its own buckets' events
            f = self.flat
            if self._update_stream is None:
                self._update_stream = torch.cuda.Stream(device=f.device)
            side = self._update_stream
            coef.record_stream(side)  # (before the wait: record_stream counts as a main-stream access)
            side.wait_stream(torch.cuda.current_stream(f.device))
            with torch.cuda.stream(side):
                for b in forward_order(f.buckets):
                    s0, s1 = b.start, b.end
                    ops.adamw_step_(f.data[s0:s1], self.master[s0:s1], f.grad[s0:s1], self.exp_avg[s0:s1],
                                    self.exp_avg_sq[s0:s1], lr=lr, beta1=self.beta1, beta2=self.beta2,
                                    eps=self.eps, weight_decay=self.weight_decay if b.decay else 0.0,
                                    step=self.step_count, grad_scale=coef)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    self._pending[b.index] = (_StreamEvent(ev), None)
        elif self.zero_stage == 0:
            for pv, ms, g, m, v, decay, region in self._segments():
                ops.adamw_step_(pv, ms, g, m, v, lr=lr, beta1=self.beta1, beta2=self.beta2, eps=self.eps,
                                weight_decay=self.weight_decay if decay else 0.0, step=self.step_count,
                                grad_scale=coef)
        else:
            # update shard -> all-gather, bucket by bucket in forward (flat-offset) order: the
            # RCCL gather of bucket i runs while AdamW updates bucket i+1, and with
            # ``overlap_param_gather`` the waits move to the next forward (per-module hooks)
            f = self.flat
            for b in forward_order(f.buckets):
                off, c = self.shard_offsets[b.index]
                s = b.start + self.dp_rank * c
                ops.adamw_step_(f.data[s:s + c], self.master[off:off + c], self.grad_shard[off:off + c],
                                self.exp_avg[off:off + c], self.exp_avg_sq[off:off + c], lr=lr, beta1=self.beta1,
                                beta2=self.beta2, eps=self.eps,
                                weight_decay=self.weight_decay if b.decay else 0.0, step=self.step_count,
                                grad_scale=coef)
                self._gather_bucket(b)
            if not self.overlap_param_gather:
                self.wait_params()
        self.last_grad_norm = norm
        return norm

    def _gather_bucket(self, b: Bucket) -> None:
        if self.dp == 1:
            return
        off, c = self.shard_offsets[b.index]
        full = self.flat.data[b.start:b.end]
        mine = full[self.dp_rank * c:(self.dp_rank + 1) * c].clone()  # distinct input buffer
        work = dist.all_gather_into_tensor(full, mine, group=self.dp_group, async_op=True)
        self._pending[b.index] = (work, mine)

    def wait_params(self, bucket_indices=None) -> None:
        """Make the current stream wait for the updated parameters of the given buckets (all
        pending ones by default).  Called by forward pre-hooks and before any host-side use
        of the parameters (eval, checkpointing)."""
        if not self._pending:
            return
        keys = list(self._pending) if bucket_indices is None else [i for i in bucket_indices if i in self._pending]
        for i in keys:
            work, _ = self._pending.pop(i)
            work.wait()

    def _all_gather_params(self) -> None:
        for b in self.flat.buckets:
            self._gather_bucket(b)
        self.wait_params()

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict:
        return {"step": self.step_count, "master": self.master, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "zero_stage": self.zero_stage, "dp": self.dp,
                "dp_rank": self.dp_rank, "hyper": dict(lr=self.lr, betas=(self.beta1, self.beta2), eps=self.eps,
                                                      weight_decay=self.weight_decay)}

    def load_state_dict(self, sd: dict) -> None:
        if sd["master"].numel() != self.master.numel():
            raise ValueError("optimizer shard size mismatch (different plan?) — use reshard on load")
        self.step_count = int(sd["step"])
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
