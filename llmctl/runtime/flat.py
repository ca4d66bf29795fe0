"""Flat parameter / gradient storage.

All trainable parameters of a (stage of a) model are re-homed into ONE contiguous bf16
buffer and their ``.grad`` into ONE contiguous gradient buffer:

* the optimizer (fused AdamW HIP kernel) runs as one launch per region over flat memory
  instead of a per-tensor multi-tensor-apply loop;
* gradient buckets for the DP overlap engine are plain *views* of the flat grad buffer
  (zero-copy all-reduce / reduce-scatter over RCCL);
* ZeRO-1/2 shards are contiguous slices of each bucket.

Regions (laid out in this order, each bucketed separately):

``decay``       matrices (weight decay on)
``nodecay``     1-D params that are sharded under TP (e.g. column-parallel biases)
``replicated``  params replicated across the TP group (norm weights, row-parallel biases,
                learned position embedding) — no weight decay; under sequence
                parallelism their grads are partial per TP rank and get all-reduced over
                the TP group before the optimizer.

Every bucket is padded to ``align`` elements (a multiple of DP-size × 64) so ZeRO shards
are equal and 128-byte aligned.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

REGIONS = ("decay", "nodecay", "replicated")


def classify(name: str, p: torch.Tensor) -> str:
    if getattr(p, "tp_replicated", False):
        return "replicated"
    if p.dim() < 2:
        return "nodecay"
    return "decay"


@dataclass
class Bucket:
    index: int
    start: int  # element offset into the flat buffer (inclusive)
    end: int  # exclusive; (end - start) % align == 0
    region: str = "decay"
    params: List[nn.Parameter] = field(default_factory=list)

    @property
    def numel(self) -> int:
        return self.end - self.start

    @property
    def decay(self) -> bool:
        return self.region == "decay"


def _fold_main_grad(p: nn.Parameter) -> None:
    """Post-accumulate hook (fp32 main gradients): add the bf16 autograd gradient into the fp32
    flat view and drop it.  Also runs, with ``p.grad`` None, for GEMM-written weights."""
    g = p.grad
    if g is not None:
        p.main_grad.add_(g)
        p.grad = None


def grad_view(p: nn.Parameter) -> Optional[torch.Tensor]:
    """The flat-buffer gradient of ``p``: its fp32 main gradient if it has one, else ``.grad``."""
    g = getattr(p, "main_grad", None)
    return g if g is not None else p.grad


class FlatParameters:
    """Re-home ``named_params`` into flat buffers (in place: ``p.data`` becomes a view)."""

    def __init__(self, named_params: Sequence[Tuple[str, nn.Parameter]], *, bucket_numel: int,
                 align: int = 64, grad_dtype: Optional[torch.dtype] = None, allocate_grad: bool = True,
                 solo: Sequence[str] = ()):
        """``solo``: parameter names that get a bucket of their own (the tied embedding copies
        of a pipeline: equal-sized solo buckets make their ZeRO shards line up across stages)."""
        named_params = [(n, p) for n, p in named_params if p.requires_grad]
        if not named_params:
            raise ValueError("no trainable parameters")
        self.align = align
        dev = named_params[0][1].device
        dtype = named_params[0][1].dtype
        self.dtype, self.device = dtype, dev
        self.grad_dtype = grad_dtype or dtype

        def rup(x):
            return (x + align - 1) // align * align

        self.buckets: List[Bucket] = []
        self.offsets: Dict[int, int] = {}
        self.names: Dict[int, str] = {}
        self.regions: List[Tuple[str, int, int]] = []
        cursor = 0
        for region in REGIONS:
            plist = [(n, p) for n, p in named_params if classify(n, p) == region]
            if not plist:
                continue
            region_start = cursor
            # grads become ready roughly last-layer-first: group in REVERSE model order
            groups: List[List[Tuple[str, nn.Parameter]]] = []
            cur: List[Tuple[str, nn.Parameter]] = []
            cur_n = 0
            for n, p in reversed(plist):
                if n in solo:
                    if cur:
                        groups.append(cur)
                    groups.append([(n, p)])
                    cur, cur_n = [], 0
                    continue
                cur.append((n, p))
                cur_n += p.numel()
                if cur_n >= bucket_numel:
                    groups.append(cur)
                    cur, cur_n = [], 0
            if cur:
                groups.append(cur)
            region_buckets = []
            for g in reversed(groups):  # memory in model order
                b = Bucket(index=-1, start=cursor, end=cursor, region=region)
                for n, p in reversed(g):
                    self.offsets[id(p)] = cursor
                    self.names[id(p)] = n
                    b.params.append(p)
                    cursor += p.numel()
                cursor = rup(cursor)
                b.end = cursor
                region_buckets.append(b)
            # completion order inside a region: highest offsets first
            self.buckets.extend(sorted(region_buckets, key=lambda b: -b.start))
            self.regions.append((region, region_start, cursor))
        self.numel = cursor
        for i, b in enumerate(self.buckets):
            b.index = i
        self.param_bucket: Dict[int, Bucket] = {id(p): b for b in self.buckets for p in b.params}

        self.data = torch.zeros(self.numel, dtype=dtype, device=dev)
        self.grad = torch.zeros(self.numel, dtype=self.grad_dtype, device=dev) if allocate_grad else None
        self.params: List[nn.Parameter] = [p for _, p in named_params]
        # fp32 main gradients (grad_dtype wider than the params): a parameter's ``.grad`` cannot
        # be a view of a buffer of another dtype, so the flat fp32 view is ``p.main_grad``
        # (Megatron's convention).  GEMM-written weights accumulate straight into it in fp32
        # (llmctl.exec.linear.GradSink); autograd-produced grads (norms, embeddings) land in a
        # transient bf16 ``p.grad`` that a post-accumulate hook folds in and drops — registered
        # here, i.e. before the DP overlap engine's hooks, so a bucket launches after the fold.
        self.main_grads = self.grad is not None and self.grad_dtype != dtype
        for n, p in named_params:
            off = self.offsets[id(p)]
            view = self.data[off:off + p.numel()].view_as(p)
            view.copy_(p.data)
            p.data = view
            if self.grad is not None:
                gv = self.grad[off:off + p.numel()].view_as(p)
                if self.main_grads:
                    p.main_grad = gv
                    p.grad = None
                    p.register_post_accumulate_grad_hook(_fold_main_grad)
                else:
                    p.grad = gv

    # ------------------------------------------------------------------ helpers
    def install_sinks(self, sink, predicate) -> int:
        """Attach a :class:`llmctl.exec.linear.GradSink` to every parameter for which
        ``predicate(name, p)`` holds; their gradients are then written (beta=0 first) by
        the backward GEMM, so ``zero_grad`` skips them."""
        n = 0
        for p in self.params:
            if predicate(self.names[id(p)], p):
                sink.attach(p)
                n += 1
        self.sink = sink
        return n

    def zero_grad(self) -> None:
        if self.grad is None:
            return
        sink = getattr(self, "sink", None)
        if sink is None:
            self.grad.zero_()
        for p in self.params:
            off = self.offsets[id(p)]
            if self.main_grads:
                p.grad = None
                g = p.main_grad
            else:
                g = p.grad
                if g is None or g.data_ptr() != self.grad[off:].data_ptr():
                    p.grad = g = self.grad[off:off + p.numel()].view_as(p)
            if sink is not None:
                if getattr(p, "_llmctl_grad_sink", None) is sink:
                    sink.reset(p)
                else:
                    g.zero_()

    def view(self, start: int, end: int, which: str = "grad") -> torch.Tensor:
        buf = self.grad if which == "grad" else self.data
        return buf[start:end]

    def region_range(self, region: str) -> Optional[Tuple[int, int]]:
        for r, s, e in self.regions:
            if r == region:
                return s, e
        return None

    def state_dict_views(self) -> Dict[str, torch.Tensor]:
        return {self.names[id(p)]: p.data for p in self.params}
