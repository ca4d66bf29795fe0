"""ZeRO-3 (fully sharded parameters) over RCCL: per-layer all-gather with prefetch, per-layer
gradient reduce-scatter, fp32 master/moments sharded with the parameters.

Reference: ``zero_stage`` is a config/planner number only (``init.py:137``,
``plan.py:82-86,121-123``); DeepSpeed is imported but unused.  ZeRO-1/2 are
implemented by :mod:`llmctl.runtime.optimizer` + :mod:`llmctl.comms.overlap`
(reduce-scatter of flat gradient buckets); this module adds stage 3.

Units: every decoder layer is one unit; the remaining top-level parameters (embedding,
final norm, lm_head) form the *root* unit, gathered for the whole step.  A unit's
parameters are packed ``[decay | no-decay | replicated]`` into one flat bf16 vector padded
to ``dp * 64`` and split evenly: rank r keeps elements ``[r*c, (r+1)*c)``.

Forward: a pre-forward hook all-gathers the unit (and prefetches the next layer on a side
stream), points each parameter's ``.data`` at views of the gathered buffer, and a
post-forward hook releases it.  Backward: a tensor hook on the layer output re-gathers the
unit (prefetching the layer below) before its backward runs; when all of the unit's
gradients are written (sink callbacks / post-accumulate hooks) the full gradient buffer is
reduce-scattered into the rank's gradient shard and freed.  Peak parameter memory is
therefore ~2 layers + root, which is what lets Llama-3-70B (70.6B params, ~1.1 TB of
training state) fit on 8 × 288 GB.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from llmctl.runtime.flat import REGIONS, classify


class _Unit:
    def __init__(self, name: str, named: List[Tuple[str, nn.Parameter]], align: int, dtype, device):
        self.name = name
        order = []
        for region in REGIONS:
            order += [(n, p, region) for n, p in named if classify(n, p) == region]
        self.params: List[Tuple[str, nn.Parameter, str]] = order
        self.shapes = {id(p): p.shape for _, p, _ in order}
        self.numels = {id(p): p.numel() for _, p, _ in order}  # p.data is empty while released
        off = 0
        self.offsets: Dict[int, int] = {}
        self.region_bounds: List[Tuple[str, int, int]] = []
        for region in REGIONS:
            s = off
            for n, p, r in order:
                if r == region:
                    self.offsets[id(p)] = off
                    off += p.numel()
            if off > s:
                self.region_bounds.append((region, s, off))
        self.numel_raw = off
        self.numel = (off + align - 1) // align * align
        self.dtype, self.device = dtype, device
        self.full: Optional[torch.Tensor] = None
        self.full_grad: Optional[torch.Tensor] = None
        self.gather_work = None
        self.shard_start = 0  # offset of this unit's shard inside the rank's shard buffer
        self.pending = 0
        self.grad_done = False


class Zero3Model:
    def __init__(self, model: nn.Module, dp_group, dtype=torch.bfloat16):
        self.model = model
        self.group = dp_group
        self.dp = dist.get_world_size(dp_group)
        self.rank = dist.get_rank(dp_group)
        self.dtype = dtype
        dev = next(model.parameters()).device
        self.device = dev
        align = 64 * self.dp
        layers = list(model.layers)
        self.units: List[_Unit] = []
        layer_param_ids = set()
        for i, layer in enumerate(layers):
            named = [(f"layers.{i}.{n}", p) for n, p in layer.named_parameters()]
            layer_param_ids |= {id(p) for _, p in named}
            self.units.append(_Unit(f"layers.{i}", named, align, dtype, dev))
        root_named = [(n, p) for n, p in model.named_parameters() if id(p) not in layer_param_ids]
        self.root = _Unit("root", root_named, align, dtype, dev) if root_named else None
        all_units = ([self.root] if self.root else []) + self.units
        # ---- shard storage (the optimizer's "flat" view)
        total = sum(u.numel // self.dp for u in all_units)
        self.flat = _ShardFlat(total, dtype, dev)
        off = 0
        for u in all_units:
            u.shard_start = off
            c = u.numel // self.dp
            lo, hi = self.rank * c, (self.rank + 1) * c
            full = torch.zeros(u.numel, dtype=dtype, device=dev)
            for n, p, r in u.params:
                o = u.offsets[id(p)]
                full[o:o + p.numel()].copy_(p.data.reshape(-1))
            self.flat.data[off:off + c].copy_(full[lo:hi])
            # optimizer regions: intersections of this shard with the unit's regions
            for region, s, e in u.region_bounds:
                a, b = max(s, lo), min(e, hi)
                if a < b:
                    self.flat.regions.append((region, off + a - lo, off + b - lo))
            off += c
            for n, p, r in u.params:
                self.flat.names[id(p)] = n
                p.data = torch.empty(0, dtype=dtype, device=dev)
            del full
        self.all_units = all_units
        self.unit_of: Dict[int, _Unit] = {id(p): u for u in all_units for _, p, _ in u.params}
        self._sync_enabled = True
        self._grad_works: List = []
        self._side = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self._install_hooks(layers)

    # ------------------------------------------------------------------ gather / release
    def _shard(self, u: _Unit) -> torch.Tensor:
        c = u.numel // self.dp
        return self.flat.data[u.shard_start:u.shard_start + c]

    def _gather(self, u: _Unit, async_op: bool = False):
        if u.gather_work is not None:  # prefetched: finish it when the caller needs the data
            if not async_op:
                self._wait(u)
            return
        if u.full is not None:
            return
        u.full = torch.empty(u.numel, dtype=self.dtype, device=self.device)
        # the shard is read in place (no staging copy): every gather is waited before the
        # optimizer rewrites the shards (forward / backward use, or finish_grad_sync)
        u.gather_work = dist.all_gather_into_tensor(u.full, self._shard(u), group=self.group, async_op=True)
        if not async_op:
            self._wait(u)

    def _wait(self, u: _Unit):
        if u.gather_work is not None:
            u.gather_work.wait()
            u.gather_work = None
        for n, p, r in u.params:
            o = u.offsets[id(p)]
            p.data = u.full[o:o + u.numels[id(p)]].view(u.shapes[id(p)])

    def _release(self, u: _Unit):
        if u.gather_work is not None:
            u.gather_work.wait()
            u.gather_work = None
        for n, p, r in u.params:
            p.data = torch.empty(0, dtype=self.dtype, device=self.device)
        u.full = None

    # ------------------------------------------------------------------ hooks
    def _install_hooks(self, layers):
        from llmctl.exec.linear import GradSink

        self.sink = GradSink(transpose_dgrad=False)  # params are gathered / freed per layer
        self.flat.sink = None  # zero_grad of the shard buffer is a plain memset
        leafs = ("wqkv", "wo", "w_up", "w_down", "lm_head")
        tied = getattr(self.model.cfg, "tie_word_embeddings", False)
        for u in self.all_units:
            for n, p, r in u.params:
                if n.split(".")[-1] in leafs and not (tied and n.endswith("lm_head")):
                    self.sink.attach(p)
                else:
                    p.register_post_accumulate_grad_hook(self._on_grad)
        self.sink.callbacks.append(self._on_grad)
        n = len(layers)
        for i, layer in enumerate(layers):
            u = self.units[i]
            nxt = self.units[i + 1] if i + 1 < n else None
            prv = self.units[i - 1] if i > 0 else None

            def pre_fwd(mod, args, u=u, nxt=nxt):
                self._gather(u)
                if nxt is not None:
                    self._gather(nxt, async_op=True)

            def post_fwd(mod, args, out, u=u, prv=prv):
                if torch.is_grad_enabled():
                    tensors = [t for t in (out if isinstance(out, tuple) else (out,))
                               if torch.is_tensor(t) and t.requires_grad]
                    state = {"fired": False}

                    def pre_bwd(grad, u=u, prv=prv, state=state):
                        if not state["fired"]:
                            state["fired"] = True
                            self._begin_backward(u)
                            if prv is not None:
                                self._gather(prv, async_op=True)
                        return grad

                    for t in tensors:
                        t.register_hook(pre_bwd)
                self._release(u)
                return out

            layer.register_forward_pre_hook(pre_fwd)
            layer.register_forward_hook(post_fwd)

        def root_pre(mod, args):
            if self.root is not None:
                self._gather(self.root)
                self._begin_backward(self.root)

        self.model.register_forward_pre_hook(root_pre)

    def _begin_backward(self, u: _Unit):
        self._gather(u)
        if u.full_grad is None:
            u.full_grad = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
            for n, p, r in u.params:
                o = u.offsets[id(p)]
                p.grad = u.full_grad[o:o + u.numels[id(p)]].view(u.shapes[id(p)])
                if getattr(p, "_llmctl_grad_sink", None) is not None:
                    self.sink.reset(p)
                    p._llmctl_fresh = False  # buffer is zeroed: accumulate (beta=1)
            u.pending = len(u.params)
            u.grad_done = False

    def _on_grad(self, p):
        u = self.unit_of.get(id(p))
        if u is None or u.full_grad is None:
            return
        u.pending -= 1
        if u.pending == 0 and u is not self.root:
            self._reduce_unit(u)

    # reduce-scatters in flight per rank: enough to cover the next layer's backward, bounded so
    # the unit-sized full-gradient buffers they keep alive stay a few layers' worth
    MAX_INFLIGHT = 2

    def _reduce_unit(self, u: _Unit):
        """Reduce-scatter the unit's full gradient into this rank's shard ASYNCHRONOUSLY: the next
        layer's backward runs while RCCL reduces this one (the collective stream waits for the
        gradient writes; the shard accumulation waits for the collective).  The unit's gathered
        parameters are released right away — only its gradient buffer stays alive until the
        collective has been waited for (``_drain``)."""
        c = u.numel // self.dp
        out = torch.empty(c, dtype=self.dtype, device=self.device)
        work = dist.reduce_scatter_tensor(out, u.full_grad, group=self.group, async_op=True)
        self._grad_works.append((work, out, u.full_grad, u.shard_start, c))
        for n, p, r in u.params:
            p.grad = None
        u.full_grad = None
        u.grad_done = True
        if u is not self.root:
            self._release(u)
        self._drain(self.MAX_INFLIGHT)

    def _drain(self, keep: int = 0):
        """Wait for all but the ``keep`` newest gradient reduce-scatters and add their shards."""
        while len(self._grad_works) > keep:
            work, out, _full, start, c = self._grad_works.pop(0)
            work.wait()
            self.flat.grad[start:start + c].add_(out)

    # ------------------------------------------------------------------ engine API
    def begin_step(self):
        """Gather the root unit (embedding / head) for the whole step."""
        if self.root is not None:
            self._gather(self.root)
            self._begin_backward(self.root)

    def gather_root(self):
        """Pipeline evaluation calls embed / head outside the hooked forward."""
        if self.root is not None:
            self._gather(self.root)

    def release_root(self):
        if self.root is not None and self.root.full is not None:
            self._release(self.root)

    def set_sync(self, enabled: bool):
        self._sync_enabled = enabled

    def no_sync(self):
        import contextlib

        return contextlib.nullcontext()  # ZeRO-3 reduce-scatters every micro-step (DeepSpeed semantics)

    def finish_grad_sync(self):
        for u in self.units:
            if u.full_grad is not None:
                self._reduce_unit(u)
        if self.root is not None and self.root.full_grad is not None:
            self._reduce_unit(self.root)
            self._release(self.root)
        self._drain(0)
        for u in self.all_units:  # no gather may still read a shard the optimizer rewrites
            if u.gather_work is not None:
                u.gather_work.wait()
                u.gather_work = None

    def attach_optimizer(self, opt):
        opt.dp_sharded = True
        self.opt = opt

    def after_step(self):
        pass  # shards were updated in place by the optimizer; next forward re-gathers

    def full_named_parameters(self) -> List[Tuple[str, torch.Tensor]]:
        out = []
        for u in self.all_units:
            self._gather(u)
            for n, p, r in u.params:
                out.append((n, p.data))
        self._held = True
        return out

    def reload_shards_from_full(self):
        with torch.no_grad():
            for u in self.all_units:
                if u.full is None:
                    continue
                c = u.numel // self.dp
                self._shard(u).copy_(u.full[self.rank * c:(self.rank + 1) * c])
                self._release(u)

    def release_all(self):
        for u in self.all_units:
            if u.full is not None:
                self._release(u)


class _ShardFlat:
    """Duck-types the parts of FlatParameters the optimizer/engine use."""

    def __init__(self, n: int, dtype, device):
        self.numel = n
        self.dtype, self.device, self.grad_dtype = dtype, device, dtype
        self.data = torch.zeros(n, dtype=dtype, device=device)
        self.grad = torch.zeros(n, dtype=dtype, device=device)
        self.regions: List[Tuple[str, int, int]] = []
        self.buckets: list = []
        self.names: Dict[int, str] = {}
        self.params: list = []

    def zero_grad(self):
        self.grad.zero_()
