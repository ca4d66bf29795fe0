"""Custom one-shot all-reduce over xGMI peer memory (``llmctl/ops/csrc/custom_ar.hip``).

For the small per-layer tensor-parallel all-reduces of decode (KBs to ~1 MB) RCCL's ring
pays one link latency per step; here every rank maps the other ranks' IPC buffers once
(``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle``, handles exchanged over the process group)
and a single kernel copies, signals and reduces.  Larger messages fall back to RCCL.

The kernel keeps its epoch counter on the device, so the call is hipGraph-capturable (the
TP serving decode step captures it).  A bounded spin turns a dead peer into an error word
(:meth:`CustomAllReduce.check`) instead of a hung GPU.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from llmctl.ops._lib import native


class CustomAllReduce:
    """``max_bytes``: largest message of the one-shot kernel (decode); ``twoshot_bytes``: largest
    message of the two-shot kernel (prefill-sized: reduce-scatter + all-gather through the peer
    buffers, 2 (w-1)/w x n bytes read per rank instead of (w-1) x n), used above
    ``twoshot_min_bytes`` when world > 2.  The data buffer's two epoch-parity halves are sized for
    the larger of the two (input copy + reduced slice)."""

    def __init__(self, group=None, max_bytes: int = 2 << 20, device: Optional[torch.device] = None,
                 twoshot_bytes: int = 0, twoshot_min_bytes: int = 1 << 20):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one node)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = max_bytes
        self.twoshot_bytes = twoshot_bytes if self.world > 2 else 0
        self.twoshot_min_bytes = twoshot_min_bytes
        self.half_bytes = max(max_bytes, self.twoshot_bytes + self.twoshot_bytes // max(self.world, 1))
        ops = native()
        self.ops = ops
        self._data = ops.car_malloc(2 * self.half_bytes)  # two epoch-parity halves
        self._sig = ops.car_malloc(4 * ops.car_sig_words())
        mine = (bytes(ops.car_ipc_handle(self._data).numpy()), bytes(ops.car_ipc_handle(self._sig).numpy()))
        handles: List = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        self._opened: List[int] = []
        data, sig = [], []
        for r, (hd, hs) in enumerate(handles):
            if r == self.rank:
                data.append(self._data)
                sig.append(self._sig)
                continue
            pd = ops.car_ipc_open(torch.frombuffer(bytearray(hd), dtype=torch.uint8))
            ps = ops.car_ipc_open(torch.frombuffer(bytearray(hs), dtype=torch.uint8))
            self._opened += [pd, ps]
            data.append(pd)
            sig.append(ps)
        self.data_ptrs = torch.tensor(data, dtype=torch.int64)
        self.sig_ptrs = torch.tensor(sig, dtype=torch.int64)
        dist.barrier(group=group)

    def eligible(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.max_bytes)

    def twoshot_eligible(self, x: torch.Tensor) -> bool:
        n = x.numel() * 2
        return (self.twoshot_bytes > 0 and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % (8 * self.world) == 0 and self.twoshot_min_bytes <= n <= self.twoshot_bytes)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum of ``x`` over the group (in place unless ``out`` is given); RCCL beyond the
        buffer size or for other dtypes."""
        if self.twoshot_eligible(x) and (not self.eligible(x) or x.numel() * 2 >= self.twoshot_min_bytes):
            out = x if out is None else out
            self.ops.car_allreduce_twoshot(x, out, self.data_ptrs, self.sig_ptrs, self.rank, self.world,
                                           self.half_bytes)
            return out
        if not self.eligible(x):
            dist.all_reduce(x, group=self.group)
            if out is not None:
                out.copy_(x)
                return out
            return x
        out = x if out is None else out
        self.ops.car_allreduce(x, out, self.data_ptrs, self.sig_ptrs, self.rank, self.world, self.half_bytes)
        return out

    def all_reduce_add_rmsnorm(self, part: torch.Tensor, bias: Optional[torch.Tensor], res: torch.Tensor,
                               norm_w: torch.Tensor, eps: float):
        """(rmsnorm(res + sum(part) + bias) * norm_w, res + sum(part) + bias) in one kernel: the TP
        decode layer's row-parallel reduction fused with the next norm (``part`` [M, N] bf16)."""
        return self.ops.car_allreduce_add_rmsnorm(part, bias, res.contiguous(), norm_w, float(eps), self.data_ptrs,
                                                  self.sig_ptrs, self.rank, self.world, self.half_bytes)

    def check(self) -> None:
        if self.ops.car_error(self._sig):
            raise RuntimeError("custom all-reduce: a peer did not signal (timeout)")

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.ops.car_ipc_close(p)
        self._opened = []
        self.ops.car_free(self._data)
        self.ops.car_free(self._sig)
