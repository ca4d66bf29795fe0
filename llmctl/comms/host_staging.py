"""Host-staged gloo collectives for device tensors: multi-rank rehearsal on ONE GPU.

RCCL refuses two ranks on one device, so a TP2 x PP2 x SP2 layout cannot be exercised on a
single-GPU box over ``nccl``.  With ``distributed_backend="gloo"`` and a CUDA device, the
engine calls :func:`install`: every torch.distributed collective / point-to-point op the
framework issues (all_reduce, all_gather[_into_tensor], reduce_scatter_tensor,
all_to_all_single, broadcast, [i]send / [i]recv, batch_isend_irecv) is run by gloo on host
copies of the device tensors, and outputs are copied back on ``wait()`` (or at once for
synchronous calls).  The compute — the HIP GEMM / attention / norm kernels, the pipeline
schedule, the async-TP ring decomposition — runs unchanged on the GPU; only the transport
differs from the RCCL path.  Async semantics are kept (isend/irecv stay non-blocking), so the
deadlock-freedom of the ring and pipeline exchanges is exercised too.

Ops on CPU tensors, or on groups whose backend is not gloo, pass straight through.
"""

from __future__ import annotations

from typing import Callable, List

import torch
import torch.distributed as dist
from torch.distributed import distributed_c10d as c10d

_ORIG: dict = {}


class _Staged:
    """A work handle whose ``wait()`` also copies the host results back to the device."""

    def __init__(self, work, finish: Callable[[], None], keep=()):
        self._work, self._finish, self._keep, self._done = work, finish, keep, False

    def wait(self, timeout=None):
        if not self._done:
            if self._work is not None:
                self._work.wait()
            self._finish()
            self._done = True
            self._keep = ()
        return True

    def is_completed(self):
        return self._done

    def is_success(self):
        return True


def _gloo(group) -> bool:
    try:
        return dist.get_backend(group) == "gloo"
    except Exception:  # noqa: BLE001 - not initialised
        return False


def _dev(*ts) -> bool:
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in ts)


def _host(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu").contiguous()


def _finish_copy(pairs):
    def f():
        for dst, src in pairs:
            dst.copy_(src)
    return f


def _run(work, async_op: bool, finish, keep=()):
    st = _Staged(work, finish, keep)
    if async_op:
        return st
    st.wait()
    return None


def _all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["all_reduce"](tensor, op=op, group=group, async_op=async_op)
    h = _host(tensor)
    w = _ORIG["all_reduce"](h, op=op, group=group, async_op=async_op)
    return _run(w, async_op, _finish_copy([(tensor, h)]))


def _broadcast(tensor, src=None, group=None, async_op=False, **kw):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["broadcast"](tensor, src=src, group=group, async_op=async_op, **kw)
    h = _host(tensor)
    w = _ORIG["broadcast"](h, src=src, group=group, async_op=async_op, **kw)
    return _run(w, async_op, _finish_copy([(tensor, h)]))


def _all_gather_into_tensor(output_tensor, input_tensor, group=None, async_op=False):
    if not (_dev(output_tensor, input_tensor) and _gloo(group)):
        return _ORIG["all_gather_into_tensor"](output_tensor, input_tensor, group=group, async_op=async_op)
    ho = torch.empty(output_tensor.shape, dtype=output_tensor.dtype)
    w = _ORIG["all_gather_into_tensor"](ho, _host(input_tensor), group=group, async_op=async_op)
    return _run(w, async_op, _finish_copy([(output_tensor, ho)]))


def _reduce_scatter_tensor(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
    if not (_dev(output, input) and _gloo(group)):
        return _ORIG["reduce_scatter_tensor"](output, input, op=op, group=group, async_op=async_op)
    ho = torch.empty(output.shape, dtype=output.dtype)
    w = _ORIG["reduce_scatter_tensor"](ho, _host(input), op=op, group=group, async_op=async_op)
    return _run(w, async_op, _finish_copy([(output, ho)]))


def _all_gather(tensor_list, tensor, group=None, async_op=False):
    if not (_dev(tensor, *tensor_list) and _gloo(group)):
        return _ORIG["all_gather"](tensor_list, tensor, group=group, async_op=async_op)
    hl = [torch.empty(t.shape, dtype=t.dtype) for t in tensor_list]
    w = _ORIG["all_gather"](hl, _host(tensor), group=group, async_op=async_op)
    return _run(w, async_op, _finish_copy(list(zip(tensor_list, hl))))


def _all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None,
                       async_op=False):
    if not (_dev(output, input) and _gloo(group)):
        return _ORIG["all_to_all_single"](output, input, output_split_sizes, input_split_sizes, group=group,
                                          async_op=async_op)
    ho = torch.empty(output.shape, dtype=output.dtype)
    w = _ORIG["all_to_all_single"](ho, _host(input), output_split_sizes, input_split_sizes, group=group,
                                   async_op=async_op)
    return _run(w, async_op, _finish_copy([(output, ho)]))


def _isend(tensor, dst=None, group=None, tag=0, **kw):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["isend"](tensor, dst, group, tag, **kw)
    h = _host(tensor)
    return _Staged(_ORIG["isend"](h, dst, group, tag, **kw), lambda: None, keep=(h,))


def _irecv(tensor, src=None, group=None, tag=0, **kw):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["irecv"](tensor, src, group, tag, **kw)
    h = torch.empty(tensor.shape, dtype=tensor.dtype)
    return _Staged(_ORIG["irecv"](h, src, group, tag, **kw), _finish_copy([(tensor, h)]))


def _send(tensor, dst=None, group=None, tag=0, **kw):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["send"](tensor, dst, group, tag, **kw)
    _ORIG["send"](_host(tensor), dst, group, tag, **kw)


def _recv(tensor, src=None, group=None, tag=0, **kw):
    if not (_dev(tensor) and _gloo(group)):
        return _ORIG["recv"](tensor, src, group, tag, **kw)
    h = torch.empty(tensor.shape, dtype=tensor.dtype)
    r = _ORIG["recv"](h, src, group, tag, **kw)
    tensor.copy_(h)
    return r


def _batch_isend_irecv(p2p_op_list) -> List:
    if not any(_dev(op.tensor) and _gloo(op.group) for op in p2p_op_list):
        return _ORIG["batch_isend_irecv"](p2p_op_list)
    works = []
    for op in p2p_op_list:  # gloo p2p is already asynchronous: issue each op on its own
        fn = _isend if op.op in (_isend, _ORIG["isend"]) else _irecv
        if op.peer is not None:  # P2POp may carry both the global and the group rank
            works.append(fn(op.tensor, op.peer, op.group, op.tag))
        else:
            works.append(fn(op.tensor, None, op.group, op.tag, **{"group_dst" if fn is _isend else "group_src":
                                                                   op.group_peer}))
    return works


_PATCHES = {"all_reduce": _all_reduce, "broadcast": _broadcast, "all_gather_into_tensor": _all_gather_into_tensor,
            "reduce_scatter_tensor": _reduce_scatter_tensor, "all_gather": _all_gather,
            "all_to_all_single": _all_to_all_single, "isend": _isend, "irecv": _irecv, "send": _send,
            "recv": _recv, "batch_isend_irecv": _batch_isend_irecv}


def installed() -> bool:
    return bool(_ORIG)


def install() -> None:
    """Route device-tensor collectives on gloo groups through host copies (idempotent).
    Patched on both ``torch.distributed`` and ``distributed_c10d`` so ``P2POp``'s op check
    accepts the staged isend / irecv."""
    if _ORIG:
        return
    for name, fn in _PATCHES.items():
        _ORIG[name] = getattr(c10d, name)
        setattr(c10d, name, fn)
        setattr(dist, name, fn)


def uninstall() -> None:
    for name, fn in _ORIG.items():
        setattr(c10d, name, fn)
        setattr(dist, name, fn)
    _ORIG.clear()


__all__ = ["install", "uninstall", "installed"]
