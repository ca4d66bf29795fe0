"""Linear layer with gradient *sinks*: weight gradients are written by the backward GEMM
directly into the flat gradient buffer.

With stock autograd, ``dW = dY^T X`` lands in a fresh tensor and AccumulateGrad then adds
it into ``param.grad`` (our flat-buffer view) — an extra read-read-write pass over every
weight gradient (~40 GB/step for GPT-7B, ~7 ms of HBM time on MI355X).  Here the backward
GEMM writes the flat view itself: ``mm(..., out=view)`` on the first micro-step after
``zero_grad`` (beta = 0, so the buffer never needs zeroing) and ``addmm_`` (hipBLASLt
beta = 1 epilogue, free accumulation) on later gradient-accumulation micro-steps.  The sink
then notifies the DP overlap engine that the parameter's gradient is ready — the same
signal ``register_post_accumulate_grad_hook`` gives for ordinary parameters.
"""

from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.nn.functional as F


def _gemm_ex_ok(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    """Shapes/layouts the hand-written MFMA wgrad kernel (llmctl/ops/csrc/gemm_bf16.hip) takes:
    M = out and N = in multiples of 256, K = tokens a multiple of 32, bf16, unit inner stride."""
    if not (g.is_cuda and g.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16):
        return False
    from llmctl.ops._lib import use_native

    if not use_native(g):
        return False
    M, N, K = dy2.shape[1], x2.shape[1], dy2.shape[0]
    if M % 256 or N % 256 or K % 32 or K == 0:
        return False
    for t in (g, dy2, x2):
        if t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
            return False
    # 32-bit buffer offsets inside the kernel
    return dy2.stride(0) * K * 2 < 2**31 and x2.stride(0) * K * 2 < 2**31


def wgrad_into(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, accumulate: bool) -> None:
    """``g (+)= dy2^T @ x2``: the MFMA kernel reads both K-major operands through
    ds_read_b64_tr_b16 (+12-26 % over hipBLASLt on the GPT-7B shapes, profiles/gemm_bench_r1.json);
    other shapes go to hipBLASLt."""
    if _gemm_ex_ok(g, dy2, x2):
        from llmctl.ops._lib import native

        native().gemm_ex(dy2, x2, g, True, True, accumulate)
    elif accumulate:
        g.addmm_(dy2.t(), x2)
    else:
        torch.mm(dy2.t(), x2, out=g)


class GradSink:
    def __init__(self):
        self.callbacks: List[Callable[[torch.nn.Parameter], None]] = []

    def attach(self, p: torch.nn.Parameter) -> None:
        p._llmctl_grad_sink = self
        p._llmctl_fresh = True

    def reset(self, p: torch.nn.Parameter) -> None:
        p._llmctl_fresh = True

    def write(self, p: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor) -> None:
        g = p.grad
        if g is None:
            raise RuntimeError("grad sink parameter has no flat .grad view")
        wgrad_into(g, dy2, x2, accumulate=not p._llmctl_fresh)
        p._llmctl_fresh = False
        for cb in self.callbacks:
            cb(p)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        # keep the Parameter object itself: tensors coming back from saved_tensors can be
        # aliases (e.g. under activation checkpointing) that do not carry the sink
        ctx.wparam = w
        ctx.has_b = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dw = None
        if ctx.needs_input_grad[1]:
            sink: Optional[GradSink] = getattr(ctx.wparam, "_llmctl_grad_sink", None)
            if sink is not None:
                sink.write(ctx.wparam, dy2, x2)  # weight grad first: lets its bucket's comm start earlier
            else:
                dw = dy2.t().matmul(x2)
        dx = dy.matmul(w) if ctx.needs_input_grad[0] else None
        db = dy2.sum(0) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w^T (+ b)`` on hipBLASLt; weight grads go through the parameter's sink if any."""
    if getattr(w, "_llmctl_grad_sink", None) is None or not torch.is_grad_enabled():
        return F.linear(x, w, b)
    return _Linear.apply(x, w, b)


def weight_grad(w: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor) -> Optional[torch.Tensor]:
    """For hand-written backward passes: route ``dy2^T x2`` through ``w``'s sink (returns
    None) or return it as an ordinary gradient."""
    sink = getattr(w, "_llmctl_grad_sink", None)
    if sink is not None:
        sink.write(w, dy2, x2)
        return None
    return dy2.t().matmul(x2)
