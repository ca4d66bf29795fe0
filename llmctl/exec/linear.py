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

Data gradient through a transposed weight copy: ``dX = dY W`` (the "NN" GEMM) runs ~13 %
slower on hipBLASLt than the forward's "TN" layout at the GPT-7B shapes
(``profiles/gemm_tunable_dgradT_r1.log``: 7.27 -> 6.37 ms per layer).  Sinked weights therefore
keep a bf16 ``W^T`` copy, refreshed by the transpose HIP kernel the first time the weight is
used after an optimizer step (``GradSink.epoch``; under ZeRO-1/2 that is after the layer's
all-gather has landed), and the backward computes ``dX = F.linear(dY, W^T)``.  Cost: one
bf16 copy of the projection weights and ~2 x 13.5 GB of HBM transpose traffic per step.

Round 2: weight gradients run on the in-house 64-deep MFMA kernel (``gemm64_ex``,
llmctl/ops/csrc/gemm64.hip; 20-40 % over hipBLASLt on the GPT-7B shapes).  Data gradients: the
down projection's runs on gemm64 with the SwiGLU backward in its epilogue; the others run on
hipBLASLt's forward layout through the ``W^T`` copies, which measured 0.7 % faster per step
than gemm64 for all of them (knob ``dgrad64``, see ``dgrad64_shape_ok``).
"""

from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.nn.functional as F

from llmctl.config.knobs import knobs


# gemm64_ex config: knob gemm64_config (see gemm64_config below).  A tuning cache
# (llmctl.plugins.tuning_cache) can override it per layout or per exact shape.
GEMM64_CONFIGS: dict = {}  # layout -> config
GEMM64_SHAPE_CONFIGS: dict = {}  # (layout, M, N, K) -> config


def gemm64_config(layout: str, M: int, N: int, K: int) -> int:
    """Config of one gemm64 call: a tuning-cache entry for the exact shape or the layout, else
    knob ``gemm64_config`` (default 304: the persistent 4-wave kernel; the down projection's
    weight gradient with the SwiGLU backward as a side job runs the one-shot 4-wave kernel --
    3 rounds of bench.py: 1051.9 vs 1053.3 ms/step for 904 on every wgrad,
    profiles/ab_wgrad_persistent_r4.txt)."""
    c = GEMM64_SHAPE_CONFIGS.get((layout, M, N, K), GEMM64_CONFIGS.get(layout))
    if c is not None:
        return c
    return knobs().gemm64_config


def _gemm64_enabled() -> bool:
    return knobs().gemm64  # False: A/B against hipBLASLt


def _rows_ok(*ts: torch.Tensor) -> bool:
    for t in ts:
        if t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
            return False
    return True


def _gemm64_ok(M: int, N: int, K: int, *ts: torch.Tensor) -> bool:
    """Shapes the 64-deep MFMA kernel (llmctl/ops/csrc/gemm64.hip) takes: M, N multiples of
    256, K of 128, bf16 GPU operands with 16-byte aligned unit-stride rows."""
    if not _gemm64_enabled() or M % 256 or N % 256 or K % 128 or K == 0:
        return False
    if not all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts):
        return False
    from llmctl.ops._lib import use_native

    return use_native(ts[0]) and _rows_ok(*ts)


def fwd64_pick(M: int, N: int, K: int) -> bool:
    """Forward ``x W^T`` shapes routed to gemm64: the wide up-projection up to 8192 tokens and the
    QKV / down projections at <= 2048 tokens (serving prefill chunks); hipBLASLt keeps the
    training shapes (24576 tokens) and the rest.  Standalone sweep:
    profiles/gemm64_fwd_small_m_r2.jsonl (up at 2048: 0.278 vs 0.422 ms); in situ, inside a
    GPT-7B 2k prefill, hipBLASLt picks a better up-projection kernel (0.268 ms) and the gain is
    ~1.5 ms per prefill (TTFT p50 28.0 vs 29.5 ms, profiles/ttft_fwd64_r2.txt).
    Knob ``fwd64``: ``off`` disables, ``all`` forces every supported shape (A/B)."""
    mode = knobs().fwd64
    if mode == "off" or not _gemm64_enabled():
        return False
    if mode == "all":
        return True
    return (N >= 16384 and M <= 8192) or (M <= 2048 and (N >= 8192 or K >= 8192))


def forward_linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w^T (+ b)``: gemm64 for the shapes ``fwd64_pick`` selects, hipBLASLt otherwise."""
    N, K = w.shape
    M = x.numel() // K if x.shape[-1] == K else 0
    if M and fwd64_pick(M, N, K) and x.dtype == torch.bfloat16:
        x2 = x.reshape(M, K)
        if _gemm64_ok(M, N, K, x2, w) and 256 * x2.stride(0) * 2 < 2**31 and 256 * w.stride(0) * 2 < 2**31:
            from llmctl.ops._lib import native

            y = torch.empty(M, N, dtype=x.dtype, device=x.device)
            native().gemm64_ex(x2, w, y, False, False, False, gemm64_config("fwd", M, N, K))
            if b is not None:
                y += b
            return y.view(*x.shape[:-1], N)
    return F.linear(x, w, b)


def dgrad64_shape_ok(tokens: int, w: torch.Tensor, fused: bool = False) -> bool:
    """Will ``dx = dy W`` for ``tokens`` rows run on gemm64?  (Decided at forward time: the
    weight's W^T copy is only kept for layers whose data gradient cannot.)  ``fused``: the
    down-projection data gradient with the SwiGLU backward in its epilogue.
    Knob ``dgrad64``: fused (default) = only the SwiGLU-fused down-projection data gradient on
    gemm64, the rest on hipBLASLt's forward layout through the W^T copies; all = every data
    gradient on gemm64 (no W^T copies, ~10 GB less memory for GPT-7B); off = none.  Same-box GPT-7B
    step A/B (profiles/bench_r2_dgrad_modes.txt): fused 832.0 / 833.9 ms, 0 833.9 / 832.7 ms,
    1 837.7 / 839.7 ms."""
    out, inn = w.shape
    mode = knobs().dgrad64
    if mode == "off" or (mode == "fused" and not fused):
        return False
    return _gemm64_ok(tokens, inn, out, w) and out * w.stride(0) * 2 < 2**31


def dgrad64_ok(dy2: torch.Tensor, w: torch.Tensor, fused: bool = False) -> bool:
    """``dx = dy W`` on gemm64 (W read K-major through ds_read_b64_tr_b16: no W^T copy)."""
    return (dy2.dim() == 2 and dy2.shape[1] == w.shape[0] and dgrad64_shape_ok(dy2.shape[0], w, fused)
            and dy2.is_cuda and dy2.dtype == torch.bfloat16 and _rows_ok(dy2))


def dgrad64(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    from llmctl.ops._lib import native

    dx = torch.empty(dy2.shape[0], w.shape[1], dtype=dy2.dtype, device=dy2.device)
    cfg = gemm64_config("dgrad", dy2.shape[0], w.shape[1], w.shape[0])
    native().gemm64_ex(dy2, w, dx, False, True, False, cfg)
    return dx


def _gemm_ex_ok(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    """Shapes/layouts the hand-written MFMA wgrad kernel (llmctl/ops/csrc/gemm_bf16.hip) takes:
    M = out and N = in multiples of 256, K = tokens a multiple of 32, bf16, unit inner stride."""
    if not (g.is_cuda and g.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16):
        return False
    from llmctl.ops._lib import use_native

    if not use_native(g) or not knobs().wgrad_kernel:  # off: hipBLASLt (A/B)
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
    """``g (+)= dy2^T @ x2``: the MFMA kernels read both K-major operands through
    ds_read_b64_tr_b16 (gemm64: +20-40 % over hipBLASLt on the GPT-7B shapes,
    profiles/gemm64_variants_r2.jsonl; the 32-deep gemm_ex where K is not a multiple of 128);
    other shapes go to hipBLASLt."""
    M, N, K = dy2.shape[1], x2.shape[1], dy2.shape[0]
    if g.dtype == torch.float32:  # fp32 main gradient: accumulate without a bf16 rounding
        if (_gemm64_ok(M, N, K, dy2, x2) and g.is_cuda and g.stride(1) == 1 and g.stride(0) % 4 == 0
                and g.data_ptr() % 16 == 0 and K * dy2.stride(0) * 2 < 2**31 and K * x2.stride(0) * 2 < 2**31):
            from llmctl.ops._lib import native

            native().gemm64_ex(dy2, x2, g, True, True, accumulate, gemm64_config("wgrad", M, N, K))
        elif accumulate:
            g.add_(dy2.t().matmul(x2))
        else:
            g.copy_(dy2.t().matmul(x2))
        return
    if (_gemm64_ok(M, N, K, g, dy2, x2) and K * dy2.stride(0) * 2 < 2**31 and K * x2.stride(0) * 2 < 2**31):
        from llmctl.ops._lib import native

        native().gemm64_ex(dy2, x2, g, True, True, accumulate, gemm64_config("wgrad", M, N, K))
    elif _gemm_ex_ok(g, dy2, x2):
        from llmctl.ops._lib import native

        native().gemm_ex(dy2, x2, g, True, True, accumulate)
    elif accumulate:
        g.addmm_(dy2.t(), x2)
    else:
        torch.mm(dy2.t(), x2, out=g)


def side_chunks(M: int, N: int, K: int, T: int, F: int) -> int:
    """Chunks of 1024 elements per K-tile that ``gemm64_wgrad_swiglu``'s side job needs to cover
    ``T * F`` elements over the K-tiles of an ``[M, N] x K`` weight gradient (0: unsupported) —
    as ``side_chunks`` in gemm64.hip."""
    ktiles = (M // 256) * (N // 256) * (K // 64)
    E = T * F
    if E * 4 >= 2**31 or F % 2:
        return 0
    for ch in (1, 2):
        if ktiles * 1024 * ch >= E and ktiles * 1024 * ch < 2**32 and F >= 1024 * ch:
            return ch
    return 0


def swiglu_side_mode() -> str:
    """Where the MLP's SwiGLU backward runs (knob ``swiglu_bwd``): ``side`` (default) = as a side
    job of the down projection's weight-gradient GEMM (``gemm64_wgrad_swiglu``), the data
    gradient a plain GEMM; ``epilogue`` = in the data-gradient GEMM's store epilogue
    (``gemm64_swiglu_dgrad``, round 2); ``separate`` = separate elementwise kernel."""
    return knobs().swiglu_bwd


def wgrad_swiglu_ok(w: torch.nn.Parameter, tokens: int, F: int) -> bool:
    """Can ``w``'s (down projection, [H, F]) weight gradient over ``tokens`` rows carry the SwiGLU
    backward as a side job?  Needs the grad sink (the GEMM writes the flat gradient view)."""
    if swiglu_side_mode() != "side" or getattr(w, "_llmctl_grad_sink", None) is None or not w.is_cuda:
        return False
    H = w.shape[0]
    return (_gemm64_enabled() and w.dtype == torch.bfloat16 and H % 256 == 0 and F % 256 == 0
            and tokens % 128 == 0 and tokens > 0 and side_chunks(H, F, tokens, tokens, F) > 0)


def wgrad_swiglu_into(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, accumulate: bool,
                      dact: torch.Tensor, gu: torch.Tensor) -> Optional[torch.Tensor]:
    """``g (+)= dy2^T x2`` with ``dgu = swiglu_bwd(dact, gu)`` computed by the same kernel
    (returned); None when the operands do not fit (the caller falls back)."""
    M, N, K = dy2.shape[1], x2.shape[1], dy2.shape[0]
    if not (_gemm64_ok(M, N, K, dy2, x2) and g.is_cuda and g.dtype in (torch.bfloat16, torch.float32)
            and g.stride(1) == 1 and g.stride(0) % 8 == 0 and g.data_ptr() % 16 == 0
            and K * dy2.stride(0) * 2 < 2**31 and K * x2.stride(0) * 2 < 2**31
            and dact.is_contiguous() and gu.is_contiguous() and dact.shape == (K, N) and gu.shape == (K, 2 * N)
            and dact.dtype == torch.bfloat16 and gu.dtype == torch.bfloat16
            and side_chunks(M, N, K, K, N) > 0):
        return None
    from llmctl.ops._lib import native

    return native().gemm64_wgrad_swiglu(dy2, x2, g, accumulate, dact, gu, gemm64_config("wgrad", M, N, K))


class GradSink:
    def __init__(self, transpose_dgrad: Optional[bool] = None):
        self.callbacks: List[Callable[[torch.nn.Parameter], None]] = []
        if transpose_dgrad is None:
            transpose_dgrad = knobs().dgrad_transpose
        self.transpose_dgrad = transpose_dgrad
        self.epoch = 0  # bumped by the engine after every optimizer step / weight load

    def weight_t(self, w: torch.nn.Parameter) -> Optional[torch.Tensor]:
        """The up-to-date ``W^T`` copy of a 2-D bf16 GPU weight (None if not applicable)."""
        if not (self.transpose_dgrad and w.is_cuda and w.dim() == 2 and w.dtype == torch.bfloat16):
            return None
        from llmctl.ops._lib import native, use_native

        if not use_native(w) or w.shape[0] % 8 or w.shape[1] % 8:
            return None
        wt = getattr(w, "_llmctl_wt", None)
        if wt is None:
            wt = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device)
            w._llmctl_wt = wt
            w._llmctl_wt_epoch = -1
        if w._llmctl_wt_epoch != self.epoch:
            if self._side_stream_ok():
                # the copy is only read by the backward's data-gradient GEMM: transpose on a side
                # stream under the forward's compute-bound GEMMs; wait_weight_t() orders the
                # backward after it (and, through the backward, the next optimizer step)
                cur = torch.cuda.current_stream(w.device)
                side = self._side_stream(w.device)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    native().transpose_(w.detach(), wt)
                ev = torch.cuda.Event()
                ev.record(side)
                w._llmctl_wt_event = ev
            else:
                native().transpose_(w.detach(), wt)
                w._llmctl_wt_event = None
            w._llmctl_wt_epoch = self.epoch
        return wt

    @staticmethod
    def wait_weight_t(w: torch.nn.Parameter) -> None:
        """Order the current stream after the side-stream refresh of ``w``'s W^T copy."""
        ev = getattr(w, "_llmctl_wt_event", None)
        if ev is not None:
            torch.cuda.current_stream(w.device).wait_event(ev)

    _streams: dict = {}

    @staticmethod
    def _side_stream_ok() -> bool:
        return knobs().wt_side_stream and not torch.cuda.is_current_stream_capturing()

    @classmethod
    def _side_stream(cls, device) -> "torch.cuda.Stream":
        s = cls._streams.get(device)
        if s is None:
            s = cls._streams[device] = torch.cuda.Stream(device=device)
        return s

    def attach(self, p: torch.nn.Parameter) -> None:
        p._llmctl_grad_sink = self
        p._llmctl_fresh = True

    def reset(self, p: torch.nn.Parameter) -> None:
        p._llmctl_fresh = True

    @staticmethod
    def _target(p: torch.nn.Parameter) -> torch.Tensor:
        g = getattr(p, "main_grad", None)
        if g is None:
            g = p.grad
        if g is None:
            raise RuntimeError("grad sink parameter has no flat .grad view")
        return g

    def _written(self, p: torch.nn.Parameter) -> None:
        p._llmctl_fresh = False
        for cb in self.callbacks:
            cb(p)

    def write(self, p: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor) -> None:
        wgrad_into(self._target(p), dy2, x2, accumulate=not p._llmctl_fresh)
        self._written(p)

    def write_swiglu(self, p: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor, dact: torch.Tensor,
                     gu: torch.Tensor) -> Optional[torch.Tensor]:
        """``write`` with the SwiGLU backward riding on the weight-gradient GEMM: returns
        ``dgu = swiglu_bwd(dact, gu)``, or None (nothing written) if the kernel cannot take it."""
        dgu = wgrad_swiglu_into(self._target(p), dy2, x2, not p._llmctl_fresh, dact, gu)
        if dgu is not None:
            self._written(p)
        return dgu


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        # keep the Parameter object itself: tensors coming back from saved_tensors can be
        # aliases (e.g. under activation checkpointing) that do not carry the sink
        ctx.wparam = w
        ctx.has_b = b is not None
        sink = getattr(w, "_llmctl_grad_sink", None)
        ctx.wt = None
        if sink is not None and ctx.needs_input_grad[0] and not dgrad64_shape_ok(x.numel() // x.shape[-1], w):
            ctx.wt = sink.weight_t(w)
        return forward_linear(x, w, b)

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
            else:  # an ordinary gradient (AccumulateGrad adds it), still on the MFMA kernels when they fit
                dw = torch.empty_like(w)
                wgrad_into(dw, dy2, x2, accumulate=False)
        dx = None
        if ctx.needs_input_grad[0]:
            # an unsinked weight keeps no W^T copy, so its alternative is hipBLASLt's slower "NN"
            # layout: gemm64 (W read K-major) whenever the shape fits, unless knob dgrad64 is off
            free = getattr(ctx.wparam, "_llmctl_grad_sink", None) is None and knobs().dgrad64 != "off"
            if dgrad64_ok(dy2, w) or (free and dy2.is_cuda and dy2.dtype == torch.bfloat16 and _rows_ok(dy2)
                                      and _gemm64_ok(dy2.shape[0], w.shape[1], w.shape[0], w)
                                      and w.shape[0] * w.stride(0) * 2 < 2**31):
                dx = dgrad64(dy2, w).view(*dy.shape[:-1], w.shape[1])
            elif ctx.wt is not None:
                GradSink.wait_weight_t(ctx.wparam)
                dx = F.linear(dy, ctx.wt)
            else:
                dx = dy.matmul(w)
        db = dy2.sum(0) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x @ w^T (+ b)`` (``forward_linear``: gemm64 or hipBLASLt); weight grads go through the
    parameter's sink if any.  Whenever a gradient is needed the call goes through ``_Linear`` — the
    gemm64 forward is a plain kernel call that autograd cannot see, so an unsinked weight (MoE
    experts, tied heads) taking that route from ``forward_linear`` directly would get no gradient."""
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad
                                              or (b is not None and b.requires_grad))
    if not needs_grad:
        return forward_linear(x, w, b)
    return _Linear.apply(x, w, b)


def data_grad(dy: torch.Tensor, w: torch.nn.Parameter) -> torch.Tensor:
    """``dy @ w`` for hand-written backward passes: gemm64 when the shape fits, else through
    the weight's transposed copy when its sink keeps one."""
    dy2 = dy.reshape(-1, dy.shape[-1])
    if dgrad64_ok(dy2, w):
        return dgrad64(dy2, w).view(*dy.shape[:-1], w.shape[1])
    sink = getattr(w, "_llmctl_grad_sink", None)
    wt = sink.weight_t(w) if sink is not None else None
    if wt is not None:
        GradSink.wait_weight_t(w)
        return F.linear(dy, wt)
    return dy.matmul(w)


def data_grad_into(dy2: torch.Tensor, w: torch.nn.Parameter, out: torch.Tensor) -> None:
    """``out = dy2 @ w`` into a preallocated (row-slice) output: gemm64 writes it directly."""
    if dgrad64_ok(dy2, w) and _rows_ok(out):
        from llmctl.ops._lib import native

        native().gemm64_ex(dy2, w, out, False, True, False, gemm64_config("dgrad", dy2.shape[0], w.shape[1], w.shape[0]))
        return
    out.copy_(data_grad(dy2, w))


def swiglu_data_grad(dy: torch.Tensor, w: torch.nn.Parameter, gu: torch.Tensor) -> torch.Tensor:
    """``swiglu_bwd(dy @ w, gu)`` for the MLP down projection: on gemm64 the SwiGLU backward runs
    in the data-gradient GEMM's epilogue (``gemm64_swiglu_dgrad``: dgate / dup from the fp32 dAct
    tile, no dAct tensor); otherwise the data gradient and the elementwise kernel separately."""
    dy2 = dy.reshape(-1, dy.shape[-1])
    gu2 = gu.reshape(-1, gu.shape[-1])
    if (dgrad64_ok(dy2, w, fused=True) and gu2.is_contiguous() and gu2.data_ptr() % 16 == 0
            and swiglu_side_mode() != "separate"):  # separate: unfused (A/B)
        from llmctl.ops._lib import native

        cfg = gemm64_config("dgrad", dy2.shape[0], w.shape[1], w.shape[0])
        return native().gemm64_swiglu_dgrad(dy2, w, gu2, cfg).view(gu.shape)
    from llmctl.ops._lib import native, use_native
    from llmctl.ops import ref

    dact = data_grad(dy, w)
    return native().swiglu_bwd(dact, gu) if use_native(gu) else ref.swiglu_bwd(dact, gu)


def weight_grad(w: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor) -> Optional[torch.Tensor]:
    """For hand-written backward passes: route ``dy2^T x2`` through ``w``'s sink (returns
    None) or return it as an ordinary gradient."""
    sink = getattr(w, "_llmctl_grad_sink", None)
    if sink is not None:
        sink.write(w, dy2, x2)
        return None
    return dy2.t().matmul(x2)
