"""Decoder-only transformer (Llama-style and GPT-2-style) built on llmctl's fused ops.

Replaces the reference's HF ``AutoModelForCausalLM`` (``llmctl/runtime/engine.py:119-140``):
weights are random-initialised from the model JSON (no Hub access on the GPU box), and
every non-GEMM op is a hand-written HIP kernel (``llmctl.ops``).  GEMMs go to hipBLASLt via
``torch.nn.functional.linear`` on token-major ``[T, features]`` activations; fused weights
(``wqkv``, ``w_gate_up``) keep the GEMM count at 4 per layer.

Parallelism hooks (see ``llmctl.parallel``):
* tensor parallel — ``wqkv``/``w_gate_up`` column-parallel, ``wo``/``w_down`` row-parallel,
  vocab-parallel embedding / lm_head / cross-entropy;
* sequence parallel — residual stream sharded on tokens inside the TP group;
* pipeline parallel — a stage owns ``layers[lo:hi]`` plus optionally embed / head.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from llmctl import ops
from llmctl.config.knobs import knobs
from llmctl.exec.linear import data_grad, dgrad64, linear, swiglu_data_grad, weight_grad
from llmctl.parallel import async_tp
from llmctl.parallel import context_parallel as cp
from llmctl.parallel import tensor_parallel as tp
from .config import ModelConfig
from .moe import MoEMLP


@dataclass
class ParallelContext:
    tp_group: Optional[object] = None
    tp_size: int = 1
    tp_rank: int = 0
    sequence_parallel: bool = False
    # pipeline stage description
    layer_start: int = 0
    layer_end: Optional[int] = None
    has_embedding: bool = True
    has_head: bool = True
    # interleaved pipeline (virtual stages): this rank's model chunks as global [start, end)
    # layer ranges, in chunk order (None: the single range [layer_start, layer_end))
    layer_ranges: Optional[List[Tuple[int, int]]] = None

    @property
    def layer_index(self):
        """Local -> global layer numbering for parameter names: the offset ``layer_start`` for
        one contiguous range, or the list of global ids of the local layers (virtual stages)."""
        if self.layer_ranges is None:
            return self.layer_start
        return [i for a, b in self.layer_ranges for i in range(a, b)]
    # recompute policy: "none" | "selective" | "full"
    activation_checkpoint: str = "none"
    # context parallel (llmctl.parallel.context_parallel): "ulysses" all-to-all around
    # attention, or "ring" attention (K/V chunks rotated over the CP ring)
    cp_group: Optional[object] = None
    cp_size: int = 1
    cp_rank: int = 0
    cp_mode: str = "ulysses"
    cp_zigzag: bool = False  # ring mode: rank r holds pieces r and 2cp-1-r of the sequence
    # expert parallel (MoE models; llmctl.models.moe): all-to-all group of ep_size DP ranks
    ep_group: Optional[object] = None
    ep_size: int = 1
    ep_rank: int = 0


def _init_linear(w: torch.Tensor, std: float) -> None:
    with torch.no_grad():
        w.normal_(0.0, std)


class _SwiGLUDown(torch.autograd.Function):
    """``down(swiglu(gu))`` with the SwiGLU backward fused into the down projection's data
    gradient (``swiglu_data_grad``: gemm64's store pass computes dgate / dup from the fp32 dAct
    tile, so dAct never round-trips through HBM).  ``recompute`` (selective activation
    checkpointing): save only ``gu`` and recompute the [T, ffn] activation in backward — one extra
    memory-bound pass in exchange for T*ffn*2 bytes per layer."""

    @staticmethod
    def forward(ctx, gu, w_down, recompute=False):
        from llmctl.exec.linear import wgrad_swiglu_ok
        from llmctl.ops._lib import native, use_native
        from llmctl.ops import ref

        act = native().swiglu_fwd(gu) if use_native(gu) else ref.swiglu_fwd(gu)
        out = F.linear(act, w_down)
        T = gu.numel() // gu.shape[-1]
        ctx.side = gu.requires_grad and wgrad_swiglu_ok(w_down, T, w_down.shape[1])
        # the plain data gradient: gemm64 reading W K-major when knob dgrad64 = all, else
        # hipBLASLt's forward layout through the W^T copy
        ctx.dgrad_g64 = ctx.side and knobs().dgrad64 == "all"
        if ctx.side and not ctx.dgrad_g64:
            _prep_weight_t(w_down, T)
        ctx.recompute = recompute
        if recompute:
            ctx.save_for_backward(gu, w_down)
        else:
            ctx.save_for_backward(gu, w_down, act)
        ctx.wparam = w_down  # the Parameter (carries the grad sink)
        return out

    @staticmethod
    def backward(ctx, dout):
        from llmctl.ops._lib import native, use_native
        from llmctl.ops import ref

        if ctx.recompute:
            gu, w_down = ctx.saved_tensors
            act = native().swiglu_fwd(gu) if use_native(gu) else ref.swiglu_fwd(gu)
        else:
            gu, w_down, act = ctx.saved_tensors
        dout2 = dout.reshape(-1, dout.shape[-1])
        act2 = act.reshape(-1, act.shape[-1])
        if ctx.side:
            # plain data gradient, then the weight gradient computing dgu on the side (gemm64.hip
            # "side job"): the HBM-bound SwiGLU backward streams under the wgrad's MFMAs
            if ctx.dgrad_g64 and _gemm64_dgrad_ok(dout2, w_down):
                dact = dgrad64(dout2, w_down)
            else:
                dact = data_grad(dout2, ctx.wparam)
            dgu = ctx.wparam._llmctl_grad_sink.write_swiglu(ctx.wparam, dout2, act2, dact, gu.reshape(-1, gu.shape[-1]))
            if dgu is not None:
                return dgu.view(gu.shape), None, None
            from llmctl.ops._lib import native, use_native

            dw = weight_grad(ctx.wparam, dout2, act2)
            return (native().swiglu_bwd(dact, gu) if use_native(gu) else ref.swiglu_bwd(dact, gu)), dw, None
        dw = weight_grad(ctx.wparam, dout2, act2)
        dgu = swiglu_data_grad(dout, ctx.wparam, gu)
        return dgu, dw, None


def _gemm64_dgrad_ok(dy2: torch.Tensor, w: torch.Tensor) -> bool:
    """``dy2 @ w`` on gemm64 (shape / alignment / 32-bit offset limits of ``gemm64_ex``)."""
    from llmctl.exec.linear import _gemm64_ok

    T, H = dy2.shape
    return (_gemm64_ok(T, w.shape[1], H, dy2, w) and w.is_contiguous() and H * w.stride(0) * 2 < 2**31)


def _fused_fwd_enabled() -> bool:
    """Training-forward GEMMs with fused epilogues (gemm64 ``EPI_ROPE_QKV`` / ``EPI_UP_SWIGLU``)
    when knob ``fused_fwd``.  Off by default: on the GPT-7B step the saved RoPE / SwiGLU passes
    (~0.45 ms per layer) are outweighed by gemm64's forward running 4-7 % below hipBLASLt's tuned
    forward kernels (1474-1477 vs 1543-1588 TF on the QKV / gate-up shapes): 842 / 845 ms per step
    fused vs 837 / 839 ms unfused, same box (profiles/fused_fwd_ab_r3.txt); at micro-batch 16 with the
    re-tuned hipBLASLt solutions and the in-place RoPE pass, 1111.8 / 1112.9 vs 1091.9 / 1094.3 ms."""
    return knobs().fused_fwd


def _gemm64_rows(x2: torch.Tensor, w: torch.Tensor) -> bool:
    from llmctl.exec.linear import _gemm64_enabled, _rows_ok
    from llmctl.ops._lib import use_native

    T, K = x2.shape
    return (_gemm64_enabled() and x2.is_cuda and use_native(x2) and x2.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.is_contiguous() and T % 256 == 0 and K % 128 == 0
            and _rows_ok(x2) and 256 * x2.stride(0) * 2 < 2**31)


def _prep_weight_t(w: nn.Parameter, tokens: int) -> None:
    """Start the side-stream W^T refresh now (forward) if this weight's data gradient will not
    run on gemm64 — as ``_Linear.forward`` does."""
    from llmctl.exec.linear import dgrad64_shape_ok

    sink = getattr(w, "_llmctl_grad_sink", None)
    if sink is not None and not dgrad64_shape_ok(tokens, w):
        sink.weight_t(w)


class _QKVRopeAttention(torch.autograd.Function):
    """QKV projection + RoPE + causal flash attention with the RoPE and the head split in the
    projection GEMM's epilogue (``gemm64_qkv_rope``: no qkv tensor, no rope_qkv_fwd pass) and,
    in backward, the RoPE backward in the attention backward's stores (``flash_attn_bwd_qkv``
    writes d(qkv) directly), followed by the projection's weight gradient (grad sink) and data
    gradient.  Replaces ``linear(x, wqkv)`` + ``ops.rope_flash_attention`` — reference step
    ``llmctl/runtime/engine.py:283-300``."""

    @staticmethod
    def forward(ctx, x, w, cos, sin, nq, nkv, B, S, positions, doc_start):
        from llmctl.exec.linear import gemm64_config
        from llmctl.ops._lib import native

        x2 = x.reshape(-1, x.shape[-1])
        T = x2.shape[0]
        pos = positions.reshape(-1).int().contiguous() if positions is not None else None
        q, k, v = native().gemm64_qkv_rope(x2, w, cos, sin, pos, nq, nkv, S,
                                           gemm64_config("fwd", T, w.shape[0], x2.shape[1]) % 1000)
        if ctx.needs_input_grad[0]:
            _prep_weight_t(w, T)
        D = 128
        q, k, v = q.view(B, S, nq, D), k.view(B, S, nkv, D), v.view(B, S, nkv, D)
        scale = D ** -0.5
        o, lse = native().flash_attn_fwd(q, k, v, scale, True, doc_start)
        ctx.save_for_backward(x2, q, k, v, o, lse, cos, sin, pos if pos is not None else torch.empty(0))
        ctx.wparam, ctx.has_pos, ctx.S, ctx.scale, ctx.doc_start = w, pos is not None, S, scale, doc_start
        ctx.xshape = x.shape
        return o

    @staticmethod
    def backward(ctx, do):
        from llmctl.ops._lib import native

        x2, q, k, v, o, lse, cos, sin, pos = ctx.saved_tensors
        dqkv = native().flash_attn_bwd_qkv(do.contiguous(), q, k, v, o, lse, ctx.scale, True, ctx.doc_start, cos,
                                           sin, pos if ctx.has_pos else None, ctx.S)
        dw = weight_grad(ctx.wparam, dqkv, x2) if ctx.needs_input_grad[1] else None
        dx = data_grad(dqkv, ctx.wparam).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, dw, None, None, None, None, None, None, None, None


class _UpSwiGLUDown(torch.autograd.Function):
    """Gate/up projection with SwiGLU in its epilogue (``gemm64_up_swiglu`` stores gu for the
    backward and act for the down projection: no swiglu_fwd pass) + the down projection; the
    backward is ``_SwiGLUDown``'s (SwiGLU backward in the down data-gradient epilogue) followed by
    the up projection's weight / data gradients."""

    @staticmethod
    def forward(ctx, x, w_up, w_down):
        from llmctl.exec.linear import forward_linear, gemm64_config, wgrad_swiglu_ok
        from llmctl.ops._lib import native

        x2 = x.reshape(-1, x.shape[-1])
        T = x2.shape[0]
        gu, act = native().gemm64_up_swiglu(x2, w_up, gemm64_config("fwd", T, w_up.shape[0], x2.shape[1]) % 1000)
        out = forward_linear(act, w_down)
        if ctx.needs_input_grad[0]:
            _prep_weight_t(w_up, T)
        # the SwiGLU backward as the down projection wgrad's side job (swiglu_bwd = side), as
        # _SwiGLUDown; the down data gradient then runs plain (gemm64 or hipBLASLt through W^T).
        # (gu is made inside this Function, so gu.requires_grad is always False here: whether dgu
        # is needed comes from the inputs -- round 4 read gu.requires_grad and never took the side
        # path, running the down dgrad on the slower fused-epilogue kernel instead)
        ctx.side = (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]) and wgrad_swiglu_ok(w_down, T, w_down.shape[1])
        ctx.dgrad_g64 = ctx.side and knobs().dgrad64 == "all"
        if ctx.side and not ctx.dgrad_g64:
            _prep_weight_t(w_down, T)
        ctx.save_for_backward(x2, gu, act)
        ctx.w_up, ctx.w_down, ctx.xshape = w_up, w_down, x.shape
        return out.view(*x.shape[:-1], w_down.shape[0])

    @staticmethod
    def backward(ctx, dout):
        x2, gu, act = ctx.saved_tensors
        dout2 = dout.reshape(-1, dout.shape[-1])
        dgu = None
        if ctx.side:
            if ctx.dgrad_g64 and _gemm64_dgrad_ok(dout2, ctx.w_down):
                dact = dgrad64(dout2, ctx.w_down)
            else:
                dact = data_grad(dout2, ctx.w_down)
            dgu = ctx.w_down._llmctl_grad_sink.write_swiglu(ctx.w_down, dout2, act, dact, gu)
            dw_down = None
            if dgu is None:  # operands the side kernel cannot take: weight gradient + elementwise pass
                from llmctl.ops._lib import native

                dw_down = weight_grad(ctx.w_down, dout2, act)
                dgu = native().swiglu_bwd(dact, gu)
        else:
            dw_down = weight_grad(ctx.w_down, dout2, act)
            dgu = swiglu_data_grad(dout2, ctx.w_down, gu)
        dw_up = weight_grad(ctx.w_up, dgu, x2) if ctx.needs_input_grad[1] else None
        dx = data_grad(dgu, ctx.w_up).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, dw_up, dw_down


class DecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, pc: ParallelContext, layer_idx: int, device=None, dtype=None):
        super().__init__()
        self.cfg, self.pc, self.idx = cfg, pc, layer_idx
        t = pc.tp_size
        if cfg.heads % t or cfg.kv_heads % t or cfg.ffn % t:
            raise ValueError(f"heads/kv_heads/ffn must divide tp={t}")
        if pc.cp_mode not in ("ulysses", "ring"):
            raise ValueError(f"unknown context-parallel mode {pc.cp_mode!r} (ulysses | ring)")
        if pc.cp_mode == "ulysses" and ((cfg.kv_heads // t) % pc.cp_size or (cfg.heads // t) % pc.cp_size):
            raise ValueError(f"(kv_)heads / tp must divide context_parallel={pc.cp_size} (ulysses; "
                             f"ring attention has no head constraint)")
        self.nq, self.nkv, self.D = cfg.heads // t, cfg.kv_heads // t, cfg.head_dim
        self.f = cfg.ffn // t
        h = cfg.hidden
        kw = dict(device=device, dtype=dtype)
        ln = cfg.norm == "layernorm"
        self.attn_norm_w = nn.Parameter(torch.ones(h, **kw))
        self.mlp_norm_w = nn.Parameter(torch.ones(h, **kw))
        self.attn_norm_b = nn.Parameter(torch.zeros(h, **kw)) if ln else None
        self.mlp_norm_b = nn.Parameter(torch.zeros(h, **kw)) if ln else None
        self.wqkv = nn.Parameter(torch.empty((self.nq + 2 * self.nkv) * self.D, h, **kw))
        self.wo = nn.Parameter(torch.empty(h, self.nq * self.D, **kw))
        gated = cfg.gated_mlp
        self.moe = None
        if cfg.is_moe:
            if t > 1:
                raise NotImplementedError("MoE layers with tensor parallelism (use expert parallelism)")
            self.w_up = self.w_down = None
        else:
            self.w_up = nn.Parameter(torch.empty((2 if gated else 1) * self.f, h, **kw))
            self.w_down = nn.Parameter(torch.empty(h, self.f, **kw))
        if ln:  # GPT-2 style biases (row-parallel biases are replicated, added after the reduce)
            self.bqkv = nn.Parameter(torch.zeros((self.nq + 2 * self.nkv) * self.D, **kw))
            self.bo = nn.Parameter(torch.zeros(h, **kw))
            self.b_up = nn.Parameter(torch.zeros((2 if gated else 1) * self.f, **kw))
            self.b_down = nn.Parameter(torch.zeros(h, **kw))
        else:
            self.bqkv = self.bo = self.b_up = self.b_down = None
        std = 0.02
        _init_linear(self.wqkv, std)
        if self.w_up is not None:
            _init_linear(self.w_up, std)
        _init_linear(self.wo, std / math.sqrt(2 * cfg.layers))
        if self.w_down is not None:
            _init_linear(self.w_down, std / math.sqrt(2 * cfg.layers))
        if cfg.is_moe:
            self.moe = MoEMLP(cfg, cfg.layers, pc.ep_group, pc.ep_size, pc.ep_rank, **kw)
        for p in (self.attn_norm_w, self.mlp_norm_w, self.attn_norm_b, self.mlp_norm_b, self.bo, self.b_down):
            if p is not None:
                p.tp_replicated = True  # identical on every TP rank (partial grads under SP)

    # -- norm helpers --------------------------------------------------------------
    def _norm(self, x, w, b):
        eps = self.cfg.layer_norm_eps
        return ops.layernorm(x, w, b, eps) if b is not None else ops.rmsnorm(x, w, eps)

    def _add_norm(self, x, res, w, b):
        eps = self.cfg.layer_norm_eps
        return ops.add_layernorm(x, res, w, b, eps) if b is not None else ops.add_rmsnorm(x, res, w, eps)

    def _col_in(self, x):
        pc = self.pc
        if pc.tp_size == 1:
            return x
        return tp.gather_from_sp(x, pc.tp_group) if pc.sequence_parallel else tp.copy_to_tp(x, pc.tp_group)

    def _row_out(self, x):
        pc = self.pc
        if pc.tp_size == 1:
            return x
        return tp.reduce_scatter_to_sp(x, pc.tp_group) if pc.sequence_parallel else tp.reduce_from_tp(x, pc.tp_group)

    def _async_sp(self) -> bool:
        return self.pc.tp_size > 1 and self.pc.sequence_parallel and async_tp.enabled()

    def _fused_qkv_ok(self, x, rope) -> bool:
        if not (_fused_fwd_enabled() and rope is not None and self.bqkv is None and self.D == 128
                and self.nq % 2 == 0 and self.nkv % 2 == 0 and self.pc.cp_size == 1 and not self._async_sp()
                and torch.is_grad_enabled() and knobs().fused_rope_attn):
            return False
        return _gemm64_rows(x.reshape(-1, x.shape[-1]), self.wqkv) and rope[0].shape[-1] == 64

    def attention(self, xn, B, S, rope, positions=None, doc_start=None):
        if self._fused_qkv_ok(xn, rope):
            x = self._col_in(xn)
            o = _QKVRopeAttention.apply(x, self.wqkv, rope[0], rope[1], self.nq, self.nkv, B, S, positions, doc_start)
            return self._attn_out(o, B, S)
        if self._async_sp():  # SP all-gather overlapped with the QKV GEMM
            qkv = async_tp.column_parallel_sp(xn, self.wqkv, self.bqkv, self.pc.tp_group)
        else:
            qkv = linear(self._col_in(xn), self.wqkv, self.bqkv)
        if rope is not None and self.pc.cp_size == 1 and knobs().fused_rope_attn:
            # RoPE + attention with the RoPE backward fused into the attention backward's stores
            o = ops.rope_flash_attention(qkv, rope[0], rope[1], self.nq, self.nkv, B, S, positions, doc_start,
                                         inplace=True)
            return self._attn_out(o, B, S)
        if rope is not None:
            q, k, v = ops.rope_qkv(qkv, rope[0], rope[1], self.nq, self.nkv, S, positions)
        else:
            T = qkv.shape[0]
            x = qkv.view(T, self.nq + 2 * self.nkv, self.D)
            q, k, v = x[:, :self.nq].contiguous(), x[:, self.nq:self.nq + self.nkv].contiguous(), \
                x[:, self.nq + self.nkv:].contiguous()
        q = q.view(B, S, self.nq, self.D)
        k = k.view(B, S, self.nkv, self.D)
        v = v.view(B, S, self.nkv, self.D)
        if self.pc.cp_size > 1 and self.pc.cp_mode == "ring":  # K/V chunks around the CP ring
            o = cp.ring_attention(q, k, v, self.pc.cp_group, zigzag=self.pc.cp_zigzag)
        elif self.pc.cp_size > 1:  # sequence chunk, all heads <-> all tokens, head chunk
            g = self.pc.cp_group
            o = cp.head_to_seq(ops.flash_attention(cp.seq_to_head(q, g), cp.seq_to_head(k, g),
                                                   cp.seq_to_head(v, g), causal=True), g)
        else:
            o = ops.flash_attention(q, k, v, causal=True, doc_start=doc_start)
        return self._attn_out(o, B, S)

    def _attn_out(self, o, B, S):
        if self._async_sp():  # o-proj GEMM with the SP reduce-scatter overlapped
            out = async_tp.row_parallel_sp(o.reshape(B * S, self.nq * self.D), self.wo, self.pc.tp_group)
        else:
            out = self._row_out(linear(o.reshape(B * S, self.nq * self.D), self.wo))
        if self.bo is not None:
            out = out + self.bo
        return out

    def mlp(self, xn):
        if self.moe is not None:
            return self.moe(xn)
        if self._async_sp() and self.pc.activation_checkpoint != "selective":
            # SP all-gather / reduce-scatter overlapped with the up / down GEMMs
            g = self.pc.tp_group
            h = async_tp.column_parallel_sp(xn, self.w_up, self.b_up, g)
            h = ops.swiglu(h) if self.cfg.gated_mlp else ops.gelu(h)
            out = async_tp.row_parallel_sp(h, self.w_down, g)
        else:
            x = self._col_in(xn)
            if (self.cfg.gated_mlp and _fused_fwd_enabled() and self.b_up is None and torch.is_grad_enabled()
                    and self.pc.activation_checkpoint != "selective" and self.w_up.shape[0] % 256 == 0
                    and _gemm64_rows(x.reshape(-1, x.shape[-1]), self.w_up)):
                out = _UpSwiGLUDown.apply(x, self.w_up, self.w_down)
            elif self.cfg.gated_mlp:
                gu = linear(x, self.w_up, self.b_up)
                out = _SwiGLUDown.apply(gu, self.w_down, self.pc.activation_checkpoint == "selective")
            else:
                hdn = ops.gelu(linear(x, self.w_up, self.b_up))
                out = linear(hdn, self.w_down)
            out = self._row_out(out)
        if self.b_down is not None:
            out = out + self.b_down
        return out

    def forward(self, x, residual, B, S, rope, positions=None, doc_start=None):
        """Pre-norm block with fused residual-add + norm.

        ``residual`` is the running residual stream (None for the first layer);
        ``x`` is the previous block's output to be added into it.
        Returns (block_output, residual) — the add of block_output is deferred into the
        next layer's fused add+norm kernel."""
        if residual is None:
            residual = x
            xn = self._norm(x, self.attn_norm_w, self.attn_norm_b)
        else:
            xn, residual = self._add_norm(x, residual, self.attn_norm_w, self.attn_norm_b)
        a = self.attention(xn, B, S, rope, positions, doc_start)
        xn2, residual = self._add_norm(a, residual, self.mlp_norm_w, self.mlp_norm_b)
        m = self.mlp(xn2)
        return m, residual


class DecoderLM(nn.Module):
    """Causal LM.  ``forward(input_ids [B,S], labels [B,S]|None)`` -> mean loss or logits."""

    def __init__(self, cfg: ModelConfig, pc: Optional[ParallelContext] = None, device=None,
                 dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        self.pc = pc = pc or ParallelContext()
        end = pc.layer_end if pc.layer_end is not None else cfg.layers
        kw = dict(device=device, dtype=dtype)
        t = pc.tp_size
        h = cfg.hidden
        if cfg.vocab_size % t:
            raise ValueError(f"vocab {cfg.vocab_size} not divisible by tp={t}")
        self.vocab_local = cfg.vocab_size // t
        self.vocab_start = pc.tp_rank * self.vocab_local
        self.embed = None
        self.pos_embed = None
        if pc.has_embedding:
            self.embed = nn.Parameter(torch.empty(self.vocab_local, h, **kw))
            _init_linear(self.embed, 0.02)
            if cfg.position == "learned":
                self.pos_embed = nn.Parameter(torch.empty(cfg.max_position_embeddings, h, **kw))
                _init_linear(self.pos_embed, 0.01)
        ranges = pc.layer_ranges or [(pc.layer_start, end)]
        self.layers = nn.ModuleList([DecoderLayer(cfg, pc, i, **kw) for a, b in ranges for i in range(a, b)])
        # local [start, end) slice of every model chunk (one chunk unless virtual stages)
        self.chunk_slices, o = [], 0
        for a, b in ranges:
            self.chunk_slices.append((o, o + b - a))
            o += b - a
        self.final_norm_w = self.final_norm_b = self.lm_head = None
        if pc.has_head:
            self.final_norm_w = nn.Parameter(torch.ones(h, **kw))
            if cfg.norm == "layernorm":
                self.final_norm_b = nn.Parameter(torch.zeros(h, **kw))
            if not (cfg.tie_word_embeddings and pc.has_embedding):
                self.lm_head = nn.Parameter(torch.empty(self.vocab_local, h, **kw))
                _init_linear(self.lm_head, 0.02)
        for p in (self.pos_embed, self.final_norm_w, self.final_norm_b):
            if p is not None:
                p.tp_replicated = True
        self._rope_cache = {}
        # called at the top of ``head()``: the engine's ZeRO-1/2 (and side-stream optimizer)
        # overlap waits here for the final-norm / LM-head buckets, which are gathered last
        self.pre_head_hook = None

    # ------------------------------------------------------------------ helpers
    def head_weight(self):
        return self.lm_head if self.lm_head is not None else self.embed

    def rope_tables(self, S: int, device):
        if self.cfg.position != "rope":
            return None
        key = (max(S, 1), str(device))
        if key not in self._rope_cache:
            r = self.cfg.rope or {}
            n = max(S, self.cfg.max_position_embeddings)
            self._rope_cache[key] = ops.ref.rope_tables(
                n, self.cfg.head_dim, base=float(r.get("base", 10000)), scaling=r.get("scaling", "linear"),
                factor=float(r.get("factor", 1.0)), short_factor=r.get("short_factor"),
                long_factor=r.get("long_factor"), original_max_position=r.get("original_max_position"),
                device=device)
        return self._rope_cache[key]

    def embed_tokens(self, input_ids: torch.Tensor, positions: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, S = input_ids.shape
        ids = input_ids.reshape(-1)
        pc = self.pc
        if pc.tp_size > 1:
            x = tp.vocab_parallel_embedding(ids, self.embed, self.vocab_start, pc.tp_group, pc.sequence_parallel)
        else:
            x = F.embedding(ids, self.embed)
        if self.pos_embed is not None:
            if positions is not None:  # explicit (e.g. per-document) positions
                pos = self.pos_embed[positions.long()]
            elif pc.cp_size > 1:  # this rank's part of the sequence: global positions
                pos = self.pos_embed[cp.local_positions(B, S, pc.cp_rank, ids.device, pc.cp_size,
                                                        pc.cp_zigzag).long()]
            else:
                pos = self.pos_embed[:S].repeat(B, 1)
            if pc.tp_size > 1 and pc.sequence_parallel:
                pos = tp._split_tokens(pos, pc.tp_group)
            x = x + pos
        return x

    def run_layers(self, x, B, S, residual=None, positions=None, doc_start=None, chunk: Optional[int] = None):
        """Run the local decoder layers (only model chunk ``chunk`` under virtual stages)."""
        if self.pc.cp_size > 1 and positions is None:
            positions = cp.local_positions(B, S, self.pc.cp_rank, x.device, self.pc.cp_size, self.pc.cp_zigzag)
        if doc_start is not None and positions is None:  # packed documents: RoPE restarts per document
            positions = (torch.arange(S, device=x.device, dtype=torch.int32).view(1, S) - doc_start).reshape(-1)
        rope = self.rope_tables(S * self.pc.cp_size, x.device)
        ac = self.pc.activation_checkpoint
        layers = self.layers if chunk is None else self.layers[self.chunk_slices[chunk][0]:self.chunk_slices[chunk][1]]
        for layer in layers:
            if ac == "full" and self.training and torch.is_grad_enabled():
                if residual is None:
                    x, residual = torch.utils.checkpoint.checkpoint(
                        lambda a, l=layer: l(a, None, B, S, rope, positions, doc_start), x, use_reentrant=False)
                else:
                    x, residual = torch.utils.checkpoint.checkpoint(
                        lambda a, r, l=layer: l(a, r, B, S, rope, positions, doc_start), x, residual,
                        use_reentrant=False)
            else:
                x, residual = layer(x, residual, B, S, rope, positions, doc_start)
        return x, residual

    def head(self, x, residual):
        cfg = self.cfg
        if self.pre_head_hook is not None:
            self.pre_head_hook()
        if residual is None:
            xn = (ops.layernorm(x, self.final_norm_w, self.final_norm_b, cfg.layer_norm_eps)
                  if self.final_norm_b is not None else ops.rmsnorm(x, self.final_norm_w, cfg.layer_norm_eps))
        else:
            xn, _ = (ops.add_layernorm(x, residual, self.final_norm_w, self.final_norm_b, cfg.layer_norm_eps)
                     if self.final_norm_b is not None
                     else ops.add_rmsnorm(x, residual, self.final_norm_w, cfg.layer_norm_eps))
        pc = self.pc
        if pc.tp_size > 1:
            xn = tp.gather_from_sp(xn, pc.tp_group) if pc.sequence_parallel else tp.copy_to_tp(xn, pc.tp_group)
        return linear(xn, self.head_weight())

    def loss(self, logits, labels, denom: Optional[float] = None):
        pc = self.pc
        lab = labels.reshape(-1)
        if denom is None:
            denom = float(lab.numel())
        if pc.tp_size > 1:
            return tp.vocab_parallel_cross_entropy(logits, lab, self.vocab_start, pc.tp_group, denom)
        return ops.cross_entropy(logits, lab, reduction_denom=denom)

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None,
                loss_denom: Optional[float] = None, doc_start: Optional[torch.Tensor] = None):
        """``doc_start`` (int32 [B,S], packed sequences): attention and positions restart at
        every document boundary (see ``llmctl.ops.ref.document_starts``)."""
        B, S = input_ids.shape
        positions = None
        if doc_start is not None:
            if self.pc.cp_size > 1:
                raise NotImplementedError("packed sequences with context parallelism")
            positions = (torch.arange(S, device=input_ids.device, dtype=torch.int32).view(1, S) - doc_start).reshape(-1)
        x = self.embed_tokens(input_ids, positions)
        x, residual = self.run_layers(x, B, S, positions=positions, doc_start=doc_start)
        logits = self.head(x, residual)
        if labels is None:
            return logits
        loss = self.loss(logits, labels, loss_denom)
        if self.cfg.is_moe and self.cfg.router_aux_loss_coef:
            # load-balancing loss, averaged over layers; scaled like the CE term so gradient
            # accumulation over micro-batches averages it
            aux = [l.moe.aux_loss for l in self.layers if l.moe is not None and l.moe.aux_loss is not None]
            if aux:
                scale = labels.numel() / float(loss_denom if loss_denom is not None else labels.numel())
                loss = loss + self.cfg.router_aux_loss_coef * scale * torch.stack(aux).mean().to(loss.dtype)
        return loss


def build_model(cfg: ModelConfig, device=None, dtype=torch.bfloat16, pc: Optional[ParallelContext] = None,
                seed: Optional[int] = None) -> DecoderLM:
    if seed is not None:
        torch.manual_seed(seed)
    return DecoderLM(cfg, pc=pc, device=device, dtype=dtype)
