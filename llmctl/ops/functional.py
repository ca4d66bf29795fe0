"""Autograd-facing fused ops.  GPU tensors run the hand-written CDNA4 HIP kernels in
``csrc/`` (``torch.ops.llmctl.*``); CPU tensors run the fp32 oracle in :mod:`.ref`.

Every op keeps the layouts the GEMMs (hipBLASLt) produce/consume so no transposes or
copies are needed between kernels:

* activations are token-major ``[T, features]`` (T = batch*seq);
* attention takes ``q [B,S,Hq,D]``, ``k/v [B,S,Hkv,D]`` (GQA), returns ``o [B,S,Hq,D]``
  which *is* the ``[T, Hq*D]`` input of the output projection;
* RoPE is fused with the QKV split: ``[T,(Hq+2Hkv)D] -> q,k (rotated), v``.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from llmctl.config.knobs import knobs

from . import ref
from ._lib import native, use_native


# =============================================================================== norms
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        x2 = x.reshape(-1, x.shape[-1])
        if use_native(x):
            y, rstd = native().rmsnorm_fwd(x2, w, eps)
        else:
            y, rstd = ref.rmsnorm_fwd(x2, w, eps)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        if use_native(dy):
            dx, dw = native().rmsnorm_bwd(dy2, x2, w, rstd, None)
        else:
            dx, dw = ref.rmsnorm_bwd(dy2, x2, w, rstd)
        return dx.view(ctx.shape), dw, None


class _AddRMSNorm(torch.autograd.Function):
    """res_out = x + residual ; y = rmsnorm(res_out) * w.  One HBM pass for both."""

    @staticmethod
    def forward(ctx, x, residual, w, eps):
        H = x.shape[-1]
        x2, r2 = x.reshape(-1, H), residual.reshape(-1, H)
        if use_native(x):
            y, res_out, rstd = native().add_rmsnorm_fwd(x2, r2, w, eps)
        else:
            res_out = (x2.float() + r2.float()).to(x.dtype)
            y, rstd = ref.rmsnorm_fwd(res_out, w, eps)
        ctx.save_for_backward(res_out, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape), res_out.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dres):
        res_out, w, rstd = ctx.saved_tensors
        H = res_out.shape[-1]
        dy2 = dy.reshape(-1, H).contiguous()
        dres2 = dres.reshape(-1, H).contiguous() if dres is not None else None
        if use_native(dy):
            dx, dw = native().rmsnorm_bwd(dy2, res_out, w, rstd, dres2)
        else:
            dx, dw = ref.rmsnorm_bwd(dy2, res_out, w, rstd, dres2)
        dx = dx.view(ctx.shape)
        return dx, dx, dw, None


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        x2 = x.reshape(-1, x.shape[-1])
        if use_native(x):
            y, mu, rstd = native().layernorm_fwd(x2, w, b, eps)
        else:
            y, mu, rstd = ref.layernorm_fwd(x2, w, b, eps)
        ctx.save_for_backward(x2, w, mu, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mu, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        if use_native(dy):
            dx, dw, db = native().layernorm_bwd(dy2, x2, w, mu, rstd, None)
        else:
            dx, dw, db = ref.layernorm_bwd(dy2, x2, w, mu, rstd)
        return dx.view(ctx.shape), dw, db, None


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, eps):
        H = x.shape[-1]
        x2, r2 = x.reshape(-1, H), residual.reshape(-1, H)
        if use_native(x):
            y, res_out, mu, rstd = native().add_layernorm_fwd(x2, r2, w, b, eps)
        else:
            res_out = (x2.float() + r2.float()).to(x.dtype)
            y, mu, rstd = ref.layernorm_fwd(res_out, w, b, eps)
        ctx.save_for_backward(res_out, w, mu, rstd)
        ctx.shape = x.shape
        return y.view(x.shape), res_out.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dres):
        res_out, w, mu, rstd = ctx.saved_tensors
        H = res_out.shape[-1]
        dy2 = dy.reshape(-1, H).contiguous()
        dres2 = dres.reshape(-1, H).contiguous() if dres is not None else None
        if use_native(dy):
            dx, dw, db = native().layernorm_bwd(dy2, res_out, w, mu, rstd, dres2)
        else:
            dx, dw, db = ref.layernorm_bwd(dy2, res_out, w, mu, rstd, dres2)
        dx = dx.view(ctx.shape)
        return dx, dx, dw, db, None


def rmsnorm(x, w, eps: float = 1e-5):
    return _RMSNorm.apply(x, w, eps)


def add_rmsnorm(x, residual, w, eps: float = 1e-5):
    return _AddRMSNorm.apply(x, residual, w, eps)


def layernorm(x, w, b, eps: float = 1e-5):
    return _LayerNorm.apply(x, w, b, eps)


def add_layernorm(x, residual, w, b, eps: float = 1e-5):
    return _AddLayerNorm.apply(x, residual, w, b, eps)


# =============================================================================== rope
class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, nq, nkv, seq_len, positions):
        if use_native(qkv):
            q, k, v = native().rope_qkv_fwd(qkv, cos, sin, nq, nkv, seq_len, positions)
        else:
            q, k, v = ref.rope_qkv_fwd(qkv, cos, sin, nq, nkv, seq_len, positions)
        ctx.save_for_backward(cos, sin, positions if positions is not None else torch.empty(0))
        ctx.has_pos = positions is not None
        ctx.seq_len = seq_len
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin, pos = ctx.saved_tensors
        pos = pos if ctx.has_pos else None
        dq, dk, dv = dq.contiguous(), dk.contiguous(), dv.contiguous()
        if use_native(dq):
            dqkv = native().rope_qkv_bwd(dq, dk, dv, cos, sin, ctx.seq_len, pos)
        else:
            dqkv = ref.rope_qkv_bwd(dq, dk, dv, cos, sin, ctx.seq_len, pos)
        return dqkv, None, None, None, None, None, None


def rope_qkv(qkv, cos, sin, nq: int, nkv: int, seq_len: int, positions: Optional[torch.Tensor] = None):
    """``qkv [T,(nq+2nkv)*D]`` -> ``q [T,nq,D], k [T,nkv,D], v [T,nkv,D]`` with RoPE on q,k."""
    return _RopeQKV.apply(qkv, cos, sin, nq, nkv, seq_len, positions)


def rope_qkv_cache(qkv, cos, sin, nq: int, nkv: int, seq_len: int, positions, k_cache, v_cache, slots):
    """Inference: ``rope_qkv`` that also writes the rotated K and V rows into the paged cache at
    ``slots`` (int64 [T], -1 = skip) in the same pass."""
    if use_native(qkv):
        return native().rope_qkv_cache_fwd(qkv, cos, sin, nq, nkv, seq_len, positions, k_cache, v_cache, slots)
    q, k, v = ref.rope_qkv_fwd(qkv, cos, sin, nq, nkv, seq_len, positions)
    ref.kv_cache_write(k, v, k_cache, v_cache, slots)
    return q, k, v


# =============================================================================== attention
class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, doc_start):
        if use_native(q):
            o, lse = native().flash_attn_fwd(q, k, v, scale, causal, doc_start)
        else:
            o, lse = ref.attention_fwd(q, k, v, scale, causal, doc_start)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale, ctx.causal, ctx.doc_start = scale, causal, doc_start
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        if use_native(do):
            dq, dk, dv = native().flash_attn_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal, ctx.doc_start)
        else:
            dq, dk, dv = ref.attention_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal, ctx.doc_start)
        return dq, dk, dv, None, None, None


def flash_attention(q, k, v, causal: bool = True, softmax_scale: Optional[float] = None,
                    doc_start: Optional[torch.Tensor] = None):
    """Causal flash attention.  q ``[B,S,Hq,D]``, k/v ``[B,S,Hkv,D]`` (Hq % Hkv == 0).
    ``doc_start`` (int32 ``[B,S]``, packed sequences): attention stays inside each document."""
    scale = softmax_scale if softmax_scale is not None else q.shape[-1] ** -0.5
    return _FlashAttn.apply(q, k, v, scale, causal, doc_start)


class _RopeFlashAttn(torch.autograd.Function):
    """``rope_qkv`` + ``flash_attention`` with the RoPE backward fused into the attention
    backward's dQ / dK stores (``flash_attn_bwd_qkv``): the backward writes the QKV-projection
    gradient dqkv [T, (nq+2nkv)*D] directly — no dq/dk/dv tensors and no rope_bwd pass."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, nq, nkv, B, S, positions, doc_start, inplace=False):
        if inplace:
            # the caller owns qkv (a projection output nothing else saved): rotate its q / k heads
            # in place and attend strided views of it — V is neither copied nor re-read
            native().rope_qk_inplace_(qkv, cos, sin, nq, nkv, S, positions)
            D = qkv.shape[-1] // (nq + 2 * nkv)
            qkv4 = qkv.view(B, S, nq + 2 * nkv, D)
            q, k, v = qkv4[:, :, :nq], qkv4[:, :, nq:nq + nkv], qkv4[:, :, nq + nkv:]
        else:
            q, k, v = native().rope_qkv_fwd(qkv, cos, sin, nq, nkv, S, positions)
            D = q.shape[-1]
            q, k, v = q.view(B, S, nq, D), k.view(B, S, nkv, D), v.view(B, S, nkv, D)
        scale = D ** -0.5
        o, lse = native().flash_attn_fwd(q, k, v, scale, True, doc_start)
        pos = positions.reshape(-1).int().contiguous() if positions is not None else None
        ctx.save_for_backward(q, k, v, o, lse, cos, sin, pos if pos is not None else torch.empty(0))
        ctx.has_pos, ctx.S, ctx.scale, ctx.doc_start = pos is not None, S, scale, doc_start
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cos, sin, pos = ctx.saved_tensors
        dqkv = native().flash_attn_bwd_qkv(do.contiguous(), q, k, v, o, lse, ctx.scale, True, ctx.doc_start, cos, sin,
                                           pos if ctx.has_pos else None, ctx.S)
        return dqkv, None, None, None, None, None, None, None, None, None


def rope_flash_attention(qkv, cos, sin, nq: int, nkv: int, B: int, S: int, positions=None, doc_start=None,
                         inplace: bool = False):
    """Causal attention on the QKV projection output: RoPE(q, k) -> flash attention -> o
    ``[B,S,nq,D]``; the backward returns d(qkv) in one fused pass on the HIP path.  ``inplace``
    (HIP path; the caller's qkv must not be needed afterwards): RoPE rotates qkv's q / k heads in
    place and attention reads strided views (knob ``rope_inplace`` off disables)."""
    if use_native(qkv) and qkv.is_contiguous():
        inplace = inplace and knobs().rope_inplace
        return _RopeFlashAttn.apply(qkv, cos, sin, nq, nkv, B, S, positions, doc_start, inplace)
    q, k, v = rope_qkv(qkv, cos, sin, nq, nkv, S, positions)
    D = q.shape[-1]
    return flash_attention(q.view(B, S, nq, D), k.view(B, S, nkv, D), v.view(B, S, nkv, D), causal=True,
                           doc_start=doc_start)


# =============================================================================== MLP
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu) if use_native(gu) else ref.swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dact):
        (gu,) = ctx.saved_tensors
        dact = dact.contiguous()
        return native().swiglu_bwd(dact, gu) if use_native(dact) else ref.swiglu_bwd(dact, gu)


class _GELU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return native().gelu_fwd(x) if use_native(x) else ref.gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        return native().gelu_bwd(dy, x) if use_native(dy) else ref.gelu_bwd(dy, x)


def swiglu(gu):
    """``gu [..., 2F]`` laid out ``[gate | up]`` -> ``silu(gate) * up``."""
    return _SwiGLU.apply(gu)


def gelu(x):
    return _GELU.apply(x)


# =============================================================================== loss
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, denom):
        if use_native(logits):
            loss, lse = native().cross_entropy_fwd(logits, labels, ignore_index)
        else:
            loss, lse = ref.cross_entropy_fwd(logits, labels, ignore_index)
        ctx.save_for_backward(logits, lse, labels)
        ctx.ignore_index, ctx.denom = ignore_index, denom
        return loss.sum() / denom

    @staticmethod
    def backward(ctx, g):
        logits, lse, labels = ctx.saved_tensors
        dloss = (g / ctx.denom).float().expand(labels.shape).contiguous()
        if use_native(logits):
            # logits are dead after this: write dlogits in place (saves a [T,V] buffer)
            dl = native().cross_entropy_bwd(dloss, logits, lse, labels, ctx.ignore_index, True)
        else:
            dl = ref.cross_entropy_bwd(dloss, logits, lse, labels, ctx.ignore_index)
        return dl, None, None, None


def cross_entropy(logits, labels, ignore_index: int = -100, reduction_denom: Optional[float] = None):
    """Mean token cross-entropy over non-ignored labels; logits ``[T,V]`` bf16/fp32."""
    if reduction_denom is None:
        reduction_denom = float(max(int((labels != ignore_index).sum()), 1)) if not labels.is_cuda else None
    if reduction_denom is None:
        # avoid a host sync on GPU: callers that know the count pass it; default = all tokens
        reduction_denom = float(labels.numel())
    return _CrossEntropy.apply(logits, labels, ignore_index, reduction_denom)


# =============================================================================== optimizer
def adamw_step_(param, master, grad, exp_avg, exp_avg_sq, *, lr: float, beta1: float, beta2: float,
                eps: float, weight_decay: float, step: int, grad_scale: Optional[torch.Tensor] = None):
    """One fused AdamW update over flat buffers (bf16 param, fp32 master/m/v, bf16|fp32 grad).
    ``grad_scale`` is a 1-element fp32 device tensor (e.g. the clip coefficient) so clipping
    needs no host sync."""
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if use_native(param):
        native().adamw_step_(param, master, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                             bc1, bc2, grad_scale)
    else:
        gs = float(grad_scale) if grad_scale is not None else 1.0
        ref.adamw_step_(param, master, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, gs)


def l2norm_sq(t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum of squares of ``t`` accumulated (fp32) into ``out`` (allocated if None)."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=t.device)
    if use_native(t):
        native().l2norm_sq_(t, out)
    else:
        out += ref.l2norm_sq(t)
    return out


# =============================================================================== serving
def transpose_(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """``dst[C, R] = src[R, C]`` (bf16, HIP kernel on GPU)."""
    if use_native(src):
        native().transpose_(src, dst)
    else:
        dst.copy_(src.t())
    return dst


def kv_cache_write(k, v, k_cache, v_cache, slot_mapping):
    if use_native(k):
        native().kv_cache_write(k, v, k_cache, v_cache, slot_mapping)
    else:
        ref.kv_cache_write(k, v, k_cache, v_cache, slot_mapping)


def paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale: Optional[float] = None):
    scale = scale if scale is not None else q.shape[-1] ** -0.5
    if use_native(q):
        return native().paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale)
    return ref.paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale)


def attn_merge_(o_acc, lse_acc, o_j, lse_j) -> None:
    """Merge a partial attention output into an fp32 accumulator by log-sum-exp (in place)."""
    if use_native(o_acc):
        native().attn_merge_(o_acc, lse_acc, o_j, lse_j)
    else:
        ref.attn_merge_(o_acc, lse_acc, o_j, lse_j)


def prefill_work_list(cu_q, q_block: int = 128) -> List[int]:
    """(sequence << 16) | q-block items for ``paged_prefill_attention``, heaviest (longest
    causal span: the last q-blocks of long chunks) first."""
    items = []
    for n in range(len(cu_q) - 1):
        qlen = int(cu_q[n + 1]) - int(cu_q[n])
        for b in range((qlen + q_block - 1) // q_block):
            items.append((b * q_block, (n << 16) | b))
    items.sort(key=lambda t: -t[0])
    return [w for _, w in items]


def paged_prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale: Optional[float] = None,
                            work=None):
    """Chunked / prefix-reusing prefill attention over the paged KV cache (see
    ``csrc/paged_prefill.hip``).  ``cu_q`` / ``ctx_lens`` / ``block_tables`` int32; ``work``
    (optional) is the precomputed :func:`prefill_work_list` as an int32 tensor."""
    scale = scale if scale is not None else q.shape[-1] ** -0.5
    if use_native(q):
        if work is None:
            work = torch.tensor(prefill_work_list(cu_q.tolist()), dtype=torch.int32, device=q.device)
        return native().paged_prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, work, scale)
    return ref.paged_prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale)


SKINNY_CONFIGS: dict = {}  # (M, N, K) -> tuned config (0 = hipBLASLt), from a tuning cache


def decode_linear(x, w, b=None):
    """``x @ w^T (+ b)`` for decode-shaped inputs: the weight-streaming MFMA kernels
    (``csrc/skinny_gemm.hip``) where they beat hipBLASLt on uncached weights
    (``profiles/skinny_sweep_r2*.jsonl``): every projection up to 16 tokens (at 16 tokens the
    LDS-staged v2 kernel: QKV 3.78 vs 3.55 TB/s, up 3.89 vs 3.35, down 3.16 vs 2.07) and the
    4096 x 4096 o-projection up to 32; wide projections at 17-32 tokens stay on hipBLASLt, and so
    does the vocabulary projection (out features >= 16384) from 8 tokens (GPT-7B LM head at 16
    tokens: 59.7 vs 68.5 us, ``profiles/decode_gemm_nt_r5.txt``).
    Knob ``skinny_gemm``: ``off`` / ``all`` force the library / kernel path (A/B)."""
    from llmctl.exec.linear import forward_linear

    mode = knobs().skinny_gemm
    M = x.shape[0] if x.dim() == 2 else 0
    tuned = SKINNY_CONFIGS.get((M, w.shape[0], w.shape[1])) if SKINNY_CONFIGS and x.dim() == 2 else None
    if tuned is not None and mode == "auto" and use_native(x):
        if tuned == 0:
            return torch.nn.functional.linear(x, w, b)
        if x.is_contiguous() and w.is_contiguous() and x.dtype == w.dtype == torch.bfloat16:
            return native().skinny_linear_cfg(x, w, b, tuned)
    if (mode != "off" and use_native(x) and x.dim() == 2 and M <= 32 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.shape[0] % 16 == 0 and x.shape[1] % 128 == 0
            and x.is_contiguous() and w.is_contiguous() and (b is None or b.is_contiguous())
            and (mode == "all" or (M <= 16 and not (M >= 8 and w.shape[0] >= 16384))
                 or (w.shape[0] <= 4096 and x.shape[1] <= 4096))):
        return native().skinny_linear(x, w, b)
    return forward_linear(x, w, b)


def _dequant(w, w_scale, dtype):
    """bf16 image of an fp8 (e4m3fn) weight with fp32 row scales (fallback paths)."""
    return w if w_scale is None else (w.float() * w_scale.float().unsqueeze(1)).to(dtype)


def decode_linear_fp8(x, w, w_scale, b=None):
    """``x @ (w * w_scale[:, None])^T (+ b)`` for decode-shaped inputs with fp8 (OCP e4m3fn)
    weights and fp32 row scales (W8A16: ``csrc/skinny_gemm.hip``'s fp8 weight stream, half the
    bytes of the bf16 one)."""
    if decode_fused_ok(x, w):
        return native().decode_linear_fp8(x, w, w_scale, b)
    return decode_linear(x, _dequant(w, w_scale, x.dtype), b)


def decode_fused_ok(x, w) -> bool:
    """Can this decode projection run with a fused epilogue (``csrc/skinny_gemm.hip``: the v2
    weight-streaming GEMM's K-chunk partials summed by a finalize pass that also applies RoPE +
    paged-cache write, SwiGLU or residual + RMSNorm)?  <= 16 tokens, bf16, out features a
    multiple of 64, in features of 128.  Knob ``decode_fused`` off disables (A/B)."""
    return (knobs().decode_fused and use_native(x) and x.dim() == 2
            and 1 <= x.shape[0] <= 16 and x.dtype == torch.bfloat16
            and w.dtype in (torch.bfloat16, torch.float8_e4m3fn) and x.is_contiguous()
            and w.is_contiguous() and w.shape[0] % 64 == 0 and x.shape[1] % 128 == 0)


def decode_qkv_rope_cache(x, w, b, cos, sin, nq: int, nkv: int, positions, k_cache, v_cache, slots,
                          w_scale=None):
    """Decode QKV projection + RoPE + paged-cache write of K/V in one finalize pass; returns
    ``q [T, nq, D]``.  Same result as ``rope_qkv_cache(decode_linear(x, w, b), ...)[0]``.
    ``w_scale``: fp32 row scales of an fp8 (e4m3fn) ``w``."""
    if decode_fused_ok(x, w):
        return native().decode_qkv_rope_cache(x, w, b, cos, sin, nq, nkv, positions.to(torch.int32).contiguous(),
                                              k_cache, v_cache, slots, w_scale)
    return rope_qkv_cache(decode_linear(x, _dequant(w, w_scale, x.dtype), b), cos, sin, nq, nkv, 0, positions,
                          k_cache, v_cache, slots)[0]


def decode_attention_qkv(x, w, b, cos, sin, nq: int, nkv: int, positions, k_cache, v_cache, slots, block_tables,
                         ctx_lens, scale: Optional[float] = None, w_scale=None):
    """Decode QKV projection -> RoPE -> paged-cache write (one finalize pass) -> paged attention.
    (Round 2's variant that summed the projection partials inside the attention kernel measured
    0.1-0.2 ms slower per 16 x 2k GPT-7B step, profiles/serve_r2_session6.txt, and was retired.)"""
    D = w.shape[0] // (nq + 2 * nkv)
    scale = scale if scale is not None else D ** -0.5
    q = decode_qkv_rope_cache(x, w, b, cos, sin, nq, nkv, positions, k_cache, v_cache, slots, w_scale)
    return paged_attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)


def up_swiglu(x, w, b=None):
    """``silu(gate) * up`` of the gate/up projection ``x @ w^T (+ b)`` (w = [W_gate; W_up]).
    Serving prefill: tokens a multiple of 256 run the gemm64 kernel with the SwiGLU in its
    epilogue (``gemm64_swiglu_fwd``: gate and matching up rows in one output tile, only the
    [T, F] activation stored — no gu tensor, no SwiGLU pass).  Knob ``prefill_swiglu`` off
    disables (A/B)."""
    x2 = x.reshape(-1, x.shape[-1])
    T, F = x2.shape[0], w.shape[0] // 2
    if (b is None and knobs().prefill_swiglu and use_native(x) and T % 256 == 0
            and F % 128 == 0 and x2.shape[1] % 128 == 0 and x2.dtype == w.dtype == torch.bfloat16
            and x2.stride(1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and w.is_contiguous()
            and w.data_ptr() % 16 == 0):
        from llmctl.exec.linear import gemm64_config

        act = native().gemm64_swiglu_fwd(x2, w, gemm64_config("fwd", T, 2 * F, x2.shape[1]) % 1000)
        return act.view(*x.shape[:-1], F)
    from llmctl.exec.linear import forward_linear

    return swiglu(forward_linear(x, w, b))


def decode_up_swiglu(x, w, b=None, w_scale=None):
    """Decode gate/up projection with SwiGLU in its finalize pass: ``silu(g) * u`` of
    ``x @ w^T (+ b)`` (gate = first half of the out features)."""
    if decode_fused_ok(x, w):
        return native().decode_up_swiglu(x, w, b, w_scale)
    return swiglu(decode_linear(x, _dequant(w, w_scale, x.dtype), b))


# ----------------------------------------------------------- prefill with the RMSNorm folded in
# Serving prefill (llmctl/serve/engine.py ``_prefill_layers_folded``): rmsnorm(h) * w_n @ W^T equals
# rstd(h)[:, None] * (h @ (W * w_n)^T), so with the norm weight folded into the projection's K
# columns (once, at engine start) the norm reduces to a per-row statistic that the GEMM applies in its
# epilogue, and no normalised copy of h is written or read.

def rms_rstd(x, eps: float):
    """``rsqrt(mean(x^2, -1) + eps)`` per row of a 2-D bf16 ``x`` (fp32 [T])."""
    if use_native(x):
        return native().rms_rstd(x.contiguous(), eps)
    return torch.rsqrt(x.float().pow(2).mean(-1) + eps)


def rowscale_ok(x, w) -> bool:
    """Shapes the row-scaled gemm64 forms take: x [T, K], w [N, K], T and N multiples of 256, K of
    128 and >= 256, bf16 GPU operands, 16-byte aligned rows."""
    return (use_native(x) and x.dim() == 2 and w.dim() == 2 and x.dtype == w.dtype == torch.bfloat16
            and x.shape[0] % 256 == 0 and x.shape[0] > 0 and w.shape[0] % 256 == 0 and x.shape[1] == w.shape[1]
            and x.shape[1] % 128 == 0 and x.shape[1] >= 256 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and w.is_contiguous() and w.data_ptr() % 16 == 0)


def linear_rowscale(x, w, rstd):
    """``(x @ w^T) * rstd[:, None]`` rounded once to bf16 (gemm64 persistent kernel, row scale in
    its epilogue)."""
    if rowscale_ok(x, w):
        from llmctl.exec.linear import gemm64_config

        return native().gemm64_rs(x, w, rstd, gemm64_config("fwd", x.shape[0], w.shape[0], x.shape[1]))
    return ((x.float() @ w.float().t()) * rstd.float()[:, None]).to(x.dtype)


def up_swiglu_rowscale(x, w, rstd):
    """``silu(g) * u`` of ``(x @ w^T) * rstd[:, None]`` (w = [W_gate; W_up]): the SwiGLU and the row
    scale in the gate/up GEMM's epilogue."""
    F = w.shape[0] // 2
    if rowscale_ok(x, w) and F % 128 == 0:
        from llmctl.exec.linear import gemm64_config

        return native().gemm64_swiglu_fwd(x, w, gemm64_config("fwd", x.shape[0], w.shape[0], x.shape[1]) % 1000, rstd)
    gu = ((x.float() @ w.float().t()) * rstd.float()[:, None]).to(x.dtype)
    return swiglu(gu)


def linear_acc_(x, w, out):
    """``out += x @ w^T`` in place (the residual add riding on the projection's epilogue)."""
    if rowscale_ok(x, w) and out.is_contiguous() and out.shape == (x.shape[0], w.shape[0]):
        from llmctl.exec.linear import gemm64_config

        native().gemm64_ex(x, w, out, False, False, True, gemm64_config("fwd", x.shape[0], w.shape[0], x.shape[1]))
        return out
    return out.addmm_(x, w.t())


def decode_linear_add_rmsnorm(x, w, b, residual, norm_w, eps: float, w_scale=None):
    """Decode row projection + residual add + RMSNorm in one finalize pass:
    ``(rmsnorm(y + residual) * norm_w, y + residual)`` with ``y = x @ w^T (+ b)``."""
    if decode_fused_ok(x, w) and w.shape[0] <= 16384:
        return native().decode_linear_add_rmsnorm(x, w, b, residual, norm_w, eps, w_scale)
    y = decode_linear(x, _dequant(w, w_scale, x.dtype), b)
    return add_rmsnorm(y, residual, norm_w, eps)


def sample(logits, temperature, top_k, top_p, uniform):
    if use_native(logits):
        return native().sample(logits, temperature, top_k, top_p, uniform)
    return ref.sample(logits, temperature, top_k, top_p, uniform)


__all__ = [
    "transpose_",
    "rmsnorm", "add_rmsnorm", "layernorm", "add_layernorm", "rope_qkv", "flash_attention", "rope_flash_attention",
    "swiglu",
    "gelu", "cross_entropy", "adamw_step_", "l2norm_sq", "kv_cache_write", "paged_attention_decode",
    "sample", "decode_linear", "decode_linear_fp8", "decode_fused_ok", "decode_qkv_rope_cache", "decode_up_swiglu", "decode_attention_qkv", "up_swiglu",
    "decode_linear_add_rmsnorm", "rope_qkv_cache", "paged_prefill_attention", "prefill_work_list", "attn_merge_",
    "rms_rstd", "rowscale_ok", "linear_rowscale", "up_swiglu_rowscale", "linear_acc_",
]
