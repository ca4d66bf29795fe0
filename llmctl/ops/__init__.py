"""Hand-written CDNA4 (gfx950) HIP kernels for the hot ops + their autograd wrappers.

Kernel sources live in ``llmctl/ops/csrc/*.hip`` and build in-tree into
``llmctl/ops/_llmctl_hip.so`` (``python -m llmctl.ops.build``).  See ``functional.py`` for
the op surface and ``ref.py`` for the fp32 oracles.
"""

from . import ref
from ._lib import available as native_available
from .functional import (
    adamw_step_,
    add_layernorm,
    add_rmsnorm,
    cross_entropy,
    decode_attention_qkv,
    decode_fused_ok,
    decode_linear,
    decode_linear_fp8,
    decode_linear_add_rmsnorm,
    decode_qkv_rope_cache,
    decode_up_swiglu,
    flash_attention,
    gelu,
    kv_cache_write,
    l2norm_sq,
    layernorm,
    linear_acc_,
    linear_rowscale,
    paged_attention_decode,
    paged_prefill_attention,
    attn_merge_,
    prefill_work_list,
    rms_rstd,
    rmsnorm,
    rope_qkv,
    rope_flash_attention,
    rope_qkv_cache,
    sample,
    swiglu,
    transpose_,
    up_swiglu,
    up_swiglu_rowscale,
)

__all__ = [
    "ref", "native_available", "adamw_step_", "add_layernorm", "add_rmsnorm", "cross_entropy", "decode_linear",
    "decode_attention_qkv", "decode_fused_ok", "decode_linear_add_rmsnorm", "decode_qkv_rope_cache", "decode_up_swiglu",
    "flash_attention", "gelu", "kv_cache_write", "l2norm_sq", "layernorm", "paged_attention_decode",
    "paged_prefill_attention", "prefill_work_list", "attn_merge_",
    "rmsnorm", "rope_qkv", "rope_flash_attention", "rope_qkv_cache", "sample", "swiglu", "transpose_", "up_swiglu",
    "rms_rstd", "linear_rowscale", "up_swiglu_rowscale", "linear_acc_",
]
