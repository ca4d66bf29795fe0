"""Kernel plugin group: named HIP kernels (``torch.ops.llmctl.*``) with their fp32 oracles.
The reference's docs name ``flash_attention_v3`` / ``fused_rmsnorm`` plugins
(``USER_GUIDE.md:263-270``); here they resolve to the real CDNA4 kernels."""

from __future__ import annotations


def _ops():
    from llmctl import ops

    return ops


KERNELS = {
    "flash_attention": lambda: _ops().flash_attention,
    "flash_attention_v3": lambda: _ops().flash_attention,  # reference plugin name
    "fused_rmsnorm": lambda: _ops().rmsnorm,
    "fused_add_rmsnorm": lambda: _ops().add_rmsnorm,
    "rope": lambda: _ops().rope_qkv,
    "swiglu": lambda: _ops().swiglu,
    "cross_entropy": lambda: _ops().cross_entropy,
    "fused_adamw": lambda: _ops().adamw_step_,
    "paged_attention": lambda: _ops().paged_attention_decode,
    "sampling": lambda: _ops().sample,
}


def register(reg) -> None:
    for k, f in KERNELS.items():
        reg.add("kernels", k, f)
