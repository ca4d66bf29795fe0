"""FLOPs / MFU accounting against MI355X dense peaks (no sparsity)."""

from __future__ import annotations

import torch

# dense peak per GPU (MI355X_MICROARCH.md: ~2.5 PF bf16/fp16, ~5 PF fp8, 157 TF fp32)
MI355X_PEAK = {torch.bfloat16: 2.5e15, torch.float16: 2.5e15, torch.float32: 157.3e12}
MI355X_HBM_BW = 8.0e12  # spec; ~6.3e12 achievable
MI355X_HBM_BYTES = 288e9
MI355X_XGMI_LINKS = 7
MI355X_XGMI_LINK_BW = 153e9


def device_peak_flops(dtype=torch.bfloat16) -> float:
    try:
        name = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
    except Exception:
        name = ""
    peak = MI355X_PEAK.get(dtype, 2.5e15)
    if name and not name.startswith("gfx950"):
        # unknown part: keep MI355X numbers but callers can tell from the arch string
        pass
    return peak


def mfu(tokens_per_sec: float, flops_per_token: float, n_gpus: int, dtype=torch.bfloat16) -> float:
    return tokens_per_sec * flops_per_token / (device_peak_flops(dtype) * max(n_gpus, 1))
