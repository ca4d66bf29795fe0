"""Weight quantizers (plugin group ``quantizers``).

* ``int8``  — symmetric per-output-channel absmax round-to-nearest (int8 + fp32 scales);
* ``int4``  — the same at 4 bits, two values packed per byte;
* ``fp8``   — OCP e4m3 (``torch.float8_e4m3fn``, the gfx950 MFMA fp8 format — NOT the
  MI300 ``fnuz`` variant) with per-channel fp32 scales.
The reference's names ``int8-awq`` / ``int4-gptq`` are accepted as aliases of RTN int8 /
int4: AWQ/GPTQ need calibration activations that an offline export does not have, so the
export records ``method: rtn`` and warns.
"""

from __future__ import annotations

from typing import Dict, Tuple

import torch

ALIASES = {"int8-awq": "int8", "int4-gptq": "int4"}


def _per_channel_absmax(w: torch.Tensor) -> torch.Tensor:
    return w.float().abs().amax(dim=1, keepdim=True).clamp_min(1e-12)


def quantize_int8(w: torch.Tensor) -> Dict[str, torch.Tensor]:
    s = _per_channel_absmax(w) / 127.0
    q = torch.clamp(torch.round(w.float() / s), -127, 127).to(torch.int8)
    return {"qweight": q, "scale": s.squeeze(1)}


def quantize_int4(w: torch.Tensor) -> Dict[str, torch.Tensor]:
    s = _per_channel_absmax(w) / 7.0
    q = torch.clamp(torch.round(w.float() / s), -8, 7).to(torch.int8)
    if q.shape[1] % 2:
        q = torch.nn.functional.pad(q, (0, 1))
    lo = (q[:, 0::2] & 0xF).to(torch.uint8)
    hi = (q[:, 1::2] & 0xF).to(torch.uint8)
    return {"qweight": lo | (hi << 4), "scale": s.squeeze(1)}


def quantize_fp8(w: torch.Tensor) -> Dict[str, torch.Tensor]:
    fmax = 448.0  # e4m3fn max
    s = _per_channel_absmax(w) / fmax
    q = (w.float() / s).clamp(-fmax, fmax).to(torch.float8_e4m3fn)
    return {"qweight": q, "scale": s.squeeze(1)}


def dequantize(name: str, t: Dict[str, torch.Tensor], shape: Tuple[int, int]) -> torch.Tensor:
    name = ALIASES.get(name, name)
    s = t["scale"].float().unsqueeze(1)
    if name == "int8":
        return t["qweight"].float() * s
    if name == "fp8":
        return t["qweight"].float() * s
    if name == "int4":
        p = t["qweight"]
        lo = (p & 0xF).to(torch.int8)
        hi = ((p >> 4) & 0xF).to(torch.int8)
        lo = torch.where(lo > 7, lo - 16, lo)
        hi = torch.where(hi > 7, hi - 16, hi)
        q = torch.stack([lo, hi], dim=2).reshape(p.shape[0], -1)[:, :shape[1]]
        return q.float() * s
    raise KeyError(name)


QUANTIZERS = {"int8": quantize_int8, "int4": quantize_int4, "fp8": quantize_fp8}


def register(reg) -> None:
    for k, fn in QUANTIZERS.items():
        reg.add("quantizers", k, fn)
    for alias, target in ALIASES.items():
        reg.add("quantizers", alias, QUANTIZERS[target])
