"""GPU telemetry for AMD Instinct: utilisation, memory, power, temperature.

Order of sources: the ``amdsmi`` Python bindings (ROCm), the amdgpu sysfs nodes
(``gpu_busy_percent``, ``mem_info_vram_used``, hwmon power/temp), then torch's allocator
view.  Replaces the reference's hard-coded ``gpu_utilization = 0.0`` placeholder
(``observability.py:135``) and its NVML usage.
"""

from __future__ import annotations

import glob
import os
from typing import Any, Dict, List


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _sysfs_cards() -> List[str]:
    cards = []
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        vendor = _read(os.path.join(dev, "vendor"))
        if vendor == "0x1002" and os.path.exists(os.path.join(dev, "gpu_busy_percent")):
            cards.append(dev)
    return cards


def gpu_stats() -> List[Dict[str, Any]]:
    out: List[Dict[str, Any]] = []
    try:  # amdsmi
        import amdsmi  # type: ignore

        amdsmi.amdsmi_init()
        try:
            for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
                act = amdsmi.amdsmi_get_gpu_activity(h)
                vram = amdsmi.amdsmi_get_gpu_vram_usage(h)
                d = {"id": i, "utilization": float(act.get("gfx_activity", 0)),
                     "memory_used_gb": float(vram.get("vram_used", 0)) / 1024,
                     "memory_total_gb": float(vram.get("vram_total", 0)) / 1024}
                try:
                    d["power_w"] = float(amdsmi.amdsmi_get_power_info(h).get("average_socket_power", 0))
                except Exception:
                    pass
                out.append(d)
        finally:
            amdsmi.amdsmi_shut_down()
        if out:
            return out
    except Exception:
        pass
    for i, dev in enumerate(_sysfs_cards()):
        d: Dict[str, Any] = {"id": i, "utilization": float(_read(os.path.join(dev, "gpu_busy_percent")) or 0)}
        used = _read(os.path.join(dev, "mem_info_vram_used"))
        tot = _read(os.path.join(dev, "mem_info_vram_total"))
        if used and tot:
            d["memory_used_gb"] = int(used) / 1e9
            d["memory_total_gb"] = int(tot) / 1e9
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            p = _read(os.path.join(hw, "power1_average")) or _read(os.path.join(hw, "power1_input"))
            if p:
                d["power_w"] = int(p) / 1e6
            t = _read(os.path.join(hw, "temp1_input"))
            if t:
                d["temperature_c"] = int(t) / 1e3
        out.append(d)
    if out:
        return out
    try:
        import torch

        if torch.cuda.is_available():
            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                out.append({"id": i, "utilization": 0.0, "memory_used_gb": (total - free) / 1e9,
                            "memory_total_gb": total / 1e9})
    except Exception:
        pass
    return out
