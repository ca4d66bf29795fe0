"""Process / device environment helpers.

One process per GPU: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT come from
torchrun (or our own launcher, ``llmctl.runtime.launcher``).  On ROCm the HIP device is
exposed through the ``torch.cuda`` namespace and the ``"nccl"`` backend is RCCL.
"""

from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class DistEnv:
    rank: int
    local_rank: int
    world_size: int
    master_addr: str
    master_port: int

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


def dist_env() -> DistEnv:
    return DistEnv(
        rank=int(os.environ.get("RANK", "0")),
        local_rank=int(os.environ.get("LOCAL_RANK", "0")),
        world_size=int(os.environ.get("WORLD_SIZE", "1")),
        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
        master_port=int(os.environ.get("MASTER_PORT", "29500")),
    )


def is_rocm_gpu_available() -> bool:
    try:
        import torch
    except Exception:  # pragma: no cover
        return False
    return bool(torch.cuda.is_available() and getattr(torch.version, "hip", None))


def local_device(prefer: str = "auto"):
    """Return the torch.device this process should compute on."""
    import torch

    if prefer == "cpu":
        return torch.device("cpu")
    if torch.cuda.is_available():
        return torch.device("cuda", dist_env().local_rank % max(torch.cuda.device_count(), 1))
    if prefer in ("cuda", "gpu", "hip"):
        raise RuntimeError("a GPU was requested but torch.cuda.is_available() is False")
    return torch.device("cpu")
