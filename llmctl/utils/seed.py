"""Seeding / determinism (the reference never applies its --seed: SURVEY App. C #5)."""

from __future__ import annotations

import os
import random


def set_seed(seed: int, deterministic: bool = False) -> None:
    import numpy as np
    import torch

    random.seed(seed)
    np.random.seed(seed % (2**32))
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    os.environ.setdefault("PYTHONHASHSEED", str(seed))
    if deterministic:
        # HIP analogue of CUDA_LAUNCH_BLOCKING; our own kernels are deterministic by design
        # (no float atomics on the training path except the flash-attn dQ sum, which has a
        # deterministic mode).
        os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
        os.environ["LLMCTL_DETERMINISTIC"] = "1"
        torch.use_deterministic_algorithms(True, warn_only=True)
