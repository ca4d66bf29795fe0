"""Small shared utilities (device/env/seed/logging helpers)."""

from .env import dist_env, is_rocm_gpu_available, local_device
from .seed import set_seed

__all__ = ["dist_env", "is_rocm_gpu_available", "local_device", "set_seed"]
