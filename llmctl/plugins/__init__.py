"""Plugins: autotuner + registries for the entry-point groups the reference declares
(``pyproject.toml:77-81``: kernels, quantizers, exporters, schedulers)."""

from .autotuning import AutoTuner, TuningConfig, TuningResult, create_auto_tuner

__all__ = ["AutoTuner", "TuningConfig", "TuningResult", "create_auto_tuner"]
