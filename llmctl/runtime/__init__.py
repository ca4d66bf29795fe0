"""Runtime: launchers/orchestrator (process boundary), training engine, flat params,
optimizer.  Mirrors the reference's ``llmctl/runtime/__init__.py:3-12`` exports."""

from .engine import TrainingConfig, TrainingEngine, create_training_config
from .launcher import LaunchConfig, ProcessOrchestrator, create_launcher

__all__ = ["LaunchConfig", "ProcessOrchestrator", "create_launcher", "TrainingEngine", "TrainingConfig",
           "create_training_config"]
