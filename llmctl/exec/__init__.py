"""Execution layer: grad-sink linear, selective recompute, HIP-graph capture, streams."""

from .linear import GradSink, linear, weight_grad

__all__ = ["GradSink", "linear", "weight_grad"]
