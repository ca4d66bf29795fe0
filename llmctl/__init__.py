"""llmctl — MI355X-native distributed LLM training and inference system.

Capability parity target: ambicuity/Distributed-LLM-Training-and-Inference-System
(`llmctl/__init__.py:5` there declares version 0.1.0).  This package is a from-scratch
re-design for AMD Instinct MI355X (gfx950 / CDNA4): hand-written HIP kernels for the hot
ops (``llmctl.ops``), RCCL-over-xGMI collectives (``llmctl.comms``), and a native C++
runtime for the host-side allocator / scheduler / data loader (``llmctl.native``).
"""

__version__ = "0.2.0"
__all__ = ["__version__"]
