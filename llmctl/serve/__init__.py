"""Serving: paged KV cache, continuous batching, hipGraph decode, FastAPI server.
Exports mirror the reference (``serve/__init__.py:3-5``)."""

from .server import InferenceServer, create_inference_server

__all__ = ["InferenceServer", "create_inference_server"]
