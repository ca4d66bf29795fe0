"""Benchmark / evaluation / tracing implementations behind `llmctl bench|eval|trace`."""
