"""Metrics: FLOPs/MFU, observability (Prometheus/OTel/JSONL), health monitoring."""
