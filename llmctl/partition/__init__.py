"""Partitioner: cost model + plan search + shard maps (reference: plan.py:18-202)."""
