"""Scheduler plugin group: serving batch schedulers and LR schedules."""

from __future__ import annotations


def register(reg) -> None:
    from llmctl.runtime.optimizer import LRSchedule
    from llmctl.serve.scheduler import ContinuousBatchScheduler

    reg.add("schedulers", "dynamic", lambda kv, **kw: ContinuousBatchScheduler(kv, policy="dynamic", **kw))
    reg.add("schedulers", "static", lambda kv, **kw: ContinuousBatchScheduler(kv, policy="static", **kw))
    for kind in ("linear", "cosine", "constant"):
        reg.add("schedulers", f"lr-{kind}", lambda base_lr, kind=kind, **kw: LRSchedule(base_lr, kind, **kw))
