"""Test utilities shipped with the framework: a multi-process gloo harness and rank workers
used by the distributed-equivalence tests (the reference has no distributed tests at all,
SURVEY §4)."""
