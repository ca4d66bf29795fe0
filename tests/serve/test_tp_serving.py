"""Tensor-parallel serving (llmctl.serve.tp) on CPU/gloo: TP=2 must generate exactly the
tokens of the single-process engine (same random-init model, greedy)."""

from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import serve_generate


def test_tp2_serving_matches_single_process():
    ref = serve_generate(0, 1)
    out = run_ranks(serve_generate, 2)
    assert out[0]["tokens"] == ref["tokens"]
    assert out[0]["kv_heads_local"] * 2 == ref["kv_heads_local"]  # each rank caches half the KV heads
