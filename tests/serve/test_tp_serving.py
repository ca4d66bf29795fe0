"""Tensor-parallel serving (llmctl.serve.tp) on CPU/gloo: TP=2 must generate exactly the
tokens of the single-process engine (same random-init model, greedy)."""

from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import serve_generate


def test_tp2_serving_matches_single_process():
    ref = serve_generate(0, 1)
    out = run_ranks(serve_generate, 2)
    assert out[0]["tokens"] == ref["tokens"]
    assert out[0]["kv_heads_local"] * 2 == ref["kv_heads_local"]  # each rank caches half the KV heads


def _row_err(a, b):
    return ((a - b).abs().amax(dim=1) / b.abs().amax(dim=1).clamp_min(1e-6)).max().item()


def test_tp2_sequence_prefill_matches_single_process():
    """``TPInferenceEngine.prefill`` called with ``Sequence`` objects (whole prompts)."""
    ref = serve_generate(0, 1)
    out = run_ranks(serve_generate, 2)
    assert out[0]["prefill_logits"].shape == ref["prefill_logits"].shape == (2, 512)
    assert _row_err(out[0]["prefill_logits"], ref["prefill_logits"]) < 1e-4


def test_tp8_serving_matches_single_process():
    """BASELINE config #5's degree: 8 ranks, 8 query / 8 KV heads (one of each per rank),
    vocab-parallel embedding and LM head over 8 shards."""
    ref = serve_generate(0, 1, 8, "tiny-wide")
    out = run_ranks(serve_generate, 8, 8, "tiny-wide", timeout=400)
    assert out[0]["kv_heads_local"] == 1 and ref["kv_heads_local"] == 8
    assert _row_err(out[0]["prefill_logits"], ref["prefill_logits"]) < 1e-4
    assert out[0]["tokens"] == ref["tokens"]
