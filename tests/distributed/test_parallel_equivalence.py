"""DP / ZeRO / TP / SP (/ PP) produce the same training trajectory as one process (gloo, fp32)."""

import pytest
import torch

from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import pp_tied_fresh, train_layout, train_reference, zero3_pp_tied_error

STEPS = 3


@pytest.fixture(scope="module")
def ref_dp2():
    return train_reference(STEPS, dp=2)


@pytest.fixture(scope="module")
def ref_dp1():
    return train_reference(STEPS, dp=1)


def _close(state_a, state_b, atol=1.5e-3, rtol=1e-3):
    """Adam normalises near-zero gradients, so fp32 summation-order noise can move single
    elements by up to ~lr; a layout bug moves whole tensors by >= lr (1e-3)."""
    assert state_a.keys() == state_b.keys()
    for k in state_a:
        a, b = state_a[k].float(), state_b[k].float()
        assert a.shape == b.shape, k
        d = (a - b).abs()
        assert torch.allclose(a, b, atol=atol, rtol=rtol), f"{k}: max|d|={d.max().item():.3e}"
        assert d.mean().item() < 2e-6, f"{k}: mean|d|={d.mean().item():.3e}"


def _losses_close(a, b, tol=1e-4):
    for x, y in zip(a, b):
        assert abs(x - y) < tol, (a, b)


@pytest.mark.parametrize("zero", [0, 1, 2])
def test_dp2_matches_single(ref_dp2, zero):
    out = run_ranks(train_layout, 2, STEPS, {"zero": zero})
    _losses_close(out[0]["losses"], ref_dp2["losses"])
    _close(out[0]["state"], ref_dp2["state"])


@pytest.mark.parametrize("sp", [False, True])
def test_tp2_matches_single(ref_dp1, sp):
    out = run_ranks(train_layout, 2, STEPS, {"tp": 2, "sp": sp})
    _losses_close(out[0]["losses"], ref_dp1["losses"])
    _close(out[0]["state"], ref_dp1["state"])


@pytest.mark.parametrize("world", [2, 3])
def test_async_tp_linears_match_unsharded(world):
    """AG-GEMM / GEMM-RS ring decompositions (fwd + both grads) equal the unsharded products."""
    from llmctl.testing.workers import async_tp_check

    out = run_ranks(async_tp_check, world)
    for r in range(world):
        for name in ("y", "dx", "dw1", "db1", "dw2"):
            assert torch.allclose(out[r][name], out[r][name + "_ref"], atol=1e-5, rtol=1e-4), (r, name)


def test_tp2_sp_plain_collectives_match_single(ref_dp1, monkeypatch):
    """Knob async_tp off: Megatron-SP with the synchronous all-gather / reduce-scatter."""
    monkeypatch.setenv("LLMCTL_KNOBS", "async_tp=0")
    out = run_ranks(train_layout, 2, STEPS, {"tp": 2, "sp": True})
    _losses_close(out[0]["losses"], ref_dp1["losses"])
    _close(out[0]["state"], ref_dp1["state"])


def test_tp2_dp2_zero1_matches_single(ref_dp2):
    out = run_ranks(train_layout, 4, STEPS, {"tp": 2, "zero": 1, "sp": True})
    _losses_close(out[0]["losses"], ref_dp2["losses"])
    _close(out[0]["state"], ref_dp2["state"])


def test_selective_and_full_recompute_match(ref_dp1):
    for ac in ("selective", "full"):
        out = run_ranks(train_layout, 1, STEPS, {"ac": ac})
        _losses_close(out[0]["losses"], ref_dp1["losses"])
        _close(out[0]["state"], ref_dp1["state"])


@pytest.fixture(scope="module")
def ref_dp1_m4():
    return train_reference(STEPS, dp=1, micro_per_rank=4)


@pytest.fixture(scope="module")
def ref_dp2_m4():
    return train_reference(STEPS, dp=2, micro_per_rank=4)


def test_pp2_1f1b_matches_single(ref_dp1_m4):
    out = run_ranks(train_layout, 2, STEPS, {"pp": 2, "microbatches": 4})
    _losses_close(out[0]["losses"], ref_dp1_m4["losses"])
    _close(out[0]["state"], ref_dp1_m4["state"])


@pytest.mark.parametrize("staging", [False, True])
def test_pp2_tp2_sp_matches_single(ref_dp1_m4, staging):
    """TP2 x PP2 with SP (async-TP ring steps); ``staging``: with the one-GPU rehearsal's
    host-staging patches installed, which must pass CPU tensors through untouched."""
    out = run_ranks(train_layout, 4, STEPS, {"pp": 2, "tp": 2, "sp": True, "microbatches": 4, "staging": staging})
    _losses_close(out[0]["losses"], ref_dp1_m4["losses"])
    _close(out[0]["state"], ref_dp1_m4["state"])


def test_pp2_dp2_zero1_matches_single(ref_dp2_m4):
    out = run_ranks(train_layout, 4, STEPS, {"pp": 2, "zero": 1, "microbatches": 4})
    _losses_close(out[0]["losses"], ref_dp2_m4["losses"])
    _close(out[0]["state"], ref_dp2_m4["state"])


def test_pp2_tied_embeddings_matches_single():
    """GPT-2 style tied LM head split over two stages: the last stage's copy gets the summed
    gradient and the clip norm counts the matrix once."""
    ref = train_reference(STEPS, dp=1, model="tiny-tied", micro_per_rank=4)
    out = run_ranks(train_layout, 2, STEPS, {"pp": 2, "microbatches": 4}, "tiny-tied")
    _losses_close(out[0]["losses"], ref["losses"])
    _close(out[0]["state"], ref["state"])


@pytest.mark.parametrize("pp,vstages,micro", [(2, 2, 4), (2, 4, 2), (4, 2, 4)])
def test_interleaved_pp_matches_single(pp, vstages, micro):
    """Virtual pipeline stages (interleaved 1F1B): rank r owns chunks r, r+pp, ... of an
    8-layer model; the trajectory equals one process accumulating the same micro-batches."""
    ref = train_reference(STEPS, dp=1, model="tiny-deep", micro_per_rank=micro)
    out = run_ranks(train_layout, pp, STEPS, {"pp": pp, "vstages": vstages, "microbatches": micro}, "tiny-deep")
    _losses_close(out[0]["losses"], ref["losses"])
    _losses_close([out[0]["eval"]], [ref["eval"]])
    _close(out[0]["state"], ref["state"])
    # bounded send backlog: at most INFLIGHT_ROUNDS rounds x (one activation + one gradient)
    # sent tensors alive on any rank, not every micro-batch's (M * V) for the whole step
    from llmctl.parallel.pipeline import PipelineSchedule

    for o in out:
        assert o["peak_inflight"] is not None and o["peak_inflight"] <= 2 * PipelineSchedule.INFLIGHT_ROUNDS


def test_interleaved_pp2_dp2_zero1_matches_single():
    ref = train_reference(STEPS, dp=2, model="tiny-deep", micro_per_rank=4)
    out = run_ranks(train_layout, 4, STEPS, {"pp": 2, "vstages": 2, "zero": 1, "microbatches": 4}, "tiny-deep")
    _losses_close(out[0]["losses"], ref["losses"])
    _close(out[0]["state"], ref["state"])


def test_pp2_tied_fresh_init_stays_tied():
    """From the engine's own init (no load_full_state_dict re-seeding the fp32 masters), the
    last stage's lm_head copy equals stage 0's embed after optimizer steps."""
    out = run_ranks(pp_tied_fresh, 2, 2)
    assert torch.equal(out[0]["tied"], out[1]["tied"])


def test_zero3_pp_tied_rejected():
    out = run_ranks(zero3_pp_tied_error, 4)
    assert all("ZeRO-3" in o["error"] for o in out), out


@pytest.mark.parametrize("zero", [0, 1, 2])
def test_pp2_tied_dp2_matches_single(zero):
    ref = train_reference(STEPS, dp=2, model="tiny-tied", micro_per_rank=4)
    out = run_ranks(train_layout, 4, STEPS, {"pp": 2, "microbatches": 4, "zero": zero}, "tiny-tied")
    _losses_close(out[0]["losses"], ref["losses"])
    _close(out[0]["state"], ref["state"])


@pytest.mark.parametrize("cp_mode", ["ulysses", "ring"])
def test_pp2_cp2_matches_single(ref_dp1_m4, cp_mode):
    out = run_ranks(train_layout, 4, STEPS, {"pp": 2, "cp": 2, "cp_mode": cp_mode, "microbatches": 4})
    _losses_close(out[0]["losses"], ref_dp1_m4["losses"])
    _losses_close([out[0]["eval"]], [ref_dp1_m4["eval"]])  # CP-split, pipelined evaluation
    _close(out[0]["state"], ref_dp1_m4["state"])


def test_pp2_packed_sequences_matches_single():
    """Packed documents: every stage rebuilds the document map, the last masks separators."""
    ref = train_reference(STEPS, dp=1, micro_per_rank=4, pack=True)
    out = run_ranks(train_layout, 2, STEPS, {"pp": 2, "microbatches": 4, "pack": True})
    _losses_close(out[0]["losses"], ref["losses"])
    _losses_close([out[0]["eval"]], [ref["eval"]])
    _close(out[0]["state"], ref["state"])


def test_zero3_dp2_matches_single(ref_dp2):
    out = run_ranks(train_layout, 2, STEPS, {"zero": 3})
    _losses_close(out[0]["losses"], ref_dp2["losses"])
    _close(out[0]["state"], ref_dp2["state"])


def test_zero3_pp2_dp2_matches_single(ref_dp2_m4):
    out = run_ranks(train_layout, 4, STEPS, {"zero": 3, "pp": 2, "microbatches": 4})
    _losses_close(out[0]["losses"], ref_dp2_m4["losses"])
    _losses_close([out[0]["eval"]], [ref_dp2_m4["eval"]])  # gathered root unit on both stages
    _close(out[0]["state"], ref_dp2_m4["state"])


def test_cp2_ulysses_matches_single(ref_dp1):
    """Context parallel: each rank holds half of every sequence; all-to-all around attention."""
    out = run_ranks(train_layout, 2, STEPS, {"cp": 2})
    _losses_close(out[0]["losses"], ref_dp1["losses"])
    _losses_close([out[0]["eval"]], [ref_dp1["eval"]])
    _close(out[0]["state"], ref_dp1["state"])


def test_cp2_ring_matches_single(ref_dp1):
    """Ring attention (zigzag pieces, the default): K/V chunks travel around the CP ring."""
    out = run_ranks(train_layout, 2, STEPS, {"cp": 2, "cp_mode": "ring"})
    _losses_close(out[0]["losses"], ref_dp1["losses"])
    _losses_close([out[0]["eval"]], [ref_dp1["eval"]])
    _close(out[0]["state"], ref_dp1["state"])


def test_cp2_ring_contiguous_matches_single(ref_dp1, monkeypatch):
    monkeypatch.setenv("LLMCTL_KNOBS", "cp_zigzag=0")
    out = run_ranks(train_layout, 2, STEPS, {"cp": 2, "cp_mode": "ring"})
    _losses_close(out[0]["losses"], ref_dp1["losses"])
    _close(out[0]["state"], ref_dp1["state"])


def test_cp2_dp2_zero1_matches_single(ref_dp2):
    out = run_ranks(train_layout, 4, STEPS, {"cp": 2, "zero": 1})
    _losses_close(out[0]["losses"], ref_dp2["losses"])
    _close(out[0]["state"], ref_dp2["state"])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("zigzag", [False, True])
def test_ring_attention_matches_full_attention(world, zigzag):
    """Ring attention (fwd + bwd, GQA) over 2 / 3 CP ranks equals full causal attention, with
    contiguous chunks and with the load-balanced zigzag pieces."""
    from llmctl.testing.workers import ring_attention_check

    out = run_ranks(ring_attention_check, world, zigzag)
    for r in range(world):
        for name in ("o", "dq", "dk", "dv"):
            assert torch.allclose(out[r][name], out[r][name + "_ref"], atol=2e-5, rtol=1e-4), (r, name)


@pytest.fixture(scope="module")
def ref_moe_dp2():
    return train_reference(STEPS, 2, model="tiny-moe")


@pytest.mark.parametrize("ep,zero", [(1, 1), (2, 0), (2, 1)])
def test_moe_expert_parallel_matches_single(ref_moe_dp2, ep, zero):
    """Mixture of experts: DP=2 with the experts sharded over EP ranks (all-to-all token
    dispatch, expert grads reduced over expert-DP) follows the single-process trajectory."""
    out = run_ranks(train_layout, 2, STEPS, {"ep": ep, "zero": zero}, "tiny-moe")
    _losses_close(out[0]["losses"], ref_moe_dp2["losses"])
    _close(out[0]["state"], ref_moe_dp2["state"])


def test_moe_dp4_ep2_zero1_matches_single():
    """EP=2 inside DP=4: two EP blocks, expert gradients all-reduced over expert-DP pairs."""
    ref = train_reference(STEPS, 4, model="tiny-moe")
    out = run_ranks(train_layout, 4, STEPS, {"ep": 2, "zero": 1}, "tiny-moe")
    _losses_close(out[0]["losses"], ref["losses"])
    _close(out[0]["state"], ref["state"])


@pytest.mark.parametrize("zero", [0, 1])
def test_dp2_tp2_multi_param_buckets_match_single(zero):
    """DP x TP on the 8-layer model, where a DP bucket holds several GEMM-written (sinked)
    weights (wo + wqkv): the bucket must launch only after its LAST gradient is written.
    Regression: autograd also runs a sinked weight's post-accumulate hook (grad None), the sync
    engine counted it twice and all-reduced the bucket before wqkv's gradient existed."""
    ref = train_reference(STEPS, dp=2, model="tiny-deep")
    out = run_ranks(train_layout, 4, STEPS, {"tp": 2, "zero": zero}, "tiny-deep")
    _losses_close(out[0]["losses"], ref["losses"])
    _close(out[0]["state"], ref["state"])
