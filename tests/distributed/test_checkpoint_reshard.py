"""Checkpoint written under one parallel layout resumes under another with the fp32 master
and Adam moments resharded (not re-initialised): the trajectory must equal one process that
saw the same global batches (gloo, fp32)."""

import pytest
import torch

from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import ckpt_resume_phase, ckpt_save_phase, train_reference_schedule


def _close(a, b, atol=1.5e-3, rtol=1e-3):
    assert a.keys() == b.keys()
    for k in a:
        x, y = a[k].float(), b[k].float()
        d = (x - y).abs()
        assert torch.allclose(x, y, atol=atol, rtol=rtol), f"{k}: max|d|={d.max().item():.3e}"
        assert d.mean().item() < 2e-6, f"{k}: mean|d|={d.mean().item():.3e}"


@pytest.mark.parametrize("src,dst", [
    ({"tp": 1, "zero": 1}, {"tp": 2, "zero": 0}),   # DP=2 ZeRO-1 shards -> TP=2 splits
    ({"tp": 2, "zero": 0}, {"tp": 1, "zero": 2}),   # TP=2 -> DP=2 ZeRO-2
    ({"tp": 1, "pp": 2, "microbatches": 1}, {"tp": 1, "zero": 1}),  # PP=2 -> DP=2 ZeRO-1
])
def test_resume_across_layouts(tmp_path, src, dst):
    run_ranks(ckpt_save_phase, 2, src, 2, str(tmp_path))
    out = run_ranks(ckpt_resume_phase, 2, dst, 2, 1, str(tmp_path))
    dp = lambda L: 2 // (L.get("tp", 1) * L.get("pp", 1))  # noqa: E731
    ref = train_reference_schedule([dp(src), dp(src), dp(dst)])
    _close(out[0]["state"], ref["state"])


def test_resume_tied_pp1_checkpoint_under_pp2(tmp_path):
    """A tied model saved under PP=1 (only ``embed`` on disk) resumes under PP=2: the last
    stage's lm_head copy and its optimizer state come from ``embed``."""
    run_ranks(ckpt_save_phase, 2, {"tp": 1, "zero": 1}, 2, str(tmp_path), "tiny-tied")
    out = run_ranks(ckpt_resume_phase, 2, {"tp": 1, "pp": 2, "microbatches": 1}, 2, 1, str(tmp_path), "tiny-tied")
    ref = train_reference_schedule([2, 2, 1], model="tiny-tied")
    _close(out[0]["state"], ref["state"])
