"""Self-checks of the kernel tests' error criterion (CPU): a single corrupted tile passes a
tensor-wide Frobenius test but fails the per-row check the GPU kernel tests gate on."""

import torch

from llmctl.testing.numerics import rel_frob, row_err


def test_row_check_catches_one_bad_gemm_tile():
    want = torch.randn(2048, 2048, generator=torch.Generator().manual_seed(1))
    got = want.clone()
    got[256:272, 512:528] += 0.15 * want.abs().amax()  # one 16x16 tile off by 15 % of the range
    assert rel_frob(got, want) < 8e-3
    assert row_err(got, want) > 0.1


def test_row_check_catches_one_bad_attention_tile():
    want = torch.randn(1, 2048, 8, 128, generator=torch.Generator().manual_seed(3))
    got = want.clone()
    got[0, 1024:1056, 3] *= 1.15  # one 32-query tile of one head 15 % off
    assert rel_frob(got, want) < 2e-2
    assert row_err(got, want) > 0.1
    assert row_err(got, want, floor=0.5) > 0.1  # the gradient checks' floored variant too


def test_row_check_passes_bf16_rounding():
    want = torch.randn(512, 1024, generator=torch.Generator().manual_seed(5))
    assert row_err(want.bfloat16(), want) < 1e-2
