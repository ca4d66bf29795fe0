"""Custom IPC all-reduce (llmctl/comms/custom_ar.py): two processes on the one GPU of the
test box map each other's buffers through hipIpc handles; results must match the exact sum."""

import pytest

from llmctl.testing.harness import run_ranks
from llmctl.testing.workers import custom_ar_check

pytestmark = pytest.mark.gpu


def test_custom_allreduce_two_processes(native_lib):
    out = run_ranks(custom_ar_check, 2, timeout=300)
    for r in (0, 1):
        # bf16 output of an fp32 sum: <= 1 bf16 ulp relative
        assert out[r]["worst_rel_err"] < 1e-2, out


def test_custom_allreduce_twoshot_four_processes(native_lib):
    """Two-shot kernel (reduce-scatter + all-gather through the peer buffers) for prefill-sized
    messages beside the one-shot for small ones: 4 processes, sizes from 8 elements to 8 MB (the
    64-KB..16-MB range takes the two-shot path), epoch parity over many calls, graph replay."""
    out = run_ranks(custom_ar_check, 4, (8, 4096, 65536, 524288, 4 << 20), 6, 16 << 20, timeout=400)
    for r in range(4):
        assert out[r]["twoshot"] and out[r]["worst_rel_err"] < 1e-2, out
