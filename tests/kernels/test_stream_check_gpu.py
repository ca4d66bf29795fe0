"""Stream-race checker (LLMCTL_STREAM_CHECK=1 -> torch.cuda._sanitizer) over a training step
through the HIP ops: every op schema's read/write annotations are tracked per stream, so an
unsynchronised cross-stream access raises.  Runs in a child process (the checker is global)."""

import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[2]

CHILD = (ROOT / "tools" / "stream_check_child.py").read_text()


def test_training_step_under_stream_checker(native_lib):
    env = dict(os.environ, LLMCTL_STREAM_CHECK="1", PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "loss" in r.stdout, r.stderr[-4000:]
    assert "CSAN" not in r.stderr and "data race" not in r.stderr.lower(), r.stderr[-4000:]
