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

CHILD = textwrap.dedent('''
    import torch
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine
    cfg = TrainingConfig(model_name_or_path="tiny", device="cuda", seq_len=128, batch_size=2, log_level="error",
                         activation_checkpoint="selective", gradient_accumulation_steps=2, output_dir="/tmp/sc")
    eng = TrainingEngine(cfg)
    g = torch.Generator(device="cuda").manual_seed(0)
    for s in range(2):
        b = [(torch.randint(1, 500, (2, 128), device="cuda", generator=g),
              torch.randint(1, 500, (2, 128), device="cuda", generator=g)) for _ in range(2)]
        out = eng.train_step(b)
    torch.cuda.synchronize()
    print("loss", float(out["loss"]))
''')


def test_training_step_under_stream_checker(native_lib):
    env = dict(os.environ, LLMCTL_STREAM_CHECK="1", PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "loss" in r.stdout, r.stderr[-4000:]
    assert "CSAN" not in r.stderr and "data race" not in r.stderr.lower(), r.stderr[-4000:]
