"""The driver's ``bench.py`` contract, exercised through the exact multi-rank launch the driver
uses (``torch.distributed.run`` one rank per device, rendezvous on 127.0.0.1) with gloo/CPU
ranks and a tiny model: one JSON line from rank 0, whole-job tokens/s, max-over-ranks time.
The 7B/RCCL numbers themselves come from the GPU runs (profiles/)."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[2]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, *extra):
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--model", "tiny", "--seq-len", "64",
           "--micro-batch", "2", "--device", "cpu", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp", env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n,extra,par", [(2, (), "dp2-zero1"), (2, ("--zero", "0"), "dp2"),
                                         (4, ("--tp", "2"), "dp2-tp2-zero1")])
def test_bench_multirank_json_line(n, extra, par):
    res = _run(n, *extra)
    assert KEYS <= set(res)
    assert res["n_gpus"] == n and res["steps"] == 2 and res["warmup"] == 1
    assert res["higher_is_better"] is True and res["scaling"] == "weak" and res["dtype"] == "bf16"
    cfg = res["config"]
    assert cfg["parallelism"] == par and cfg["seq_len"] == 64
    assert cfg["layout"] == ("planner" if not extra else "flags")  # default: the planner's layout
    dp = n // (2 if "--tp" in extra else 1)
    assert cfg["global_batch"] == 2 * dp
    # value is the whole-job aggregate: global tokens over the (max-over-ranks) timed window
    tokens = cfg["global_batch"] * 64 * res["steps"]
    assert res["value"] == pytest.approx(tokens / (res["ms_per_step"] * res["steps"] / 1000.0), rel=1e-2)
    assert res["final_loss"] == res["final_loss"]  # finite
