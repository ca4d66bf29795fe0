"""CLI integration tests.

The first four mirror the reference's ``tests/integration/test_cli.py`` (help text, hw probe,
scaffold layout, scaffold → probe → plan workflow) but run ``python -m llmctl`` (no
console-script install needed) and use ``cwd=`` instead of ``os.chdir``.  The rest cover
the commands the reference only stubs: train → replay → export → eval, admin index/gc/inspect,
short / bare forms, and the reference-compatible plan mode.
"""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[2]


def llmctl(*args, cwd=None, timeout=600):
    env = dict(os.environ, PYTHONPATH=str(ROOT), LLMCTL_DEVICE="cpu")
    return subprocess.run([sys.executable, "-m", "llmctl", *args], capture_output=True, text=True, cwd=cwd,
                          env=env, timeout=timeout)


def _ok(r):
    assert r.returncode == 0, f"rc={r.returncode}\nstdout:{r.stdout[-3000:]}\nstderr:{r.stderr[-3000:]}"
    return r


# ---------------------------------------------------------------- reference parity (tests/integration/test_cli.py)
def test_cli_help():
    r = _ok(llmctl("--help"))
    assert "Distributed LLM Training and Inference System" in r.stdout


def test_hw_probe():
    r = _ok(llmctl("hw", "probe"))
    assert "Hardware Profile" in r.stdout


def test_init_scaffold(tmp_path):
    _ok(llmctl("init", "scaffold", "--template", "gpt", "--size", "7b", "--name", "test-proj",
               "--output-dir", str(tmp_path)))
    proj = tmp_path / "test-proj"
    assert (proj / "configs" / "models" / "gpt-7b.json").exists()
    assert (proj / "configs" / "default.toml").exists()
    assert (proj / "README.md").exists()


def test_plan_workflow(tmp_path):
    _ok(llmctl("init", "scaffold", "--template", "gpt", "--size", "7b", "--name", "test-proj",
               "--output-dir", str(tmp_path)))
    proj = tmp_path / "test-proj"
    _ok(llmctl("hw", "probe", "--emit", "configs/hw/local.toml", cwd=proj))
    assert (proj / "configs" / "hw" / "local.toml").exists()
    _ok(llmctl("plan", "compute", "--model", "configs/models/gpt-7b.json", "--hardware", "configs/hw/local.toml",
               "--out", "plans/local.toml", cwd=proj))
    assert (proj / "plans" / "local.toml").exists()


# ---------------------------------------------------------------- beyond the reference
def test_bare_and_short_forms(tmp_path):
    _ok(llmctl("init", "--template", "llama", "--size", "7b", "--name", "p", "--output-dir", str(tmp_path)))
    proj = tmp_path / "p"
    assert (proj / "configs" / "models" / "llama-7b.json").exists()
    _ok(llmctl("plan", "--model", "configs/models/llama-7b.json", "--hardware", str(ROOT / "configs/presets/mi355x8.toml"),
               "--out", "plans/p.toml", cwd=proj))
    from llmctl.config.toml_io import load_toml

    plan = load_toml(proj / "plans" / "p.toml")
    par = plan["parallelism"]
    assert par["tensor_parallel"] * par["pipeline_parallel"] * par["data_parallel"] == 8
    assert par["estimated_memory_gb"] <= 288


def test_plan_compat_reference_golden(tmp_path):
    hw = tmp_path / "a100x8.toml"
    hw.write_text('[gpu]\ncount = 8\n')
    out = tmp_path / "plan.toml"
    _ok(llmctl("plan", "compute", "--model", str(ROOT / "configs/models/llama-7b.json"), "--hardware", str(hw),
               "--compat-reference", "--out", str(out)))
    from llmctl.config.toml_io import load_toml

    par = load_toml(out)["parallelism"]
    assert (par["tensor_parallel"], par["pipeline_parallel"], par["data_parallel"], par["zero_stage"],
            par["micro_batch_size"], par["global_batch_size"]) == (8, 1, 1, 0, 1, 4)
    assert abs(par["estimated_memory_gb"] - 7.97) < 0.01


def test_train_replay_export_eval(tmp_path):
    out = tmp_path / "run"
    _ok(llmctl("train", "launch", "--model", "tiny", "--device", "cpu", "--max-steps", "3", "--batch-size", "2",
               "--seq-len", "64", "--output-dir", str(out)))
    assert (out / "final" / "model.safetensors").exists()
    man = json.loads((out / "run_manifest.json").read_text())
    assert man["status"] == "complete" and man["history"]
    r = _ok(llmctl("replay", "run", "--run-id", str(out)))
    assert json.loads(r.stdout[r.stdout.index("{"):])["match"] is True
    _ok(llmctl("export", "convert", "--ckpt", str(out), "--format", "safetensors", "--quant", "int8",
               "--out", str(tmp_path / "exp")))
    assert (tmp_path / "exp" / "model.safetensors").exists()
    r = llmctl("export", "convert", "--ckpt", str(out), "--format", "tensorrt", "--out", str(tmp_path / "x"))
    assert r.returncode != 0
    ev = tmp_path / "eval.json"
    _ok(llmctl("eval", "run", "--ckpt", str(out), "--device", "cpu", "--seq-len", "64", "--out", str(ev)))
    res = json.loads(ev.read_text())
    assert 1.0 < res["perplexity"]["perplexity"] < 5000
    _ok(llmctl("admin", "inspect", "--checkpoint", str(out / "final")))
    _ok(llmctl("admin", "gc", "--root", str(out), "--keep", "1", "--dry-run"))


def test_admin_index(tmp_path):
    src = tmp_path / "corpus.jsonl"
    src.write_text("\n".join(json.dumps({"text": f"document {i} ü"}) for i in range(5)) + "\n")
    r = _ok(llmctl("admin", "index", "--dataset", str(src)))
    toks = Path(tmp_path / "corpus.bin")
    assert toks.exists()
    import numpy as np

    arr = np.fromfile(toks, dtype=np.uint16)
    assert arr.size == sum(len(f"document {i} ü".encode()) + 1 for i in range(5))


def test_health_check_json(tmp_path):
    rep = tmp_path / "h.json"
    _ok(llmctl("health", "check", "--component", "system", "--save-report", str(rep)))
    assert "system" in json.loads(rep.read_text())


def test_elastic_restart_after_rank_kill(tmp_path):
    """Fault injection (LLMCTL_FAULT) kills rank 1 after step 3 of a 2-process gloo run.
    torchrun's own restart (not the orchestrator's whole-job relaunch) re-forms the group on a
    fresh store key space, resumes from checkpoint-2 (committed asynchronously right after its
    write, before the fault) and finishes all 5 steps.  The run is its own process group and is
    killed as a whole on timeout; ranks dump their stacks if they hang."""
    import signal
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "run"
    env = dict(os.environ, PYTHONPATH=str(ROOT), LLMCTL_DEVICE="cpu", LLMCTL_FAULT="kill_rank:1@step:3",
               LLMCTL_MASTER_PORT=str(port), OMP_NUM_THREADS="2", LLMCTL_HANG_DUMP="150")
    p = subprocess.Popen([sys.executable, "-m", "llmctl", "train", "launch", "--model", "tiny", "--device", "cpu",
                          "--gpus-per-node", "2", "--max-steps", "5", "--batch-size", "2", "--seq-len", "32",
                          "--save-steps", "2", "--max-restarts", "1", "--mixed-precision", "fp32",
                          "--output-dir", str(out)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=env, start_new_session=True)
    try:
        stdout, _ = p.communicate(timeout=300)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        stdout, _ = p.communicate()
        raise AssertionError("elastic run hung; output tail:\n" + stdout[-6000:])
    finally:
        try:
            os.killpg(p.pid, signal.SIGKILL)  # nothing of the run may outlive the test
        except ProcessLookupError:
            pass
    assert p.returncode == 0, stdout[-6000:]
    assert (out / ".faults" / "kill_rank-1-3").exists()
    assert "[orchestrator] exit code" not in stdout, "recovered by the orchestrator, not torchrun"
    import re

    flat = " ".join(stdout.split())  # the console wraps long log lines
    assert re.search(r"resumed from \S+ at step 2 \(restart attempt 1\)", flat), stdout[-4000:]
    st = json.loads((out / "final" / "training_state.json").read_text())
    assert st["global_step"] == 5
    man = json.loads((out / "run_manifest.json").read_text())
    assert man["status"] == "complete"
