"""The user-facing CLI flow on the GPU: ``llmctl train launch`` (tiny model, a few steps on
``cuda``) -> ``llmctl eval run`` on the trained checkpoint -> ``llmctl serve start`` of that
checkpoint as a child process, queried over HTTP (completion, streaming, health, metrics) and
stopped by its own PID.  The CPU suite covers the same commands on ``--device cpu``
(tests/integration/test_cli.py); this runs them through the HIP kernels, hipGraph decode and the
native runtime the way a user would."""

import json
import os
import socket
import subprocess
import sys
import time
import urllib.request
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[2]


def llmctl(*args, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    env.pop("LLMCTL_DEVICE", None)
    return subprocess.run([sys.executable, "-m", "llmctl", *args], capture_output=True, text=True, env=env,
                          timeout=timeout)


def _ok(r):
    assert r.returncode == 0, f"rc={r.returncode}\nstdout:{r.stdout[-3000:]}\nstderr:{r.stderr[-3000:]}"
    return r


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url, timeout=10):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.read().decode()


def _post(url, body, timeout=120):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.read().decode()


def test_train_eval_serve_on_gpu(native_lib, tmp_path):
    out = tmp_path / "run"
    _ok(llmctl("train", "launch", "--model", "tiny", "--device", "cuda", "--max-steps", "4", "--batch-size", "2",
               "--seq-len", "128", "--output-dir", str(out)))
    man = json.loads((out / "run_manifest.json").read_text())
    assert man["status"] == "complete" and len(man["history"]) >= 1
    assert (out / "final" / "model.safetensors").exists()
    ev = tmp_path / "eval.json"
    _ok(llmctl("eval", "run", "--ckpt", str(out), "--device", "cuda", "--seq-len", "128", "--out", str(ev)))
    assert 1.0 < json.loads(ev.read_text())["perplexity"]["perplexity"] < 5000

    port = _free_port()
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    log = open(tmp_path / "serve.log", "w")
    proc = subprocess.Popen([sys.executable, "-m", "llmctl", "serve", "start", "--artifact", str(out / "final"),
                             "--host", "127.0.0.1", "--port", str(port), "--device", "cuda", "--max-batch-size", "4",
                             "--kv-cache-fraction", "0.05"], stdout=log, stderr=subprocess.STDOUT, env=env)
    base = f"http://127.0.0.1:{port}"
    try:
        deadline = time.time() + 180
        health = None
        while time.time() < deadline:
            assert proc.poll() is None, (tmp_path / "serve.log").read_text()[-3000:]
            try:
                health = json.loads(_get(base + "/health"))
                if health["status"] == "healthy":
                    break
            except OSError:
                pass
            time.sleep(1.0)
        assert health is not None and health["status"] == "healthy", health
        assert health["device"].startswith("cuda")
        body = json.loads(_post(base + "/v1/completions", {"prompt": "hello world", "max_tokens": 12,
                                                           "temperature": 0.0, "ignore_eos": True}))
        assert body["usage"]["completion_tokens"] == 12 and body["finish_reason"] == "length"
        again = json.loads(_post(base + "/v1/completions", {"prompt": "hello world", "max_tokens": 12,
                                                            "temperature": 0.0, "ignore_eos": True}))
        assert again["text"] == body["text"]  # greedy decode is deterministic across requests
        stream = _post(base + "/v1/completions", {"prompt": [5, 6, 7], "max_tokens": 4, "stream": True,
                                                  "temperature": 0.0, "ignore_eos": True})
        lines = [l for l in stream.splitlines() if l.startswith("data: ")]
        assert lines[-1] == "data: [DONE]"
        chunks = [json.loads(l[6:]) for l in lines[:-1]]
        assert len([c for c in chunks if c["choices"][0]["finish_reason"] is None]) == 4
        assert "llmctl_inference_requests_total" in _get(base + "/metrics")
    finally:
        proc.terminate()  # our own child, by PID
        try:
            proc.wait(timeout=30)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait(timeout=30)
        log.close()
