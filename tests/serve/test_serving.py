"""Serving engine + HTTP server on CPU (tiny random-init model).

Includes the regression the reference lacks: ``max_tokens > 1`` must complete (the
reference server hung forever) and concurrent requests must all finish.
"""

import json
import threading

import pytest
import torch

from llmctl.serve.block_manager import PyKVManager, make_kv_manager
from llmctl.serve.engine import InferenceEngine
from llmctl.serve.scheduler import ContinuousBatchScheduler, SamplingParams, Sequence


@pytest.fixture(scope="module")
def engine():
    return InferenceEngine("tiny", device="cpu", max_batch_size=4, num_kv_blocks=48, block_size=8,
                           max_model_len=256, max_batch_tokens=512)


def test_greedy_decode_matches_full_forward(engine):
    seqs = engine.generate([[1, 2, 3, 4, 5], [9] * 13, [7, 7]], SamplingParams(max_tokens=10, temperature=0.0))
    for s in seqs:
        assert len(s.output_ids) == 10 and s.finish_reason == "length"
        logits = engine.model(torch.tensor([s.all_ids[:-1]]))
        ref_next = logits.view(-1, logits.shape[-1]).argmax(-1)[len(s.prompt_ids) - 1:].tolist()
        assert ref_next == s.output_ids


def test_kv_blocks_released(engine):
    free0 = engine.kv.num_free_blocks
    engine.generate([[1] * 30, [2] * 3], SamplingParams(max_tokens=5, temperature=0.0))
    assert engine.kv.num_free_blocks == free0


def test_preemption_under_kv_pressure():
    e = InferenceEngine("tiny", device="cpu", max_batch_size=8, num_kv_blocks=12, block_size=4, max_model_len=128)
    seqs = e.generate([[i + 1] * 6 for i in range(6)], SamplingParams(max_tokens=8, temperature=0.0))
    assert all(len(s.output_ids) == 8 for s in seqs)
    assert sum(s.preemptions for s in seqs) > 0
    # recomputation after preemption must not change greedy outputs
    e2 = InferenceEngine("tiny", device="cpu", max_batch_size=1, num_kv_blocks=64, block_size=4, max_model_len=128)
    ref = e2.generate([[i + 1] * 6 for i in range(6)], SamplingParams(max_tokens=8, temperature=0.0))
    assert [s.output_ids for s in seqs] == [s.output_ids for s in ref]


@pytest.mark.parametrize("impl", ["py", "native"])
def test_kv_manager_semantics(impl):
    kv = PyKVManager(10, 4) if impl == "py" else make_kv_manager(10, 4, prefer_native=True)
    assert kv.add_sequence(1, 5)
    assert kv.num_free_blocks == 8
    slots = [kv.append_token(1) for _ in range(4)]
    assert slots[-1] // 4 == kv.block_table(1)[2]
    kv.fork(1, 2)
    kv.free_sequence(1)
    assert kv.num_free_blocks == 7  # shared blocks survive
    kv.free_sequence(2)
    assert kv.num_free_blocks == 10
    bt = kv.block_tables([], 3)
    assert bt.shape == (0, 3)


def test_scheduler_token_budget():
    kv = PyKVManager(100, 16)
    s = ContinuousBatchScheduler(kv, max_batch_size=8, max_batch_tokens=40, block_size=16)
    for n in (30, 20, 5):
        s.add(Sequence(prompt_ids=[1] * n, params=SamplingParams()))
    out = s.schedule()
    assert [len(q.prompt_ids) for q in out.prefill] == [30]  # 30 + 20 > 40
    out = s.schedule()
    assert len(out.decode) == 1 and [len(q.prompt_ids) for q in out.prefill] == [20, 5]


def test_scheduler_prefill_first_policy():
    kv = PyKVManager(100, 16)
    s = ContinuousBatchScheduler(kv, max_batch_size=8, max_batch_tokens=40, block_size=16, policy="prefill_first")
    for n in (30, 20, 5):
        s.add(Sequence(prompt_ids=[1] * n, params=SamplingParams()))
    out = s.schedule()
    assert [len(q.prompt_ids) for q in out.prefill] == [30] and not out.decode
    out = s.schedule()  # admissions pending: the running sequence pauses
    assert not out.decode and [len(q.prompt_ids) for q in out.prefill] == [20, 5]
    out = s.schedule()  # queue drained: everyone decodes
    assert len(out.decode) == 3 and not out.prefill


def test_engine_prefill_first_matches_dynamic():
    p = SamplingParams(max_tokens=6, temperature=0.0)
    prompts = [[1, 2, 3], [4, 5, 6, 7, 8], [9] * 20]
    outs = []
    for pol in ("dynamic", "prefill_first"):
        e = InferenceEngine("tiny", device="cpu", max_batch_size=2, num_kv_blocks=64, block_size=8,
                            max_model_len=128, scheduler=pol)
        outs.append([s.output_ids for s in e.generate(prompts, p)])
    assert outs[0] == outs[1]


@pytest.fixture(scope="module")
def client():
    from fastapi.testclient import TestClient

    from llmctl.serve.server import InferenceServer

    eng = InferenceEngine("tiny", device="cpu", max_batch_size=4, num_kv_blocks=64, block_size=8,
                          max_model_len=256)
    srv = InferenceServer("tiny", engine=eng, max_concurrent=16)
    with TestClient(srv.app) as c:
        yield c


def test_http_routes(client):
    h = client.get("/health").json()
    assert h["status"] == "healthy" and "active_requests" in h and "pending_requests" in h
    m = client.get("/v1/models").json()
    assert m["object"] == "list" and m["data"][0]["owned_by"] == "llmctl"
    r = client.post("/v1/completions", json={"prompt": "hello world", "max_tokens": 20, "temperature": 0.7,
                                            "top_k": 50, "top_p": 0.9})
    assert r.status_code == 200
    body = r.json()
    assert body["usage"]["completion_tokens"] == 20 and body["finish_reason"] == "length"
    assert body["usage"]["prompt_tokens"] == len("hello world".encode())
    assert "ttft_s" in body["timing"]
    assert "llmctl_inference_requests_total" in client.get("/metrics").text


def test_http_concurrent_requests(client):
    results = []

    def go(i):
        r = client.post("/v1/completions", json={"prompt": [i + 1, 2, 3], "max_tokens": 15 + i,
                                                "temperature": 0.0})
        results.append(r.json())

    ts = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert len(results) == 6
    assert sorted(r["usage"]["completion_tokens"] for r in results) == [15, 16, 17, 18, 19, 20]


def test_http_streaming(client):
    with client.stream("POST", "/v1/completions", json={"prompt": "abc", "max_tokens": 5, "stream": True,
                                                        "temperature": 0.0}) as r:
        lines = [l for l in r.iter_lines() if l.startswith("data: ")]
    assert lines[-1] == "data: [DONE]"
    toks = [json.loads(l[6:]) for l in lines[:-1]]
    assert len([t for t in toks if t["choices"][0]["finish_reason"] is None]) == 5
