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
    engine.prefix_cache.clear()
    free0 = engine.kv.num_free_blocks
    engine.generate([[1] * 30, [2] * 3], SamplingParams(max_tokens=5, temperature=0.0))
    # finished sequences keep only the blocks the prefix cache indexes
    assert engine.kv.num_free_blocks == free0 - len(engine.prefix_cache)
    engine.prefix_cache.clear()
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


def _run(s, out):
    """What the engine does after executing a step: mark the work computed and append a
    (dummy) sampled token to every sequence whose known tokens are now all cached."""
    for q in out.decode:
        s.computed(q, 1)
        q.output_ids.append(0)
    for c in out.prefill:
        s.computed(c.seq, c.count)
        if c.final:
            c.seq.output_ids.append(0)


def _chunks(out):
    return [(len(c.seq.prompt_ids), c.start, c.count) for c in out.prefill]


def test_scheduler_token_budget_chunks_prefills():
    """Budget 40: the 30-token prompt fits, the 20-token one is split 10 + 10 across steps
    (chunked prefill) and the 5-token one joins the second step beside the first decode."""
    kv = PyKVManager(100, 16)
    s = ContinuousBatchScheduler(kv, max_batch_size=8, max_batch_tokens=40, block_size=16)
    for n in (30, 20, 5):
        s.add(Sequence(prompt_ids=[1] * n, params=SamplingParams()))
    out = s.schedule()
    assert _chunks(out) == [(30, 0, 30), (20, 0, 10)] and not out.decode
    assert [c.final for c in out.prefill] == [True, False]
    _run(s, out)
    out = s.schedule()
    assert len(out.decode) == 1 and _chunks(out) == [(20, 10, 10), (5, 0, 5)]
    _run(s, out)
    out = s.schedule()
    assert len(out.decode) == 3 and not out.prefill


def test_scheduler_prefill_first_policy():
    kv = PyKVManager(100, 16)
    s = ContinuousBatchScheduler(kv, max_batch_size=8, max_batch_tokens=40, block_size=16, policy="prefill_first")
    for n in (30, 20, 5):
        s.add(Sequence(prompt_ids=[1] * n, params=SamplingParams()))
    out = s.schedule()
    assert _chunks(out) == [(30, 0, 30), (20, 0, 10)] and not out.decode
    _run(s, out)
    out = s.schedule()  # admissions pending: the running sequence pauses
    assert not out.decode and _chunks(out) == [(20, 10, 10), (5, 0, 5)]
    _run(s, out)
    out = s.schedule()  # queue drained: everyone decodes
    assert len(out.decode) == 3 and not out.prefill


def test_prefix_cache_reuses_blocks_and_evicts():
    from llmctl.serve.prefix_cache import PrefixCache

    kv = PyKVManager(8, 4)
    pc = PrefixCache(kv, 4)
    s = ContinuousBatchScheduler(kv, max_batch_size=4, max_batch_tokens=64, block_size=4, prefix_cache=pc)
    a = Sequence(prompt_ids=list(range(1, 11)), params=SamplingParams())  # 10 tokens: 2 full blocks
    s.add(a)
    out = s.schedule()
    _run(s, out)
    assert len(pc) == 2  # blocks [1..4], [5..8] indexed
    s.finish(a, "length")
    assert kv.num_free_blocks == 6  # the two cached blocks stay resident
    b = Sequence(prompt_ids=list(range(1, 9)) + [42, 43], params=SamplingParams())
    s.add(b)
    out = s.schedule()
    assert _chunks(out) == [(10, 8, 2)] and b.cached_tokens == 8  # only the new tail is computed
    _run(s, out)
    s.finish(b, "length")
    # a prompt needing every block evicts the unused cached ones
    c = Sequence(prompt_ids=[7] * 25, params=SamplingParams())
    s.add(c)
    out = s.schedule()
    assert _chunks(out) == [(25, 0, 25)] and pc.stats["evicted"] >= 1


@pytest.mark.parametrize("impl", ["py", "native"])
def test_admission_eviction_never_frees_its_own_prefix(impl):
    """8 blocks of 4 slots, a cached 2-block prefix, one other running sequence and a 28-token
    prompt sharing the prefix: reserving the prompt's 6 other blocks must not evict the 2 blocks
    match() just returned (they are held only by the cache until the sequence is added) — the
    admission waits instead, and succeeds with the prefix re-attached once space frees up."""
    from llmctl.serve.prefix_cache import PrefixCache

    kv = PyKVManager(8, 4) if impl == "py" else make_kv_manager(8, 4, prefer_native=True)
    pc = PrefixCache(kv, 4)
    s = ContinuousBatchScheduler(kv, max_batch_size=4, max_batch_tokens=64, block_size=4, prefix_cache=pc)
    a = Sequence(prompt_ids=list(range(1, 11)), params=SamplingParams())
    s.add(a)
    _run(s, s.schedule())
    s.finish(a, "length")
    assert len(pc) == 2 and kv.num_free_blocks == 6
    r = Sequence(prompt_ids=[50] * 3, params=SamplingParams())
    s.add(r)
    _run(s, s.schedule())
    c = Sequence(prompt_ids=list(range(1, 9)) + [99] * 20, params=SamplingParams())
    s.add(c)
    out = s.schedule()  # must not raise ("incref of a free block")
    assert c.status == "waiting" and all(q.seq is not c for q in out.prefill)
    assert len(pc) == 2 and pc.stats["evicted"] == 0
    s.finish(r, "length")
    out = s.schedule()
    assert c.status == "running" and c.cached_tokens == 8
    assert [(q.start, q.count) for q in out.prefill if q.seq is c] == [(8, 20)]


def test_can_admit_counts_evictable_cached_blocks():
    """prefill_first: blocks held only by the prefix cache count as free, so a full cache does
    not stop the policy from pausing decodes for an admission."""
    from llmctl.serve.prefix_cache import PrefixCache

    kv = PyKVManager(8, 4)
    pc = PrefixCache(kv, 4)
    s = ContinuousBatchScheduler(kv, max_batch_size=4, max_batch_tokens=64, block_size=4, prefix_cache=pc,
                                 policy="prefill_first")
    a = Sequence(prompt_ids=list(range(1, 18)), params=SamplingParams())  # 4 full blocks
    s.add(a)
    _run(s, s.schedule())
    s.finish(a, "length")
    r = Sequence(prompt_ids=[5] * 3, params=SamplingParams())
    s.add(r)
    _run(s, s.schedule())
    assert kv.num_free_blocks == 3 and len(pc) == 4 and not kv.can_allocate(14)
    s.add(Sequence(prompt_ids=[9] * 10, params=SamplingParams()))  # needs 4 blocks
    assert s._can_admit()
    out = s.schedule()
    assert not out.decode and _chunks(out) == [(10, 0, 10)]


def test_prefix_keys_are_keyed_digests():
    from llmctl.serve.prefix_cache import PrefixCache, _block_hash

    h1 = _block_hash(b"", [1, 2, 3, 4])
    assert isinstance(h1, bytes) and len(h1) == 16
    assert _block_hash(h1, [5, 6, 7, 8]) != _block_hash(b"", [5, 6, 7, 8])
    pc = PrefixCache(PyKVManager(4, 4), 4)
    assert pc._hashes([1, 2, 3, 4, 5, 6, 7, 8], 2) == [h1, _block_hash(h1, [5, 6, 7, 8])]


def test_preempted_sequence_resumes_from_cached_blocks():
    """A sequence preempted after its prompt was computed re-attaches its full blocks when it
    is readmitted: only the tail past the last full block is recomputed."""
    from llmctl.serve.prefix_cache import PrefixCache

    kv = PyKVManager(64, 4)
    pc = PrefixCache(kv, 4)
    s = ContinuousBatchScheduler(kv, max_batch_size=4, max_batch_tokens=64, block_size=4, prefix_cache=pc)
    a = Sequence(prompt_ids=list(range(1, 15)), params=SamplingParams())  # 14 tokens
    s.add(a)
    _run(s, s.schedule())
    for _ in range(2):  # prompt (14) + two decodes computed = 16; 17 tokens known
        _run(s, s.schedule())
    assert a.num_computed == 16
    s._preempt(a)
    assert a.status == "waiting" and a.preemptions == 1
    out = s.schedule()
    assert a.cached_tokens == 16 and _chunks(out) == [(14, 16, 1)]


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


@pytest.mark.parametrize("impl", ["py", "native"])
def test_kv_manager_shared_prefix(impl):
    kv = PyKVManager(10, 4) if impl == "py" else make_kv_manager(10, 4, prefer_native=True)
    assert kv.add_sequence(1, 8)
    shared = kv.block_table(1)
    kv.incref_block(shared[0])  # an outside holder (the prefix cache)
    assert kv.add_sequence_shared(2, 10, shared)  # 2 shared + 1 fresh
    assert kv.block_table(2)[:2] == shared and kv.num_free_blocks == 10 - 3
    assert kv.refcount(shared[0]) == 3 and kv.refcount(shared[1]) == 2
    kv.free_sequence(1)
    kv.free_sequence(2)
    assert kv.num_free_blocks == 9 and kv.decref_block(shared[0]) and kv.num_free_blocks == 10
    assert not kv.add_sequence_shared(3, 44, [])  # 11 blocks > 10: refused, nothing taken
    assert kv.num_free_blocks == 10


def _greedy(e, prompts, n=6):
    return [s.output_ids for s in e.generate(prompts, SamplingParams(max_tokens=n, temperature=0.0))]


def test_chunked_prefill_matches_single_shot():
    """A 16-token step budget splits every prompt into several prefill chunks (each attending
    its cached earlier chunks through the paged cache); greedy outputs equal the one-shot run."""
    prompts = [[(7 * i + 3) % 250 + 1 for i in range(45)], [5] * 17, [1, 2, 3]]
    kw = dict(device="cpu", max_batch_size=4, num_kv_blocks=64, block_size=8, max_model_len=256,
              prefix_caching=False)
    chunked = InferenceEngine("tiny", max_batch_tokens=16, **kw)
    ref = InferenceEngine("tiny", max_batch_tokens=4096, **kw)
    assert _greedy(chunked, prompts) == _greedy(ref, prompts)
    assert chunked.stats["prefill_tokens"] == ref.stats["prefill_tokens"] == 45 + 17 + 3


def test_prefix_cache_hit_skips_prefix_compute():
    """A second request sharing a 32-token prefix computes only its own tail, and its tokens
    equal an engine without prefix caching."""
    base = [(11 * i) % 200 + 1 for i in range(32)]
    p1, p2 = base + [9, 9, 9], base + [4, 5]
    kw = dict(device="cpu", max_batch_size=2, num_kv_blocks=64, block_size=8, max_model_len=256)
    e = InferenceEngine("tiny", **kw)
    out1 = _greedy(e, [p1])
    before = e.stats["prefill_tokens"]
    out2 = _greedy(e, [p2])
    assert e.stats["prefill_tokens"] - before == len(p2) - 32  # 4 cached blocks re-attached
    ref = InferenceEngine("tiny", prefix_caching=False, **kw)
    assert out1 + out2 == _greedy(ref, [p1]) + _greedy(ref, [p2])


def test_preemption_resume_reuses_cached_blocks():
    """A sequence preempted mid-generation re-attaches its full cached blocks when resumed:
    only the tail past its last full block is recomputed, and greedy tokens are unchanged."""
    prompt = [(5 * i) % 97 + 1 for i in range(21)]
    # synchronous decode: the test reads the scheduler state between steps
    kw = dict(device="cpu", max_batch_size=2, num_kv_blocks=64, block_size=4, max_model_len=128,
              perf_knobs={"async_decode": False})
    e = InferenceEngine("tiny", **kw)
    seq = e.add_request(prompt, SamplingParams(max_tokens=10, temperature=0.0))
    for _ in range(4):  # prefill + 3 decodes: 24 positions computed
        e.step()
    assert seq.num_computed == 24
    e.scheduler._preempt(seq)
    before = e.stats["prefill_tokens"]
    while seq.status != "finished":
        e.step()
    assert seq.cached_tokens == 24 and e.stats["prefill_tokens"] - before == 1  # 25 known, 24 re-attached
    ref = InferenceEngine("tiny", prefix_caching=False, **kw)
    assert seq.output_ids == _greedy(ref, [prompt], 10)[0]


@pytest.mark.parametrize("prefix", [False, True])
def test_mixed_prefill_decode_steps_match_separate(monkeypatch, prefix):
    """A step with both decode tokens and prefill chunks runs ONE forward (decode rows appended to
    the chunk batch, attention split by row kind): greedy outputs equal the two-forward steps."""
    prompts = [[1, 2, 3, 4, 5] * 6, [9] * 37, [7, 7, 3], [3, 1, 4, 1, 5, 9, 2, 6] * 5]
    kw = dict(device="cpu", max_batch_size=4, num_kv_blocks=64, block_size=8, max_model_len=256,
              max_batch_tokens=48, prefix_caching=prefix)
    p = SamplingParams(max_tokens=9, temperature=0.0)
    e = InferenceEngine("tiny", perf_knobs={"mixed_steps": True}, **kw)
    a = [s.output_ids for s in e.generate(prompts, p)]
    assert e.stats.get("mixed_steps", 0) > 0
    e2 = InferenceEngine("tiny", perf_knobs={"mixed_steps": False}, **kw)
    b = [s.output_ids for s in e2.generate(prompts, p)]
    assert e2.stats.get("mixed_steps", 0) == 0
    assert a == b


def test_engines_keep_their_own_knobs():
    """A second engine in the same process (other perf_knobs) must not change the first one's
    routing: each engine re-activates its own resolved knobs on every step."""
    from llmctl.config.knobs import knobs
    from llmctl.serve.scheduler import SamplingParams

    kw = dict(device="cpu", max_batch_size=2, num_kv_blocks=32, block_size=8, max_model_len=128)
    a = InferenceEngine("tiny", perf_knobs={"mixed_steps": False}, **kw)
    b = InferenceEngine("tiny", perf_knobs={"mixed_steps": True}, **kw)
    assert knobs().mixed_steps  # b's
    a.add_request([1, 2, 3], SamplingParams(max_tokens=2, temperature=0.0))
    a.step()
    assert not knobs().mixed_steps and not a._mixed_ok()
    b.add_request([1, 2, 3], SamplingParams(max_tokens=2, temperature=0.0))
    b.step()
    assert knobs().mixed_steps


@pytest.mark.parametrize("temp", [0.0, 0.9])
def test_async_decode_pipeline_matches_sync_cpu(temp):
    """The pipelined decode loop (step N + 1 launched before step N's tokens are read, ids fed
    from step N's sampled tokens) gives the synchronous loop's tokens, greedy and sampled; it
    stops continuing at length limits and when a request waits for admission."""
    from llmctl.serve.scheduler import SamplingParams

    prompts = [[1, 2, 3, 4, 5], [9] * 11, [7, 7], [3] * 17]
    p = SamplingParams(max_tokens=9, temperature=temp, top_k=20, top_p=0.9, ignore_eos=True)
    outs = []
    for a in (True, False):
        e = InferenceEngine("tiny", device="cpu", max_batch_size=4, num_kv_blocks=64, block_size=8,
                            max_model_len=128, seed=5, perf_knobs={"async_decode": a}, prefix_caching=False)
        seqs = e.generate(prompts, p)
        late = e.add_request([4, 4, 4], p)  # arrives while nothing runs
        while late.status != "finished":
            e.step()
        outs.append(([s.output_ids for s in seqs], late.output_ids))
        assert all(len(s.output_ids) == 9 for s in seqs) and len(late.output_ids) == 9
        if a:
            assert e.stats.get("async_continued", 0) >= 4
        assert e.kv.num_free_blocks == 64  # every block back (speculative rows included)
    assert outs[0] == outs[1]


def test_engine_fp8_kv_cache_cpu():
    """kv_cache_dtype="fp8": the cache holds float8_e4m3fn (a quarter of the CPU oracle's fp32 bytes,
    so four times the blocks for the same budget), the oracle paths quantise on write and widen
    on read, and the first greedy token (prefill attends the un-quantised K/V) is unchanged."""
    import torch

    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams

    prompts = [[(7 * i + r) % 200 + 1 for i in range(24 + 5 * r)] for r in range(3)]
    p = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    engs = {k: InferenceEngine("tiny", device="cpu", max_batch_size=3, kv_cache_dtype=k) for k in ("auto", "fp8")}
    assert engs["fp8"].kv_cache.k.dtype == torch.float8_e4m3fn
    assert engs["fp8"].kv_cache.num_blocks == 4 * engs["auto"].kv_cache.num_blocks
    outs = {k: [s.output_ids for s in e.generate(prompts, p)] for k, e in engs.items()}
    assert all(len(o) == 6 for o in outs["fp8"])
    assert [o[0] for o in outs["fp8"]] == [o[0] for o in outs["auto"]]
    with pytest.raises(ValueError):
        InferenceEngine("tiny", device="cpu", kv_cache_dtype="int4")


@pytest.mark.parametrize("temp", [0.0, 0.9])
def test_tp_async_decode_matches_tp1(temp):
    """TP = 2 (gloo) with the pipelined decode loop: every rank samples in the decode step from the
    same gathered logits and the uniforms rank 0 publishes with the plan, and a continued step
    feeds the device-side ids back on every rank.  Tokens equal the TP = 2 synchronous loop and the
    TP = 1 engine, greedy and seeded-sampled, and the host RNG advanced by the same number of draws
    (no second draw per step on the TP path)."""
    from llmctl.testing.harness import run_ranks
    from llmctl.testing.workers import serve_sampled

    one = run_ranks(serve_sampled, 1, True, temp)[0]
    tp_async = run_ranks(serve_sampled, 2, True, temp)[0]
    tp_sync = run_ranks(serve_sampled, 2, False, temp)[0]
    assert tp_async["continued"] >= 3 and tp_sync["continued"] == 0
    assert tp_async["tokens"] == tp_sync["tokens"] == one["tokens"]
    assert tp_async["rng_next"] == tp_sync["rng_next"] == one["rng_next"]


@pytest.mark.parametrize("async_decode", [True, False])
def test_async_decode_early_stop_with_prefix_cache(async_decode):
    """Sequences that stop on EOS (or a stop string) while a speculative step N + 1 for them is in
    flight, with prefix caching on: outputs and finish reasons equal the synchronous loop, and
    every KV block comes back (free, or held only by the prefix cache)."""
    from llmctl.serve.scheduler import SamplingParams

    prompts = [[1, 2, 3, 4, 5, 6, 7, 8, 9], [9] * 11, [1, 2, 3, 4, 5, 6, 7, 8, 9, 10], [3] * 17]
    mk = lambda a: InferenceEngine("tiny", device="cpu", max_batch_size=4, num_kv_blocks=64, block_size=4,
                                   max_model_len=128, seed=5, perf_knobs={"async_decode": a}, prefix_caching=True)
    probe = mk(False)
    free = [s.output_ids for s in probe.generate(prompts, SamplingParams(max_tokens=12, temperature=0.0,
                                                                          ignore_eos=True))]
    # a token some sequence first produces mid-stream: that row (and any other hitting it) stops there
    si, pos = next((i, j) for i, o in enumerate(free) for j in range(2, len(o)) if o[j] not in o[:j])
    eos = free[si][pos]
    outs = {}
    for a in (async_decode, False):
        e = mk(a)
        e.tokenizer.eos_token_id = eos
        seqs = e.generate(prompts, SamplingParams(max_tokens=12, temperature=0.0))
        stop = e.add_request([2, 2, 2, 2, 2], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True,
                                                             stop=[e.tokenizer.decode(free[0][2:3])]))
        while stop.status != "finished":
            e.step()
        outs[a] = ([s.output_ids for s in seqs], [s.finish_reason for s in seqs], stop.output_ids,
                   stop.finish_reason)
        assert e.kv.num_free_blocks + e.prefix_cache.num_evictable() == 64
        e.prefix_cache.clear()
        assert e.kv.num_free_blocks == 64
    assert outs[async_decode] == outs[False]
    assert outs[False][1][si] == "stop" and len(outs[False][0][si]) == pos + 1


def test_engine_close_is_deterministic_and_idempotent():
    """``close()`` (and the context-manager exit) drops the pipelined step, the graphs, the KV
    cache and the fp8 copies without waiting for garbage collection; a second close is a no-op."""
    from llmctl.serve.scheduler import SamplingParams

    with InferenceEngine("tiny", device="cpu", max_batch_size=2, num_kv_blocks=16, block_size=8,
                         max_model_len=64) as e:
        e.generate([[1, 2, 3]], SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
        assert e.kv_cache is not None
    assert e.kv_cache is None and e._pending is None and not e._graphs and e._nf is None
    e.close()


def test_kv_manager_native_matches_python_model():
    """Model-based property test (hypothesis state machine): the native C++ KVManager and the
    Python PyKVManager, driven by the same random operation sequence (add / add with a shared
    prefix / append / fork / free / external prefix-cache references, OOM included), return the
    same results and hold the same block tables, token counts, slots and reference counts; every
    block's count equals its table occurrences plus the external references."""
    from hypothesis import settings
    from hypothesis import strategies as st
    from hypothesis.stateful import RuleBasedStateMachine, initialize, invariant, precondition, rule

    native = make_kv_manager(1, 1)
    if isinstance(native, PyKVManager):
        pytest.skip("native runtime not built")

    class Machine(RuleBasedStateMachine):
        @initialize(nb=st.integers(1, 24), bs=st.sampled_from([1, 2, 4, 16]))
        def setup(self, nb, bs):
            self.n, self.p = make_kv_manager(nb, bs), PyKVManager(nb, bs)
            self.nb, self.bs, self.next_id, self.ext = nb, bs, 0, []

        def _both(self, name, *args):
            outs = []
            for m in (self.n, self.p):
                try:
                    outs.append(("ok", getattr(m, name)(*args)))
                except Exception as e:  # the same failure on both sides
                    outs.append(("err", type(e).__name__ in ("RuntimeError", "ValueError", "IndexError")))
            assert outs[0] == outs[1] or (outs[0][0] == outs[1][0] == "err"), (name, args, outs)
            return outs[0]

        @property
        def seqs(self):
            return sorted(self.p.tables)

        @rule(tokens=st.integers(0, 40))
        def add(self, tokens):
            self._both("add_sequence", self.next_id, tokens)
            self.next_id += 1

        @precondition(lambda self: self.p.tables)
        @rule(data=st.data(), tokens=st.integers(1, 40))
        def add_shared(self, data, tokens):
            src = data.draw(st.sampled_from(self.seqs))
            full = self.p.num_tokens(src) // self.bs
            k = data.draw(st.integers(0, min(full, self.p.blocks_needed(tokens))))
            self._both("add_sequence_shared", self.next_id, tokens, self.p.block_table(src)[:k])
            self.next_id += 1

        @precondition(lambda self: self.p.tables)
        @rule(data=st.data())
        def append(self, data):
            self._both("append_token", data.draw(st.sampled_from(self.seqs)))

        @precondition(lambda self: self.p.tables)
        @rule(data=st.data())
        def fork(self, data):
            self._both("fork", data.draw(st.sampled_from(self.seqs)), self.next_id)
            self.next_id += 1

        @precondition(lambda self: self.p.tables)
        @rule(data=st.data())
        def free(self, data):
            self._both("free_sequence", data.draw(st.sampled_from(self.seqs)))

        @precondition(lambda self: any(self.p.tables.values()))
        @rule(data=st.data())
        def cache_ref(self, data):  # the prefix cache takes a reference on a live block
            s = data.draw(st.sampled_from([s for s in self.seqs if self.p.tables[s]]))
            b = data.draw(st.sampled_from(self.p.block_table(s)))
            self._both("incref_block", b)
            self.ext.append(b)

        @precondition(lambda self: self.ext)
        @rule(data=st.data())
        def cache_release(self, data):
            b = self.ext.pop(data.draw(st.integers(0, len(self.ext) - 1)))
            self._both("decref_block", b)

        @invariant()
        def same_state(self):
            if not hasattr(self, "p"):
                return
            assert self.n.num_free_blocks == self.p.num_free_blocks
            assert self.n.num_sequences == self.p.num_sequences
            occ = [0] * self.nb
            for s in self.seqs:
                t = self.p.block_table(s)
                assert list(self.n.block_table(s)) == t and self.n.num_tokens(s) == self.p.num_tokens(s)
                for b in t:
                    occ[b] += 1
                if t:
                    n_slots = min(self.p.num_tokens(s), len(t) * self.bs)
                    assert list(self.n.slots(s, 0, n_slots)) == list(self.p.slots(s, 0, n_slots))
            for b in self.ext:
                occ[b] += 1
            for b in range(self.nb):
                assert self.n.refcount(b) == self.p.refcount(b) == occ[b], (b, occ[b])
            assert self.p.num_free_blocks == occ.count(0)

    Machine.TestCase.settings = settings(max_examples=120, stateful_step_count=40, deadline=None)
    Machine.TestCase().runTest()


def test_scheduler_simulation_property():
    """Property test (hypothesis): the continuous-batching scheduler driven by a fake engine
    (the engine's synchronous step: decode rows then prefill chunks, ``computed`` then token
    append, finish at max_tokens) over random request mixes -- shared prompt prefixes, every
    policy, tight KV pools that force preemption, small token budgets, prefix cache on / off.
    Every step respects the token budget and batch size, every chunk continues exactly where its
    sequence stopped and addresses reserved KV slots, every request finishes with its max_tokens,
    the run makes progress (no livelock), and at the end every KV block is free or held only by
    the prefix cache with consistent reference counts."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    from llmctl.serve.prefix_cache import PrefixCache
    from llmctl.serve.scheduler import ContinuousBatchScheduler, SamplingParams, Sequence

    requests = st.lists(st.tuples(st.integers(0, 3), st.integers(1, 40), st.integers(1, 12)), min_size=1, max_size=9)

    @settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.too_slow])
    @given(requests, st.sampled_from(["dynamic", "prefill_first", "static"]), st.sampled_from([1, 4, 16]),
           st.integers(1, 6), st.integers(8, 96), st.booleans(), st.booleans())
    def run(reqs, policy, bs, max_bs, budget, use_pc, native):
        max_len = 64
        nb = (max_len + 2 * bs) // bs + 3  # any single sequence fits: preemption always makes progress
        kv = make_kv_manager(nb, bs, prefer_native=native)
        pc = PrefixCache(kv, bs) if use_pc else None
        sched = ContinuousBatchScheduler(kv, max_bs, budget, max_len, policy, bs, pc)
        bases = [[(7 * j + 3 * k) % 50 + 1 for k in range(40)] for j in range(4)]
        seqs = []
        for base, n, mt in reqs:
            s = Sequence(prompt_ids=bases[base][:n], params=SamplingParams(max_tokens=mt, ignore_eos=True))
            sched.add(s)
            seqs.append(s)
        idle = steps = 0
        while sched.has_work():
            out = sched.schedule()
            steps += 1
            assert steps < 2000
            assert sum(c.count for c in out.prefill) + len(out.decode) <= budget
            assert len(out.decode) <= max_bs and len(sched.running) <= max_bs
            idle = idle + 1 if not (out.prefill or out.decode) else 0
            assert idle < 3, "scheduler made no progress"
            for seq in out.decode:
                assert seq.num_computed == seq.num_tokens - 1 and seq.kv_len == seq.num_tokens
                assert seq._decode_slot == kv.slot(seq.seq_id, seq.num_tokens - 1)
            for c in out.prefill:
                assert c.start == c.seq.num_computed and c.count > 0
                assert c.start + c.count <= c.seq.kv_len == c.seq.num_tokens
                kv.slots(c.seq.seq_id, c.start, c.count)  # reserved positions (raises otherwise)
            for seq in out.decode:
                sched.computed(seq, 1)
            for c in out.prefill:
                sched.computed(c.seq, c.count)
            for seq in list(out.decode) + [c.seq for c in out.prefill if c.final]:
                seq.output_ids.append((seq.seq_id * 31 + len(seq.output_ids)) % 50 + 1)
                if len(seq.output_ids) >= seq.params.max_tokens or seq.num_tokens >= max_len:
                    sched.finish(seq, "length")
        for s in seqs:
            assert s.status == "finished"
            assert len(s.output_ids) == min(s.params.max_tokens, max_len - len(s.prompt_ids)), s
        held = set(pc._owner) if pc is not None else set()
        assert kv.num_free_blocks == nb - len(held)
        assert kv.num_sequences == 0
        for b in range(nb):
            assert kv.refcount(b) == (1 if b in held else 0)

    run()


def test_sampling_oracle_property():
    """Property test (hypothesis) of the sampling oracle (``llmctl.ops.ref.sample``, the semantics
    ``csrc/sampling.hip`` is tested against): temperature <= 0 is the argmax; otherwise the token
    is in the kept set {x >= max(k-th largest, top-p threshold)} with a nonzero weight, the argmax
    is always drawable, the draw is monotone in the uniform (inverse CDF in vocabulary order) and
    u = 0 picks the first drawable token."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from llmctl.ops import ref

    @settings(max_examples=300, deadline=None)
    @given(st.integers(1, 64), st.integers(0, 2**31 - 1), st.one_of(st.just(0.0), st.floats(0.05, 3.0)),
           st.integers(0, 70),
           st.floats(0.05, 1.0), st.floats(0.0, 0.999999), st.floats(0.0, 0.999999))
    def check(V, seed, temp, k, p, u1, u2):
        g = torch.Generator().manual_seed(seed)
        logits = torch.randn(1, V, generator=g) * 3
        if seed % 3 == 0:
            logits = logits.round()  # ties
        T, K, P = torch.tensor([temp]), torch.tensor([k]), torch.tensor([p])
        lo, hi = min(u1, u2), max(u1, u2)
        a = int(ref.sample(logits, T, K, P, torch.tensor([lo]))[0])
        b = int(ref.sample(logits, T, K, P, torch.tensor([hi]))[0])
        if temp <= 0:
            assert a == b == int(torch.argmax(logits[0]))
            return
        x = logits[0].float() / temp
        thr = -float("inf")
        if 0 < k < V:
            thr = float(torch.topk(x, k).values[-1])
        if p < 1.0:
            e = torch.exp(x - x.max())
            sx, si = torch.sort(x, descending=True)
            cum = torch.cumsum(e[si], 0)
            n = int((cum < p * float(e.sum())).sum())
            thr = max(thr, float(sx[min(n, V - 1)]))
        keep = x >= thr
        # drawable: kept with a nonzero weight (a kept token whose exp underflows is never drawn)
        drawable = keep & (torch.exp(x - x.max()) > 0)
        assert bool(drawable[int(torch.argmax(x))])
        assert bool(drawable[a]) and bool(drawable[b])
        assert a <= b
        first = int(torch.nonzero(drawable)[0])
        assert int(ref.sample(logits, T, K, P, torch.tensor([0.0]))[0]) == first

    check()


def test_prefill_work_list_property():
    """Property test (hypothesis): the paged-prefill work list holds every (chunk, 128-row q-block)
    exactly once, decodable from ``(chunk << 16) | block``, ordered by non-increasing causal span."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from llmctl.ops.functional import prefill_work_list

    @settings(max_examples=300, deadline=None)
    @given(st.lists(st.integers(0, 3000), min_size=1, max_size=40))
    def check(lens):
        cu = [0]
        for n in lens:
            cu.append(cu[-1] + n)
        work = prefill_work_list(cu)
        got = [(w >> 16, w & 0xFFFF) for w in work]
        want = {(i, b) for i, n in enumerate(lens) for b in range((n + 127) // 128)}
        assert len(got) == len(want) and set(got) == want
        assert all(a[1] >= b[1] for a, b in zip(got, got[1:]))

    check()
