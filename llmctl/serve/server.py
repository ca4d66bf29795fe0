"""HTTP inference server (FastAPI + uvicorn) around :class:`InferenceEngine`.

Routes (same as the reference, ``server.py:286-311``): ``POST /v1/completions``,
``GET /v1/models``, ``GET /health``; plus ``GET /metrics`` (Prometheus) and SSE streaming
when ``stream=true`` (ignored by the reference).  Request/response schemas keep the
reference fields (``GenerationRequest`` / ``GenerationResponse``, ``server.py:25-37``) and add
OpenAI-style ``choices``.

Concurrency model (fixes SURVEY App. C #1): the engine runs on its own thread, looping
``engine.step()`` while there is work; HTTP handlers enqueue a request and await an
``asyncio.Future`` (or an async token queue for streaming) that the engine thread resolves
via ``loop.call_soon_threadsafe`` — no polling, the event loop is never blocked by model
compute, and unfinished sequences stay scheduled until they finish.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, Field

log = logging.getLogger("llmctl.serve.server")


class GenerationRequest(BaseModel):
    prompt: Union[str, List[int]]
    max_tokens: int = 100
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    stream: bool = False
    stop: Optional[Union[str, List[str]]] = None
    ignore_eos: bool = False
    model: Optional[str] = None


class GenerationResponse(BaseModel):
    id: str
    text: str
    finish_reason: str
    usage: Dict[str, int]
    object: str = "text_completion"
    created: int = 0
    model: str = ""
    choices: List[Dict[str, Any]] = Field(default_factory=list)
    timing: Dict[str, float] = Field(default_factory=dict)


class InferenceServer:
    def __init__(self, model_path: str, host: str = "0.0.0.0", port: int = 8080, max_batch_size: int = 8,
                 max_batch_tokens: int = 8192, max_concurrent: int = 128, scheduler: str = "dynamic",
                 device: str = "auto", kv_cache_fraction: float = 0.85, block_size: int = 16, use_graphs: bool = True,
                 tensor_parallel: int = 1, engine=None, kv_cache_dtype: str = "auto", weight_dtype: str = "auto"):
        from fastapi import FastAPI, HTTPException
        from fastapi.middleware.cors import CORSMiddleware
        from fastapi.responses import PlainTextResponse, StreamingResponse

        self.model_path, self.host, self.port = model_path, host, port
        self.max_concurrent = max_concurrent
        self.engine_kwargs = dict(model_path=model_path, device=device, max_batch_size=max_batch_size,
                                  max_batch_tokens=max_batch_tokens, kv_cache_fraction=kv_cache_fraction,
                                  block_size=block_size, scheduler=scheduler, use_graphs=use_graphs,
                                  kv_cache_dtype=kv_cache_dtype, weight_dtype=weight_dtype)
        if tensor_parallel != 1 and engine is None:
            raise ValueError("TP serving runs one engine per rank under torchrun: use llmctl.serve.tp "
                             "(`llmctl serve start --tensor-parallel N` launches it)")
        self.engine = engine
        self.active_requests: Dict[str, Any] = {}
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        from llmctl.metrics.observability import ObservabilityManager

        self.obs = ObservabilityManager(enable_prometheus=True, prometheus_port=0, collection_interval=5.0)
        from llmctl.metrics.health import HealthManager

        self.health = HealthManager(check_interval=30.0)

        app = FastAPI(title="llmctl inference server", version="0.2.0")
        app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                           allow_headers=["*"])
        self.app = app

        @app.on_event("startup")
        async def _startup():
            self.loop = asyncio.get_running_loop()
            self.start_engine()

        @app.on_event("shutdown")
        async def _shutdown():
            self.stop_engine()
            if getattr(self, "_own_engine", False) and self.engine is not None:
                self.engine.close()
                self.engine = None

        @app.post("/v1/completions")
        async def completions(req: GenerationRequest):
            if len(self.active_requests) >= self.max_concurrent:
                raise HTTPException(status_code=503, detail="Server at capacity")
            if req.stream:
                return StreamingResponse(self._stream(req), media_type="text/event-stream")
            try:
                return await self.handle_generation_request(req)
            except ValueError as e:
                raise HTTPException(status_code=400, detail=str(e))

        @app.get("/v1/models")
        async def models():
            return {"object": "list", "data": [{"id": self.model_name, "object": "model", "created": int(time.time()),
                                                "owned_by": "llmctl"}]}

        @app.get("/health")
        async def health():
            e = self.engine
            sched = e.scheduler if e else None
            return {"status": "healthy" if e is not None else "loading",
                    "active_requests": len(self.active_requests),
                    "pending_requests": sched.num_waiting if sched else 0,
                    "running_sequences": sched.num_running if sched else 0,
                    "kv_cache_usage": round(e.kv.usage(), 4) if e else 0.0,
                    "device": str(e.device) if e else None}

        @app.get("/metrics")
        async def metrics():
            return PlainTextResponse(self.obs.prometheus_exporter.render().decode())

    # ------------------------------------------------------------------ engine thread
    @property
    def model_name(self) -> str:
        return self.engine.cfg.name if self.engine is not None else str(self.model_path)

    def start_engine(self):
        if self.engine is None:
            from .engine import InferenceEngine

            self.engine = InferenceEngine(**self.engine_kwargs)
            self._own_engine = True  # closed by this server's shutdown (a passed-in engine is the caller's)
        if self._thread is None:
            self._stop = False
            self._thread = threading.Thread(target=self._engine_loop, name="llmctl-engine", daemon=True)
            self._thread.start()

    def stop_engine(self):
        self._stop = True
        self._wake.set()
        if self._thread:
            self._thread.join(timeout=10)
            self._thread = None

    def _engine_loop(self):
        e = self.engine
        while not self._stop:
            with self._lock:
                busy = e.scheduler.has_work()
            if not busy:
                self._wake.wait(timeout=0.05)
                self._wake.clear()
                continue
            try:
                with self._lock:
                    e.step()
            except Exception as ex:  # fail all in-flight requests loudly instead of hanging
                with self._lock:
                    for seq in list(e.scheduler.running) + list(e.scheduler.waiting):
                        e.scheduler.finish(seq, f"error: {ex}") if seq.status == "running" else None
                        seq.status = "finished"
                        seq.finish_reason = f"error: {ex}"
                        if seq.on_finish:
                            seq.on_finish(seq)
                    e.scheduler.waiting.clear()
                from .control import PeerLostError

                if isinstance(ex, PeerLostError):
                    # a TP rank is gone: the group cannot serve again.  Give the failed requests a
                    # moment to be answered, then leave non-zero so the launcher tears down the job
                    log.error("TP peer lost, server exiting: %s", ex)
                    threading.Timer(0.5, os._exit, (70,)).start()
                    return

    # ------------------------------------------------------------------ request handling
    def _make_params(self, req: GenerationRequest):
        from .scheduler import SamplingParams

        stop = [req.stop] if isinstance(req.stop, str) else (req.stop or [])
        return SamplingParams(max_tokens=max(1, req.max_tokens), temperature=req.temperature, top_p=req.top_p,
                              top_k=req.top_k, stop=stop, ignore_eos=req.ignore_eos)

    def _encode(self, prompt) -> List[int]:
        if isinstance(prompt, list):
            return [int(t) for t in prompt]
        return self.engine.tokenizer.encode(prompt)

    async def handle_generation_request(self, req: GenerationRequest) -> GenerationResponse:
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()
        rid = f"cmpl-{uuid.uuid4().hex[:16]}"
        t0 = time.time()
        ids = self._encode(req.prompt)

        def on_finish(seq):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(seq))

        with self._lock:
            self.active_requests[rid] = True
            try:
                seq = self.engine.add_request(ids, self._make_params(req), rid, on_finish=on_finish)
            except ValueError:
                self.active_requests.pop(rid, None)
                raise
        self._wake.set()
        try:
            seq = await fut
        finally:
            self.active_requests.pop(rid, None)
        text = self.engine.tokenizer.decode(seq.output_ids)
        lat = time.time() - t0
        ttft = (seq.first_token_time - seq.arrival_time) if seq.first_token_time else lat
        n = len(seq.output_ids)
        tpot = (seq.finish_time - seq.first_token_time) / max(n - 1, 1) if seq.first_token_time and seq.finish_time else 0.0
        self.obs.record_inference_request(lat, ttft=ttft, tpot=tpot)
        self.health.record_inference_request(lat, success=not str(seq.finish_reason).startswith("error"))
        usage = {"prompt_tokens": len(ids), "completion_tokens": n, "total_tokens": len(ids) + n}
        return GenerationResponse(id=rid, text=text, finish_reason=seq.finish_reason or "stop", usage=usage,
                                  created=int(t0), model=self.model_name,
                                  choices=[{"index": 0, "text": text, "finish_reason": seq.finish_reason}],
                                  timing={"latency_s": lat, "ttft_s": ttft, "tpot_s": tpot})

    async def _stream(self, req: GenerationRequest):
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        rid = f"cmpl-{uuid.uuid4().hex[:16]}"

        def on_token(seq, tok):
            loop.call_soon_threadsafe(q.put_nowait, ("tok", tok))

        def on_finish(seq):
            loop.call_soon_threadsafe(q.put_nowait, ("end", seq.finish_reason))

        with self._lock:
            self.active_requests[rid] = True
            self.engine.add_request(self._encode(req.prompt), self._make_params(req), rid, on_token=on_token,
                                    on_finish=on_finish)
        self._wake.set()
        try:
            while True:
                kind, val = await q.get()
                if kind == "tok":
                    payload = {"id": rid, "object": "text_completion", "model": self.model_name,
                               "choices": [{"index": 0, "text": self.engine.tokenizer.decode([val]), "token": val,
                                            "finish_reason": None}]}
                    yield f"data: {json.dumps(payload)}\n\n"
                else:
                    payload = {"id": rid, "choices": [{"index": 0, "text": "", "finish_reason": val}]}
                    yield f"data: {json.dumps(payload)}\n\n"
                    yield "data: [DONE]\n\n"
                    break
        finally:
            self.active_requests.pop(rid, None)

    # ------------------------------------------------------------------ run
    def run(self):
        import uvicorn

        uvicorn.run(self.app, host=self.host, port=self.port, log_level="info")

    async def start_server(self):
        import uvicorn

        config = uvicorn.Config(self.app, host=self.host, port=self.port, log_level="info")
        await uvicorn.Server(config).serve()


def create_inference_server(model_path: str, **kwargs) -> InferenceServer:
    return InferenceServer(model_path, **kwargs)
