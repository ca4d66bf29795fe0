"""Auto-tuner (reference API: ``llmctl/plugins/autotuning.py:21-457``).

Same classes (``TuningConfig``, ``TuningResult``, ``Tunable``, ``MatMulTuner``,
``AttentionTuner``, ``CommunicationTuner``, ``AutoTuner``, ``create_auto_tuner``), same
cache-key and JSON formats — but every knob changes what runs (the
reference's knobs were mostly no-ops and its comm tuning was a random-number simulation):

* MatMul: implementation (hipBLASLt via torch / llmctl's MFMA GEMM kernel), operand layout
  (NT vs NN), dtype; CPU: intra-op thread count and layout;
* Attention: implementation (llmctl flash-attn HIP kernel / torch SDPA / eager), causal;
* Communication: bucket size and op (all-reduce vs reduce-scatter+all-gather) measured on
  the live process group (RCCL on GPU, gloo on CPU); without a process group it measures
  the local chunked copy path and says so in the result (``mode: "local"``);
* HIP kernel knobs (round 2): the gemm64 tile-order group / schedule variant per GEMM
  layout (``Gemm64Tuner``), the paged-decode context split count (``DecodeSplitTuner``), the
  flash-attention forward K/V split (``FlashSplitTuner``) and the decode-GEMM configuration
  (``SkinnyTuner``).  ``save_results`` writes ``tuning_cache.json``; TrainingEngine /
  InferenceEngine read it back through :mod:`llmctl.plugins.tuning_cache` and dispatch the
  tuned configurations.

``max_iterations``, ``warmup`` and ``measurement`` iterations and ``tolerance`` are all
honoured (the reference read only ``timeout``/``tolerance``).
"""

from __future__ import annotations

import itertools
import json
import time
from abc import ABC, abstractmethod
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import torch


@dataclass
class TuningConfig:
    max_iterations: int = 50
    min_runtime: float = 0.1
    warmup_iterations: int = 5
    measurement_iterations: int = 10
    tolerance: float = 0.05
    timeout: float = 300.0


@dataclass
class TuningResult:
    best_config: Dict[str, Any]
    best_performance: float
    improvement: float
    total_time: float
    iterations: int
    all_results: List[Tuple[Dict[str, Any], float]] = field(default_factory=list)


def _dev(device: str) -> torch.device:
    if device == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _time(fn, dev, warmup: int, iters: int) -> float:
    for _ in range(warmup):
        fn()
    _sync(dev)
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(dev)
    return (time.perf_counter() - t) / iters


class Tunable(ABC):
    @abstractmethod
    def get_parameter_space(self) -> Dict[str, List[Any]]:
        ...

    @abstractmethod
    def set_parameters(self, params: Dict[str, Any]) -> None:
        ...

    @abstractmethod
    def benchmark(self, config: TuningConfig) -> float:
        """Seconds per call (lower is better)."""

    def validate_parameters(self, params: Dict[str, Any]) -> bool:
        return True


class MatMulTuner(Tunable):
    def __init__(self, shape: Tuple[int, int, int], device: str = "auto"):
        self.m, self.k, self.n = shape
        self.dev = _dev(device)
        self.params: Dict[str, Any] = {}

    def get_parameter_space(self):
        if self.dev.type == "cuda":
            return {"implementation": ["hipblaslt", "llmctl_mfma"], "layout": ["NT", "NN"],
                    "dtype": ["bfloat16", "float16"]}
        import os

        n = os.cpu_count() or 4
        return {"num_threads": sorted({1, max(n // 2, 1), n}), "layout": ["NT", "NN"]}

    def validate_parameters(self, p):
        if p.get("implementation") == "llmctl_mfma":
            return p.get("dtype") == "bfloat16" and p.get("layout") == "NT" and self.k % 64 == 0 and \
                self.m % 256 == 0 and self.n % 256 == 0
        return True

    def set_parameters(self, params):
        self.params = params
        dt = getattr(torch, params.get("dtype", "float32")) if self.dev.type == "cuda" else torch.float32
        g = torch.Generator(device="cpu").manual_seed(0)
        self.a = torch.randn(self.m, self.k, generator=g).to(self.dev, dt)
        b = torch.randn(self.n, self.k, generator=g).to(self.dev, dt)
        self.b = b if params.get("layout") == "NT" else b.t().contiguous()
        if "num_threads" in params:
            torch.set_num_threads(int(params["num_threads"]))

    def benchmark(self, config: TuningConfig) -> float:
        p = self.params
        if p.get("implementation") == "llmctl_mfma":
            from llmctl.ops import _lib

            ops = _lib.native()
            fn = lambda: ops.gemm_bf16(self.a, self.b)  # noqa: E731
        elif p.get("layout") == "NT":
            fn = lambda: self.a @ self.b.t()  # noqa: E731
        else:
            fn = lambda: self.a @ self.b  # noqa: E731
        return _time(fn, self.dev, config.warmup_iterations, config.measurement_iterations)


class AttentionTuner(Tunable):
    def __init__(self, seq_len: int, head_dim: int, batch_size: int = 8, num_heads: int = 8, device: str = "auto"):
        self.S, self.D, self.B, self.H = seq_len, head_dim, batch_size, num_heads
        self.dev = _dev(device)
        self.params: Dict[str, Any] = {}

    def get_parameter_space(self):
        impl = ["llmctl_flash", "sdpa", "eager"] if self.dev.type == "cuda" else ["sdpa", "eager"]
        return {"implementation": impl, "causal_mask": [True, False]}

    def validate_parameters(self, p):
        return not (p["implementation"] == "llmctl_flash" and self.D not in (64, 128))

    def set_parameters(self, params):
        self.params = params
        dt = torch.bfloat16 if self.dev.type == "cuda" else torch.float32
        g = torch.Generator(device="cpu").manual_seed(0)
        self.q, self.k, self.v = (torch.randn(self.B, self.S, self.H, self.D, generator=g).to(self.dev, dt)
                                  for _ in range(3))

    def benchmark(self, config):
        p = self.params
        causal = bool(p.get("causal_mask"))
        scale = self.D ** -0.5
        if p["implementation"] == "llmctl_flash":
            from llmctl.ops import _lib

            ops = _lib.native()
            fn = lambda: ops.flash_attn_fwd(self.q, self.k, self.v, scale, causal)  # noqa: E731
        elif p["implementation"] == "sdpa":
            qt, kt, vt = (t.transpose(1, 2) for t in (self.q, self.k, self.v))
            fn = lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)  # noqa
        else:
            from llmctl.ops import ref

            fn = lambda: ref.attention_fwd(self.q, self.k, self.v, scale, causal)  # noqa: E731
        return _time(fn, self.dev, max(1, config.warmup_iterations // 2), max(1, config.measurement_iterations // 2))


class CommunicationTuner(Tunable):
    def __init__(self, tensor_shape: Tuple[int, ...], dtype=torch.float32, device: str = "auto"):
        self.shape = tensor_shape
        self.dtype = dtype
        self.dev = _dev(device)
        self.params: Dict[str, Any] = {}
        import torch.distributed as dist

        self.live = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.mode = "process_group" if self.live else "local"

    def get_parameter_space(self):
        return {"bucket_mb": [1, 4, 16, 64, 256], "algorithm": ["allreduce", "reduce_scatter_all_gather"]}

    def set_parameters(self, params):
        self.params = params
        self.x = torch.ones(*self.shape, dtype=self.dtype, device=self.dev)

    def benchmark(self, config):
        import torch.distributed as dist

        flat = self.x.reshape(-1)
        esz = flat.element_size()
        chunk = max(1, int(self.params["bucket_mb"] * 2 ** 20 // esz))
        algo = self.params["algorithm"]
        if self.live:
            ws = dist.get_world_size()

            def fn():
                for s in range(0, flat.numel(), chunk):
                    v = flat[s:s + chunk]
                    if algo == "allreduce" or v.numel() % ws:
                        dist.all_reduce(v)
                    else:
                        out = torch.empty(v.numel() // ws, dtype=v.dtype, device=v.device)
                        dist.reduce_scatter_tensor(out, v)
                        dist.all_gather_into_tensor(v, out)
        else:
            dst = torch.empty_like(flat)

            def fn():
                for s in range(0, flat.numel(), chunk):
                    dst[s:s + chunk].copy_(flat[s:s + chunk])
                    if algo != "allreduce":
                        flat[s:s + chunk].copy_(dst[s:s + chunk])
        return _time(fn, self.dev, max(1, config.warmup_iterations // 2), config.measurement_iterations)


def _knob(name: str, value: int):
    """A performance knob (llmctl.config.knobs; native ones reach the HIP launchers' table) set
    for the duration of one measurement."""
    from llmctl.config.knobs import override

    return override(**{name: value})


class Gemm64Tuner(Tunable):
    """gemm64_ex configuration (tile-order group + 100 * schedule variant) for one GEMM of a
    linear layer: ``layout`` fwd (x W^T), dgrad (dy W) or wgrad (dy^T x) with M tokens.  The
    schedules: 1xx the 8-wave kernel, 3xx the persistent 4-wave kernel, 9xx the one-shot 4-wave
    kernel; group 4 or 8 tile-rows per tile-order group."""

    LAYOUTS = {"fwd": (False, False), "dgrad": (False, True), "wgrad": (True, True)}

    def __init__(self, M: int, N: int, K: int, layout: str = "dgrad", device: str = "auto"):
        self.M, self.N, self.K, self.layout = M, N, K, layout
        self.dev = _dev(device)

    def get_parameter_space(self):
        return {"config": [104, 108, 304, 308, 904, 908]}

    def validate_parameters(self, p):
        return self.dev.type == "cuda" and self.M % 256 == 0 and self.N % 256 == 0 and self.K % 128 == 0

    def set_parameters(self, params):
        self.params = params
        at, bt = self.LAYOUTS[self.layout]
        g = torch.Generator(device="cpu").manual_seed(0)
        A = (torch.rand(self.M, self.K, generator=g) * 2 - 1).to(self.dev, torch.bfloat16)
        B = (torch.rand(self.N, self.K, generator=g) * 2 - 1).to(self.dev, torch.bfloat16)
        self.a = A.t().contiguous() if at else A
        self.b = B.t().contiguous() if bt else B
        self.out = torch.empty(self.M, self.N, device=self.dev, dtype=torch.bfloat16)
        self.flags = (at, bt)

    def benchmark(self, config):
        from llmctl.ops import _lib

        ops = _lib.native()
        c = int(self.params["config"])
        fn = lambda: ops.gemm64_ex(self.a, self.b, self.out, self.flags[0], self.flags[1], False, c)  # noqa: E731
        return _time(fn, self.dev, config.warmup_iterations, config.measurement_iterations)


class DecodeSplitTuner(Tunable):
    """Paged-attention decode: context splits per (sequence, kv-head) (knob ``decode_splits``)."""

    def __init__(self, batch: int, ctx: int, heads: int = 32, kv_heads: int = 32, head_dim: int = 128,
                 block_size: int = 16, device: str = "auto"):
        self.N, self.ctx, self.H, self.Hkv, self.D, self.bs = batch, ctx, heads, kv_heads, head_dim, block_size
        self.dev = _dev(device)

    def get_parameter_space(self):
        return {"splits": [1, 2, 4, 8, 16]}

    def validate_parameters(self, p):
        return self.dev.type == "cuda"

    def set_parameters(self, params):
        self.params = params
        nbs = (self.ctx + self.bs - 1) // self.bs
        nb = self.N * nbs
        self.kc = torch.randn(nb, self.bs, self.Hkv, self.D, device=self.dev, dtype=torch.bfloat16)
        self.vc = torch.randn_like(self.kc)
        self.bt = torch.randperm(nb, device=self.dev).to(torch.int32).view(self.N, nbs).contiguous()
        self.lens = torch.full((self.N,), self.ctx, device=self.dev, dtype=torch.int32)
        self.q = torch.randn(self.N, self.H, self.D, device=self.dev, dtype=torch.bfloat16)

    def benchmark(self, config):
        from llmctl.ops import _lib

        ops = _lib.native()
        with _knob("decode_splits", int(self.params["splits"])):
            fn = lambda: ops.paged_attention_decode(self.q, self.kc, self.vc, self.bt, self.lens, self.D ** -0.5)  # noqa
            return _time(fn, self.dev, config.warmup_iterations, config.measurement_iterations)


class FlashSplitTuner(Tunable):
    """Flash-attention forward: split every causal q-block's K/V range over two workgroups
    (+ combine) or not (knob ``fa_split``); pays off on small grids (short prefills)."""

    def __init__(self, batch: int, seq_len: int, heads: int = 32, head_dim: int = 128, device: str = "auto"):
        self.B, self.S, self.H, self.D = batch, seq_len, heads, head_dim
        self.dev = _dev(device)

    def get_parameter_space(self):
        return {"split": [0, 1]}

    def validate_parameters(self, p):
        return self.dev.type == "cuda" and self.D in (64, 128)

    def set_parameters(self, params):
        self.params = params
        g = torch.Generator(device="cpu").manual_seed(0)
        self.q, self.k, self.v = (torch.randn(self.B, self.S, self.H, self.D, generator=g).to(self.dev, torch.bfloat16)
                                  for _ in range(3))

    def benchmark(self, config):
        from llmctl.ops import _lib

        ops = _lib.native()
        with _knob("fa_split", int(self.params["split"])):
            fn = lambda: ops.flash_attn_fwd(self.q, self.k, self.v, self.D ** -0.5, True, None)  # noqa: E731
            return _time(fn, self.dev, config.warmup_iterations, config.measurement_iterations)


class SkinnyTuner(Tunable):
    """Decode GEMM (M <= 32 tokens): hipBLASLt (config 0 here) or one of the weight-streaming
    MFMA kernel's configurations (``skinny_linear_cfg``), on uncached weights."""

    def __init__(self, M: int, N: int, K: int, device: str = "auto"):
        self.M, self.N, self.K = M, N, K
        self.dev = _dev(device)

    def get_parameter_space(self):
        return {"config": [0, 1, 2, 3, 4, 5, 7]}

    def validate_parameters(self, p):
        return self.dev.type == "cuda" and self.M <= 32 and self.N % 32 == 0 and self.K % 128 == 0

    def set_parameters(self, params):
        self.params = params
        pool = max(2, int(1e9 // (self.N * self.K * 2)))
        self.ws = [torch.randn(self.N, self.K, device=self.dev, dtype=torch.bfloat16) for _ in range(pool)]
        self.x = torch.randn(self.M, self.K, device=self.dev, dtype=torch.bfloat16)

    def benchmark(self, config):
        from llmctl.ops import _lib

        ops = _lib.native()
        c = int(self.params["config"])
        it = [0]

        def fn():
            w = self.ws[it[0] % len(self.ws)]
            it[0] += 1
            return torch.nn.functional.linear(self.x, w) if c == 0 else ops.skinny_linear_cfg(self.x, w, None, c)
        return _time(fn, self.dev, config.warmup_iterations, config.measurement_iterations)


class AutoTuner:
    def __init__(self, config: Optional[TuningConfig] = None):
        self.config = config or TuningConfig()
        self.cache: Dict[str, TuningResult] = {}

    def grid_search(self, tunable: Tunable, key: Optional[str] = None) -> TuningResult:
        if key and key in self.cache:
            return self.cache[key]
        space = tunable.get_parameter_space()
        names = list(space)
        t0 = time.time()
        results: List[Tuple[Dict[str, Any], float]] = []
        best_cfg, best = None, float("inf")
        for values in itertools.product(*(space[n] for n in names)):
            if len(results) >= self.config.max_iterations or time.time() - t0 > self.config.timeout:
                break
            params = dict(zip(names, values))
            if not tunable.validate_parameters(params):
                continue
            try:
                tunable.set_parameters(params)
                perf = tunable.benchmark(self.config)
            except Exception as e:  # unsupported combination on this device
                results.append((dict(params, error=str(e)[:120]), float("inf")))
                continue
            results.append((params, perf))
            if perf < best:
                best, best_cfg = perf, params
        finite = [p for _, p in results if p != float("inf")]
        baseline = finite[0] if finite else float("inf")
        improvement = 100.0 * (baseline - best) / baseline if finite and baseline > 0 else 0.0
        res = TuningResult(best_cfg or {}, best, improvement, time.time() - t0, len(results), results)
        if key:
            self.cache[key] = res
        return res

    def tune_matmul(self, shape: Tuple[int, int, int], device: str = "auto") -> TuningResult:
        d = _dev(device)
        return self.grid_search(MatMulTuner(shape, device), f"matmul_{tuple(shape)}_{d.type}")

    def tune_attention(self, seq_len: int, head_dim: int, batch_size: int = 8, num_heads: int = 8,
                       device: str = "auto") -> TuningResult:
        d = _dev(device)
        return self.grid_search(AttentionTuner(seq_len, head_dim, batch_size, num_heads, device),
                                f"attention_{seq_len}_{head_dim}_{d.type}")

    def tune_communication(self, tensor_shape: Tuple[int, ...], dtype=torch.float32, device: str = "auto"
                           ) -> TuningResult:
        t = CommunicationTuner(tensor_shape, dtype, device)
        res = self.grid_search(t, f"comm_{tuple(tensor_shape)}_{dtype}")
        res.best_config = dict(res.best_config, mode=t.mode)
        return res

    # ---- HIP kernel knobs (consumed by llmctl.plugins.tuning_cache)
    def tune_gemm64(self, M: int, N: int, K: int, layout: str = "dgrad", device: str = "auto") -> TuningResult:
        return self.grid_search(Gemm64Tuner(M, N, K, layout, device), f"gemm64_{layout}_{M}x{N}x{K}")

    def tune_decode_splits(self, batch: int, ctx: int, heads: int = 32, kv_heads: int = 32, head_dim: int = 128,
                           device: str = "auto") -> TuningResult:
        return self.grid_search(DecodeSplitTuner(batch, ctx, heads, kv_heads, head_dim, device=device),
                                f"decode_splits_{batch}x{ctx}x{kv_heads}")

    def tune_fa_split(self, batch: int, seq_len: int, heads: int = 32, head_dim: int = 128,
                      device: str = "auto") -> TuningResult:
        return self.grid_search(FlashSplitTuner(batch, seq_len, heads, head_dim, device),
                                f"fa_split_{batch}x{seq_len}x{heads}x{head_dim}")

    def tune_skinny(self, M: int, N: int, K: int, device: str = "auto") -> TuningResult:
        return self.grid_search(SkinnyTuner(M, N, K, device), f"skinny_{M}x{N}x{K}")

    def save_results(self, filepath: str) -> None:
        data = {k: {"best_config": r.best_config, "best_performance": r.best_performance,
                    "improvement": r.improvement, "total_time": r.total_time, "iterations": r.iterations}
                for k, r in self.cache.items()}
        with open(filepath, "w") as f:
            json.dump(data, f, indent=2)

    def load_results(self, filepath: str) -> None:
        with open(filepath) as f:
            data = json.load(f)
        for k, v in data.items():
            self.cache[k] = TuningResult(v["best_config"], v["best_performance"], v["improvement"],
                                         v["total_time"], v["iterations"])


def create_auto_tuner(config: Optional[TuningConfig] = None) -> AutoTuner:
    return AutoTuner(config)
