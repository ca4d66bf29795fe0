"""Observability: metrics collection, Prometheus / OpenTelemetry / JSONL export.

API parity with the reference (``llmctl/metrics/observability.py:26-428``): the
``SystemMetrics``/``TrainingMetrics``/``InferenceMetrics`` dataclasses, ``MetricsCollector``,
``PrometheusExporter`` (same ``llmctl_*`` metric names), ``OpenTelemetryExporter`` (spans
``training_step`` / ``inference_request``), ``ObservabilityManager``,
``setup_observability`` / ``get_observability_manager``.  Differences: it is actually wired
into training (:func:`attach_training_metrics`) and serving; GPU utilisation/memory/power
come from amdsmi/sysfs (``llmctl.metrics.gpu``); MFU, TTFT and TPOT are exported; OTel is
optional (the package is not installed on this image) and degrades to a no-op; every rank
can stream JSONL records.
"""

from __future__ import annotations

import json
import os
import threading
import time
from collections import deque
from dataclasses import asdict, dataclass, field
from typing import Any, Deque, Dict, List, Optional

from rich.console import Console

console = Console()


@dataclass
class SystemMetrics:
    cpu_percent: float = 0.0
    memory_percent: float = 0.0
    memory_used_gb: float = 0.0
    memory_total_gb: float = 0.0
    gpu_utilization: List[float] = field(default_factory=list)
    gpu_memory_used: List[float] = field(default_factory=list)
    gpu_memory_total: List[float] = field(default_factory=list)
    gpu_power_w: List[float] = field(default_factory=list)
    network_sent_mbps: float = 0.0
    network_recv_mbps: float = 0.0
    disk_read_mbps: float = 0.0
    disk_write_mbps: float = 0.0


@dataclass
class TrainingMetrics:
    loss: float = 0.0
    learning_rate: float = 0.0
    gradient_norm: float = 0.0
    tokens_per_second: float = 0.0
    samples_per_second: float = 0.0
    step: int = 0
    epoch: int = 0
    flops_per_second: float = 0.0
    mfu: float = 0.0
    step_time: float = 0.0


@dataclass
class InferenceMetrics:
    request_latency: float = 0.0
    tokens_per_second: float = 0.0
    batch_size: int = 0
    queue_length: int = 0
    active_requests: int = 0
    throughput_requests_per_second: float = 0.0
    ttft: float = 0.0
    tpot: float = 0.0


class MetricsCollector:
    """Background thread sampling system/GPU metrics; holds the latest training/inference
    metrics and a bounded history (1000 points, as the reference)."""

    def __init__(self, collection_interval: float = 1.0, history: int = 1000):
        self.collection_interval = collection_interval
        self.system_metrics = SystemMetrics()
        self.training_metrics = TrainingMetrics()
        self.inference_metrics = InferenceMetrics()
        self.system_history: Deque[Dict[str, Any]] = deque(maxlen=history)
        self.training_history: Deque[Dict[str, Any]] = deque(maxlen=history)
        self.inference_history: Deque[Dict[str, Any]] = deque(maxlen=history)
        self._lock = threading.Lock()
        self._running = False
        self._thread: Optional[threading.Thread] = None
        self._last_net = None
        self._last_disk = None
        self._last_t = None

    def start_collection(self):
        if self._running:
            return
        self._running = True
        self._thread = threading.Thread(target=self._collection_loop, daemon=True)
        self._thread.start()

    def stop_collection(self):
        self._running = False
        if self._thread:
            self._thread.join(timeout=2 * self.collection_interval + 1)

    def _collection_loop(self):
        while self._running:
            try:
                self._collect_system_metrics()
            except Exception:
                pass
            time.sleep(self.collection_interval)

    def _collect_system_metrics(self):
        import psutil

        from .gpu import gpu_stats

        now = time.time()
        vm = psutil.virtual_memory()
        net = psutil.net_io_counters()
        disk = psutil.disk_io_counters()
        sm = SystemMetrics(cpu_percent=psutil.cpu_percent(interval=None), memory_percent=vm.percent,
                           memory_used_gb=vm.used / 1e9, memory_total_gb=vm.total / 1e9)
        if self._last_t is not None:
            dt = max(now - self._last_t, 1e-6)
            if net and self._last_net:
                sm.network_sent_mbps = (net.bytes_sent - self._last_net.bytes_sent) * 8 / 1e6 / dt
                sm.network_recv_mbps = (net.bytes_recv - self._last_net.bytes_recv) * 8 / 1e6 / dt
            if disk and self._last_disk:
                sm.disk_read_mbps = (disk.read_bytes - self._last_disk.read_bytes) / 1e6 / dt
                sm.disk_write_mbps = (disk.write_bytes - self._last_disk.write_bytes) / 1e6 / dt
        self._last_net, self._last_disk, self._last_t = net, disk, now
        for g in gpu_stats():
            sm.gpu_utilization.append(float(g.get("utilization", 0.0)))
            sm.gpu_memory_used.append(float(g.get("memory_used_gb", 0.0)))
            sm.gpu_memory_total.append(float(g.get("memory_total_gb", 0.0)))
            sm.gpu_power_w.append(float(g.get("power_w", 0.0)))
        with self._lock:
            self.system_metrics = sm
            self.system_history.append({"t": now, **asdict(sm)})

    def update_training_metrics(self, **kwargs):
        with self._lock:
            for k, v in kwargs.items():
                if hasattr(self.training_metrics, k):
                    setattr(self.training_metrics, k, v)
            self.training_history.append({"t": time.time(), **asdict(self.training_metrics)})

    def update_inference_metrics(self, **kwargs):
        with self._lock:
            for k, v in kwargs.items():
                if hasattr(self.inference_metrics, k):
                    setattr(self.inference_metrics, k, v)
            self.inference_history.append({"t": time.time(), **asdict(self.inference_metrics)})

    def get_summary(self) -> Dict[str, Any]:
        with self._lock:
            return {"system": asdict(self.system_metrics), "training": asdict(self.training_metrics),
                    "inference": asdict(self.inference_metrics),
                    "history_sizes": {"system": len(self.system_history), "training": len(self.training_history),
                                      "inference": len(self.inference_history)}}


class PrometheusExporter:
    """Reference metric names (``observability.py:237-251``) + MFU, grad-norm, TTFT/TPOT."""

    def __init__(self, port: int = 8000, registry=None):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

        self.port = port
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.training_loss = Gauge("llmctl_training_loss", "Current training loss", registry=r)
        self.training_lr = Gauge("llmctl_training_learning_rate", "Current learning rate", registry=r)
        self.training_step = Counter("llmctl_training_steps_total", "Total training steps", registry=r)
        self.training_tokens_per_sec = Gauge("llmctl_training_tokens_per_second", "Training tokens per second",
                                             registry=r)
        self.training_mfu = Gauge("llmctl_training_mfu", "Model FLOPs utilisation vs dense bf16 peak", registry=r)
        self.training_grad_norm = Gauge("llmctl_training_grad_norm", "Global gradient norm", registry=r)
        self.inference_latency = Histogram("llmctl_inference_latency_seconds", "Request latency", registry=r)
        self.inference_ttft = Histogram("llmctl_inference_ttft_seconds", "Time to first token", registry=r,
                                        buckets=(.005, .01, .025, .05, .1, .25, .5, 1, 2.5, 5, 10))
        self.inference_tpot = Histogram("llmctl_inference_tpot_seconds", "Time per output token", registry=r,
                                        buckets=(.001, .0025, .005, .01, .025, .05, .1, .25))
        self.inference_requests = Counter("llmctl_inference_requests_total", "Total inference requests", registry=r)
        self.inference_active = Gauge("llmctl_inference_active_requests", "Active inference requests", registry=r)
        self.inference_throughput = Gauge("llmctl_inference_tokens_per_second", "Inference tokens per second",
                                          registry=r)
        self.system_cpu = Gauge("llmctl_system_cpu_percent", "CPU utilization", registry=r)
        self.system_memory = Gauge("llmctl_system_memory_percent", "Memory utilization", registry=r)
        self.system_gpu_memory = Gauge("llmctl_system_gpu_memory_used_gb", "GPU memory used", ["gpu_id"],
                                       registry=r)
        self.system_gpu_util = Gauge("llmctl_system_gpu_utilization_percent", "GPU busy percent", ["gpu_id"],
                                     registry=r)
        self._server = None

    def start_server(self):
        from prometheus_client import start_http_server

        if self.port and self._server is None:
            self._server = start_http_server(self.port, registry=self.registry)

    def update_metrics(self, collector: MetricsCollector):
        s = collector.get_summary()
        sysm, tr = s["system"], s["training"]
        self.system_cpu.set(sysm["cpu_percent"])
        self.system_memory.set(sysm["memory_percent"])
        for i, (u, m) in enumerate(zip(sysm["gpu_utilization"], sysm["gpu_memory_used"])):
            self.system_gpu_memory.labels(gpu_id=str(i)).set(m)
            self.system_gpu_util.labels(gpu_id=str(i)).set(u)
        self.training_loss.set(tr["loss"])
        self.training_lr.set(tr["learning_rate"])
        self.training_tokens_per_sec.set(tr["tokens_per_second"])
        self.training_mfu.set(tr["mfu"])
        self.training_grad_norm.set(tr["gradient_norm"])

    def render(self) -> bytes:
        from prometheus_client import generate_latest

        return generate_latest(self.registry)


class OpenTelemetryExporter:
    """OTLP/HTTP traces + metrics when ``opentelemetry`` is importable, else a no-op."""

    def __init__(self, endpoint: Optional[str] = None):
        self.endpoint = endpoint or os.environ.get("LLMCTL_OTLP_ENDPOINT", "http://localhost:4318")
        self.enabled = False
        try:
            from opentelemetry import metrics, trace  # type: ignore
            from opentelemetry.exporter.otlp.proto.http.metric_exporter import OTLPMetricExporter  # type: ignore
            from opentelemetry.exporter.otlp.proto.http.trace_exporter import OTLPSpanExporter  # type: ignore
            from opentelemetry.sdk.metrics import MeterProvider  # type: ignore
            from opentelemetry.sdk.metrics.export import PeriodicExportingMetricReader  # type: ignore
            from opentelemetry.sdk.trace import TracerProvider  # type: ignore
            from opentelemetry.sdk.trace.export import BatchSpanProcessor  # type: ignore

            tp = TracerProvider()
            tp.add_span_processor(BatchSpanProcessor(OTLPSpanExporter(endpoint=f"{self.endpoint}/v1/traces")))
            trace.set_tracer_provider(tp)
            reader = PeriodicExportingMetricReader(OTLPMetricExporter(endpoint=f"{self.endpoint}/v1/metrics"),
                                                   export_interval_millis=5000)
            metrics.set_meter_provider(MeterProvider(metric_readers=[reader]))
            self.tracer = trace.get_tracer("llmctl")
            self.meter = metrics.get_meter("llmctl")
            self.training_loss_histogram = self.meter.create_histogram("llmctl.training.loss")
            self.inference_latency_histogram = self.meter.create_histogram("llmctl.inference.latency", unit="s")
            self.enabled = True
        except Exception:
            self.tracer = None

    def record_training_step(self, loss: float, step: int, **attributes):
        if not self.enabled:
            return
        with self.tracer.start_as_current_span("training_step") as span:
            span.set_attribute("step", step)
            span.set_attribute("loss", loss)
            for k, v in attributes.items():
                span.set_attribute(k, v)
            self.training_loss_histogram.record(loss, attributes)

    def record_inference_request(self, latency: float, **attributes):
        if not self.enabled:
            return
        with self.tracer.start_as_current_span("inference_request") as span:
            span.set_attribute("latency", latency)
            self.inference_latency_histogram.record(latency, attributes)


class JSONLExporter:
    """One JSON object per record, per rank (structured logs the reference lacks)."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "a", buffering=1)
        self._lock = threading.Lock()

    def write(self, kind: str, rec: Dict[str, Any]):
        with self._lock:
            self._f.write(json.dumps({"kind": kind, "time": time.time(), **rec}, default=float) + "\n")

    def close(self):
        self._f.close()


class ObservabilityManager:
    def __init__(self, enable_prometheus: bool = True, prometheus_port: int = 8000, enable_otlp: bool = False,
                 otlp_endpoint: Optional[str] = None, collection_interval: float = 1.0,
                 jsonl_path: Optional[str] = None):
        self.collector = MetricsCollector(collection_interval)
        self.prometheus_exporter = PrometheusExporter(prometheus_port) if enable_prometheus else None
        self.otlp_exporter = OpenTelemetryExporter(otlp_endpoint) if enable_otlp else None
        self.jsonl = JSONLExporter(jsonl_path) if jsonl_path else None
        self._updating = False
        self._update_thread: Optional[threading.Thread] = None

    def start(self):
        self.collector.start_collection()
        if self.prometheus_exporter and self.prometheus_exporter.port:
            try:
                self.prometheus_exporter.start_server()
            except OSError as e:
                console.print(f"[yellow]prometheus exporter not started: {e}[/yellow]")
        self._updating = True
        self._update_thread = threading.Thread(target=self._update_loop, daemon=True)
        self._update_thread.start()

    def stop(self):
        self._updating = False
        self.collector.stop_collection()
        if self.jsonl:
            self.jsonl.close()

    def _update_loop(self):
        while self._updating:
            if self.prometheus_exporter:
                try:
                    self.prometheus_exporter.update_metrics(self.collector)
                except Exception:
                    pass
            time.sleep(5.0)

    def record_training_step(self, **kwargs):
        self.collector.update_training_metrics(**kwargs)
        if self.prometheus_exporter:
            self.prometheus_exporter.training_step.inc()
            self.prometheus_exporter.update_metrics(self.collector)
        if self.otlp_exporter:
            self.otlp_exporter.record_training_step(kwargs.get("loss", 0.0), kwargs.get("step", 0))
        if self.jsonl:
            self.jsonl.write("train_step", kwargs)

    def record_inference_request(self, latency: float, **kwargs):
        self.collector.update_inference_metrics(request_latency=latency, **kwargs)
        if self.prometheus_exporter:
            pe = self.prometheus_exporter
            pe.inference_latency.observe(latency)
            pe.inference_requests.inc()
            if kwargs.get("ttft") is not None:
                pe.inference_ttft.observe(kwargs["ttft"])
            if kwargs.get("tpot"):
                pe.inference_tpot.observe(kwargs["tpot"])
        if self.otlp_exporter:
            self.otlp_exporter.record_inference_request(latency)
        if self.jsonl:
            self.jsonl.write("inference_request", {"latency": latency, **kwargs})

    def get_metrics_summary(self) -> Dict[str, Any]:
        return self.collector.get_summary()


_manager: Optional[ObservabilityManager] = None


def get_observability_manager() -> Optional[ObservabilityManager]:
    return _manager


def setup_observability(**kwargs) -> ObservabilityManager:
    global _manager
    if _manager is not None:
        _manager.stop()
    _manager = ObservabilityManager(**kwargs)
    _manager.start()
    return _manager


def attach_training_metrics(engine, jsonl_path: Optional[str] = None, prometheus_port: int = 0,
                            otlp_endpoint: Optional[str] = None):
    """Wire an :class:`ObservabilityManager` and the health monitor into a TrainingEngine's
    logging hook (loss, lr, grad-norm, tokens/s, MFU per logged step)."""
    from .health import get_health_manager, setup_health_monitoring

    mgr = ObservabilityManager(enable_prometheus=bool(prometheus_port), prometheus_port=prometheus_port,
                               enable_otlp=bool(otlp_endpoint or os.environ.get("LLMCTL_OTLP_ENDPOINT")),
                               otlp_endpoint=otlp_endpoint, jsonl_path=jsonl_path, collection_interval=5.0)
    mgr.start()
    hm = get_health_manager() or setup_health_monitoring(check_interval=60.0, start=False)

    def hook(rec: Dict[str, Any]):
        mgr.record_training_step(loss=rec["loss"], learning_rate=rec["lr"], gradient_norm=rec["grad_norm"],
                                 tokens_per_second=rec["tokens_per_sec"], step=rec["step"], mfu=rec["mfu"],
                                 step_time=rec["step_time"])
        hm.update_training_metrics(loss=rec["loss"], grad_norm=rec["grad_norm"], step=rec["step"])

    engine.metrics_hooks.append(hook)
    engine.observability = mgr
    return mgr
