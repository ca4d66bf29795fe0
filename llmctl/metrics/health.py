"""Health monitoring (reference: ``llmctl/metrics/health.py:19-437``, same API).

Monitors: system (CPU / memory / disk / GPU memory with the reference thresholds — keyed
correctly this time, SURVEY App. C #9 — plus GPU temperature from amdgpu hwmon), training
(staleness < 300 s, finite loss, 0.001 < grad-norm < 100, NaN streak), inference (error rate
< 5 %, mean latency < 10 s, activity < 600 s, active < 100).  ``HealthManager`` runs them
on a thread, keeps a 1000-entry history, fires alert callbacks, and saves the JSON report
``{component: {component, status, checks, metrics, message, timestamp}}``.
"""

from __future__ import annotations

import json
import math
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from enum import Enum
from typing import Callable, Deque, Dict, List, Optional

from rich.console import Console

console = Console()


class HealthStatus(Enum):
    HEALTHY = "healthy"
    WARNING = "warning"
    CRITICAL = "critical"
    UNKNOWN = "unknown"


@dataclass
class HealthCheck:
    name: str
    check_function: Callable[[], bool]
    critical: bool = False
    warning_threshold: Optional[float] = None
    critical_threshold: Optional[float] = None
    description: str = ""


@dataclass
class HealthReport:
    component: str
    status: HealthStatus
    checks: Dict[str, bool] = field(default_factory=dict)
    metrics: Dict[str, float] = field(default_factory=dict)
    message: str = ""
    timestamp: float = field(default_factory=time.time)

    def to_dict(self):
        return {"component": self.component, "status": self.status.value, "checks": self.checks,
                "metrics": self.metrics, "message": self.message, "timestamp": self.timestamp}


def _grade(value: float, warn: float, crit: float) -> HealthStatus:
    if value >= crit:
        return HealthStatus.CRITICAL
    if value >= warn:
        return HealthStatus.WARNING
    return HealthStatus.HEALTHY


def _worst(statuses: List[HealthStatus]) -> HealthStatus:
    order = [HealthStatus.CRITICAL, HealthStatus.WARNING, HealthStatus.UNKNOWN, HealthStatus.HEALTHY]
    for s in order:
        if s in statuses:
            return s
    return HealthStatus.HEALTHY


class SystemHealthMonitor:
    THRESHOLDS = {"cpu_usage": (80.0, 95.0), "memory_usage": (85.0, 95.0), "disk_usage": (85.0, 95.0),
                  "gpu_memory_usage": (90.0, 98.0), "gpu_temperature": (90.0, 100.0)}

    def __init__(self, cpu_sample_interval: float = 0.2):
        self.cpu_sample_interval = cpu_sample_interval
        self.checks = [HealthCheck(n, lambda: True, critical=n != "cpu_usage", warning_threshold=w,
                                   critical_threshold=c) for n, (w, c) in self.THRESHOLDS.items()]

    def _metrics(self) -> Dict[str, float]:
        import psutil

        from .gpu import gpu_stats

        m = {"cpu_usage": psutil.cpu_percent(interval=self.cpu_sample_interval),
             "memory_usage": psutil.virtual_memory().percent, "disk_usage": psutil.disk_usage("/").percent}
        gs = gpu_stats()
        if gs:
            fr = [100.0 * g.get("memory_used_gb", 0) / g["memory_total_gb"] for g in gs if g.get("memory_total_gb")]
            if fr:
                m["gpu_memory_usage"] = max(fr)
            temps = [g["temperature_c"] for g in gs if "temperature_c" in g]
            if temps:
                m["gpu_temperature"] = max(temps)
            m["gpu_count"] = float(len(gs))
        return m

    def get_health_report(self) -> HealthReport:
        m = self._metrics()
        checks, statuses = {}, []
        for k, (w, c) in self.THRESHOLDS.items():
            if k in m:
                s = _grade(m[k], w, c)
                checks[k] = s == HealthStatus.HEALTHY
                statuses.append(s)
        st = _worst(statuses) if statuses else HealthStatus.UNKNOWN
        bad = [k for k, ok in checks.items() if not ok]
        return HealthReport("system", st, checks, m, "all checks passed" if not bad else "issues: " + ", ".join(bad))


class TrainingHealthMonitor:
    def __init__(self, stale_after_s: float = 300.0):
        self.stale_after_s = stale_after_s
        self.last_update: Optional[float] = None
        self.metrics: Dict[str, float] = {}
        self.nan_streak = 0

    def update_training_metrics(self, **kwargs):
        self.metrics.update({k: float(v) for k, v in kwargs.items() if isinstance(v, (int, float))})
        self.last_update = time.time()
        loss = kwargs.get("loss")
        if loss is not None and not math.isfinite(float(loss)):
            self.nan_streak += 1
        elif loss is not None:
            self.nan_streak = 0

    def get_health_report(self) -> HealthReport:
        if self.last_update is None:
            return HealthReport("training", HealthStatus.UNKNOWN, message="no training metrics received")
        checks = {"active": time.time() - self.last_update < self.stale_after_s}
        loss = self.metrics.get("loss")
        if loss is not None:
            checks["loss_finite"] = math.isfinite(loss)
        gn = self.metrics.get("grad_norm")
        if gn is not None:
            checks["grad_norm_ok"] = (0.001 < gn < 100.0) if math.isfinite(gn) else False
        status = HealthStatus.HEALTHY
        if not checks.get("loss_finite", True) or self.nan_streak >= 3:
            status = HealthStatus.CRITICAL
        elif not all(checks.values()):
            status = HealthStatus.WARNING
        m = dict(self.metrics)
        m["seconds_since_update"] = time.time() - self.last_update
        bad = [k for k, v in checks.items() if not v]
        return HealthReport("training", status, checks, m, "training healthy" if not bad else "issues: " + ", ".join(bad))


class InferenceHealthMonitor:
    def __init__(self, window: int = 1000):
        self.latencies: Deque[float] = deque(maxlen=window)
        self.successes: Deque[bool] = deque(maxlen=window)
        self.active = 0
        self.last_request: Optional[float] = None

    def record_request(self, latency: float, success: bool = True):
        self.latencies.append(latency)
        self.successes.append(success)
        self.last_request = time.time()

    def update_active_requests(self, count: int):
        self.active = count

    def get_health_report(self) -> HealthReport:
        if not self.latencies:
            return HealthReport("inference", HealthStatus.UNKNOWN, message="no inference requests recorded")
        err = 1.0 - sum(self.successes) / len(self.successes)
        avg = sum(self.latencies) / len(self.latencies)
        since = time.time() - (self.last_request or time.time())
        checks = {"error_rate": err < 0.05, "latency": avg < 10.0, "recent_activity": since < 600.0,
                  "load": self.active < 100}
        status = HealthStatus.CRITICAL if err >= 0.2 else (HealthStatus.WARNING if not all(checks.values())
                                                           else HealthStatus.HEALTHY)
        m = {"error_rate": err, "avg_latency": avg, "active_requests": float(self.active),
             "seconds_since_request": since, "requests": float(len(self.latencies))}
        return HealthReport("inference", status, checks, m)


class HealthManager:
    def __init__(self, check_interval: float = 30.0, history: int = 1000):
        self.check_interval = check_interval
        self.system_monitor = SystemHealthMonitor()
        self.training_monitor = TrainingHealthMonitor()
        self.inference_monitor = InferenceHealthMonitor()
        self.health_history: Deque[Dict[str, HealthReport]] = deque(maxlen=history)
        self.alert_callbacks: List[Callable[[HealthReport], None]] = []
        self._running = False
        self._thread: Optional[threading.Thread] = None

    def add_alert_callback(self, callback: Callable[[HealthReport], None]):
        self.alert_callbacks.append(callback)

    def start_monitoring(self):
        if self._running:
            return
        self._running = True
        self._thread = threading.Thread(target=self._monitoring_loop, daemon=True)
        self._thread.start()

    def stop_monitoring(self):
        self._running = False
        if self._thread:
            self._thread.join(timeout=1.0)

    def _monitoring_loop(self):
        while self._running:
            try:
                self._perform_health_checks()
            except Exception:
                pass
            time.sleep(self.check_interval)

    def _perform_health_checks(self) -> Dict[str, HealthReport]:
        reports = self.get_current_health()
        self.health_history.append(reports)
        for r in reports.values():
            if r.status in (HealthStatus.WARNING, HealthStatus.CRITICAL):
                for cb in self.alert_callbacks:
                    cb(r)
        return reports

    def get_current_health(self) -> Dict[str, HealthReport]:
        return {"system": self.system_monitor.get_health_report(),
                "training": self.training_monitor.get_health_report(),
                "inference": self.inference_monitor.get_health_report()}

    def get_overall_status(self, reports: Optional[Dict[str, HealthReport]] = None) -> HealthStatus:
        reports = reports or self.get_current_health()
        known = [r.status for r in reports.values() if r.status != HealthStatus.UNKNOWN]
        return _worst(known) if known else HealthStatus.UNKNOWN

    def update_training_metrics(self, **kwargs):
        self.training_monitor.update_training_metrics(**kwargs)

    def record_inference_request(self, latency: float, success: bool = True):
        self.inference_monitor.record_request(latency, success)

    def update_active_requests(self, count: int):
        self.inference_monitor.update_active_requests(count)

    def save_health_report(self, filepath: str, reports: Optional[Dict[str, HealthReport]] = None):
        reports = reports or self.get_current_health()
        with open(filepath, "w") as f:
            json.dump({k: v.to_dict() for k, v in reports.items()}, f, indent=2)


def create_default_alert_callback() -> Callable[[HealthReport], None]:
    def alert_callback(report: HealthReport):
        color = "red" if report.status == HealthStatus.CRITICAL else "yellow"
        console.print(f"[{color}]HEALTH {report.status.value.upper()}: {report.component}: {report.message}[/{color}]")

    return alert_callback


_manager: Optional[HealthManager] = None


def get_health_manager() -> Optional[HealthManager]:
    return _manager


def setup_health_monitoring(check_interval: float = 30.0, start: bool = True, **kwargs) -> HealthManager:
    global _manager
    _manager = HealthManager(check_interval=check_interval, **kwargs)
    _manager.add_alert_callback(create_default_alert_callback())
    if start:
        _manager.start_monitoring()
    return _manager
