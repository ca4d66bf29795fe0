"""``llmctl health`` — health check and drift detection (reference: ``cli/commands/health.py:15-186``).

Same flags: ``check --component all --save-report --monitor-duration --check-interval 30``
and ``drift --baseline-file --tolerance 10`` (exit 1 on drift).
"""

from __future__ import annotations

import json
import time
from pathlib import Path
from typing import Optional

import typer
from rich.console import Console
from rich.table import Table

console = Console()
app = typer.Typer(help="Cluster health checks")


def _display(reports, overall):
    t = Table(title="System Health")
    for c in ("Component", "Status", "Checks", "Message"):
        t.add_column(c)
    colors = {"healthy": "green", "warning": "yellow", "critical": "red", "unknown": "dim"}
    for name, r in reports.items():
        st = r.status.value
        checks = ", ".join(f"{k}={'✓' if v else '✗'}" for k, v in r.checks.items())
        t.add_row(name, f"[{colors[st]}]{st}[/{colors[st]}]", checks, r.message)
    console.print(t)
    console.print(f"Overall: [bold]{overall.value}[/bold]")


@app.command()
def check(
    component: str = typer.Option("all", help="Component to check (all, system, training, inference)"),
    save_report: Optional[Path] = typer.Option(None, help="Save health report to file"),
    monitor_duration: Optional[int] = typer.Option(None, help="Monitor for N seconds"),
    check_interval: float = typer.Option(30.0, help="Check interval in seconds"),
) -> None:
    """Run health checks."""
    from llmctl.metrics.health import setup_health_monitoring

    hm = setup_health_monitoring(check_interval=check_interval, start=False)
    end = time.time() + (monitor_duration or 0)
    while True:
        reports = hm.get_current_health()
        if component != "all":
            reports = {k: v for k, v in reports.items() if k == component}
        _display(reports, hm.get_overall_status(reports))
        if time.time() >= end:
            break
        time.sleep(min(check_interval, max(end - time.time(), 0)))
    if save_report:
        hm.save_health_report(str(save_report), reports)
        console.print(f"[green]✓ Health report saved to {save_report}[/green]")


@app.command()
def drift(
    baseline_file: Path = typer.Option(..., help="Baseline health report"),
    tolerance: float = typer.Option(10.0, help="Tolerance percentage for drift detection"),
) -> None:
    """Compare current metrics against a baseline report; exit 1 on drift."""
    from llmctl.metrics.health import setup_health_monitoring

    base = json.loads(baseline_file.read_text())
    cur = {k: v.to_dict() for k, v in setup_health_monitoring(start=False).get_current_health().items()}
    drifts = []
    for comp, rep in base.items():
        for k, bv in (rep.get("metrics") or {}).items():
            cv = (cur.get(comp, {}).get("metrics") or {}).get(k)
            if cv is None or not isinstance(bv, (int, float)):
                continue
            if bv == 0:
                pct = 0.0 if cv == 0 else 100.0
            else:
                pct = abs(cv - bv) / abs(bv) * 100.0
            if pct > tolerance:
                drifts.append({"component": comp, "metric": k, "baseline": bv, "current": cv, "drift_pct": pct})
    if drifts:
        t = Table(title="Drift detected")
        for c in ("component", "metric", "baseline", "current", "drift %"):
            t.add_column(c)
        for d in drifts:
            t.add_row(d["component"], d["metric"], f"{d['baseline']:.3g}", f"{d['current']:.3g}", f"{d['drift_pct']:.1f}")
        console.print(t)
        raise typer.Exit(1)
    console.print(f"[green]✓ No drift beyond {tolerance}%[/green]")
