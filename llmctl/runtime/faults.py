"""Opt-in fault injection for recovery tests (the reference has none).

``LLMCTL_FAULT`` holds comma-separated actions ``<kind>[:<rank>]@step:<N>``:

* ``kill_rank:R@step:N`` — rank ``R`` dies (``os._exit(43)``, no cleanup, like a node loss)
  right after optimizer step ``N``.  It fires once per output directory (a marker under
  ``<output_dir>/.faults/`` is written first), so an elastic restart that resumes from the
  last checkpoint runs through.
* ``nan_grad@step:N`` — every rank's loss of step ``N`` is multiplied by NaN before
  backward: the global grad norm is non-finite and the optimizer's skip-step policy must
  leave the model untouched.
* ``raise@step:N`` — ``RuntimeError`` on every rank after step ``N``.
"""

from __future__ import annotations

import os
import re
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional

EXIT_CODE = 43
_RE = re.compile(r"^(kill_rank|nan_grad|raise)(?::(\d+))?@step:(\d+)$")


@dataclass
class Fault:
    kind: str
    rank: Optional[int]
    step: int

    @property
    def tag(self) -> str:
        return f"{self.kind}-{self.rank if self.rank is not None else 'all'}-{self.step}"


def parse(spec: Optional[str]) -> List[Fault]:
    out = []
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        m = _RE.match(part)
        if not m:
            raise ValueError(f"LLMCTL_FAULT: cannot parse '{part}' (expected kind[:rank]@step:N)")
        out.append(Fault(m.group(1), int(m.group(2)) if m.group(2) else None, int(m.group(3))))
    return out


class FaultInjector:
    def __init__(self, rank: int, output_dir: str, spec: Optional[str] = None):
        self.rank = rank
        self.faults = parse(spec if spec is not None else os.environ.get("LLMCTL_FAULT"))
        self.marker_dir = Path(output_dir) / ".faults"

    def __bool__(self) -> bool:
        return bool(self.faults)

    def nan_loss(self, step: int) -> bool:
        """True when the loss of (1-based) step ``step`` must be poisoned."""
        return any(f.kind == "nan_grad" and f.step == step for f in self.faults)

    def after_step(self, step: int) -> None:
        for f in self.faults:
            if f.step != step or f.kind == "nan_grad":
                continue
            if f.rank is not None and f.rank != self.rank:
                continue
            if f.kind == "raise":
                raise RuntimeError(f"injected fault at step {step}")
            marker = self.marker_dir / f.tag
            if marker.exists():
                continue  # already fired in an earlier attempt of this run
            self.marker_dir.mkdir(parents=True, exist_ok=True)
            marker.write_text(str(step))
            os._exit(EXIT_CODE)
