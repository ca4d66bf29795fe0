"""Pre-tuned library GEMM selection (PyTorch TunableOp) for the projection GEMMs.

The forward / dgrad projections run on hipBLASLt through torch.  Its default heuristic pick is
not always the fastest solution on gfx950: an exhaustive TunableOp search over the hipBLASLt and
rocBLAS solutions (``tools/gemm_tunable.py``, ``profiles/gemm_tunableop_study_r1.log``) found
e.g. the GPT-7B up-projection forward at 2.55 ms instead of 2.91 ms (1.74 vs 1.52 PFLOP/s).
The winning solution per (op, shape) is committed as a CSV and loaded with tuning OFF, so a run
never spends time searching; shapes not in the file keep the default heuristic.

The CSV's validator lines pin the PyTorch / HIP / hipBLASLt / rocBLAS versions and the GPU
arch; on any mismatch TunableOp ignores the file (default heuristics, never wrong results).
"""

from __future__ import annotations

import logging
import os
import tempfile
from pathlib import Path
from typing import Optional

log = logging.getLogger("llmctl.gemm_tuning")

DEFAULT_FILE = Path(__file__).resolve().parents[2] / "configs" / "tuning" / "tunableop_mi355x_gpt7b.csv"
_state = {"enabled": None}


def enable_tuned_gemms(path: Optional[str] = None) -> bool:
    """Load pre-tuned GEMM solutions (idempotent).  knob ``gemm_tuning`` off disables;
    ``LLMCTL_GEMM_TUNING_FILE`` overrides the file."""
    if _state["enabled"] is not None:
        return _state["enabled"]
    _state["enabled"] = False
    import torch

    from llmctl.config.knobs import knobs

    if not knobs().gemm_tuning or not torch.cuda.is_available() or torch.version.hip is None:
        return False
    f = Path(path or os.environ.get("LLMCTL_GEMM_TUNING_FILE", str(DEFAULT_FILE)))
    if not f.is_file():
        return False
    try:
        import torch.cuda.tunable as tun

        tun.enable(True)
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        ok = bool(tun.read_file(str(f)))
        # any write-back at exit goes to a scratch file, never over the committed results
        tun.set_filename(os.path.join(tempfile.gettempdir(), f"llmctl_tunableop_{os.getpid()}.csv"))
    except Exception as e:  # pragma: no cover - version dependent
        log.warning("TunableOp results not loaded (%s); using default GEMM heuristics", e)
        ok = False
    if not ok:
        try:
            torch.cuda.tunable.enable(False)
        except Exception:
            pass
    _state["enabled"] = ok
    if ok:
        log.info("loaded tuned GEMM solutions from %s", f)
    return ok
