"""Performance knobs: every kernel-selection / scheduling choice in one typed record.

Round 1-3 grew ~50 ``LLMCTL_*`` environment variables read ad hoc on hot paths; a run that set
one could not be reproduced from its manifest.  Here every *performance* choice is a field of
:class:`PerfKnobs` with its measured default.  Precedence (lowest first):

    defaults  <  TrainingConfig.perf_knobs / [perf] TOML table / serve ``perf_knobs``
              <  LLMCTL_KNOBS="name=value,..."  (one debug/A-B override for experiments)

:func:`apply` makes a resolved record the process-wide active one (``knobs()``), pushes the
native ones into the HIP library's knob table (``torch.ops.llmctl.set_knob``, read by the
launchers in ``llmctl/ops/csrc``) and is called by the training and serving engines at init;
the run manifest (``run_manifest.json: perf_knobs``) and every checkpoint's
``training_state.json`` record ``asdict`` of the engine's resolved knobs, so ``llmctl replay``
restores them.  Each engine keeps its own resolved record (``engine.knobs``) and re-activates it
(:func:`use`) on entry to its hot paths.

The remaining environment variables are debugging aids only (``LLMCTL_DEBUG``,
``LLMCTL_HANG_DUMP``, ``LLMCTL_FAULT``, ``LLMCTL_STREAM_CHECK``, ``LLMCTL_SANITIZE``,
``LLMCTL_FORCE_REF``, ``LLMCTL_HIP_LIB``, ...; see README "Environment").

Reference: the reference has no such layer -- its engine options are the TrainingConfig fields
of ``llmctl/runtime/engine.py:30-70``.
"""

from __future__ import annotations

import contextlib
import dataclasses
import os
from dataclasses import dataclass, fields
from typing import Any, Dict, Iterator, Optional

ENV = "LLMCTL_KNOBS"


@dataclass(frozen=True)
class PerfKnobs:
    # ---- training GEMM routing (llmctl/exec/linear.py, llmctl/models/transformer.py)
    gemm64: bool = True            # in-house MFMA GEMMs (False: hipBLASLt everywhere -- A/B only)
    gemm64_config: int = 304       # gemm64 config: tile-order group + 100 * schedule variant + 1000 * split
    fwd64: str = "auto"            # forward x W^T on gemm64: auto (small-M / wide shapes) | all | off
    dgrad64: str = "fused"         # data gradients on gemm64: fused (down projection) | all | off
    wgrad_kernel: bool = True      # weight gradients on the MFMA kernels (False: hipBLASLt)
    swiglu_bwd: str = "side"       # SwiGLU backward: side (wgrad side job) | epilogue | separate
    dgrad_transpose: bool = True   # hipBLASLt data gradients through a W^T copy
    wt_side_stream: bool = True    # ... refreshed on a side stream under the forward
    fused_fwd: bool = False        # QKV+RoPE / up+SwiGLU epilogues in the forward GEMMs
    rope_inplace: bool = True      # RoPE applied in place on the q / k views
    fused_rope_attn: bool = True   # RoPE folded into the attention kernels' Q/K loads
    moe_pad: bool = True           # MoE expert rows padded to multiples of 256 (gemm64 expert GEMMs)
    overlap_optimizer: bool = False  # ZeRO-0: per-bucket AdamW under the backward (measured neutral)
    gemm_tuning: bool = True       # hipBLASLt TunableOp solutions (configs/gemm_tuning/*.csv)
    # ---- attention kernels (native: flash_attn_fwd.hip / flash_attn_bwd.hip)
    fa_split: int = -1             # forward causal K/V split: -1 auto, 0 off, 1 on
    fa_prio: int = 1               # s_setprio around the forward MFMA clusters
    fa_nw: int = 4                 # forward waves per workgroup: 4 or 8
    dkv: int = 2                   # dK/dV kernel: 0 plain, 1 pipelined, 2 persistent
    dkv_nwg: int = 0               # persistent dK/dV workgroups (0: one per CU; debug)
    # ---- parallelism
    async_tp: bool = True          # chunked all-gather / reduce-scatter rings overlapped with GEMMs
    async_tp_save_full: bool = False
    cp_zigzag: bool = True         # load-balanced (zig-zag) causal ring attention
    # ---- serving (llmctl/serve, llmctl/ops/functional.py; native: paged_attn.hip, skinny_gemm.hip)
    decode_fused: bool = True      # decode projections with fused epilogues
    decode_splits: int = 0         # paged-attention context splits (0: auto)
    decode_v3: int = 1             # skinny decode GEMM v3 schedule
    skinny_gemm: str = "auto"      # decode-size GEMMs on the skinny kernel: auto | all | off
    prefill_swiglu: bool = True    # serving prefill gate/up GEMM with the SwiGLU epilogue
    prefill_fa: bool = True        # fresh prompts through the packed flash-attention kernel
    prefill_norm_fold: bool = True  # prefill RMSNorms folded into the QKV / gate-up GEMMs (row-scaled epilogue)
    mixed_steps: bool = True       # decode rows ride on prefill chunk steps
    custom_ar: bool = True         # TP all-reduces through the xGMI peer-memory kernel
    tp_graphs: bool = True         # TP decode steps captured in hipGraphs
    async_decode: bool = True      # pure decode steps pipelined: step N+1 launched (ids fed on the
                                   # device from step N's in-graph sampling) before step N's tokens are read
    tp_fused_decode: bool = True   # TP decode: all-reduce + residual + RMSNorm in one kernel

    def as_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


NATIVE = ("fa_split", "fa_prio", "fa_nw", "dkv", "dkv_nwg", "decode_splits", "decode_v3")
_FIELDS = {f.name: f for f in fields(PerfKnobs)}


def _coerce(name: str, value: Any) -> Any:
    if name not in _FIELDS:
        raise KeyError(f"unknown performance knob {name!r} (known: {', '.join(sorted(_FIELDS))})")
    typ = _FIELDS[name].type
    if typ in ("bool", bool):
        if isinstance(value, str):
            v = value.strip().lower()
            if v not in ("1", "0", "true", "false", "on", "off", "yes", "no"):
                raise ValueError(f"knob {name}: expected a boolean, got {value!r}")
            return v in ("1", "true", "on", "yes")
        return bool(value)
    if typ in ("int", int):
        return int(value)
    return str(value)


def parse_env(spec: Optional[str]) -> Dict[str, Any]:
    """``"a=1,b=off"`` -> {"a": True, "b": ...} (typed per field; unknown names raise)."""
    out: Dict[str, Any] = {}
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "=" not in part:
            raise ValueError(f"{ENV}: expected name=value, got {part!r}")
        k, v = part.split("=", 1)
        out[k.strip()] = _coerce(k.strip(), v.strip())
    return out


# per-feature variables of rounds 1-3 that are now knobs (LLMCTL_<NAME> for a knob NAME, plus these)
_RETIRED_ENV = ("LLMCTL_SIDE_DGRAD", "LLMCTL_DECODE_ATTN_QKV", "LLMCTL_GEMM64_CONFIG", "LLMCTL_SKINNY")
_warned: set = set()


def _warn_retired_env() -> None:
    import warnings

    names = [f"LLMCTL_{n.upper()}" for n in _FIELDS] + list(_RETIRED_ENV)
    for n in names:
        if n in os.environ and n not in _warned:
            _warned.add(n)
            warnings.warn(f"{n} is no longer read (performance switches are knobs now): set "
                          f"{ENV}=\"{n[7:].lower()}=<value>\" or the [perf] config table instead", stacklevel=3)


def resolve(overrides: Optional[Dict[str, Any]] = None, env: bool = True) -> PerfKnobs:
    """Defaults < ``overrides`` (config) < ``LLMCTL_KNOBS`` (when ``env``)."""
    _warn_retired_env()
    kw = {k: _coerce(k, v) for k, v in (overrides or {}).items()}
    if env:
        kw.update(parse_env(os.environ.get(ENV)))
    return PerfKnobs(**kw)


_ACTIVE: PerfKnobs = resolve()


def knobs() -> PerfKnobs:
    """The process-wide active knobs (cheap: a module global)."""
    return _ACTIVE


def push_native(k: Optional[PerfKnobs] = None) -> bool:
    """Copy the native knobs into the HIP library's table (no-op before the library loads)."""
    k = k or _ACTIVE
    try:
        from llmctl.ops import _lib

        if not _lib.loaded():
            return False
        import torch

        for name in NATIVE:
            torch.ops.llmctl.set_knob(name, int(getattr(k, name)))
        return True
    except Exception:  # pragma: no cover - library without the knob op
        return False


def apply(k: PerfKnobs) -> PerfKnobs:
    global _ACTIVE
    _ACTIVE = k
    push_native(k)
    return k


def use(k: PerfKnobs) -> PerfKnobs:
    """Make an engine's own resolved knobs the active ones (no-op when they already are).  Engines
    call this on entry to their step / prefill / decode paths, so a second engine built in the
    same process (with other ``perf_knobs``) does not change the first one's kernel routing or
    the knob state its hipGraphs are captured under."""
    if k is not _ACTIVE:
        apply(k)
    return k


def with_env(k: PerfKnobs) -> PerfKnobs:
    """Re-apply the ``LLMCTL_KNOBS`` overrides on top of ``k`` (they stay highest in precedence
    when a tuning cache refines the config-resolved knobs)."""
    env = parse_env(os.environ.get(ENV))
    return dataclasses.replace(k, **env) if env else k


def configure(overrides: Optional[Dict[str, Any]] = None) -> PerfKnobs:
    """Resolve (config overrides + ``LLMCTL_KNOBS``) and make the result active."""
    return apply(resolve(overrides))


@contextlib.contextmanager
def override(**kw: Any) -> Iterator[PerfKnobs]:
    """Temporarily replace fields of the active knobs (tests, A/B within one process)."""
    old = _ACTIVE
    new = dataclasses.replace(old, **{k: _coerce(k, v) for k, v in kw.items()})
    apply(new)
    try:
        yield new
    finally:
        apply(old)
