"""Validated config schemas (pydantic v2) for every file format the reference reads/writes.

The reference declares "validated schemas" (``README.md:24``) but its configs are bare dict
literals with no validation.  Each model below accepts the
reference's files unchanged (``extra="allow"``) and documents the MI355X additions.
Precedence when resolving a run (``resolve_training_config``):
defaults < preset/profile < ``--config`` file < plan file < explicitly-set CLI flags.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, ConfigDict, Field, field_validator


class _Open(BaseModel):
    model_config = ConfigDict(extra="allow", populate_by_name=True)


# ----------------------------------------------------------------------------- model JSON
class RopeConfig(_Open):
    base: float = 10000
    scaling: Optional[str] = "linear"


class ModelSchema(_Open):
    """``configs/models/*.json`` (ref ``init.py:16-51``, ``configs/models/llama-7b.json``)."""
    name: str
    arch: str = "decoder-only"
    layers: int = Field(gt=0)
    hidden: int = Field(gt=0)
    ffn: Optional[int] = None
    heads: int = Field(gt=0)
    vocab_size: int = Field(gt=0)
    rope: Optional[RopeConfig] = None
    kv_heads: Optional[int] = None
    head_dim: Optional[int] = None

    @field_validator("hidden")
    @classmethod
    def _h(cls, v):
        if v % 8:
            raise ValueError("hidden must be a multiple of 8 (16-byte bf16 vectors)")
        return v


# ----------------------------------------------------------------------------- hardware TOML
class GPUDevice(_Open):
    id: int
    name: str = ""
    memory_gb: float = 0.0
    compute_capability: Optional[str] = None
    multiprocessors: Optional[int] = None
    gcn_arch: Optional[str] = None
    compute_units: Optional[int] = None


class GPUSection(_Open):
    count: int = 0
    devices: List[GPUDevice] = []
    total_memory_gb: float = 0.0
    driver_version: Optional[str] = None
    cuda_version: Optional[str] = None
    hip_version: Optional[str] = None


class Limits(_Open):
    estimated_flops: float = 0.0
    memory_bw_gbps: float = 0.0
    intra_node_bw_gbps: float = 0.0
    inter_node_bw_gbps: float = 0.0


class HardwareSchema(_Open):
    """``hw probe --emit`` output (ref ``hw.py:168-185``, ``configs/presets/a100x8.toml``)."""
    system: Dict[str, Any] = {}
    cpu: Dict[str, Any] = {}
    memory: Dict[str, Any] = {}
    gpu: GPUSection = GPUSection()
    interconnect: Dict[str, Any] = {}
    limits: Limits = Limits()


# ----------------------------------------------------------------------------- training TOML
class OptimizerSection(_Open):
    type: str = "adamw"
    lr: float = 2e-4
    betas: List[float] = [0.9, 0.95]
    weight_decay: float = 0.1
    eps: float = 1e-8
    scheduler: Dict[str, Any] = {"type": "cosine", "warmup_steps": 2000}


class ParallelSection(_Open):
    strategy: str = "auto"
    tensor_parallel: int = 1
    pipeline_parallel: int = 1
    virtual_stages: int = 1  # interleaved pipeline: model chunks per pipeline rank
    sequence_parallel: bool = False
    context_parallel: int = 1
    context_parallel_mode: str = "ulysses"  # ulysses | ring
    expert_parallel: int = 1  # MoE models: experts sharded over this many DP ranks
    zero_stage: int = Field(1, ge=0, le=3)
    activation_checkpoint: Union[str, bool] = "selective"
    micro_batch_size: int = 1
    global_batch_size: int = 64
    gradient_accumulation_steps: Optional[int] = None


class CheckpointSection(_Open):
    path: str = "checkpoints"
    interval_steps: int = 1000
    sharded: bool = True
    async_: bool = Field(True, alias="async")
    keep_latest: Optional[int] = None


class TrainingSection(_Open):
    max_steps: Optional[int] = None
    eval_interval: Optional[int] = None
    save_interval: Optional[int] = None
    log_interval: Optional[int] = None
    gradient_clipping: Optional[float] = None
    mixed_precision: Optional[str] = None
    flash_attention: Optional[bool] = None
    compile_model: Optional[bool] = None


class TrainConfigSchema(_Open):
    """``configs/default.toml`` (ref ``init.py:104-158``, ``llama-7b-a100x8.toml``)."""
    model: Dict[str, Any] = {}
    optimizer: OptimizerSection = OptimizerSection()
    data: Dict[str, Any] = {}
    hardware: Dict[str, Any] = {}
    parallel: ParallelSection = ParallelSection()
    limits: Dict[str, Any] = {}
    checkpoint: CheckpointSection = CheckpointSection()
    training: TrainingSection = TrainingSection()
    telemetry: Dict[str, Any] = {}
    # performance knobs (llmctl.config.knobs.PerfKnobs fields): kernel / schedule choices
    perf: Dict[str, Any] = {}

    @field_validator("perf")
    @classmethod
    def _known_knobs(cls, v: Dict[str, Any]) -> Dict[str, Any]:
        from llmctl.config.knobs import _coerce

        return {k: _coerce(k, x) for k, x in v.items()}  # unknown names / bad values raise


class DataConfigSchema(_Open):
    """``configs/data/*.toml`` (ref ``init.py:166-179``)."""
    name: str = "dataset"
    format: str = "json"
    sources: List[Dict[str, Any]] = []
    preprocessing: Dict[str, Any] = {}


class PlanParallelism(_Open):
    tensor_parallel: int
    pipeline_parallel: int
    data_parallel: int
    zero_stage: int
    micro_batch_size: int
    global_batch_size: int
    estimated_memory_gb: Optional[float] = None  # written by `plan compute`; optional in hand-written plans
    estimated_comm_gb: Optional[float] = None
    estimated_flops: Optional[float] = None
    sequence_parallel: bool = False
    context_parallel: int = 1
    expert_parallel: int = 1
    activation_checkpoint: str = "none"
    grad_accum: int = 1
    virtual_stages: int = 1
    num_microbatches: Optional[int] = None


class PlanSchema(_Open):
    """``plan compute --out`` (ref ``plan.py:341-358``) + ``[shard_map]``."""
    metadata: Dict[str, Any] = {}
    parallelism: PlanParallelism
    model: Dict[str, Any] = {}
    hardware: Dict[str, Any] = {}
    shard_map: Optional[Dict[str, Any]] = None


def validate(kind: str, data: Dict[str, Any]) -> BaseModel:
    cls = {"model": ModelSchema, "hardware": HardwareSchema, "train": TrainConfigSchema, "data": DataConfigSchema,
           "plan": PlanSchema}[kind]
    return cls.model_validate(data)


def resolve_training_config(train_file: Optional[Dict[str, Any]] = None, plan: Optional[Dict[str, Any]] = None,
                            cli: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Merge a training TOML, a plan and explicitly-set CLI values into TrainingConfig kwargs
    (precedence: file < plan < CLI)."""
    out: Dict[str, Any] = {}
    if train_file:
        t = TrainConfigSchema.model_validate(train_file)
        out["learning_rate"] = t.optimizer.lr
        out["weight_decay"] = t.optimizer.weight_decay
        out["betas"] = tuple(t.optimizer.betas)
        out["eps"] = t.optimizer.eps
        sch = t.optimizer.scheduler or {}
        out["scheduler"] = sch.get("type", "cosine")
        out["warmup_steps"] = int(sch.get("warmup_steps", 0))
        p = t.parallel
        out.update(tensor_parallel=p.tensor_parallel, pipeline_parallel=p.pipeline_parallel,
                   virtual_stages=p.virtual_stages,
                   sequence_parallel=p.sequence_parallel, zero_stage=p.zero_stage,
                   context_parallel=p.context_parallel, context_parallel_mode=p.context_parallel_mode,
                   expert_parallel=p.expert_parallel, batch_size=p.micro_batch_size)
        ac = p.activation_checkpoint
        out["activation_checkpoint"] = ("selective" if ac is True else "none" if ac in (False, None) else str(ac))
        if p.gradient_accumulation_steps:
            out["gradient_accumulation_steps"] = p.gradient_accumulation_steps
        ck = t.checkpoint
        out.update(save_steps=ck.interval_steps, async_checkpoint=ck.async_, sharded_checkpoint=ck.sharded)
        if ck.keep_latest:
            out["keep_latest"] = ck.keep_latest
        tr = t.training
        if tr.max_steps:
            out["max_steps"] = tr.max_steps
        if tr.eval_interval:
            out["eval_steps"] = tr.eval_interval
        if tr.save_interval:
            out["save_steps"] = tr.save_interval
        if tr.log_interval:
            out["logging_steps"] = tr.log_interval
        if tr.gradient_clipping is not None:
            out["gradient_clipping"] = tr.gradient_clipping
        if tr.mixed_precision:
            out["mixed_precision"] = tr.mixed_precision
        prof = (t.telemetry or {}).get("profiling") if isinstance(t.telemetry, dict) else None
        if isinstance(prof, dict) and prof.get("enable"):
            out["profile_dir"] = str(prof.get("dir", "profiles"))
            if prof.get("schedule"):
                out["profile_schedule"] = str(prof["schedule"])
        mx = t.data.get("max_length") if isinstance(t.data, dict) else None
        if mx:
            out["seq_len"] = int(mx)
        if t.perf:
            out["perf_knobs"] = dict(t.perf)
        if t.model.get("config_file"):
            out["model_name_or_path"] = t.model["config_file"]
        elif t.model.get("name"):
            out["model_name_or_path"] = t.model["name"]
    if plan:
        pp = PlanSchema.model_validate(plan).parallelism
        out.update(tensor_parallel=pp.tensor_parallel, pipeline_parallel=pp.pipeline_parallel,
                   zero_stage=pp.zero_stage, batch_size=pp.micro_batch_size,
                   sequence_parallel=pp.sequence_parallel, activation_checkpoint=pp.activation_checkpoint,
                   context_parallel=pp.context_parallel, expert_parallel=pp.expert_parallel,
                   gradient_accumulation_steps=max(pp.grad_accum, 1), virtual_stages=pp.virtual_stages)
        if pp.pipeline_parallel > 1 and pp.num_microbatches:
            out["num_microbatches"] = pp.num_microbatches
    if cli:
        out.update({k: v for k, v in cli.items() if v is not None})
    return out
