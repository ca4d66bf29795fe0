"""Model configuration: the reference's model-JSON schema, extended.

Reference schema: ``name, arch, layers, hidden, ffn, heads, vocab_size,
rope{base, scaling}`` written by ``llmctl/cli/commands/init.py:16-51`` and the fuller
``configs/models/llama-7b.json:1-23`` (``head_dim, max_position_embeddings, attention{},
activation, layer_norm_eps, tie_word_embeddings, estimated_params``).

Additions (all optional, so reference files load unchanged):
``kv_heads`` (GQA), ``norm`` ("rmsnorm" | "layernorm"), ``position`` ("rope" | "learned"),
``rope.factor`` (linear), ``rope.short_factor/long_factor/original_max_position`` ("su").
"""

from __future__ import annotations

import copy
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Optional


@dataclass
class ModelConfig:
    name: str = "gpt-7b"
    arch: str = "decoder-only"
    layers: int = 32
    hidden: int = 4096
    ffn: int = 11008
    heads: int = 32
    kv_heads: Optional[int] = None
    vocab_size: int = 32000
    head_dim: Optional[int] = None
    max_position_embeddings: int = 4096
    activation: str = "silu"  # silu => SwiGLU MLP, gelu => GPT-2 MLP
    norm: str = "rmsnorm"
    position: str = "rope"
    layer_norm_eps: float = 1e-5
    tie_word_embeddings: bool = False
    rope: Dict[str, Any] = field(default_factory=lambda: {"base": 10000, "scaling": "linear"})
    attention: Dict[str, Any] = field(default_factory=lambda: {"type": "causal", "bias": False, "dropout": 0.0})
    # mixture of experts (0 = dense): every layer's MLP becomes num_experts SwiGLU experts of
    # width moe_ffn (default ffn) with top-``experts_per_token`` softmax routing
    num_experts: int = 0
    experts_per_token: int = 2
    moe_ffn: Optional[int] = None
    router_aux_loss_coef: float = 0.01
    extra: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self) -> None:
        if self.kv_heads is None:
            self.kv_heads = self.heads
        if self.head_dim is None:
            self.head_dim = self.hidden // self.heads
        if self.heads % self.kv_heads:
            raise ValueError(f"heads={self.heads} not divisible by kv_heads={self.kv_heads}")
        if self.num_experts:
            if self.moe_ffn is None:
                self.moe_ffn = self.ffn
            if not (0 < self.experts_per_token <= self.num_experts):
                raise ValueError("experts_per_token must be in [1, num_experts]")
            if not self.gated_mlp:
                raise ValueError("MoE layers use SwiGLU experts (activation silu)")

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    # ------------------------------------------------------------------ derived sizes
    @property
    def q_size(self) -> int:
        return self.heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.kv_heads * self.head_dim

    @property
    def gated_mlp(self) -> bool:
        return self.activation in ("silu", "swiglu")

    def num_parameters(self, include_embedding: bool = True) -> int:
        """Exact parameter count of :class:`llmctl.models.transformer.DecoderLM`."""
        h, f, L, V = self.hidden, self.ffn, self.layers, self.vocab_size
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        mlp = (3 if self.gated_mlp else 2) * h * f
        if self.is_moe:  # router + every expert
            mlp = self.num_experts * h + self.num_experts * 3 * h * self.moe_ffn
        norms = (2 * h) if self.norm == "rmsnorm" else (4 * h)
        biases = 0
        if self.norm == "layernorm":  # GPT-2 style linear biases
            biases = (self.q_size + 2 * self.kv_size) + h + (f if not self.gated_mlp else 2 * f) + h
        per_layer = attn + mlp + norms + biases
        final_norm = h if self.norm == "rmsnorm" else 2 * h
        n = L * per_layer + final_norm
        if include_embedding:
            n += V * h
            if not self.tie_word_embeddings:
                n += V * h
            if self.position == "learned":
                n += self.max_position_embeddings * h
        return n

    def active_parameters(self) -> int:
        """Parameters a token touches (MoE: top-k experts of each layer, not all of them)."""
        n = self.num_parameters(include_embedding=False)
        if self.is_moe:
            n -= self.layers * (self.num_experts - self.experts_per_token) * 3 * self.hidden * self.moe_ffn
        return n

    def flops_per_token(self, seq_len: int, training: bool = True) -> float:
        """Model FLOPs per token (6N + attention; PaLM-style MFU accounting, causal halved;
        MoE counts the active experts only)."""
        n = self.active_parameters() + self.vocab_size * self.hidden  # lm_head matmul
        attn = 2 * 2 * self.layers * self.q_size * seq_len / 2  # QK^T + PV, causal half
        fwd = 2 * n + attn
        return 3 * fwd if training else fwd

    # ------------------------------------------------------------------ (de)serialisation
    _KNOWN = {
        "name", "arch", "layers", "hidden", "ffn", "heads", "kv_heads", "vocab_size", "head_dim",
        "max_position_embeddings", "activation", "norm", "position", "layer_norm_eps",
        "tie_word_embeddings", "rope", "attention", "num_experts", "experts_per_token", "moe_ffn",
        "router_aux_loss_coef",
    }

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        d = copy.deepcopy(dict(d))
        kw = {k: d.pop(k) for k in list(d) if k in cls._KNOWN}
        # accept a few HF-style aliases
        aliases = {
            "num_hidden_layers": "layers", "hidden_size": "hidden", "intermediate_size": "ffn",
            "num_attention_heads": "heads", "num_key_value_heads": "kv_heads", "rms_norm_eps": "layer_norm_eps",
            "num_local_experts": "num_experts", "num_experts_per_tok": "experts_per_token",
            "router_aux_loss_coef": "router_aux_loss_coef",
        }
        for a, k in aliases.items():
            if a in d and k not in kw:
                kw[k] = d.pop(a)
        if "n_kv_heads" in d and "kv_heads" not in kw:
            kw["kv_heads"] = d.pop("n_kv_heads")
        kw["extra"] = d
        return cls(**kw)

    @classmethod
    def from_file(cls, path: str | Path) -> "ModelConfig":
        path = Path(path)
        if path.suffix == ".json":
            data = json.loads(path.read_text())
        else:
            from llmctl.config.toml_io import load_toml

            data = load_toml(path)
            data = data.get("model", data) if "layers" not in data else data
        return cls.from_dict(data)

    def to_dict(self) -> Dict[str, Any]:
        moe = ("num_experts", "experts_per_token", "moe_ffn", "router_aux_loss_coef")
        d = {k: getattr(self, k) for k in sorted(self._KNOWN) if self.is_moe or k not in moe}
        d.update(self.extra)
        d["estimated_params"] = self.num_parameters()
        return d


# ---------------------------------------------------------------------------------------
# Templates.  gpt/7b, gpt/13b, llama/7b mirror reference init.py:16-51 exactly; the rest
# are additions promised by the reference docs (USER_GUIDE.md:61 lists 30b/70b sizes) and
# the BASELINE configs (GPT-2-125M plumbing run, Llama-3-70B ZeRO-3 run).
# ---------------------------------------------------------------------------------------
MODEL_TEMPLATES: Dict[str, Dict[str, Dict[str, Any]]] = {
    "gpt": {
        "125m": {
            "name": "gpt-125m", "arch": "decoder-only", "layers": 12, "hidden": 768, "ffn": 3072,
            "heads": 12, "vocab_size": 50304, "norm": "layernorm", "activation": "gelu",
            "position": "learned", "max_position_embeddings": 2048, "tie_word_embeddings": True,
            "rope": {"base": 10000, "scaling": "linear"},
        },
        "7b": {
            "name": "gpt-7b", "arch": "decoder-only", "layers": 32, "hidden": 4096, "ffn": 11008,
            "heads": 32, "vocab_size": 32000, "rope": {"base": 10000, "scaling": "su"},
        },
        "13b": {
            "name": "gpt-13b", "arch": "decoder-only", "layers": 40, "hidden": 5120, "ffn": 13824,
            "heads": 40, "vocab_size": 32000, "rope": {"base": 10000, "scaling": "su"},
        },
    },
    "gpt2": {
        "125m": {
            "name": "gpt2-125m", "arch": "decoder-only", "layers": 12, "hidden": 768, "ffn": 3072,
            "heads": 12, "vocab_size": 50304, "norm": "layernorm", "activation": "gelu",
            "position": "learned", "max_position_embeddings": 2048, "tie_word_embeddings": True,
            "rope": {"base": 10000, "scaling": "linear"},
        },
    },
    "llama": {
        "7b": {
            "name": "llama-7b", "arch": "decoder-only", "layers": 32, "hidden": 4096, "ffn": 11008,
            "heads": 32, "vocab_size": 32000, "rope": {"base": 10000, "scaling": "linear"},
        },
        "13b": {
            "name": "llama-13b", "arch": "decoder-only", "layers": 40, "hidden": 5120, "ffn": 13824,
            "heads": 40, "vocab_size": 32000, "rope": {"base": 10000, "scaling": "linear"},
        },
        "30b": {
            "name": "llama-30b", "arch": "decoder-only", "layers": 60, "hidden": 6656, "ffn": 17920,
            "heads": 52, "vocab_size": 32000, "rope": {"base": 10000, "scaling": "linear"},
        },
        "70b": {
            "name": "llama3-70b", "arch": "decoder-only", "layers": 80, "hidden": 8192, "ffn": 28672,
            "heads": 64, "kv_heads": 8, "vocab_size": 128256, "max_position_embeddings": 8192,
            "rope": {"base": 500000, "scaling": "linear"},
        },
    },
    "mixtral": {
        "8x7b": {
            "name": "mixtral-8x7b", "arch": "decoder-only", "layers": 32, "hidden": 4096, "ffn": 14336,
            "heads": 32, "kv_heads": 8, "vocab_size": 32000, "max_position_embeddings": 32768,
            "rope": {"base": 1000000, "scaling": "linear"}, "num_experts": 8, "experts_per_token": 2,
        },
    },
    "tiny": {
        "moe": {
            "name": "tiny-moe", "arch": "decoder-only", "layers": 2, "hidden": 256, "ffn": 704,
            "heads": 4, "kv_heads": 2, "vocab_size": 512, "max_position_embeddings": 512,
            "rope": {"base": 10000, "scaling": "linear"}, "num_experts": 4, "experts_per_token": 2,
            "moe_ffn": 256,
        },
        "test": {
            "name": "tiny-test", "arch": "decoder-only", "layers": 2, "hidden": 256, "ffn": 704,
            "heads": 4, "kv_heads": 2, "vocab_size": 512, "max_position_embeddings": 512,
            "rope": {"base": 10000, "scaling": "linear"},
        },
        "deep": {  # 8 thin layers: enough pipeline stages for interleaved (virtual-stage) tests
            "name": "tiny-deep", "arch": "decoder-only", "layers": 8, "hidden": 128, "ffn": 352,
            "heads": 4, "kv_heads": 2, "vocab_size": 512, "max_position_embeddings": 512,
            "rope": {"base": 10000, "scaling": "linear"},
        },
        "deep64": {  # 8 layers at head_dim 64: the deep pipeline layouts on the GPU kernels (D 64 / 128)
            "name": "tiny-deep64", "arch": "decoder-only", "layers": 8, "hidden": 256, "ffn": 704,
            "heads": 4, "kv_heads": 2, "vocab_size": 512, "max_position_embeddings": 512,
            "rope": {"base": 10000, "scaling": "linear"},
        },
        "wide": {  # 8 query / 8 KV heads: enough heads for TP=8 (BASELINE config #5's degree)
            "name": "tiny-wide", "arch": "decoder-only", "layers": 2, "hidden": 512, "ffn": 1024,
            "heads": 8, "kv_heads": 8, "vocab_size": 512, "max_position_embeddings": 512,
            "rope": {"base": 10000, "scaling": "linear"},
        },
        "tied": {  # GPT-2 style (layernorm, GELU, learned positions, tied LM head)
            "name": "tiny-tied", "arch": "decoder-only", "layers": 2, "hidden": 256, "ffn": 1024,
            "heads": 4, "vocab_size": 512, "norm": "layernorm", "activation": "gelu",
            "position": "learned", "max_position_embeddings": 512, "tie_word_embeddings": True,
        },
    },
}

ALIASES = {
    "gpt2": ("gpt2", "125m"), "gpt2-125m": ("gpt2", "125m"), "gpt-125m": ("gpt", "125m"),
    "gpt-7b": ("gpt", "7b"), "gpt-13b": ("gpt", "13b"), "llama-7b": ("llama", "7b"),
    "llama-13b": ("llama", "13b"), "llama-30b": ("llama", "30b"), "llama3-70b": ("llama", "70b"),
    "llama-70b": ("llama", "70b"), "tiny": ("tiny", "test"), "tiny-test": ("tiny", "test"),
    "mixtral-8x7b": ("mixtral", "8x7b"), "tiny-moe": ("tiny", "moe"),
    "tiny-tied": ("tiny", "tied"), "tiny-deep": ("tiny", "deep"), "tiny-wide": ("tiny", "wide"),
    "tiny-deep64": ("tiny", "deep64"),
}


def get_model_config(name_or_path: str) -> ModelConfig:
    """Resolve a template alias (``gpt-7b``), ``template/size`` or a JSON/TOML path."""
    p = Path(name_or_path)
    if p.suffix in (".json", ".toml") and p.exists():
        return ModelConfig.from_file(p)
    key = name_or_path.lower()
    if key in ALIASES:
        t, s = ALIASES[key]
        return ModelConfig.from_dict(MODEL_TEMPLATES[t][s])
    if "/" in key:
        t, s = key.split("/", 1)
        if t in MODEL_TEMPLATES and s in MODEL_TEMPLATES[t]:
            return ModelConfig.from_dict(MODEL_TEMPLATES[t][s])
    if p.is_dir() and (p / "config.json").exists():
        return ModelConfig.from_file(p / "config.json")
    raise KeyError(f"unknown model '{name_or_path}' (templates: {sorted(ALIASES)})")
