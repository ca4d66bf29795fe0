"""Model definitions (Llama-style RMSNorm/RoPE/SwiGLU/GQA and GPT-2-style LN/GELU)."""

from .config import ALIASES, MODEL_TEMPLATES, ModelConfig, get_model_config
from .transformer import DecoderLayer, DecoderLM, ParallelContext, build_model

__all__ = ["ALIASES", "MODEL_TEMPLATES", "ModelConfig", "get_model_config", "DecoderLayer", "DecoderLM",
           "ParallelContext", "build_model"]
