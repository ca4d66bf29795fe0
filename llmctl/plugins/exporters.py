"""Checkpoint exporters (plugin group ``exporters``) behind ``llmctl export convert``.

``safetensors``: one consolidated, layout-independent ``model.safetensors`` + ``config.json``
(TP/PP shards merged).  ``hf``: HF-Llama tensor names (``model.layers.N.self_attn.q_proj``
…, fused QKV / gate-up split back out) + an HF ``config.json`` so ``transformers`` can load
it.  Optional quantization per ``llmctl.plugins.quantizers`` for 2-D projection weights.
``onnx`` / ``tensorrt`` / ``gguf`` are not available on this platform.
"""

from __future__ import annotations

import json
import warnings
from pathlib import Path
from typing import Any, Dict, Optional

import torch

UNSUPPORTED = {"onnx": "ONNX export needs onnx/onnxruntime (not installed)",
               "tensorrt": "TensorRT is NVIDIA-only; no MI355X equivalent in this stack",
               "gguf": "GGUF writer not implemented"}


def to_hf_llama(sd: Dict[str, torch.Tensor], cfg) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {}
    q, kv, D = cfg.q_size, cfg.kv_size, cfg.head_dim
    for k, v in sd.items():
        if k == "embed":
            out["model.embed_tokens.weight"] = v
        elif k == "lm_head":
            out["lm_head.weight"] = v
        elif k == "final_norm_w":
            out["model.norm.weight"] = v
        elif k.startswith("layers."):
            _, i, leaf = k.split(".", 2)
            p = f"model.layers.{i}"
            if leaf == "wqkv":
                out[f"{p}.self_attn.q_proj.weight"] = v[:q]
                out[f"{p}.self_attn.k_proj.weight"] = v[q:q + kv]
                out[f"{p}.self_attn.v_proj.weight"] = v[q + kv:]
            elif leaf == "wo":
                out[f"{p}.self_attn.o_proj.weight"] = v
            elif leaf == "w_up":
                f = v.shape[0] // 2
                out[f"{p}.mlp.gate_proj.weight"] = v[:f]
                out[f"{p}.mlp.up_proj.weight"] = v[f:]
            elif leaf == "w_down":
                out[f"{p}.mlp.down_proj.weight"] = v
            elif leaf == "moe.w_router":  # Mixtral naming
                out[f"{p}.block_sparse_moe.gate.weight"] = v
            elif leaf.startswith("moe.experts_up."):
                e = leaf.rsplit(".", 1)[1]
                f = v.shape[0] // 2
                out[f"{p}.block_sparse_moe.experts.{e}.w1.weight"] = v[:f]
                out[f"{p}.block_sparse_moe.experts.{e}.w3.weight"] = v[f:]
            elif leaf.startswith("moe.experts_down."):
                e = leaf.rsplit(".", 1)[1]
                out[f"{p}.block_sparse_moe.experts.{e}.w2.weight"] = v
            elif leaf == "attn_norm_w":
                out[f"{p}.input_layernorm.weight"] = v
            elif leaf == "mlp_norm_w":
                out[f"{p}.post_attention_layernorm.weight"] = v
            else:
                out[f"{p}.{leaf}"] = v
        else:
            out[k] = v
    if cfg.tie_word_embeddings and "lm_head.weight" not in out:
        pass
    return out


def hf_config(cfg) -> Dict[str, Any]:
    return {"architectures": ["LlamaForCausalLM"], "model_type": "llama", "hidden_size": cfg.hidden,
            "intermediate_size": cfg.ffn, "num_hidden_layers": cfg.layers, "num_attention_heads": cfg.heads,
            "num_key_value_heads": cfg.kv_heads, "vocab_size": cfg.vocab_size, "rms_norm_eps": cfg.layer_norm_eps,
            "max_position_embeddings": cfg.max_position_embeddings,
            "rope_theta": float((cfg.rope or {}).get("base", 10000)), "tie_word_embeddings": cfg.tie_word_embeddings,
            "torch_dtype": "bfloat16", "hidden_act": "silu"}


def export_checkpoint(ckpt: str, fmt: str, out: str, quant: Optional[str] = None) -> Dict[str, Any]:
    from safetensors.torch import save_file

    from llmctl.io.artifact import resolve_checkpoint_dir
    from llmctl.io.checkpoint import load_full_state_dict
    from llmctl.models.config import ModelConfig

    if fmt in UNSUPPORTED:
        raise NotImplementedError(f"format {fmt!r}: {UNSUPPORTED[fmt]}")
    if fmt not in ("safetensors", "hf"):
        raise NotImplementedError(f"unknown format {fmt!r}")
    ck = resolve_checkpoint_dir(ckpt)
    if ck is None:
        raise FileNotFoundError(f"no checkpoint (config.json) under {ckpt}")
    cfg = ModelConfig.from_file(ck / "config.json")
    sd = {k: v.contiguous() for k, v in load_full_state_dict(ck, cfg).items()}
    if fmt == "hf":
        if cfg.norm != "rmsnorm" or not cfg.gated_mlp:
            raise NotImplementedError("hf export supports Llama-style (RMSNorm/SwiGLU) models")
        sd = to_hf_llama(sd, cfg)
    qinfo = None
    if quant:
        from llmctl.plugins.quantizers import ALIASES, QUANTIZERS

        name = ALIASES.get(quant, quant)
        if name not in QUANTIZERS:
            raise NotImplementedError(f"unknown quantizer {quant!r}")
        if quant in ALIASES:
            warnings.warn(f"{quant}: no calibration data offline; using round-to-nearest {name}")
        qsd = {}
        for k, v in sd.items():
            if v.dim() == 2 and ("proj" in k or k.split(".")[-1] in ("wqkv", "wo", "w_up", "w_down")):
                r = QUANTIZERS[name](v)
                qsd[k + ".qweight"] = r["qweight"].contiguous()
                qsd[k + ".scale"] = r["scale"].contiguous()
            else:
                qsd[k] = v
        sd = qsd
        qinfo = {"method": "rtn", "format": name, "requested": quant, "granularity": "per-output-channel"}
    outp = Path(out)
    outp.mkdir(parents=True, exist_ok=True)
    save_file(sd, str(outp / "model.safetensors"), metadata={"format": "pt", "llmctl_export": fmt})
    conf = hf_config(cfg) if fmt == "hf" else cfg.to_dict()
    if qinfo:
        conf["quantization_config"] = qinfo
    (outp / "config.json").write_text(json.dumps(conf, indent=2))
    for f in ("tokenizer.json", "tokenizer_config.json"):
        if (ck / f).exists():
            (outp / f).write_bytes((ck / f).read_bytes())
    return {"source": str(ck), "format": fmt, "tensors": len(sd), "out": str(outp), "quantization": qinfo,
            "bytes": sum(v.numel() * v.element_size() for v in sd.values())}


def register(reg) -> None:
    reg.add("exporters", "safetensors", lambda ckpt, out, quant=None: export_checkpoint(ckpt, "safetensors", out, quant))
    reg.add("exporters", "hf", lambda ckpt, out, quant=None: export_checkpoint(ckpt, "hf", out, quant))
