"""Inference engine: batched prefill + paged-KV decode on llmctl's HIP kernels, with
hipGraph-captured decode steps.

Reference ``InferenceEngine`` (``server.py:127-251``) re-ran a full-prefix HF forward for
every generated token with ``use_cache=True`` but discarded the cache, right-padded
batches and read the logits of the padded last position (wrong tokens for shorter
prompts), and sampled with a host sync per request per token.  Here:

* prefill (round 2): CHUNKED and prefix-aware.  The scheduler hands out chunks (sequence,
  first position, count) under a per-step token budget; the chunks of all sequences are packed
  back to back (no padding), RoPE'd and written into the paged cache in one fused pass, and
  attend through ``paged_prefill_attention`` (csrc/paged_prefill.hip): every query reads its
  keys from the block table, so a cached prefix (earlier chunk, prefix-cache hit, resumed
  sequence) and the chunk itself are one key range.  Logits are taken only at the last token
  of chunks that complete a sequence's known tokens;
* decode: one token per running sequence; per layer ``rope_qkv`` (explicit positions) ->
  ``kv_cache_write`` -> ``paged_attention_decode`` (block tables, GQA) -> o-proj -> MLP;
  the whole decode step (embedding .. lm_head) is captured once per batch-size bucket in
  a HIP graph and replayed with static input buffers (no per-layer launch overhead);
* sampling: one batched kernel (temperature / top-k / top-p / greedy) with uniforms drawn
  once per step; the only host sync per step is reading the sampled ids.
"""

from __future__ import annotations

import logging
import math
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from llmctl import ops
from llmctl.config.knobs import use as use_knobs
from llmctl.io.artifact import load_model
from llmctl.models import DecoderLM
from llmctl.utils.env import graph_capture_gc_guard

from .block_manager import PagedKVCache, make_kv_manager
from .prefix_cache import PrefixCache
from .scheduler import ContinuousBatchScheduler, PrefillChunk, SamplingParams, Sequence
from .tokenizer import load_tokenizer

log = logging.getLogger("llmctl.serve")


class InferenceEngine:
    def __init__(self, model_path: str = "tiny", device: str = "auto", dtype=torch.bfloat16, max_batch_size: int = 8,
                 max_batch_tokens: int = 8192, max_model_len: Optional[int] = None, kv_cache_fraction: float = 0.85,
                 block_size: int = 16, num_kv_blocks: Optional[int] = None, scheduler: str = "dynamic",
                 use_graphs: bool = True, seed: int = 0, pc=None, prefix_caching: bool = True,
                 tuning_cache: Optional[str] = None, perf_knobs: Optional[Dict] = None,
                 kv_cache_dtype: str = "auto", weight_dtype: str = "auto"):
        from llmctl.config import knobs as perf

        self.knobs = perf.configure(perf_knobs)  # defaults + perf_knobs + LLMCTL_KNOBS
        if device == "auto":
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.device.type == "cpu" and dtype == torch.bfloat16:
            dtype = torch.float32  # the CPU oracle path
        if self.device.type == "cuda":  # pre-tuned prefill projection GEMMs (llmctl.exec.gemm_tuning)
            from llmctl.exec.gemm_tuning import enable_tuned_gemms

            enable_tuned_gemms()
        from llmctl.plugins import tuning_cache as _tc

        tc = _tc.resolve(tuning_cache)
        self.tuned = _tc.apply_serving(tc) if tc is not None else {}
        self.knobs = perf.knobs()  # perf_knobs + tuning cache + LLMCTL_KNOBS: this engine's routing
        self.dtype = dtype
        self.model_path = model_path
        self.model: DecoderLM
        self.pc = pc
        self.tp = pc.tp_size if pc is not None else 1
        self.model, self.cfg, self.ckpt = self._load(model_path, dtype, seed)
        self.model.eval()
        self.tokenizer = load_tokenizer(str(self.ckpt) if self.ckpt else None)
        cfg = self.cfg
        self.max_model_len = max_model_len or cfg.max_position_embeddings
        self.block_size = block_size
        self.max_blocks_per_seq = (self.max_model_len + block_size - 1) // block_size
        # decode projection weights: the model's ("auto"), or an fp8 (OCP e4m3fn) copy with fp32 row
        # scales ("fp8", W8A16) that the fused decode path streams instead (half the bytes of the
        # HBM-bound decode GEMMs); prefill keeps the bf16 weights.  Made before the KV cache is sized.
        self._w8: Optional[List[Dict[str, Tuple[torch.Tensor, torch.Tensor]]]] = None
        self._w8_head: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        if weight_dtype in ("fp8", "fp8_e4m3", "float8_e4m3fn"):
            if self.device.type == "cuda":
                self._w8 = self._quantize_decode_weights()
        elif weight_dtype not in ("auto", "model", "bf16", "bfloat16"):
            raise ValueError(f"weight_dtype must be auto / bf16 / fp8, got {weight_dtype!r}")
        self.weight_dtype = "fp8" if self._w8 is not None else "auto"
        # prefill with the RMSNorms folded into the QKV / gate-up projections (knob
        # prefill_norm_fold): copies of those weights with the norm weight multiplied into their K
        # columns ((H + 2 kv) D + 2 F) H bf16 per layer, made before the KV cache is sized
        self._nf: Optional[List[Tuple[torch.Tensor, torch.Tensor]]] = (
            self._fold_norm_weights() if self.knobs.prefill_norm_fold else None)
        # KV cache element: the model dtype ("auto"), or OCP fp8 e4m3fn ("fp8": half the bytes per
        # token, so twice the blocks and half the decode attention's HBM stream; saturating at +-448)
        if kv_cache_dtype in ("auto", "model", "bf16", "bfloat16"):
            self.kv_dtype = dtype
        elif kv_cache_dtype in ("fp8", "fp8_e4m3", "float8_e4m3fn"):
            self.kv_dtype = torch.float8_e4m3fn
        else:
            raise ValueError(f"kv_cache_dtype must be auto / bf16 / fp8, got {kv_cache_dtype!r}")
        if num_kv_blocks is None:
            if self.device.type == "cuda":
                torch.cuda.synchronize()
                free, _ = torch.cuda.mem_get_info(self.device)
                budget = free * kv_cache_fraction
            else:
                budget = 256 * 2 ** 20
            num_kv_blocks = PagedKVCache.blocks_for_memory(budget, cfg.layers, block_size, cfg.kv_heads // self.tp,
                                                           cfg.head_dim, torch.tensor([], dtype=self.kv_dtype).element_size())
            num_kv_blocks = min(num_kv_blocks, 1 << 20)
            num_kv_blocks = self._agree_min(num_kv_blocks)
        # each TP rank caches only its own KV heads
        self.kv_cache = PagedKVCache(cfg.layers, num_kv_blocks, block_size, cfg.kv_heads // self.tp, cfg.head_dim,
                                     self.kv_dtype, self.device)
        self.kv = make_kv_manager(num_kv_blocks, block_size)
        self.prefix_cache = PrefixCache(self.kv, block_size) if prefix_caching else None
        self.scheduler = ContinuousBatchScheduler(self.kv, max_batch_size, max_batch_tokens, self.max_model_len,
                                                  scheduler, block_size, prefix_cache=self.prefix_cache)
        self.max_batch_size = max_batch_size
        self.rope = self.model.rope_tables(self.max_model_len, self.device)
        # MoE routing sizes the expert segments on the host: decode runs eagerly
        self.use_graphs = use_graphs and self.device.type == "cuda" and not cfg.is_moe
        self._graphs: Dict[int, Tuple[torch.cuda.CUDAGraph, Dict[str, torch.Tensor]]] = {}
        # sampling uniforms come from the host (one H2D copy with the step's other inputs), so
        # in-graph sampling and the eager path draw the same stream
        self._np_rng = np.random.default_rng(seed)
        self._pending: Optional[Dict] = None  # an in-flight asynchronous decode step
        self._last_toks: Optional[torch.Tensor] = None  # eager path: the last step's sampled ids
        self.stats = {"steps": 0, "prefill_tokens": 0, "decode_tokens": 0, "graph_replays": 0}
        log.info("engine: %s on %s, %d KV blocks x %d tokens (%.1f GB)", cfg.name, self.device, num_kv_blocks,
                 block_size, self.kv_cache.nbytes / 1e9)

    def _fold_norm_weights(self) -> Optional[List[Tuple[torch.Tensor, torch.Tensor]]]:
        """(W_qkv * w_attn_norm, W_up * w_mlp_norm) per layer, or None when the model does not fit
        the folded prefill (GPU, TP=1, RMSNorm, RoPE, dense SwiGLU MLP without biases, gemm64 shapes)."""
        cfg, m = self.cfg, self.model
        if (self.device.type != "cuda" or self.tp != 1 or cfg.is_moe or not cfg.gated_mlp or cfg.norm != "rmsnorm"
                or cfg.position != "rope" or cfg.hidden % 128 or cfg.hidden < 256):
            return None
        out = []
        for layer in m.layers:
            if (layer.moe is not None or layer.bqkv is not None or layer.bo is not None or layer.b_up is not None
                    or layer.b_down is not None or layer.wqkv.shape[0] % 256 or layer.w_up.shape[0] % 256
                    or layer.w_down.shape[0] % 256):
                return None
            out.append(((layer.wqkv.float() * layer.attn_norm_w.float()).to(layer.wqkv.dtype).contiguous(),
                        (layer.w_up.float() * layer.mlp_norm_w.float()).to(layer.w_up.dtype).contiguous()))
        return out

    def _norm_fold_ok(self, T: int) -> bool:
        return self._nf is not None and self.knobs.prefill_norm_fold and T > 0 and T % 256 == 0

    def _prefill_layers_folded(self, x, pos, slots, fa, doc, bt, cu, ctx, work):
        """The prefill layers with each RMSNorm folded into the projection that consumes it: per layer
        rstd(h) -> QKV GEMM scaling its rows by rstd -> RoPE + cache write -> attention -> h += o W_o^T
        (hipBLASLt beta = 1) -> rstd(h) -> gate/up GEMM with row scale and SwiGLU -> h += act W_down^T
        (gemm64 accumulate epilogue).  Returns the residual stream h [T, H] after the last layer (the
        final norm is applied to the selected rows only)."""
        T = x.shape[0]
        eps = self.cfg.layer_norm_eps
        kc, vc = self.kv_cache.k, self.kv_cache.v
        h = x.contiguous()
        for li, layer in enumerate(self.model.layers):
            wqkv_f, wup_f = self._nf[li]
            qkv = ops.linear_rowscale(h, wqkv_f, ops.rms_rstd(h, eps))
            q, k, v = ops.rope_qkv_cache(qkv, self.rope[0], self.rope[1], layer.nq, layer.nkv, self.max_model_len,
                                         pos, kc[li], vc[li], slots)
            if fa:
                o = ops.flash_attention(q.view(1, T, layer.nq, layer.D), k.view(1, T, layer.nkv, layer.D),
                                        v.view(1, T, layer.nkv, layer.D), causal=True, doc_start=doc)
            else:
                o = ops.paged_prefill_attention(q.view(T, layer.nq, layer.D), kc[li], vc[li], bt, cu, ctx,
                                                work=work)
            h.addmm_(o.reshape(T, -1), layer.wo.t())
            act = ops.up_swiglu_rowscale(h, wup_f, ops.rms_rstd(h, eps))
            ops.linear_acc_(act, layer.w_down, h)
        return h

    # ------------------------------------------------------------------ TP hooks (identity at tp=1)
    def _load(self, model_path: str, dtype, seed: int):
        return load_model(model_path, device=self.device, dtype=dtype, seed=seed)

    def _agree_min(self, n: int) -> int:
        return n

    def _reduce(self, x: torch.Tensor) -> torch.Tensor:
        return x

    def _gather_vocab(self, logits: torch.Tensor) -> torch.Tensor:
        return logits

    def _fused_reduce_ok(self) -> bool:
        """TP > 1: can the row-parallel reductions fuse the bias / residual / RMSNorm (TP engine)."""
        return False

    def _reduce_add_rmsnorm(self, part, bias, res, norm_w, eps):
        """(rmsnorm(res + reduce(part) + bias) * norm_w, new residual) — TP=1: no reduction."""
        y = part if bias is None else part + bias
        return ops.add_rmsnorm(y, res, norm_w, eps)

    # ------------------------------------------------------------------ model pieces
    def _embed(self, ids: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        m = self.model
        if self.tp > 1:  # vocab-parallel table: local rows + all-reduce
            local = ids - m.vocab_start
            ok = (local >= 0) & (local < m.embed.shape[0])
            x = F.embedding(local.clamp(0, m.embed.shape[0] - 1), m.embed) * ok.unsqueeze(-1).to(m.embed.dtype)
            x = self._reduce(x)
        else:
            x = F.embedding(ids, m.embed)
        if m.pos_embed is not None:
            x = x + m.pos_embed[positions]
        return x

    def _norm(self, layer, x, res, which: str):
        w = layer.attn_norm_w if which == "attn" else layer.mlp_norm_w
        b = layer.attn_norm_b if which == "attn" else layer.mlp_norm_b
        eps = self.cfg.layer_norm_eps
        if res is None:
            return (ops.layernorm(x, w, b, eps) if b is not None else ops.rmsnorm(x, w, eps)), x
        return ops.add_layernorm(x, res, w, b, eps) if b is not None else ops.add_rmsnorm(x, res, w, eps)

    def _qkv(self, layer, xn, positions, seq_len, kc, vc, slots):
        """QKV projection, RoPE and the paged-cache write of this step's K/V rows (one fused
        pass with RoPE)."""
        qkv = ops.decode_linear(xn, layer.wqkv, layer.bqkv)
        if self.rope is not None:
            return ops.rope_qkv_cache(qkv, self.rope[0], self.rope[1], layer.nq, layer.nkv, seq_len, positions,
                                      kc, vc, slots)
        T = qkv.shape[0]
        x = qkv.view(T, layer.nq + 2 * layer.nkv, layer.D)
        q, k, v = (x[:, :layer.nq].contiguous(), x[:, layer.nq:layer.nq + layer.nkv].contiguous(),
                   x[:, layer.nq + layer.nkv:].contiguous())
        ops.kv_cache_write(k, v, kc, vc, slots)
        return q, k, v

    def _mlp(self, layer, xn):
        if layer.moe is not None:  # routed experts (host-side split sizes: eager, no graphs)
            return layer.moe(xn)
        if self.cfg.gated_mlp:
            # prefill-sized (T % 256 == 0): the SwiGLU rides on the gate/up GEMM's epilogue
            act = (ops.up_swiglu(xn, layer.w_up, layer.b_up) if xn.shape[0] >= 256 and xn.shape[0] % 256 == 0
                   else ops.swiglu(ops.decode_linear(xn, layer.w_up, layer.b_up)))
            out = ops.decode_linear(act, layer.w_down)
        else:
            out = ops.decode_linear(ops.gelu(ops.decode_linear(xn, layer.w_up, layer.b_up)), layer.w_down)
        out = self._reduce(out)  # row-parallel down projection
        if layer.b_down is not None:
            out = out + layer.b_down
        return out

    def _final(self, x, res):
        m = self.model
        eps = self.cfg.layer_norm_eps
        if m.final_norm_b is not None:
            xn, _ = ops.add_layernorm(x, res, m.final_norm_w, m.final_norm_b, eps)
        else:
            xn, _ = ops.add_rmsnorm(x, res, m.final_norm_w, eps)
        return self._gather_vocab(ops.decode_linear(xn, m.head_weight()))

    # ------------------------------------------------------------------ prefill
    def prefill_plan(self, chunks: List[PrefillChunk]) -> Dict:
        """Host-side description of a (chunked, packed) prefill step — what TP ranks receive."""
        ids, pos, slots, cu, ctx, last = [], [], [], [0], [], []
        for i, c in enumerate(chunks):
            toks = c.seq.all_ids
            ids.extend(toks[c.start:c.start + c.count])
            pos.extend(range(c.start, c.start + c.count))
            slots.append(np.asarray(self.kv.slots(c.seq.seq_id, c.start, c.count), dtype=np.int64))
            cu.append(cu[-1] + c.count)
            ctx.append(c.start + c.count)
            if c.final:
                last.append(cu[-1] - 1)
        bt = np.asarray(self.kv.block_tables([c.seq.seq_id for c in chunks], self.max_blocks_per_seq))
        # every chunk is a whole fresh prompt (no cached prefix): its keys are exactly the chunk's
        # own rows, so attention can run as packed-document flash attention (doc_start per token)
        fresh = bool(chunks) and all(c.start == 0 for c in chunks)
        doc = np.repeat(np.asarray(cu[:-1], dtype=np.int32), np.diff(cu)) if fresh else None
        return {"op": "prefill", "ids": np.asarray(ids, dtype=np.int64), "pos": np.asarray(pos, dtype=np.int32),
                "slots": np.concatenate(slots) if slots else np.zeros(0, dtype=np.int64), "cu": cu, "ctx": ctx,
                "bt": bt, "last": last, "work": ops.prefill_work_list(cu), "doc": doc}

    @torch.inference_mode()
    def prefill(self, chunks) -> torch.Tensor:
        """Run prefill chunks (``PrefillChunk`` list, or sequences: whole prompts); returns the
        logits [n_final, V] of the chunks that complete their sequence, in chunk order."""
        if chunks and isinstance(chunks[0], Sequence):
            chunks = [PrefillChunk(s, 0, s.num_tokens) for s in chunks]
        return self.prefill_exec(self.prefill_plan(chunks))

    @torch.inference_mode()
    def prefill_exec(self, plan: Dict) -> torch.Tensor:
        use_knobs(self.knobs)
        d = self.device
        T = len(plan["ids"])
        ids = torch.from_numpy(plan["ids"]).to(d, non_blocking=True)
        pos = torch.from_numpy(plan["pos"]).to(d, non_blocking=True)
        slots = torch.from_numpy(plan["slots"]).to(d, non_blocking=True)
        bt = torch.from_numpy(plan["bt"]).to(d, non_blocking=True)
        cu = torch.tensor(plan["cu"], dtype=torch.int32).to(d, non_blocking=True)
        ctx = torch.tensor(plan["ctx"], dtype=torch.int32).to(d, non_blocking=True)
        work = torch.tensor(plan["work"], dtype=torch.int32).to(d, non_blocking=True)
        # fresh prompts: the training flash-attention kernel over packed documents, K/V straight
        # from the RoPE pass (16 x 2k burst TTFT p50 224.6 -> 218.6 ms, single 2k prompt 27.5 ->
        # 26.2 ms, profiles/serve_r2_session6.txt); knob prefill_fa off keeps the paged kernel
        doc = None
        fa = plan.get("doc") is not None and d.type == "cuda" and self.knobs.prefill_fa
        if fa and len(plan["cu"]) > 2:  # several prompts packed: document boundaries
            doc = torch.from_numpy(plan["doc"]).to(d, non_blocking=True).view(1, T)
        # (one prompt: plain causal attention, which also lets the kernel split the K/V range of
        # its few q-blocks over two workgroups — the split is off for packed documents)
        x = self._embed(ids, pos.long())
        if self._norm_fold_ok(T):
            h = self._prefill_layers_folded(x, pos, slots, fa, doc, bt, cu, ctx, work)
            self.stats["prefill_tokens"] += T
            if not plan["last"]:
                return torch.empty(0, self.cfg.vocab_size, device=d, dtype=h.dtype)
            hl = h.index_select(0, torch.tensor(plan["last"], device=d))
            xn = ops.rmsnorm(hl, self.model.final_norm_w, self.cfg.layer_norm_eps)
            return self._gather_vocab(ops.decode_linear(xn, self.model.head_weight()))
        res = None
        kc, vc = self.kv_cache.k, self.kv_cache.v
        for li, layer in enumerate(self.model.layers):
            xn, res = self._norm(layer, x, res, "attn")
            q, k, v = self._qkv(layer, xn, pos, self.max_model_len, kc[li], vc[li], slots)
            if fa:
                o = ops.flash_attention(q.view(1, T, layer.nq, layer.D), k.view(1, T, layer.nkv, layer.D),
                                        v.view(1, T, layer.nkv, layer.D), causal=True, doc_start=doc)
            else:
                o = ops.paged_prefill_attention(q.view(T, layer.nq, layer.D), kc[li], vc[li], bt, cu, ctx,
                                                work=work)
            a = self._reduce(ops.decode_linear(o.view(T, -1), layer.wo))
            if layer.bo is not None:
                a = a + layer.bo
            xn, res = self._norm(layer, a, res, "mlp")
            x = self._mlp(layer, xn)
        self.stats["prefill_tokens"] += T
        if not plan["last"]:
            return torch.empty(0, self.cfg.vocab_size, device=d, dtype=x.dtype)
        last = torch.tensor(plan["last"], device=d)
        return self._final(x.index_select(0, last), res.index_select(0, last))

    # ------------------------------------------------------------------ mixed prefill + decode
    def mixed_plan(self, chunks: List[PrefillChunk], seqs: List[Sequence]) -> Dict:
        """One step's prefill chunks AND decode tokens as one token batch (decode rows last)."""
        p, d = self.prefill_plan(chunks), self.decode_plan(seqs)
        return {"op": "mixed", "prefill": p, "decode": d}

    @torch.inference_mode()
    def mixed(self, chunks: List[PrefillChunk], seqs: List[Sequence]) -> torch.Tensor:
        return self.mixed_exec(self.mixed_plan(chunks, seqs))

    @torch.inference_mode()
    def mixed_exec(self, plan: Dict) -> torch.Tensor:
        """Mixed step (continuous batching's fused step): the decode tokens of the running batch
        ride in the prefill chunks' forward — every projection / MLP GEMM streams its weights
        once for both kinds of rows — and only attention splits by row kind: prefill rows through
        the (paged or fresh-prompt flash) prefill attention, decode rows through the paged decode
        kernel.  Returns logits [n_final_chunks + n_decode, V]: the final chunks' rows first, in
        chunk order, then the decode rows (eager: the graph-captured decode step is for
        decode-only steps).  Reference batching: ``llmctl/serve/server.py:89-125, 372-386``."""
        use_knobs(self.knobs)
        d = self.device
        pp, dp = plan["prefill"], plan["decode"]
        Tp, Td = len(pp["ids"]), len(dp["ids"])
        ids = torch.cat([torch.from_numpy(pp["ids"]), torch.tensor(dp["ids"], dtype=torch.long)]).to(d, non_blocking=True)
        pos = torch.cat([torch.from_numpy(pp["pos"]), torch.tensor(dp["positions"], dtype=torch.int32)]).to(d, non_blocking=True)
        slots = torch.cat([torch.from_numpy(pp["slots"]), torch.tensor(dp["slots"], dtype=torch.long)]).to(d, non_blocking=True)
        bt = torch.from_numpy(pp["bt"]).to(d, non_blocking=True)
        cu = torch.tensor(pp["cu"], dtype=torch.int32).to(d, non_blocking=True)
        ctx = torch.tensor(pp["ctx"], dtype=torch.int32).to(d, non_blocking=True)
        work = torch.tensor(pp["work"], dtype=torch.int32).to(d, non_blocking=True)
        bt_d = torch.from_numpy(dp["bt"]).to(d, non_blocking=True)
        ctx_d = torch.tensor(dp["ctx"], dtype=torch.int32).to(d, non_blocking=True)
        fa = pp.get("doc") is not None and d.type == "cuda" and self.knobs.prefill_fa
        doc = torch.from_numpy(pp["doc"]).to(d, non_blocking=True).view(1, Tp) if fa and len(pp["cu"]) > 2 else None
        x = self._embed(ids, pos.long())
        res = None
        kc, vc = self.kv_cache.k, self.kv_cache.v
        for li, layer in enumerate(self.model.layers):
            xn, res = self._norm(layer, x, res, "attn")
            q, k, v = self._qkv(layer, xn, pos, self.max_model_len, kc[li], vc[li], slots)
            if fa:
                op = ops.flash_attention(q[:Tp].reshape(1, Tp, layer.nq, layer.D),
                                         k[:Tp].reshape(1, Tp, layer.nkv, layer.D),
                                         v[:Tp].reshape(1, Tp, layer.nkv, layer.D), causal=True, doc_start=doc)
            else:
                op = ops.paged_prefill_attention(q[:Tp].reshape(Tp, layer.nq, layer.D), kc[li], vc[li], bt, cu, ctx,
                                                 work=work)
            od = ops.paged_attention_decode(q[Tp:].reshape(Td, layer.nq, layer.D).contiguous(), kc[li], vc[li], bt_d,
                                            ctx_d)
            o = torch.cat([op.reshape(Tp, -1), od.reshape(Td, -1)])
            a = self._reduce(ops.decode_linear(o, layer.wo))
            if layer.bo is not None:
                a = a + layer.bo
            xn, res = self._norm(layer, a, res, "mlp")
            x = self._mlp(layer, xn)
        self.stats["prefill_tokens"] += Tp
        self.stats["decode_tokens"] += Td
        self.stats["mixed_steps"] = self.stats.get("mixed_steps", 0) + 1
        rows = torch.tensor(list(pp["last"]) + list(range(Tp, Tp + Td)), device=d)
        return self._final(x.index_select(0, rows), res.index_select(0, rows))

    def _mixed_ok(self) -> bool:
        """Knob ``mixed_steps`` off runs a step's decode and prefill as two forwards (A/B)."""
        return self.knobs.mixed_steps

    # ------------------------------------------------------------------ decode
    def _fused_decode(self) -> bool:
        """Decode layers on the fused-epilogue projections (``ops.decode_qkv_rope_cache`` /
        ``decode_up_swiglu`` / ``decode_linear_add_rmsnorm``): 10 kernels per layer instead of 13
        (the RoPE/cache-write, SwiGLU and add+RMSNorm passes ride on the projections' finalize).  Needs the GPU path,
        RMSNorm, RoPE and a gated MLP; at TP > 1 the row-parallel projections' all-reduce, bias,
        residual add and next RMSNorm are one custom-all-reduce kernel
        (``_reduce_add_rmsnorm``); knob ``decode_fused`` off keeps the unfused layer (A/B)."""
        cfg, m = self.cfg, self.model
        return (self.device.type == "cuda" and (self.tp == 1 or self._fused_reduce_ok()) and self.rope is not None
                and cfg.gated_mlp
                and not cfg.is_moe and m.final_norm_b is None
                and all(l.attn_norm_b is None and l.mlp_norm_b is None for l in m.layers)
                and self.knobs.decode_fused)

    def _decode_body(self, ids, positions, slots, block_tables, ctx_lens) -> torch.Tensor:
        if self._fused_decode():
            return self._decode_body_fused(ids, positions, slots, block_tables, ctx_lens)
        x = self._embed(ids, positions)
        res = None
        kc, vc = self.kv_cache.k, self.kv_cache.v
        for li, layer in enumerate(self.model.layers):
            xn, res = self._norm(layer, x, res, "attn")
            q, k, v = self._qkv(layer, xn, positions, self.max_model_len, kc[li], vc[li], slots)
            o = ops.paged_attention_decode(q, kc[li], vc[li], block_tables, ctx_lens)
            a = self._reduce(ops.decode_linear(o.view(o.shape[0], -1), layer.wo))
            if layer.bo is not None:
                a = a + layer.bo
            xn, res = self._norm(layer, a, res, "mlp")
            x = self._mlp(layer, xn)
        return self._final(x, res)

    _W8_NAMES = ("wqkv", "wo", "w_up", "w_down")

    @torch.no_grad()
    def _quantize_decode_weights(self) -> List[Dict[str, Tuple[torch.Tensor, torch.Tensor]]]:
        """Per layer: fp8 (e4m3fn) copies of the decode projection weights + fp32 row scales
        (``llmctl.plugins.quantizers.quantize_fp8``: absmax / 448 per output row)."""
        from llmctl.plugins.quantizers import quantize_fp8

        out = []
        for layer in self.model.layers:
            d = {}
            for name in self._W8_NAMES:
                w = getattr(layer, name, None)
                # only weights the fused fp8 kernels take (ops.decode_fused_ok: out % 64, in % 128)
                if w is None or w.dim() != 2 or w.shape[0] % 64 or w.shape[1] % 128:
                    continue
                qd = quantize_fp8(w.detach())
                d[name] = (qd["qweight"].contiguous(), qd["scale"].float().contiguous())
            out.append(d)
        hw = self.model.head_weight()
        if hw.dim() == 2 and hw.shape[0] % 64 == 0 and hw.shape[1] % 128 == 0:  # the (local shard of the) LM head
            qd = quantize_fp8(hw.detach())
            self._w8_head = (qd["qweight"].contiguous(), qd["scale"].float().contiguous())
        return out

    W8_MAX_ROWS = 16  # the fused fp8 decode kernels take at most 16 token rows (ops.decode_fused_ok)

    def _dw(self, li: int, layer, name: str, n: int):
        """(weight, row scales or None) the fused decode path streams for ``layer.name`` at ``n``
        token rows: the fp8 copy only where the fused fp8 kernel takes it, else the bf16 weight
        (which is kept) -- never a per-step dequantised fp32 image of the fp8 one."""
        if self._w8 is not None and 1 <= n <= self.W8_MAX_ROWS and name in self._w8[li]:
            q = self._w8[li][name]
            if name not in ("wo", "w_down") or q[0].shape[0] <= 16384:  # add+RMSNorm finalize limit
                return q
        return getattr(layer, name), None

    def _decode_body_fused(self, ids, positions, slots, block_tables, ctx_lens) -> torch.Tensor:
        m = self.model
        eps = self.cfg.layer_norm_eps
        layers = m.layers
        kc, vc = self.kv_cache.k, self.kv_cache.v
        x = self._embed(ids, positions)
        xn, res = ops.rmsnorm(x, layers[0].attn_norm_w, eps), x
        tp = self.tp > 1
        def lin(x, w, s):  # a plain decode projection (TP row-parallel partial): bf16 or fp8 weights
            return ops.decode_linear(x, w) if s is None else ops.decode_linear_fp8(x, w, s)

        n = ids.shape[0]
        for li, layer in enumerate(layers):
            (wqkv, sqkv), (wo, so) = self._dw(li, layer, "wqkv", n), self._dw(li, layer, "wo", n)
            (wu, su), (wd, sd) = self._dw(li, layer, "w_up", n), self._dw(li, layer, "w_down", n)
            o = ops.decode_attention_qkv(xn, wqkv, layer.bqkv, self.rope[0], self.rope[1], layer.nq,
                                         layer.nkv, positions, kc[li], vc[li], slots, block_tables, ctx_lens,
                                         w_scale=sqkv)
            if tp:  # row-parallel o-proj partial -> one kernel: all-reduce + bias + residual + RMSNorm
                xn, res = self._reduce_add_rmsnorm(lin(o.view(o.shape[0], -1), wo, so), layer.bo,
                                                   res, layer.mlp_norm_w, eps)
            else:
                xn, res = ops.decode_linear_add_rmsnorm(o.view(o.shape[0], -1), wo, layer.bo, res,
                                                        layer.mlp_norm_w, eps, w_scale=so)
            act = ops.decode_up_swiglu(xn, wu, layer.b_up, w_scale=su)  # the local F shard
            nw = layers[li + 1].attn_norm_w if li + 1 < len(layers) else m.final_norm_w
            if tp:
                xn, res = self._reduce_add_rmsnorm(lin(act, wd, sd), layer.b_down, res, nw, eps)
            else:
                xn, res = ops.decode_linear_add_rmsnorm(act, wd, layer.b_down, res, nw, eps, w_scale=sd)
        if self._w8_head is not None and n <= self.W8_MAX_ROWS:
            return self._gather_vocab(ops.decode_linear_fp8(xn, *self._w8_head))
        return self._gather_vocab(ops.decode_linear(xn, m.head_weight()))

    def _bucket(self, n: int) -> int:
        b = 1
        while b < n:
            b *= 2
        return min(b, max(self.max_batch_size, n))

    _STAGED = ("ids", "positions", "slots", "block_tables", "ctx_lens", "u")

    def _static(self, nb: int) -> Dict:
        d = self.device
        bufs = {"ids": torch.zeros(nb, dtype=torch.long, device=d),
                "positions": torch.zeros(nb, dtype=torch.int32, device=d),
                "slots": torch.full((nb,), -1, dtype=torch.long, device=d),
                "block_tables": torch.zeros(nb, self.max_blocks_per_seq, dtype=torch.int32, device=d),
                "ctx_lens": torch.ones(nb, dtype=torch.int32, device=d),
                # in-graph sampling: per-row parameters (rewritten when the batch's change) and uniforms
                "u": torch.zeros(nb, dtype=torch.float32, device=d),
                "temp": torch.zeros(nb, dtype=torch.float32, device=d),
                "topk": torch.zeros(nb, dtype=torch.int32, device=d),
                "topp": torch.ones(nb, dtype=torch.float32, device=d)}
        # pinned host staging of the step inputs, two sets: an asynchronous step refills one while
        # the other's H2D copies may still be queued behind the step in flight (a non_blocking
        # copy from pageable memory would be synchronous)
        pin = self.device.type == "cuda"
        stage = []
        for _ in range(2):
            # initialised from the device defaults: rows past the live batch are copied too and
            # must stay valid (block id 0, context 1) for the padded graph rows
            h = {k: bufs[k].to("cpu") for k in self._STAGED}
            stage.append({k: (v.pin_memory() if pin else v) for k, v in h.items()})
        bufs["stage"] = stage
        bufs["flip"] = 0
        toks = torch.zeros(nb, dtype=torch.long)
        bufs["host_toks"] = [toks.pin_memory() if pin else toks, toks.clone().pin_memory() if pin else toks.clone()]
        bufs["tflip"] = 0
        bufs["params_key"] = None
        return bufs

    def _graph_body(self, bufs: Dict) -> None:
        """Decode step + sampling; the sampled ids also become the next step's input ids (the
        asynchronous path launches step N + 1 without reading step N's tokens first)."""
        bufs["logits"] = self._decode_body(bufs["ids"], bufs["positions"], bufs["slots"], bufs["block_tables"],
                                           bufs["ctx_lens"])
        bufs["toks"] = ops.sample(bufs["logits"].contiguous(), bufs["temp"], bufs["topk"], bufs["topp"], bufs["u"])
        bufs["ids"].copy_(bufs["toks"])

    def _capture(self, nb: int):
        bufs = self._static(nb)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up (allocator / lazy init) outside the graph
                self._graph_body(bufs)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with graph_capture_gc_guard(), torch.cuda.graph(g):
            self._graph_body(bufs)
        self._graphs[nb] = (g, bufs)

    def release_graphs(self) -> None:
        """Drop the captured decode graphs (they hold the RCCL communicator's captured
        collectives: release them before ``destroy_process_group``)."""
        if self._graphs and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for g, _ in self._graphs.values():
            g.reset()
        self._graphs.clear()

    def close(self) -> None:
        """Deterministic teardown, never left to garbage collection: drop an in-flight pipelined
        step, release the captured decode graphs (their memory pool and any captured collectives),
        drain the device and drop the KV cache / weights this engine holds.  Idempotent; the engine
        is unusable afterwards.  Also the ``with InferenceEngine(...) as e:`` exit."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        self._release_resources()

    def _release_resources(self) -> None:
        self._pending = None
        self._last_toks = None
        self.release_graphs()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.kv_cache = None
        self._w8 = self._w8_head = None
        self._nf = None
        self.rope = None
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def __enter__(self):
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def decode_plan(self, seqs: List[Sequence]) -> Dict:
        return {"op": "decode", "ids": [s.last_id for s in seqs], "positions": [s.num_tokens - 1 for s in seqs],
                "slots": [s._decode_slot for s in seqs], "ctx": [self.kv.num_tokens(s.seq_id) for s in seqs],
                "bt": np.asarray(self.kv.block_tables([s.seq_id for s in seqs], self.max_blocks_per_seq))}

    @torch.inference_mode()
    def decode(self, seqs: List[Sequence]) -> torch.Tensor:
        return self.decode_exec(self.decode_plan(seqs))

    @torch.inference_mode()
    def decode_exec(self, plan: Dict) -> torch.Tensor:
        use_knobs(self.knobs)
        ids, positions, slots, ctx, bt = plan["ids"], plan["positions"], plan["slots"], plan["ctx"], plan["bt"]
        n = len(ids)
        self.stats["decode_tokens"] += n
        if self.use_graphs:
            g, b = self._stage_and_replay(plan, cont=False)
            return b["logits"][:n]
        d = self.device
        return self._decode_body(torch.tensor(ids, device=d), torch.tensor(positions, dtype=torch.int32, device=d),
                                 torch.tensor(slots, device=d), torch.from_numpy(bt).to(d),
                                 torch.tensor(ctx, dtype=torch.int32, device=d))

    def _stage_and_replay(self, plan: Dict, cont: bool):
        """Fill one host staging set with the step's inputs, copy them (asynchronously) into the
        graph's static buffers and replay it.  ``cont``: the input ids are already on the device
        (the previous replay of this graph sampled them), only positions / slots / block tables /
        context lengths / uniforms are copied.  A sampling plan (``decode_s``) carries its uniforms
        ``u`` and per-row ``temp`` / ``topk`` / ``topp``; a logits-only plan draws nothing (the
        in-graph sampling result is unused then, and the host RNG stream stays the one every
        engine configuration consumes: one uniform per sampled row)."""
        n = len(plan["positions"])
        nb = self._bucket(n)
        if nb not in self._graphs:
            self._capture(nb)
        g, b = self._graphs[nb]
        h = b["stage"][b["flip"]]
        b["flip"] ^= 1
        hn = {k: v.numpy() for k, v in h.items()}
        if not cont:
            hn["ids"][:n] = plan["ids"]
        hn["positions"][:n] = plan["positions"]
        hn["slots"][:] = -1
        hn["slots"][:n] = plan["slots"]
        hn["block_tables"][:n] = plan["bt"]
        hn["ctx_lens"][:] = 1
        hn["ctx_lens"][:n] = plan["ctx"]
        hn["u"][:n] = plan["u"] if "u" in plan else 0.0
        if "temp" in plan:
            key = (np.asarray(plan["temp"], dtype=np.float32).tobytes(), np.asarray(plan["topk"], dtype=np.int32).tobytes(),
                   np.asarray(plan["topp"], dtype=np.float32).tobytes())
            if b["params_key"] != key:
                d = self.device
                b["temp"].zero_()
                b["topk"].zero_()
                b["topp"].fill_(1.0)
                b["temp"][:n].copy_(torch.from_numpy(np.frombuffer(key[0], dtype=np.float32).copy()).to(d))
                b["topk"][:n].copy_(torch.from_numpy(np.frombuffer(key[1], dtype=np.int32).copy()).to(d))
                b["topp"][:n].copy_(torch.from_numpy(np.frombuffer(key[2], dtype=np.float32).copy()).to(d))
                b["params_key"] = key
        for k in self._STAGED:
            if cont and k == "ids":
                continue
            b[k].copy_(h[k], non_blocking=True)
        g.replay()
        self.stats["graph_replays"] += 1
        return g, b

    # ------------------------------------------------------------------ asynchronous decode
    @staticmethod
    def _sampling_fields(seqs: List[Sequence]) -> Dict[str, np.ndarray]:
        return {"temp": np.asarray([s.params.temperature for s in seqs], dtype=np.float32),
                "topk": np.asarray([s.params.top_k if s.params.top_k and s.params.top_k > 0 else 0 for s in seqs],
                                   dtype=np.int32),
                "topp": np.asarray([s.params.top_p for s in seqs], dtype=np.float32)}

    def _publish(self, plan: Dict) -> Dict:
        """TP hook: rank 0's plan to the other ranks (identity at TP = 1)."""
        return plan

    @torch.inference_mode()
    def _launch_decode(self, seqs: List[Sequence], plan: Dict, cont: bool) -> Dict:
        """Run a decode step with sampling (the graph replay, or the eager layer stack) and queue
        the D2H copy of its tokens; the tokens are read by :meth:`_finalize`.  ``cont``: the
        input ids are the previous step's sampled tokens, already on the device.

        TP > 1: the plan -- with the step's uniforms and sampling parameters -- goes to every rank
        first; every rank runs the same step and the same in-graph sampling on the same gathered
        logits and uniforms, so all ranks hold identical sampled ids on the device without a
        broadcast of the tokens, and a continued step (``cont``) feeds them back as its input on
        every rank.  Only rank 0 reads the tokens back."""
        n = len(seqs)
        self.stats["decode_tokens"] += n
        plan = dict(plan, op="decode_s", cont=bool(cont), u=self._np_rng.random(n, dtype=np.float32),
                    **self._sampling_fields(seqs))
        if cont:
            plan.setdefault("ids", np.zeros(n, dtype=np.int64))
        toks = self._decode_sample_exec(self._publish(plan))
        d = self.device
        if self.use_graphs:
            b = self._graphs[self._bucket(n)][1]
            out = b["host_toks"][b["tflip"]]
            b["tflip"] ^= 1
            out.copy_(toks, non_blocking=True)
        else:
            out = toks.to("cpu", non_blocking=True) if d.type == "cuda" else toks
        ev = None
        if d.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        return {"seqs": list(seqs), "host": out, "event": ev, "n": n}

    @torch.inference_mode()
    def _decode_sample_exec(self, plan: Dict) -> torch.Tensor:
        """Every rank's half of :meth:`_launch_decode`: the decode step + sampling of a
        ``decode_s`` plan; returns the device tensor of sampled ids (graph: the static ``toks``
        buffer, all bucket rows)."""
        use_knobs(self.knobs)
        cont = bool(plan["cont"])
        if self.use_graphs:
            _, b = self._stage_and_replay(plan, cont)
            return b["toks"]
        d = self.device
        n = len(plan["positions"])
        ids = self._last_toks if cont else torch.as_tensor(np.asarray(plan["ids"], dtype=np.int64)).to(d)
        logits = self._decode_body(ids, torch.as_tensor(np.asarray(plan["positions"], dtype=np.int32)).to(d),
                                   torch.as_tensor(np.asarray(plan["slots"], dtype=np.int64)).to(d),
                                   torch.from_numpy(np.asarray(plan["bt"])).to(d),
                                   torch.as_tensor(np.asarray(plan["ctx"], dtype=np.int32)).to(d))
        temp = torch.from_numpy(np.asarray(plan["temp"], dtype=np.float32)).to(d)
        topk = torch.from_numpy(np.asarray(plan["topk"], dtype=np.int32)).to(d)
        topp = torch.from_numpy(np.asarray(plan["topp"], dtype=np.float32)).to(d)
        u = torch.from_numpy(np.asarray(plan["u"], dtype=np.float32)).to(d)
        toks = ops.sample(logits[:n].contiguous(), temp, topk, topp, u)
        self._last_toks = toks
        return toks

    def _finalize(self, p: Dict) -> int:
        """Read an in-flight step's tokens (the one host sync of the pipeline) and append them."""
        if p["event"] is not None:
            p["event"].synchronize()
        toks = p["host"][: p["n"]].tolist()
        produced = 0
        for seq, tok in zip(p["seqs"], toks):
            if seq.status != "running":  # finished by the previous step's tokens: speculative row
                continue
            self.scheduler.computed(seq, 1)
            self._append(seq, tok)
            produced += 1
        return produced

    def _continue_decode(self, p: Dict) -> Optional[Dict]:
        """Launch step N + 1 for the same batch before step N's tokens are known, when nothing
        else can change the batch: no request waiting for admission, every sequence of the batch
        still running and able to take two more tokens (length limits), and free KV blocks for
        one more token each (no preemption).  Its input ids are step N's sampled tokens, already
        on the device; positions / slots / context lengths advance by one."""
        seqs = p["seqs"]
        run = self.scheduler.running
        if (not self.knobs.async_decode or self.scheduler.waiting or len(run) != len(seqs)
                or any(a is not b for a, b in zip(run, seqs)) or self.kv.num_free_blocks < len(seqs)):
            return None
        for s in seqs:
            if (s.status != "running" or len(s.output_ids) + 2 > s.params.max_tokens
                    or s.num_tokens + 2 > self.max_model_len):
                return None
        for s in seqs:
            slot = self.kv.append_token(s.seq_id)
            if slot < 0:  # cannot happen with the free-block check; never launch half a batch
                raise RuntimeError("KV append failed despite free blocks")
            s._decode_slot = slot
            s.kv_len += 1
        plan = {"positions": [s.num_tokens for s in seqs], "slots": [s._decode_slot for s in seqs],
                "ctx": [self.kv.num_tokens(s.seq_id) for s in seqs],
                "bt": np.asarray(self.kv.block_tables([s.seq_id for s in seqs], self.max_blocks_per_seq))}
        self.stats["async_continued"] = self.stats.get("async_continued", 0) + 1
        return self._launch_decode(seqs, plan, cont=True)

    def _async_ok(self) -> bool:
        return self.knobs.async_decode

    # ------------------------------------------------------------------ sampling
    def sample(self, logits: torch.Tensor, seqs: List[Sequence]) -> List[int]:
        return self._sample_rows(logits, seqs).tolist()

    def _sample_rows(self, logits: torch.Tensor, seqs: List[Sequence]) -> torch.Tensor:
        """Sampled token ids (device tensor) of the rows of ``logits``, one uniform per row from
        the engine's host RNG (the same stream the in-graph sampling draws from)."""
        n = len(seqs)
        d = self.device
        # per-row sampling parameters: rebuilt (3 host->device copies) only when the batch's
        # parameters change, not every decode step
        key = tuple((s.params.temperature, s.params.top_k if s.params.top_k and s.params.top_k > 0 else 0,
                     s.params.top_p) for s in seqs)
        cached = getattr(self, "_sample_params", None)
        if cached is None or cached[0] != key:
            temp = torch.tensor([k[0] for k in key], dtype=torch.float32, device=d)
            topk = torch.tensor([k[1] for k in key], dtype=torch.int32, device=d)
            topp = torch.tensor([k[2] for k in key], dtype=torch.float32, device=d)
            self._sample_params = cached = (key, temp, topk, topp)
        _, temp, topk, topp = cached
        u = torch.from_numpy(self._np_rng.random(n, dtype=np.float32)).to(d)
        return ops.sample(logits.contiguous(), temp, topk, topp, u)

    # ------------------------------------------------------------------ step loop
    def add_request(self, prompt_ids: List[int], params: SamplingParams, request_id: str = "", on_token=None,
                    on_finish=None) -> Sequence:
        seq = Sequence(prompt_ids=list(prompt_ids), params=params, request_id=request_id, on_token=on_token,
                       on_finish=on_finish)
        self.scheduler.add(seq)
        return seq

    def _append(self, seq: Sequence, tok: int) -> None:
        now = time.time()
        if seq.first_token_time is None:
            seq.first_token_time = now
        seq.output_ids.append(tok)
        if seq.on_token:
            seq.on_token(seq, tok)
        eos = getattr(self.tokenizer, "eos_token_id", None)
        if not seq.params.ignore_eos and eos is not None and tok == eos:
            self.scheduler.finish(seq, "stop")
        elif len(seq.output_ids) >= seq.params.max_tokens:
            self.scheduler.finish(seq, "length")
        elif seq.num_tokens >= self.max_model_len:
            self.scheduler.finish(seq, "length")
        elif seq.params.stop:
            text = self.tokenizer.decode(seq.output_ids)
            if any(st and st in text for st in seq.params.stop):
                self.scheduler.finish(seq, "stop")

    def step(self) -> int:
        """One scheduling iteration; returns the number of tokens produced.  Pure decode steps
        run asynchronously (knob ``async_decode``): the step is launched and its tokens are read
        by the NEXT call, which first launches the following step when the batch cannot change."""
        use_knobs(self.knobs)
        produced = 0
        if self._pending is not None:
            p, self._pending = self._pending, None
            nxt = self._continue_decode(p)
            produced = self._finalize(p)
            if nxt is not None:
                self._pending = nxt
                self.stats["steps"] += 1
                return produced
            if not self.scheduler.has_work():
                return produced
        out = self.scheduler.schedule()
        if out.decode and out.prefill and self._mixed_ok():
            logits = self.mixed(out.prefill, out.decode)
            final = [c.seq for c in out.prefill if c.final]
            toks = self.sample(logits, final + list(out.decode))
            for c in out.prefill:
                self.scheduler.computed(c.seq, c.count)
                self.stats["prefix_hit_tokens"] = self.stats.get("prefix_hit_tokens", 0) + (
                    c.seq.cached_tokens if c.start == c.seq.cached_tokens else 0)
            for seq in out.decode:
                self.scheduler.computed(seq, 1)
            for seq, tok in zip(final + list(out.decode), toks):
                self._append(seq, tok)
                produced += 1
            self.stats["steps"] += 1
            return produced
        if out.decode and not out.prefill and "sample" not in self.__dict__:
            # sampling in the decode step (inside the graph); asynchronous: tokens read next call.
            # (an instance-level ``sample`` override -- teacher forcing, logit capture -- keeps
            # the host-sampling path below)
            pend = self._launch_decode(out.decode, self.decode_plan(out.decode), cont=False)
            self.stats["steps"] += 1
            if self._async_ok():
                self._pending = pend
                return produced
            return produced + self._finalize(pend)
        if out.decode:
            logits = self.decode(out.decode)
            for seq, tok in zip(out.decode, self.sample(logits, out.decode)):
                self.scheduler.computed(seq, 1)
                self._append(seq, tok)
                produced += 1
        if out.prefill:
            logits = self.prefill(out.prefill)
            final = [c.seq for c in out.prefill if c.final]
            for c in out.prefill:
                self.scheduler.computed(c.seq, c.count)
                self.stats["prefix_hit_tokens"] = self.stats.get("prefix_hit_tokens", 0) + (
                    c.seq.cached_tokens if c.start == c.seq.cached_tokens else 0)
            if final:
                for seq, tok in zip(final, self.sample(logits, final)):
                    self._append(seq, tok)
                    produced += 1
        self.stats["steps"] += 1
        return produced

    def generate(self, prompts: List[List[int]], params: SamplingParams) -> List[Sequence]:
        seqs = [self.add_request(p, params) for p in prompts]
        while any(s.status != "finished" for s in seqs):
            self.step()
        return seqs
