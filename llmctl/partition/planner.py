"""Parallelism planner: cost model + search over TP × PP × DP × ZeRO × SP × recompute × micro-batch.

Two planners share one interface:

``ReferenceCompatPlanner`` reproduces the reference ``ParallelismPlanner``
(``llmctl/cli/commands/plan.py:18-202``) formula-for-formula, including its known defects
(no SwiGLU third matrix / LM head / GQA in the parameter count, GB-vs-GB/s unit mix, ZeRO-1
as pure cost, no SP) so ``plan compute --compat-reference`` emits the reference's golden
plans (Llama-7B on 8×A100 -> TP=8, ZeRO-0, mb=1, gbs=4, 7.97 GB).

``ParallelismPlanner`` (default) is the MI355X model:

* exact parameter count from :class:`llmctl.models.ModelConfig` (GQA, SwiGLU, lm_head);
* training state 16 B/param (bf16 W + bf16 G + fp32 master + 2×fp32 Adam), sharded by
  TP (layers + vocab), PP (layers; embedding/head on the edge stages) and ZeRO 1/2/3 over DP;
* activation bytes per token per layer of llmctl's own kernels (flash attention: no S²
  term), reduced by selective/full recompute and by SP, times the 1F1B in-flight depth;
* step time = compute (model FLOPs / (peak × GEMM efficiency)) × pipeline bubble
  + exposed TP collectives + the non-overlapped tail of DP collectives, with collective
  costs from the ring model over the node's xGMI mesh (7 links × ~153 GB/s per MI355X,
  ``--intra-node-bw``) or the inter-node fabric when a group spans nodes;
* objective: maximise tokens/s subject to memory ≤ ``max_memory_gb`` (default 90 % of
  288 GB) — the plan records the per-GPU memory, comm volume and FLOPs estimates.
"""

from __future__ import annotations

import itertools
import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

GiB = 1024 ** 3

# MI355X constants (MI355X_MICROARCH.md): dense bf16 peak, HBM, xGMI
MI355X = {"peak_flops": 2.5e15, "hbm_gb": 288.0, "hbm_bw_gbps": 8000.0, "xgmi_links": 7, "xgmi_link_gbps": 153.0}


# ============================================================================ reference-compatible
class ReferenceCompatPlanner:
    """Exact port of the reference planner's arithmetic (for golden-value compatibility)."""

    def __init__(self, model_config: Dict[str, Any], hardware_profile: Dict[str, Any]):
        self.model = model_config
        self.hardware = hardware_profile

    def estimate_parameters(self) -> int:
        hidden = self.model.get("hidden", 4096)
        layers = self.model.get("layers", 32)
        vocab = self.model.get("vocab_size", 32000)
        ffn = self.model.get("ffn", hidden * 4)
        return vocab * hidden + layers * (4 * hidden * hidden + 2 * hidden * ffn + 4 * hidden)

    def estimate_model_memory(self) -> float:
        return self.estimate_parameters() * (2 + 2 + 8) / GiB

    def estimate_activation_memory(self, batch_size: int, seq_len: int) -> float:
        hidden = self.model.get("hidden", 4096)
        layers = self.model.get("layers", 32)
        per_layer = batch_size * seq_len * hidden * 2 / GiB
        attention = batch_size * seq_len * seq_len * 2 / GiB
        return layers * per_layer + layers * attention

    def compute_memory_requirement(self, tp, pp, zero_stage, micro_batch, seq_len=2048) -> float:
        m = self.estimate_model_memory()
        if tp > 1:
            m = m / tp
        if zero_stage >= 2:
            m *= 0.6
        if zero_stage >= 3:
            m *= 0.3
        a = self.estimate_activation_memory(micro_batch, seq_len)
        if pp > 1:
            a = a / pp
        return m + a

    def estimate_flops(self, batch_size, seq_len) -> float:
        return 2 * self.estimate_parameters() * batch_size * seq_len

    def estimate_communication_cost(self, tp, pp, zero_stage, global_batch, micro_batch) -> float:
        hidden = self.model.get("hidden", 4096)
        c = 0.0
        if tp > 1:
            c += global_batch * hidden * 2 / GiB
        if pp > 1:
            c += micro_batch * hidden * 2 / GiB
        if zero_stage >= 1:
            c += self.estimate_parameters() * 2 / GiB
        return c

    def search_optimal_plan(self, target_flops, max_memory, max_comm_bw) -> Dict[str, Any]:
        gpu_count = self.hardware.get("gpu", {}).get("count", 1)
        best, best_score = None, float("inf")
        for tp in [1, 2, 4, 8]:
            if tp > gpu_count:
                continue
            for pp in [1, 2, 4, 8]:
                if tp * pp > gpu_count:
                    continue
                for zs in [0, 1, 2, 3]:
                    for mb in [1, 2, 4, 8]:
                        mem = self.compute_memory_requirement(tp, pp, zs, mb)
                        if mem > max_memory:
                            continue
                        dp = gpu_count // (tp * pp)
                        gbs = mb * dp * 4
                        fl = self.estimate_flops(gbs, 2048)
                        if fl > target_flops:
                            continue
                        comm = self.estimate_communication_cost(tp, pp, zs, gbs, mb)
                        if comm > max_comm_bw:
                            continue
                        score = mem + comm * 10
                        if score < best_score:
                            best_score = score
                            best = dict(tensor_parallel=tp, pipeline_parallel=pp, data_parallel=dp, zero_stage=zs,
                                        micro_batch_size=mb, global_batch_size=gbs, estimated_memory_gb=mem,
                                        estimated_comm_gb=comm, estimated_flops=fl)
        if best is None:
            best = dict(tensor_parallel=1, pipeline_parallel=1, data_parallel=gpu_count, zero_stage=2,
                        micro_batch_size=1, global_batch_size=gpu_count,
                        estimated_memory_gb=self.estimate_model_memory(), estimated_comm_gb=0.1,
                        estimated_flops=self.estimate_flops(gpu_count, 2048))
        return best

    def manual_plan(self, tp, pp, zs) -> Dict[str, Any]:
        gpu_count = self.hardware.get("gpu", {}).get("count", 1)
        dp = gpu_count // (tp * pp)
        return dict(tensor_parallel=tp, pipeline_parallel=pp, data_parallel=dp, zero_stage=zs, micro_batch_size=1,
                    global_batch_size=dp * 4, estimated_memory_gb=self.compute_memory_requirement(tp, pp, zs, 1),
                    estimated_comm_gb=self.estimate_communication_cost(tp, pp, zs, dp * 4, 1),
                    estimated_flops=self.estimate_flops(dp * 4, 2048))


# ============================================================================ MI355X planner
@dataclass
class HardwareModel:
    gpus: int = 1
    gpus_per_node: int = 8
    hbm_gb: float = MI355X["hbm_gb"]
    peak_flops: float = MI355X["peak_flops"]
    intra_bw_gbps: float = MI355X["xgmi_links"] * MI355X["xgmi_link_gbps"]  # per-GPU aggregate
    inter_bw_gbps: float = 50.0
    hbm_bw_gbps: float = 8000.0
    # Per-op rates measured on MI355X (round 5 step kernel stats, GPT-7B mb 16 seq 2048, one GPU:
    # profiles/bench_r5_kernel_stats_default.txt; profiles/planner_calibration_r6.txt):
    #   projection GEMMs 1.51 PF at 32k tokens per GEMM (861 ms of GEMM kernels for 1.30 PFLOP),
    #   flash attention forward 721 TF, backward 543 TF (model FLOPs = 2.5x the forward's; the
    #   dK/dV + dQ kernels recompute S and dP), RMSNorm / SwiGLU / RoPE ~64 B per hidden element
    #   per token per layer at 6.3 TB/s, fused AdamW 28 B per parameter at 6.0 TB/s.
    gemm_efficiency: float = 0.604
    attn_fwd_efficiency: float = 0.288
    attn_bwd_efficiency: float = 0.217
    elementwise_bytes_per_hidden: float = 64.0
    hbm_efficiency: float = 0.79
    collective_efficiency: float = 0.6

    @classmethod
    def from_profile(cls, hw: Dict[str, Any]) -> "HardwareModel":
        g = hw.get("gpu", {}) or {}
        count = int(g.get("count", 0) or 0)
        devs = g.get("devices") or []
        mem = float(devs[0].get("memory_gb", 0)) if devs else 0.0
        lim = hw.get("limits", {}) or {}
        ic = hw.get("interconnect", {}) or {}
        per_gpu_flops = float(lim.get("estimated_flops", 0) or 0) / max(count, 1)
        m = cls(gpus=max(count, 1), gpus_per_node=max(int(ic.get("gpus_per_node", count) or count or 1), 1))
        if mem > 0:
            m.hbm_gb = mem
        if per_gpu_flops > 0:
            m.peak_flops = per_gpu_flops
        links = ic.get("xgmi_links")
        link_bw = ic.get("xgmi_link_bw_gbps")
        if links and link_bw:
            m.intra_bw_gbps = float(links) * float(link_bw)
        elif lim.get("intra_node_bw_gbps"):
            m.intra_bw_gbps = float(lim["intra_node_bw_gbps"])
        if lim.get("inter_node_bw_gbps"):
            m.inter_bw_gbps = float(lim["inter_node_bw_gbps"])
        return m


class ParallelismPlanner:
    """MI355X cost-model planner (see module docstring).  ``model_config`` is the model
    JSON dict; ``hardware_profile`` the ``hw probe`` dict."""

    def __init__(self, model_config: Dict[str, Any], hardware_profile: Dict[str, Any], seq_len: int = 2048,
                 hw: Optional[HardwareModel] = None):
        from llmctl.models.config import ModelConfig

        self.model_dict = model_config
        self.cfg = ModelConfig.from_dict(model_config)
        self.hardware = hardware_profile
        self.hw = hw or HardwareModel.from_profile(hardware_profile)
        self.seq_len = seq_len

    # ---------------------------------------------------------------- sizes
    def estimate_parameters(self) -> int:
        return self.cfg.num_parameters()

    def estimate_model_memory(self) -> float:
        """Full training state in GiB (16 B/param)."""
        return self.estimate_parameters() * 16 / GiB

    def _stage_params(self, tp: int, pp: int) -> float:
        c = self.cfg
        per_layer = c.num_parameters(include_embedding=False) - c.hidden  # minus final norm
        per_layer /= c.layers
        layers_first = math.ceil(c.layers / pp)
        emb = c.vocab_size * c.hidden
        edge = emb * (1 if c.tie_word_embeddings else 2) if pp == 1 else emb
        return (layers_first * per_layer + edge) / tp

    def activation_bytes_per_token_layer(self, tp: int, sp: bool, ac: str) -> float:
        c = self.cfg
        h, f = c.hidden, c.ffn
        q, kv = c.q_size, c.kv_size
        if ac == "full":
            return 2.0 * h / (tp if sp else 1)
        sharded = (q + 2 * kv + q) / tp + (2 * f + (0 if ac == "selective" else f)) / tp
        replicated = 4 * h  # layer input, normed x, residual, normed x2
        if sp and tp > 1:
            replicated /= tp
        return 2.0 * (sharded + replicated) + 8  # + lse/rstd

    def expert_parallel(self, dp: int) -> int:
        """MoE: shard experts over the largest group of DP ranks that divides the expert count
        and stays on one node (the per-layer token all-to-all rides the xGMI mesh); dense: 1."""
        c = self.cfg
        if not getattr(c, "is_moe", False):
            return 1
        return max(e for e in range(1, dp + 1)
                   if dp % e == 0 and c.num_experts % e == 0 and e <= self.hw.gpus_per_node)

    def _expert_params_stage(self, pp: int) -> float:
        c = self.cfg
        if not getattr(c, "is_moe", False):
            return 0.0
        return math.ceil(c.layers / pp) * c.num_experts * 3 * c.hidden * c.moe_ffn

    def compute_memory_requirement(self, tp: int, pp: int, dp: int, zero_stage: int, micro_batch: int,
                                   sp: bool = False, ac: str = "none", num_microbatches: int = 1) -> float:
        c = self.cfg
        P = self._stage_params(tp, pp)
        ep = self.expert_parallel(dp)
        P -= self._expert_params_stage(pp) * (1 - 1 / ep)  # each rank holds 1/ep of the experts
        w, g, opt = 2.0 * P, 2.0 * P, 12.0 * P
        if zero_stage >= 1:
            opt /= dp
        if zero_stage >= 2:
            g /= dp
        if zero_stage >= 3:
            w /= dp
            # two gathered layers in flight
            w += 2 * 2.0 * (c.num_parameters(include_embedding=False) / c.layers) / tp
        tokens = micro_batch * self.seq_len
        layers = math.ceil(c.layers / pp)
        inflight = min(pp, max(num_microbatches, 1)) if pp > 1 else 1
        act = self.activation_bytes_per_token_layer(tp, sp, ac) * tokens * layers * inflight
        if ac == "full":  # one layer's full activations during recompute
            act += self.activation_bytes_per_token_layer(tp, sp, "none") * tokens
        logits = tokens * c.vocab_size / tp * 2.0 * 2  # logits + in-place grad headroom
        workspace = 2.0 * GiB
        return (w + g + opt + act + logits + workspace) / GiB

    def estimate_flops(self, batch_size: int, seq_len: Optional[int] = None) -> float:
        s = seq_len or self.seq_len
        return self.cfg.flops_per_token(s) * batch_size * s

    # ---------------------------------------------------------------- time model
    def _link_bw(self, group_size: int, stride: int) -> float:
        """Effective per-GPU bandwidth (GB/s) for a collective whose group spans
        ``group_size`` ranks spaced ``stride`` apart."""
        span = group_size * stride
        if span <= self.hw.gpus_per_node:
            return self.hw.intra_bw_gbps * self.hw.collective_efficiency
        return self.hw.inter_bw_gbps * self.hw.collective_efficiency

    def _ring(self, nbytes: float, n: int, bw_gbps: float) -> float:
        if n <= 1:
            return 0.0
        return (n - 1) / n * nbytes / (bw_gbps * 1e9)

    def step_time(self, tp, pp, dp, zs, mb, sp, ac, accum, vs: int = 1) -> Dict[str, float]:
        """``vs``: virtual stages per pipeline rank (interleaved 1F1B): the pipeline bubble
        shrinks from (pp-1)/M to (pp-1)/(vs*M) of the compute, the stage-boundary p2p volume
        grows vs-fold."""
        c = self.cfg
        hw = self.hw
        tokens_per_rank = mb * self.seq_len * accum * pp  # pp: all micro-batches flow through every stage
        S = self.seq_len
        attn_fwd = 2 * 2 * c.layers * c.q_size * S / 2  # QK^T + PV per token, causal half
        lin = c.flops_per_token(S) - 3 * attn_fwd       # 6 x (projection + LM-head) parameters
        share = tokens_per_rank / (tp * pp)              # heads / features split over TP, layers over PP
        # GEMM rate grows with the token count per GEMM (M dimension); calibrated at 32k tokens
        T = mb * S / (tp if sp else 1)
        eff = hw.gemm_efficiency * min((T / (T + 2048.0)) / (32768.0 / 34816.0), 1.02)
        t_gemm = lin * share / (hw.peak_flops * eff)
        t_attn_f = attn_fwd * share / (hw.peak_flops * hw.attn_fwd_efficiency)
        t_attn_b = 2.5 * attn_fwd * share / (hw.peak_flops * hw.attn_bwd_efficiency)
        if ac == "full":
            t_gemm *= 4 / 3
            t_attn_f *= 2
        elif ac == "selective":  # the attention core and SwiGLU are recomputed in the backward
            t_attn_f *= 2
        elem_tokens = tokens_per_rank / ((tp if sp else 1) * pp)
        t_elem = (hw.elementwise_bytes_per_hidden * c.hidden * c.layers * elem_tokens
                  / (hw.hbm_bw_gbps * 1e9 * hw.hbm_efficiency))
        compute = t_gemm + t_attn_f + t_attn_b + t_elem
        M = accum * pp if pp > 1 else accum
        vs = max(int(vs), 1) if pp > 1 else 1
        compute_total = compute * (1 + (pp - 1) / (vs * M)) if pp > 1 else compute
        # TP collectives: 4 per layer (2 fwd + 2 bwd) of the activation size, exposed
        act_bytes = mb * self.seq_len * c.hidden * 2.0
        tp_bw = self._link_bw(tp, 1)
        tp_time = 0.0
        if tp > 1:
            per = 2 * self._ring(act_bytes, tp, tp_bw)  # all-reduce = RS + AG
            tp_time = 4 * per * math.ceil(c.layers / pp) * accum * (pp if pp > 1 else 1)
        # PP p2p
        pp_time = 0.0
        if pp > 1:
            pp_time = 2 * (vs * M + pp - 1) * act_bytes / tp / (self._link_bw(2, tp * dp) * 1e9)
        # DP gradient sync (overlapped with backward except the last bucket)
        grad_bytes = self._stage_params(tp, pp) * 2.0
        dp_bw = self._link_bw(dp, tp)
        dp_time = 2 * self._ring(grad_bytes, dp, dp_bw)
        if zs >= 3:
            dp_time *= 1.5  # params gathered in fwd and bwd
        # overlapped with the backward except the last bucket; the RCCL kernels share the CUs and
        # HBM with the backward's (uncalibrated: no multi-GPU node measured, 15 % of their time)
        exposed_dp = max(dp_time - 0.8 * compute, 0.1 * dp_time) + 0.15 * dp_time
        # MoE token all-to-all: dispatch + combine, forward and backward, per layer (exposed)
        ep_time = 0.0
        ep = self.expert_parallel(dp)
        if ep > 1:
            a2a = mb * self.seq_len * c.experts_per_token * c.hidden * 2.0 * (ep - 1) / ep
            ep_time = 4 * a2a / (self._link_bw(ep, tp) * 1e9) * math.ceil(c.layers / pp) * accum
        # fused AdamW: ~28 B of HBM traffic per parameter (bf16 grad + fp32 master/m/v read and
        # written + bf16 param), sharded over DP from ZeRO-1 on; the updated-parameter all-gather
        # of ZeRO-1/2 waits in the next forward's per-bucket hooks (mostly hidden)
        opt_time = 28.0 * self._stage_params(tp, pp) / (self.hw.hbm_bw_gbps * 1e9 * 0.75)
        if zs >= 1:
            opt_time /= dp
            if zs < 3:  # the updated-parameter all-gather: the next forward's first buckets wait on it
                exposed_dp += 0.25 * self._ring(grad_bytes, dp, dp_bw)
        total = compute_total + tp_time + pp_time + exposed_dp + ep_time + opt_time
        return dict(compute_s=compute_total, tp_s=tp_time, pp_s=pp_time, dp_s=dp_time, opt_s=opt_time, total_s=total,
                    comm_gb=(grad_bytes * 2 * (dp > 1) + (4 * act_bytes * c.layers if tp > 1 else 0)) / GiB)

    # ---------------------------------------------------------------- search
    def candidates(self, micro_batches=(1, 2, 4, 8, 16)) -> List[Dict[str, Any]]:
        c = self.cfg
        n = self.hw.gpus
        out = []
        for tp, pp in itertools.product([1, 2, 4, 8], [1, 2, 4, 8, 16]):
            if tp * pp > n or n % (tp * pp):
                continue
            if c.heads % tp or c.kv_heads % tp or c.ffn % tp or c.vocab_size % tp or tp > self.hw.gpus_per_node:
                continue
            if getattr(c, "is_moe", False) and (tp > 1 or pp > 1):
                continue  # MoE layers: expert parallelism inside DP (llmctl.models.moe)
            if pp > c.layers:
                continue
            dp = n // (tp * pp)
            for zs in (0, 1, 2, 3):
                if zs > 0 and dp == 1:
                    continue
                for sp in ((False, True) if tp > 1 else (False,)):
                    for ac in ("none", "selective", "full"):
                        for mb in micro_batches:
                            for vs in ((1, 2, 4) if pp > 1 and zs < 3 else (1,)):
                                if vs > 1 and c.layers < pp * vs:
                                    continue
                                out.append(dict(tp=tp, pp=pp, dp=dp, zs=zs, sp=sp, ac=ac, mb=mb, vs=vs))
        return out

    def evaluate(self, tp, pp, dp, zs, sp, ac, mb, global_batch: Optional[int] = None, vs: int = 1) -> Dict[str, Any]:
        if global_batch:
            accum = max(1, global_batch // (mb * dp * (pp if pp > 1 else 1)))
        else:
            accum = 1
        M = accum * pp if pp > 1 else accum
        mem = self.compute_memory_requirement(tp, pp, dp, zs, mb, sp, ac, M)
        t = self.step_time(tp, pp, dp, zs, mb, sp, ac, accum, vs)
        gbs = mb * dp * M
        tps = gbs * self.seq_len / t["total_s"]
        return dict(tensor_parallel=tp, pipeline_parallel=pp, data_parallel=dp, zero_stage=zs,
                    sequence_parallel=sp, activation_checkpoint=ac, micro_batch_size=mb,
                    expert_parallel=self.expert_parallel(dp),
                    global_batch_size=gbs, grad_accum=accum, num_microbatches=M,
                    virtual_stages=vs if pp > 1 else 1,
                    estimated_memory_gb=round(mem, 3), estimated_comm_gb=round(t["comm_gb"], 3),
                    estimated_flops=self.estimate_flops(gbs), estimated_step_time_s=float(f"{t['total_s']:.5g}"),
                    estimated_tokens_per_sec=round(tps, 1),
                    estimated_mfu=round(tps * self.cfg.flops_per_token(self.seq_len) /
                                        (self.hw.peak_flops * self.hw.gpus), 4))

    def search_optimal_plan(self, target_flops: Optional[float] = None, max_memory: Optional[float] = None,
                            max_comm_bw: Optional[float] = None, global_batch: Optional[int] = None,
                            fixed: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        max_mem = max_memory if max_memory else 0.9 * self.hw.hbm_gb
        mbs = (fixed["mb"],) if fixed and fixed.get("mb") else (1, 2, 4, 8, 16)
        feasible = []
        for cand in self.candidates(mbs):
            if fixed and any(fixed.get(k) is not None and cand[k] != fixed[k] for k in cand):
                continue
            plan = self.evaluate(global_batch=global_batch, **cand)
            if plan["estimated_memory_gb"] <= max_mem:
                feasible.append(plan)
        best = None
        if feasible:
            # throughput first; within 0.5 % of the best (the model's resolution) prefer the
            # simpler layout: lower ZeRO stage, less model parallelism, less recompute, less memory
            top = max(p["estimated_tokens_per_sec"] for p in feasible)
            acr = {"none": 0, "selective": 1, "full": 2}
            near = [p for p in feasible if p["estimated_tokens_per_sec"] >= 0.995 * top]
            best = min(near, key=lambda p: (p["zero_stage"], p["tensor_parallel"] * p["pipeline_parallel"],
                                            acr[p["activation_checkpoint"]], -p["estimated_tokens_per_sec"],
                                            p["estimated_memory_gb"]))
        if best is None:
            # nothing fits: most-sharded configuration, flagged by the memory estimate
            n = self.hw.gpus
            tp = max(t for t in (1, 2, 4, 8) if t <= min(n, self.hw.gpus_per_node) and n % t == 0
                     and self.cfg.heads % t == 0 and self.cfg.kv_heads % t == 0)  # every GPU used: tp | n
            best = self.evaluate(tp, 1, n // tp, 3 if n // tp > 1 else 0, tp > 1, "full", 1, global_batch)
        return best

    def manual_plan(self, tp: int, pp: int, zs: int, sp: bool = False, ac: str = "selective", mb: int = 1,
                    global_batch: Optional[int] = None, vs: int = 1) -> Dict[str, Any]:
        n = self.hw.gpus
        dp = max(n // (tp * pp), 1)
        return self.evaluate(tp, pp, dp, zs if dp > 1 else 0, sp and tp > 1, ac, mb, global_batch, vs)
