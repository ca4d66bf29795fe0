"""Rank workers for the parallel-equivalence tests (CPU / gloo, fp32).

Every parallel layout is checked against a single-process run that sees the same global
batch: the DP ranks' micro-batches become gradient-accumulation micro-steps of the
reference, TP/SP/PP/ZeRO must not change the math at all.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch


PACK_SEP = 7  # document separator of the packed-sequence layouts


def make_batch(vocab: int, seq: int, mb: int, step: int, dp_rank: int, micro: int = 0, pack: bool = False):
    g = torch.Generator()
    g.manual_seed(10007 * step + 101 * dp_rank + micro)
    t = torch.randint(0, vocab, (mb, seq + 1), generator=g)
    if pack:  # several documents per row
        t[:, 5::11] = PACK_SEP
    return t[:, :-1].contiguous(), t[:, 1:].contiguous()


def reference_state(model: str = "tiny", seed: int = 0) -> Dict[str, torch.Tensor]:
    from llmctl.models import build_model, get_model_config

    cfg = get_model_config(model)
    torch.manual_seed(seed)
    m = build_model(cfg, dtype=torch.float32)
    return {n: p.detach().clone() for n, p in m.named_parameters()}


def _config(**kw):
    from llmctl.runtime.engine import TrainingConfig

    base = dict(model_name_or_path="tiny", device="cpu", mixed_precision="fp32", learning_rate=1e-3,
                weight_decay=0.1, warmup_steps=0, scheduler="constant", gradient_clipping=1.0, seq_len=32,
                batch_size=2, log_level="error", bucket_mb=0.05, seed=0)
    base.update(kw)
    return TrainingConfig(**base)


def train_layout(rank: int, world: int, steps: int, layout: dict, model: str = "tiny",
                 micro_per_rank: int = 1, overrides: Optional[dict] = None) -> dict:
    """Run ``steps`` optimizer steps under ``layout`` (tp/pp/zero/sp/...) and return the
    gathered full state + losses (rank 0 meaningful).  ``overrides``: extra TrainingConfig
    fields (e.g. a larger Adam eps, so gradient elements that are zero in exact arithmetic —
    fp32 summation-order noise — do not become +-lr updates whose sign differs per layout)."""
    from llmctl.runtime.engine import TrainingEngine

    if layout.get("staging"):  # host-staging patches installed (CPU tensors pass through)
        from llmctl.comms import host_staging

        host_staging.install()
    cfg = _config(model_name_or_path=model, tensor_parallel=layout.get("tp", 1),
                  pipeline_parallel=layout.get("pp", 1), zero_stage=layout.get("zero", 0),
                  sequence_parallel=layout.get("sp", False),
                  activation_checkpoint=layout.get("ac", "none"),
                  num_microbatches=layout.get("microbatches", 0),
                  virtual_stages=layout.get("vstages", 1),
                  context_parallel=layout.get("cp", 1),
                  context_parallel_mode=layout.get("cp_mode", "ulysses"),
                  expert_parallel=layout.get("ep", 1),
                  pack_sequences=layout.get("pack", False), doc_separator=PACK_SEP, **(overrides or {}))
    eng = TrainingEngine(cfg)
    eng.load_full_state_dict(reference_state(model))
    vocab = eng.model_config.vocab_size
    losses = []
    dp_rank = eng.pg.dp_rank
    nmb = eng.pipeline.num_microbatches if eng.pipeline is not None else micro_per_rank
    for s in range(steps):
        batches = [make_batch(vocab, cfg.seq_len, cfg.batch_size, s, dp_rank, i, cfg.pack_sequences)
                   for i in range(nmb)]
        out = eng.train_step(batches)
        loss = out["loss"]
        if eng.pipeline is not None:
            losses.append(eng.pipeline.broadcast_loss(loss))
        else:
            # DP mean of the per-rank losses (CP ranks hold partial sums of one loss)
            lt = loss.detach().clone().reshape(1)
            if eng.pg.cp_group is not None:
                torch.distributed.all_reduce(lt, group=eng.pg.cp_group)
            if eng.pg.dp_group is not None:
                torch.distributed.all_reduce(lt, group=eng.pg.dp_group)
                lt /= eng.pg.layout.dp
            losses.append(float(lt))
    ev = eng.evaluate([make_batch(vocab, cfg.seq_len, cfg.batch_size, 99, 0)])
    full = eng.gather_full_state_dict()
    return {"losses": losses, "state": full if rank == 0 else None, "eval": ev,
            "peak_inflight": getattr(eng.pipeline, "peak_inflight_tensors", None)}


def train_reference(steps: int, dp: int, model: str = "tiny", micro_per_rank: int = 1,
                    pack: bool = False, overrides: Optional[dict] = None) -> dict:
    """Single process; the DP ranks' batches are accumulation micro-steps."""
    import os

    from llmctl.runtime.engine import TrainingEngine

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    cfg = _config(model_name_or_path=model, pack_sequences=pack, doc_separator=PACK_SEP, **(overrides or {}))
    eng = TrainingEngine(cfg)
    eng.load_full_state_dict(reference_state(model))
    vocab = eng.model_config.vocab_size
    losses = []
    for s in range(steps):
        batches = [make_batch(vocab, cfg.seq_len, cfg.batch_size, s, r, i, pack) for r in range(dp)
                   for i in range(micro_per_rank)]
        out = eng.train_step(batches)
        losses.append(float(out["loss"]))  # already the mean over all micro-batches
    ev = eng.evaluate([make_batch(vocab, cfg.seq_len, cfg.batch_size, 99, 0)])
    return {"losses": losses, "state": eng.gather_full_state_dict(), "eval": ev}


PROMPTS = [[1, 2, 3, 4, 5], [9] * 13, [7, 7], [3, 1, 4, 1, 5, 9, 2, 6]]


def serve_generate(rank: int, world: int, max_tokens: int = 8, model: str = "tiny") -> dict:
    """Greedy generation through the serving engine: TP=world (TPInferenceEngine) or, with
    world == 1, the single-process engine.  Rank 0 returns the produced token ids, plus the
    logits of a whole-prompt prefill called with ``Sequence`` objects (the engine's public
    ``prefill(seqs)`` form) for a row-level comparison across TP degrees."""
    import os

    import torch.distributed as dist

    from llmctl.serve.scheduler import SamplingParams

    kw = dict(device="cpu", max_batch_size=4, num_kv_blocks=48, block_size=8, max_model_len=256,
              max_batch_tokens=512, seed=0)
    if world == 1:
        from llmctl.serve.engine import InferenceEngine

        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        eng = InferenceEngine(model, **kw)
    else:
        from llmctl.serve.tp import TPInferenceEngine

        dist.init_process_group("gloo")
        eng = TPInferenceEngine(model, **kw)
        if eng.tp_rank != 0:
            eng.worker_loop()
            eng.close()
            return {}
    seqs = eng.generate(PROMPTS, SamplingParams(max_tokens=max_tokens, temperature=0.0))
    # Sequence-object prefill: two fresh prompts through the public entry point
    from llmctl.serve.scheduler import Sequence

    probe = [Sequence(prompt_ids=[11, 12, 13, 14, 15, 16], params=SamplingParams()),
             Sequence(prompt_ids=[2, 4, 6], params=SamplingParams())]
    for s in probe:
        assert eng.kv.add_sequence(s.seq_id, s.num_tokens)
    logits = eng.prefill(probe).float().cpu()
    for s in probe:
        eng.kv.free_sequence(s.seq_id)
    kv_heads_local = eng.kv_cache.k.shape[-2]
    if world > 1:
        eng.stop_workers()
        eng.close()
    return {"tokens": [s.output_ids for s in seqs], "kv_heads_local": kv_heads_local,
            "prefill_logits": logits}


def serve_tp_rccl_gpu(rank: int, world: int, max_tokens: int = 10) -> dict:
    """The TP serving engine on an RCCL process group (world 1: one GPU per rank is RCCL's
    rule) with decode hipGraphs: the vocab-parallel embedding's all-reduce and the logits gather
    run as RCCL collectives captured inside the graph.  Teardown is explicit (``close()`` then
    ``destroy_process_group``), never garbage collection; returns the TP and the plain
    engine's greedy tokens."""
    import torch.distributed as dist

    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import SamplingParams
    from llmctl.serve.tp import TPInferenceEngine

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    prompts = [[1, 2, 3, 4, 5], [9] * 37, [7, 7]]
    p = SamplingParams(max_tokens=max_tokens, temperature=0.0)
    kw = dict(device="cuda", max_batch_size=4, num_kv_blocks=128, block_size=16, max_model_len=512)
    tpe = TPInferenceEngine("tiny", use_graphs=True, **kw)
    a = [s.output_ids for s in tpe.generate(prompts, p)]
    replays = tpe.stats["graph_replays"]
    tpe.stop_workers()
    tpe.close()
    del tpe
    torch.cuda.synchronize()
    dist.destroy_process_group()
    b = [s.output_ids for s in InferenceEngine("tiny", use_graphs=False, **kw).generate(prompts, p)]
    return {"tp": a, "plain": b, "graph_replays": replays}


def custom_ar_check(rank: int, world: int, sizes=(8, 4096, 65536, 524288), iters: int = 20,
                    twoshot_bytes: int = 0) -> dict:
    """Two+ processes sharing one GPU: the IPC one-shot all-reduce must equal the sum of the
    inputs (exact fp32 sum, bf16 output) over many calls (epoch parity) and under hipGraph
    replay.  The process group is gloo (RCCL cannot put two ranks on one device)."""
    import torch
    import torch.distributed as dist

    from llmctl.comms.custom_ar import CustomAllReduce

    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    car = CustomAllReduce(max_bytes=2 << 20, device=torch.device("cuda", 0), twoshot_bytes=twoshot_bytes,
                          twoshot_min_bytes=64 << 10)
    worst = 0.0
    try:
        g = torch.Generator().manual_seed(1234 + rank)
        for n in sizes:
            for it in range(iters):
                x = (torch.randn(n, generator=g) * (1 + it)).to(torch.bfloat16)
                parts = [torch.empty_like(x) for _ in range(world)]
                dist.all_gather(parts, x)
                want = torch.stack([p.float() for p in parts]).sum(0)
                got = car.all_reduce(x.cuda()).float().cpu()
                err = ((got - want).abs() / (want.abs() + 1e-2)).max().item()
                worst = max(worst, err)
        # graph capture: one captured call, replayed with fresh inputs
        n = 16384
        static = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(static)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            car.all_reduce(static, out)
        torch.cuda.current_stream().wait_stream(s)
        dist.barrier()
        graph = torch.cuda.CUDAGraph()
        from llmctl.utils.env import graph_capture_gc_guard

        with graph_capture_gc_guard(), torch.cuda.graph(graph):
            car.all_reduce(static, out)
        dist.barrier()
        for it in range(5):
            x = (torch.randn(n, generator=g)).to(torch.bfloat16)
            parts = [torch.empty_like(x) for _ in range(world)]
            dist.all_gather(parts, x)
            want = torch.stack([p.float() for p in parts]).sum(0)
            static.copy_(x.cuda())
            torch.cuda.synchronize()
            dist.barrier()
            graph.replay()
            torch.cuda.synchronize()
            err = ((out.float().cpu() - want).abs() / (want.abs() + 1e-2)).max().item()
            worst = max(worst, err)
        car.check()
    finally:
        dist.barrier()
        car.close()
    return {"worst_rel_err": worst, "twoshot": car.twoshot_bytes > 0}


def _layout_config(layout: dict, model: str = "tiny"):
    return _config(model_name_or_path=model, tensor_parallel=layout.get("tp", 1),
                   pipeline_parallel=layout.get("pp", 1), zero_stage=layout.get("zero", 0),
                   sequence_parallel=layout.get("sp", False), num_microbatches=layout.get("microbatches", 0),
                   async_checkpoint=False)


def ckpt_save_phase(rank: int, world: int, layout: dict, steps: int, out_dir: str, model: str = "tiny") -> dict:
    """Train ``steps`` steps under ``layout`` from the reference init, then checkpoint."""
    from llmctl.io.checkpoint import CheckpointManager
    from llmctl.runtime.engine import TrainingEngine

    eng = TrainingEngine(_layout_config(layout, model))
    eng.load_full_state_dict(reference_state(model))
    vocab, cfg = eng.model_config.vocab_size, eng.config
    for s in range(steps):
        eng.train_step([make_batch(vocab, cfg.seq_len, cfg.batch_size, s, eng.pg.dp_rank, 0)])
    ck = CheckpointManager(eng, out_dir)
    ck.save("ckpt", final=True)
    ck.wait()
    return {}


def ckpt_resume_phase(rank: int, world: int, layout: dict, start: int, steps: int, out_dir: str,
                      model: str = "tiny") -> dict:
    """Resume the checkpoint under a (possibly different) ``layout`` and train more steps."""
    from llmctl.io.checkpoint import CheckpointManager
    from llmctl.runtime.engine import TrainingEngine

    eng = TrainingEngine(_layout_config(layout, model))
    CheckpointManager(eng, out_dir).load(out_dir + "/ckpt")
    vocab, cfg = eng.model_config.vocab_size, eng.config
    assert eng.global_step == start and eng.optimizer.step_count == start
    for s in range(start, start + steps):
        eng.train_step([make_batch(vocab, cfg.seq_len, cfg.batch_size, s, eng.pg.dp_rank, 0)])
    full = eng.gather_full_state_dict()
    return {"state": full if rank == 0 else None}


def train_reference_schedule(schedule, model: str = "tiny") -> dict:
    """Single process; ``schedule[s]`` = number of DP ranks whose micro-batches form step s."""
    import os

    from llmctl.runtime.engine import TrainingEngine

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    eng = TrainingEngine(_config(model_name_or_path=model))
    eng.load_full_state_dict(reference_state(model))
    vocab, cfg = eng.model_config.vocab_size, eng.config
    for s, dp in enumerate(schedule):
        eng.train_step([make_batch(vocab, cfg.seq_len, cfg.batch_size, s, r, 0) for r in range(dp)])
    return {"state": eng.gather_full_state_dict()}


def pp_tied_fresh(rank: int, world: int, steps: int = 2) -> dict:
    """PP=world tied-embedding model from its OWN init (no load_full_state_dict): return the
    first stage's ``embed`` and the last stage's ``lm_head`` after ``steps`` updates."""
    from llmctl.runtime.engine import TrainingEngine

    eng = TrainingEngine(_config(model_name_or_path="tiny-tied", pipeline_parallel=world, num_microbatches=2))
    vocab, cfg = eng.model_config.vocab_size, eng.config
    for s in range(steps):
        eng.train_step([make_batch(vocab, cfg.seq_len, cfg.batch_size, s, 0, i) for i in range(2)])
    m = eng.model
    t = m.embed if eng.pipeline.is_first else (m.lm_head if eng.pipeline.is_last else None)
    return {"tied": t.detach().clone() if t is not None else None}


def zero3_pp_tied_error(rank: int, world: int) -> dict:
    """ZeRO-3 x PP x tied embeddings must be refused, not silently untied."""
    from llmctl.runtime.engine import TrainingEngine

    try:
        TrainingEngine(_config(model_name_or_path="tiny-tied", pipeline_parallel=2, zero_stage=3))
    except NotImplementedError as e:
        return {"error": str(e)}
    return {"error": ""}


def ring_attention_check(rank: int, world: int, zigzag: bool = False, B: int = 2, S: int = 48, Hq: int = 4,
                         Hkv: int = 2, D: int = 16) -> dict:
    """Ring attention over a ``world``-rank CP group vs full causal attention (fp32, gloo):
    returns this rank's output / gradient chunks and the oracle's."""
    import torch.distributed as dist

    from llmctl.ops import ref
    from llmctl.parallel.context_parallel import ring_attention, split_sequence

    dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, S, Hq, D, generator=g)
    k = torch.randn(B, S, Hkv, D, generator=g)
    v = torch.randn(B, S, Hkv, D, generator=g)
    do = torch.randn(B, S, Hq, D, generator=g)
    scale = D ** -0.5
    o_full, lse = ref.attention_fwd(q, k, v, scale, True)
    dq_full, dk_full, dv_full = ref.attention_bwd(do, q, k, v, o_full, lse, scale, True)
    ch = lambda t: split_sequence(t, world, rank, zigzag)  # noqa: E731
    ql, kl, vl = (ch(t).requires_grad_(True) for t in (q, k, v))
    o = ring_attention(ql, kl, vl, None if world == 1 else dist.group.WORLD, scale, zigzag=zigzag)
    o.backward(ch(do))
    return {"o": o.detach(), "dq": ql.grad, "dk": kl.grad, "dv": vl.grad,
            "o_ref": ch(o_full), "dq_ref": ch(dq_full), "dk_ref": ch(dk_full), "dv_ref": ch(dv_full)}


def async_tp_check(rank: int, world: int, T: int = 24, K: int = 16, N: int = 12) -> dict:
    """Async-TP linears over a ``world``-rank TP group vs the unsharded fp32 products (gloo):
    column-parallel (AG-GEMM fwd, GEMM-RS dgrad) then row-parallel (GEMM-RS fwd, AG-GEMM dgrad)
    — the MLP pattern, ``y = RS(gelu(AG(x) W1_r^T + b_r) W2_r^T)``."""
    import torch.distributed as dist
    import torch.nn.functional as F

    from llmctl.parallel.async_tp import column_parallel_sp, row_parallel_sp

    dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(11)
    x = torch.randn(T, K, generator=g)
    w1 = torch.randn(N * world, K, generator=g) / K ** 0.5
    b1 = torch.randn(N * world, generator=g)
    w2 = torch.randn(K, N * world, generator=g) / N ** 0.5
    dy = torch.randn(T, K, generator=g)
    xr, w1r, b1r, w2r = (t.clone().requires_grad_(True) for t in (x, w1, b1, w2))
    yr = F.linear(F.gelu(F.linear(xr, w1r, b1r)), w2r)
    yr.backward(dy)
    tl = T // world
    rows = slice(rank * tl, (rank + 1) * tl)
    cols = slice(rank * N, (rank + 1) * N)
    xl = x[rows].clone().requires_grad_(True)
    w1l = w1[cols].clone().requires_grad_(True)
    b1l = b1[cols].clone().requires_grad_(True)
    w2l = w2[:, cols].clone().requires_grad_(True)
    grp = dist.group.WORLD
    y = row_parallel_sp(F.gelu(column_parallel_sp(xl, w1l, b1l, grp)), w2l, grp)
    y.backward(dy[rows])
    return {"y": y.detach(), "dx": xl.grad, "dw1": w1l.grad, "db1": b1l.grad, "dw2": w2l.grad,
            "y_ref": yr.detach()[rows], "dx_ref": xr.grad[rows], "dw1_ref": w1r.grad[cols],
            "db1_ref": b1r.grad[cols], "dw2_ref": w2r.grad[:, cols]}


def train_layout_gpu(rank: int, world: int, steps: int, layout: dict, model: str = "tiny",
                     micro_per_rank: int = 4, ref_dp: int = 1) -> dict:
    """``train_layout`` on the GPU kernel path (bf16, HIP kernels) with every rank on cuda:0:
    world > 1 runs over gloo with host-staged collectives (``llmctl.comms.host_staging`` — RCCL
    cannot put two ranks on one device), world == 1 is the single-process reference (the
    micro-batches are accumulation steps)."""
    import os

    from llmctl.ops import _lib
    from llmctl.runtime.engine import TrainingEngine

    if world == 1:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
    torch.cuda.set_device(0)
    cfg = _config(model_name_or_path=model, device="cuda:0", mixed_precision="bf16", seq_len=128, batch_size=2,
                  distributed_backend="gloo", tensor_parallel=layout.get("tp", 1),
                  pipeline_parallel=layout.get("pp", 1), zero_stage=layout.get("zero", 0),
                  sequence_parallel=layout.get("sp", False), num_microbatches=layout.get("microbatches", 0),
                  virtual_stages=layout.get("vstages", 1), context_parallel=layout.get("cp", 1),
                  context_parallel_mode=layout.get("cp_mode", "ulysses"))
    eng = TrainingEngine(cfg)
    eng.load_full_state_dict(reference_state(model))
    vocab = eng.model_config.vocab_size
    nmb = eng.pipeline.num_microbatches if eng.pipeline is not None else micro_per_rank
    dev = torch.device("cuda", 0)
    losses = []
    # world == 1 with ref_dp > 1: the single process accumulates every DP rank's micro-batches
    dps = [eng.pg.dp_rank] if world > 1 else list(range(ref_dp))
    for s in range(steps):
        batches = [tuple(t.to(dev) for t in make_batch(vocab, cfg.seq_len, cfg.batch_size, s, d, i))
                   for d in dps for i in range(nmb)]
        loss = eng.train_step(batches)["loss"]
        losses.append(eng.pipeline.broadcast_loss(loss) if eng.pipeline is not None else float(loss))
    ev = eng.evaluate([tuple(t.to(dev) for t in make_batch(vocab, cfg.seq_len, cfg.batch_size, 99, 0))])
    torch.cuda.synchronize()
    return {"losses": losses, "eval": ev, "native": bool(_lib.load()), "backend": eng.backend,
            "zero3": getattr(eng, "zero3", None) is not None, "pp": eng.pg.layout.pp, "dp": eng.pg.layout.dp,
            "max_mem_gb": torch.cuda.max_memory_allocated() / 2**30}


def train_drift(rank: int, world: int, steps: int, main_grads: str, precision: str = "bf16") -> dict:
    """DP=world x grad-accumulation 4 on the tiny model for ``steps`` steps with the given
    parameter precision and gradient-accumulation dtype; returns the per-step mean losses and
    the final parameters (fp32) on rank 0 — the fp32-main-gradient drift study."""
    from llmctl.runtime.engine import TrainingEngine

    cfg = _config(model_name_or_path="tiny", mixed_precision=precision, main_grads=main_grads,
                  gradient_accumulation_steps=4, learning_rate=3e-3, scheduler="constant")
    eng = TrainingEngine(cfg)
    eng.load_full_state_dict(reference_state("tiny"))
    losses = []
    for s in range(steps):
        out = eng.train_step([make_batch(512, cfg.seq_len, cfg.batch_size, s, eng.pg.dp_rank, i) for i in range(4)])
        lt = out["loss"].detach().float().reshape(1).clone()
        if eng.pg.dp_group is not None:
            torch.distributed.all_reduce(lt, group=eng.pg.dp_group)
            lt /= eng.pg.layout.dp
        losses.append(float(lt))
    state = {n: p.detach().float().clone() for n, p in eng.model.named_parameters()}
    return {"losses": losses, "state": state if rank == 0 else None,
            "grad_dtype": str(eng.grad_dtype), "flat_grad_dtype": str(eng.flat.grad.dtype)}


def serve_forced_gpu(rank: int, world: int, max_tokens: int = 8, model: str = "tiny", forced=None,
                     env: Optional[dict] = None, engine_kw: Optional[dict] = None) -> dict:
    """GPU serving (TP = world ranks sharing cuda:0 over gloo + the custom IPC all-reduce, decode
    steps in hipGraphs) with every sampled token replaced by ``forced[seq][step]`` (teacher
    forcing; None: greedy) and the full-vocabulary logits of every step recorded on rank 0 — so
    two configurations can be compared row by row over the same token stream.  ``env`` (e.g.
    ``{"LLMCTL_KNOBS": "decode_fused=0"}``) is set for the call and restored afterwards."""
    import os

    saved = {k: os.environ.get(k) for k in (env or {})}  # world 1 runs in the caller's process
    os.environ.update(env or {})
    try:
        return _serve_forced_gpu(rank, world, max_tokens, model, forced, engine_kw)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _serve_forced_gpu(rank, world, max_tokens, model, forced, engine_kw) -> dict:
    import os

    import torch.distributed as dist

    from llmctl.serve.scheduler import SamplingParams

    torch.cuda.set_device(0)
    kw = dict(device="cuda", max_batch_size=4, num_kv_blocks=64, block_size=16, max_model_len=256,
              max_batch_tokens=512, seed=0, use_graphs=True)
    kw.update(engine_kw or {})
    prompts = PROMPTS + [[(5 * i) % 500 + 1 for i in range(40)]]
    if world == 1:
        from llmctl.serve.engine import InferenceEngine

        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        eng = InferenceEngine(model, **kw)
    else:
        from llmctl.serve.tp import TPInferenceEngine

        dist.init_process_group("gloo")
        eng = TPInferenceEngine(model, **kw)
        assert eng.car is not None, "custom all-reduce not active"
        if eng.tp_rank != 0:
            eng.worker_loop()
            eng.close()
            return {}
    seqs = [eng.add_request(p, SamplingParams(max_tokens=max_tokens, temperature=0.0)) for p in prompts]
    idx = {s.seq_id: i for i, s in enumerate(seqs)}
    rec: Dict[int, List[torch.Tensor]] = {}
    greedy = eng.sample

    def sample(logits, batch):
        toks = greedy(logits, batch)
        out = []
        for row, s, t in zip(logits.float().cpu(), batch, toks):
            i = idx[s.seq_id]
            rec.setdefault(i, []).append(row)
            out.append(forced[i][len(s.output_ids)] if forced is not None else t)
        return out

    eng.sample = sample
    progress = os.environ.get("LLMCTL_TEST_PROGRESS")  # heartbeat lines for long multi-rank GPU runs
    n = 0
    while any(s.status != "finished" for s in seqs):
        eng.step()
        n += 1
        if progress and n % 4 == 0:
            print(f"[serve_forced_gpu rank {rank}/{world}] step {n}", flush=True)
    res = {"tokens": [s.output_ids for s in seqs], "graph_replays": eng.stats["graph_replays"],
           "fused_decode": bool(eng._fused_decode()), "mixed_steps": eng.stats.get("mixed_steps", 0),
           "logits": torch.stack([torch.stack(rec[i]) for i in range(len(seqs))])}
    if world > 1:
        eng.stop_workers()
        eng.close()
    return res


def control_channel_worker(rank, world, kind, slot_bytes=8 << 20):
    """TP plan channel (llmctl.serve.control): rank 0 publishes a stream of decode / prefill /
    mixed (nested) plans -- more than the ring has slots, and with a small ``slot_bytes`` some
    spill to the gloo fallback -- and every rank returns a digest of what it holds."""
    import numpy as np
    import torch.distributed as dist

    from llmctl.serve.control import ShmChannel, TensorChannel

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ch = ShmChannel(None, slot_bytes=slot_bytes) if kind == "shm" else TensorChannel(None)
    rng = np.random.default_rng(1)
    digests = []
    for it in range(11):
        n = 1 + it
        dec = {"op": "decode", "ids": rng.integers(0, 1000, n).tolist(), "positions": list(range(n)),
               "slots": rng.integers(0, 1 << 20, n).tolist(), "ctx": [7] * n,
               "bt": rng.integers(0, 99, (n, 5)).astype(np.int32)}
        T = 64 * (it + 1)
        pre = {"op": "prefill", "ids": rng.integers(0, 1000, T), "pos": np.arange(T, dtype=np.int32),
               "cu": [0, T], "doc": None if it % 2 else np.zeros(T, dtype=np.int32), "last": [T - 1], "x": 1.5,
               "flag": True}
        plan = [dec, pre, {"op": "mixed", "prefill": pre, "decode": dec}][it % 3]
        got = (ch.publish(plan), plan)[1] if rank == 0 else ch.receive()
        d = got["decode"] if got["op"] == "mixed" else got
        digests.append(torch.tensor([len(d["ids"]), int(np.asarray(d["ids"]).sum()),
                                     int(np.asarray(d.get("bt", d.get("pos"))).sum())], dtype=torch.int64))
        if got["op"] != "decode":
            p = got["prefill"] if got["op"] == "mixed" else got
            assert p["x"] == 1.5 and p["flag"] is True and (p["doc"] is None) == bool(it % 2)
    ch.close()
    return {"digest": torch.stack(digests), "spilled": torch.tensor(getattr(ch, "stats", {}).get("spilled", 0))}


def serve_sampled(rank: int, world: int, async_decode: bool = True, temperature: float = 0.9,
                  max_tokens: int = 8) -> dict:
    """Seeded sampled generation (temperature > 0, top-k / top-p) through the serving engine at
    TP = world (gloo) or world 1; rank 0 returns the tokens, how many decode steps ran pipelined
    (step N + 1 launched from step N's device-side ids) and the engine's host-RNG draw count (one
    uniform per sampled row, whatever the TP degree or pipelining)."""
    import os

    import torch.distributed as dist

    from llmctl.serve.scheduler import SamplingParams

    kw = dict(device="cpu", max_batch_size=4, num_kv_blocks=48, block_size=8, max_model_len=256,
              max_batch_tokens=512, seed=3, perf_knobs={"async_decode": async_decode}, prefix_caching=False)
    if world == 1:
        from llmctl.serve.engine import InferenceEngine

        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        eng = InferenceEngine("tiny", **kw)
    else:
        from llmctl.serve.tp import TPInferenceEngine

        dist.init_process_group("gloo")
        eng = TPInferenceEngine("tiny", **kw)
        if eng.tp_rank != 0:
            eng.worker_loop()
            eng.close()
            return {}
    p = SamplingParams(max_tokens=max_tokens, temperature=temperature, top_k=40, top_p=0.95, ignore_eos=True)
    seqs = eng.generate(PROMPTS, p)
    res = {"tokens": [s.output_ids for s in seqs], "continued": eng.stats.get("async_continued", 0),
           "rng_next": float(eng._np_rng.random())}
    if world > 1:
        eng.stop_workers()
        eng.close()
    return res


def serve_async_gpu(rank: int, world: int, model: str = "tiny", env=None, engine_kw=None, prompts=None,
                    max_tokens: int = 16) -> dict:
    """TP = world serving on cuda:0 (world processes sharing the GPU: gloo default group, custom
    IPC all-reduces, decode hipGraphs with in-graph sampling), greedy, with the pipelined decode
    loop on and then off on the same engine.  Rank 0 returns both runs' tokens, the pipelined
    steps, and per decode step of the pipelined run: host wall ms (``step()`` loop) and device ms
    (CUDA events around each decode launch on rank 0's stream; with the pipeline full the next
    launch's start event fires when the previous replay ends, so the sum is the busy time)."""
    import dataclasses
    import os
    import time

    import torch.distributed as dist

    from llmctl.serve.scheduler import SamplingParams

    os.environ.update(env or {})
    torch.cuda.set_device(0)
    kw = dict(device="cuda", max_batch_size=4, num_kv_blocks=64, block_size=16, max_model_len=256,
              max_batch_tokens=512, seed=0, use_graphs=True, prefix_caching=False)
    kw.update(engine_kw or {})
    prompts = prompts or PROMPTS
    if world == 1:
        from llmctl.serve.engine import InferenceEngine

        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        eng = InferenceEngine(model, **kw)
    else:
        from llmctl.serve.tp import TPInferenceEngine

        dist.init_process_group("gloo")
        eng = TPInferenceEngine(model, **kw)
        if eng.tp_rank != 0:
            eng.worker_loop()
            eng.close()
            return {}
    p = SamplingParams(max_tokens=max_tokens, temperature=0.0, ignore_eos=True)
    base = eng.knobs
    res = {}
    inner = eng._decode_sample_exec
    evs = []

    def timed(plan):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = inner(plan)
        b.record()
        evs.append((a, b))
        return out

    for mode in (True, False):
        eng.knobs = dataclasses.replace(base, async_decode=mode)
        c0 = eng.stats.get("async_continued", 0)
        seqs = [eng.add_request(list(pr), p) for pr in prompts]
        while any(s.first_token_time is None for s in seqs):  # prefills (+ first tokens)
            eng.step()
        torch.cuda.synchronize()
        start = [len(s.output_ids) for s in seqs]
        evs.clear()
        eng._decode_sample_exec = timed
        t0 = time.perf_counter()
        while any(s.status != "finished" for s in seqs):
            eng.step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        eng._decode_sample_exec = inner
        steps = max(len(s.output_ids) - s0 for s, s0 in zip(seqs, start))
        gpu = sum(a.elapsed_time(b) for a, b in evs)
        res[f"tokens_{int(mode)}"] = [s.output_ids for s in seqs]
        res[f"continued_{int(mode)}"] = eng.stats.get("async_continued", 0) - c0
        res[f"host_ms_{int(mode)}"] = wall / max(steps, 1)
        res[f"gpu_ms_{int(mode)}"] = gpu / max(len(evs), 1)
    res["graph_replays"] = eng.stats["graph_replays"]
    if world > 1:
        eng.stop_workers()
        eng.close()
    else:
        eng.release_graphs()
    return res
