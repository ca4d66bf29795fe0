"""CPU unit tests: launchers (argv/env, no exec), LR schedules, native data loader, quantizers,
plugin registry, health thresholds, autotuner, TP shard/consolidate round-trip."""

import json
import sys

import numpy as np
import pytest
import torch

from llmctl.runtime.launcher import LaunchConfig, create_launcher


# ---------------------------------------------------------------- launchers
def test_local_launcher_argv_env():
    c = LaunchConfig(nodes=1, gpus_per_node=8, master_port=29611, deterministic=True, seed=7)
    L = create_launcher(c)
    cmd = L.build_command("llmctl.runtime.worker", ["--max-steps", "2"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc_per_node=8" in cmd and "--master_addr=127.0.0.1" in cmd and "--master_port=29611" in cmd
    assert cmd[-4:] == ["-m", "llmctl.runtime.worker", "--max-steps", "2"]
    env = L.get_environment()
    assert env["WORLD_SIZE"] == "8" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert env["PYTHONHASHSEED"] == "7" and env["LLMCTL_DETERMINISTIC"] == "1"


def test_slurm_mpi_k8s_launchers():
    c = LaunchConfig(nodes=2, gpus_per_node=8, launcher="slurm")
    s = create_launcher(c).create_slurm_script("llmctl.runtime.worker", ["--seed", "1"])
    assert "#SBATCH --nodes=2" in s and "#SBATCH --ntasks-per-node=8" in s and "-m llmctl.runtime.worker" in s
    m = create_launcher(LaunchConfig(nodes=2, gpus_per_node=8, launcher="mpi")).build_command("train.py", [])
    assert m[:3] == ["mpirun", "-np", "16"]
    k = create_launcher(LaunchConfig(nodes=4, gpus_per_node=8, launcher="k8s")).render_manifest("x.py", ["--a"])
    assert "completions: 4" in k and "amd.com/gpu: 8" in k


# ---------------------------------------------------------------- LR schedules
def test_lr_schedules():
    from llmctl.runtime.optimizer import LRSchedule

    lin = LRSchedule(1.0, "linear", warmup_steps=10, total_steps=110)
    assert lin(5) == pytest.approx(0.5) and lin(10) == pytest.approx(1.0) and lin(110) == pytest.approx(0.0)
    cos = LRSchedule(1.0, "cosine", warmup_steps=0, total_steps=100, min_lr_ratio=0.1)
    assert cos(0) == pytest.approx(1.0) and cos(100) == pytest.approx(0.1) and cos(50) == pytest.approx(0.55)
    assert LRSchedule(3e-4, "constant")(1000) == 3e-4


def test_lr_schedule_matches_hf_linear():
    """0-based step index, as HF get_linear_schedule_with_warmup (the reference's scheduler,
    llmctl/runtime/engine.py:246-253): no warmup -> step 0 runs at the base LR; the last of
    ``total`` steps runs at base/(total-warmup) > 0; warmup ramps step/warmup."""
    from llmctl.runtime.optimizer import LRSchedule

    def hf(step, warmup, total):  # transformers.optimization._get_linear_schedule_with_warmup_lr_lambda
        if step < warmup:
            return step / max(1, warmup)
        return max(0.0, (total - step) / max(1, total - warmup))

    for warmup, total in ((0, 5), (3, 12), (10, 110)):
        s = LRSchedule(1.0, "linear", warmup_steps=warmup, total_steps=total)
        for step in range(total):
            assert s(step) == pytest.approx(hf(step, warmup, total)), (warmup, total, step)
        assert s(total - 1) > 0
    assert LRSchedule(2.0, "linear", warmup_steps=0, total_steps=4)(0) == 2.0


def test_engine_lr_first_and_last_step():
    """The engine applies scheduler(i) on its i-th (0-based) step: a 4-step linear run with
    warmup 0 uses the base LR first and a positive LR last."""
    import torch

    from llmctl.models import get_model_config
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine

    cfg = TrainingConfig(model_name_or_path="tiny", batch_size=2, seq_len=16, device="cpu", log_level="warning",
                         learning_rate=1e-3, max_steps=4, warmup_steps=0, scheduler="linear")
    eng = TrainingEngine(cfg, get_model_config("tiny"))
    ids = torch.randint(0, eng.model_config.vocab_size, (2, 17))
    lrs = [float(eng.train_step([(ids[:, :-1], ids[:, 1:])])["lr"]) for _ in range(4)]
    eng.shutdown()
    assert lrs[0] == pytest.approx(1e-3) and lrs[-1] == pytest.approx(2.5e-4), lrs


# ---------------------------------------------------------------- data loader
@pytest.fixture()
def token_file(tmp_path):
    arr = np.arange(64 * 33 + 1, dtype=np.uint16) % 50000
    p = tmp_path / "tok.bin"
    arr.tofile(p)
    return p


def test_memmap_tokens_dp_partition_and_resume(token_file):
    from llmctl.io.dataset import MemmapTokens

    S, B = 32, 4
    seen = []
    for r in range(2):
        ds = MemmapTokens(str(token_file), S, B, dp_rank=r, dp_size=2, seed=3)
        starts = set()
        for _ in range(8):  # 8 batches x 4 = 32 samples = one epoch per rank
            x, y = ds.next_batch()
            assert x.shape == (B, S) and torch.equal(x[:, 1:], y[:, :-1])
            starts.update(int(v) // S for v in x[:, 0])
        seen.append(starts)
    assert not (seen[0] & seen[1]), "DP ranks must read disjoint samples"
    assert len(seen[0] | seen[1]) == 64
    a = MemmapTokens(str(token_file), S, B, seed=3)
    for _ in range(3):
        a.next_batch()
    st = a.state_dict()
    want = a.next_batch()[0]
    b = MemmapTokens(str(token_file), S, B, seed=3)
    b.load_state_dict(st)
    assert torch.equal(b.next_batch()[0], want)


# ---------------------------------------------------------------- quantizers + registry
@pytest.mark.parametrize("name,tol", [("int8", 0.01), ("int4", 0.15), ("fp8", 0.07)])
def test_quantizers_roundtrip(name, tol):
    from llmctl.plugins.quantizers import QUANTIZERS, dequantize

    torch.manual_seed(0)
    w = torch.randn(64, 129)
    q = QUANTIZERS[name](w)
    back = dequantize(name, q, tuple(w.shape))
    rel = (back - w).norm() / w.norm()
    assert rel < tol, rel


def test_plugin_registry():
    from llmctl.plugins.registry import registry

    assert {"int8", "int4", "fp8", "int8-awq", "int4-gptq"} <= set(registry.names("quantizers"))
    assert {"safetensors", "hf"} <= set(registry.names("exporters"))
    assert "flash_attention_v3" in registry.names("kernels")
    sched = registry.get("schedulers", "lr-cosine")(1.0, total_steps=10)
    assert sched(10) == pytest.approx(0.1)
    with pytest.raises(KeyError):
        registry.get("exporters", "nope")


# ---------------------------------------------------------------- health
def test_training_health_thresholds():
    from llmctl.metrics.health import HealthStatus, TrainingHealthMonitor

    m = TrainingHealthMonitor()
    m.update_training_metrics(loss=2.0, grad_norm=1.0, throughput=1000.0)
    assert m.get_health_report().status == HealthStatus.HEALTHY
    m.update_training_metrics(loss=float("nan"), grad_norm=1.0, throughput=1000.0)
    assert m.get_health_report().status != HealthStatus.HEALTHY


# ---------------------------------------------------------------- autotuner
def test_autotuner_cpu_cache(tmp_path):
    from llmctl.plugins.autotuning import TuningConfig, create_auto_tuner

    t = create_auto_tuner(TuningConfig(max_iterations=4, warmup_iterations=1, measurement_iterations=2, timeout=30))
    r = t.tune_matmul((64, 64, 64), device="cpu")
    assert r.best_config and r.best_performance > 0
    f = tmp_path / "cache.json"
    t.save_results(str(f))
    t2 = create_auto_tuner()
    t2.load_results(str(f))
    assert json.loads(f.read_text())


# ---------------------------------------------------------------- TP shard/consolidate (checkpoint reshard)
@pytest.mark.parametrize("tp", [2, 4])
def test_tp_shard_consolidate_roundtrip(tp):
    from llmctl.io.checkpoint import consolidate_tp, shard_tp
    from llmctl.models import build_model, get_model_config

    cfg = get_model_config("tiny")
    m = build_model(cfg, dtype=torch.float32)
    for n, p in m.named_parameters():
        shards = [shard_tp(n, p.detach(), tp, r, cfg) for r in range(tp)]
        back = consolidate_tp(n, shards, cfg)
        assert torch.equal(back, p.detach()), n


# ---------------------------------------------------------------- packed sequences
def test_document_starts_and_mask():
    from llmctl.ops import ref

    ids = torch.tensor([[5, 6, 0, 7, 0, 0, 8, 9]])
    ds = ref.document_starts(ids, 0)
    assert ds.tolist() == [[0, 0, 0, 3, 3, 5, 6, 6]]
    q = torch.randn(1, 8, 2, 16)
    o, _ = ref.attention_fwd(q, q, q, 0.25, True, doc_start=ds)
    o2, _ = ref.attention_fwd(q[:, 3:5], q[:, 3:5], q[:, 3:5], 0.25, True)
    assert torch.allclose(o[:, 3:5], o2, atol=1e-5)


@pytest.mark.parametrize("learned_pos", [False, True])
def test_packed_model_matches_separate_documents_cpu(learned_pos):
    """RoPE (llama) and learned positions (gpt2) both restart at each document."""
    from llmctl.models import build_model, get_model_config
    from llmctl.models.config import ModelConfig
    from llmctl.ops import ref

    cfg = get_model_config("tiny")
    if learned_pos:
        cfg = ModelConfig.from_dict({"name": "gpt2-mini", "layers": 2, "hidden": 128, "ffn": 512, "heads": 2,
                                     "vocab_size": 300, "norm": "layernorm", "activation": "gelu",
                                     "position": "learned", "max_position_embeddings": 64,
                                     "tie_word_embeddings": True})
    torch.manual_seed(0)
    m = build_model(cfg, device="cpu", dtype=torch.float32)
    d1 = torch.randint(1, cfg.vocab_size, (1, 9))
    d1[0, -1] = 0
    d2 = torch.randint(1, cfg.vocab_size, (1, 7))
    packed = torch.cat([d1, d2], 1)
    with torch.no_grad():
        lp = m(packed, doc_start=ref.document_starts(packed, 0)).reshape(16, -1)
        l1, l2 = m(d1).reshape(9, -1), m(d2).reshape(7, -1)
    assert torch.allclose(lp[:9], l1, atol=1e-4) and torch.allclose(lp[9:], l2, atol=1e-4)


def test_engine_pack_sequences_step():
    """pack_sequences: separators mask labels + attention; a batch without separators trains
    exactly like the unpacked engine."""
    from llmctl.testing.workers import _config
    from llmctl.runtime.engine import TrainingEngine

    g = torch.Generator().manual_seed(0)
    x = torch.randint(1, 500, (2, 32), generator=g)
    y = torch.randint(1, 500, (2, 32), generator=g)
    losses = {}
    for pack in (False, True):
        eng = TrainingEngine(_config(pack_sequences=pack))
        losses[pack] = eng.train_step([(x, y)])["loss"].item()
    assert losses[True] == pytest.approx(losses[False], rel=1e-6)
    xs = x.clone()
    xs[:, 10] = 0
    eng = TrainingEngine(_config(pack_sequences=True))
    l_sep = eng.train_step([(xs, y)])["loss"].item()
    assert np.isfinite(l_sep)
    with pytest.raises(NotImplementedError):
        TrainingEngine(_config(pack_sequences=True, context_parallel=2))


def test_nonfinite_grad_skips_step(monkeypatch, tmp_path):
    """nan_grad fault on step 2: the fused AdamW leaves params/moments untouched and counts
    the skipped step; steps 1 and 3 update normally."""
    from llmctl.testing.workers import _config
    from llmctl.runtime.engine import TrainingEngine

    monkeypatch.setenv("LLMCTL_FAULT", "nan_grad@step:2")
    eng = TrainingEngine(_config(output_dir=str(tmp_path)))
    g = torch.Generator().manual_seed(0)
    batch = lambda: [(torch.randint(1, 500, (2, 32), generator=g), torch.randint(1, 500, (2, 32), generator=g))]
    eng.train_step(batch())
    before = eng.flat.data.clone(), eng.optimizer.exp_avg.clone()
    out = eng.train_step(batch())
    assert not torch.isfinite(out["grad_norm"]).item()
    assert torch.equal(eng.flat.data, before[0]) and torch.equal(eng.optimizer.exp_avg, before[1])
    assert int(eng.optimizer.skipped_steps) == 1
    eng.train_step(batch())
    assert not torch.equal(eng.flat.data, before[0])


def test_fault_spec_parse():
    from llmctl.runtime.faults import parse

    f = parse("kill_rank:3@step:50, nan_grad@step:2")
    assert (f[0].kind, f[0].rank, f[0].step) == ("kill_rank", 3, 50) and f[1].rank is None
    with pytest.raises(ValueError):
        parse("explode@now")


def test_scheduled_profiler_writes_trace(tmp_path):
    from llmctl.testing.workers import _config
    from llmctl.runtime.engine import TrainingEngine

    eng = TrainingEngine(_config(output_dir=str(tmp_path / "run"), max_steps=4, save_steps=0, eval_steps=0,
                                 profile_dir=str(tmp_path / "prof"), profile_schedule="step(3)", logging_steps=2))
    eng.train()
    traces = list((tmp_path / "prof").glob("trace_rank00000_step*.json"))
    assert len(traces) == 1 and "llmctl.train_step" in traces[0].read_text()


# ---------------------------------------------------------------- ZeRO gather / side-stream update overlap order
@pytest.mark.parametrize("tied", [False, True])
def test_param_gather_waits_follow_forward_order(tied):
    """The post-step parameter all-gather (ZeRO-1/2) is issued in ``forward_order``; each
    forward pre-hook may only wait for buckets up to its own layer's position in that order.
    Regression: the norm-weight bucket sat last in flat order and was waited by layer 0 (and
    the LM-head bucket by the top-level hook), which serialised the whole gather before the
    first layer."""
    import dataclasses
    from types import SimpleNamespace

    from llmctl.models import build_model, get_model_config
    from llmctl.runtime.engine import TrainingEngine
    from llmctl.runtime.flat import FlatParameters
    from llmctl.runtime.optimizer import forward_order

    cfg = dataclasses.replace(get_model_config("tiny"), tie_word_embeddings=tied)
    m = build_model(cfg, dtype=torch.float32)
    flat = FlatParameters(list(m.named_parameters()), bucket_numel=4096)
    order = {b.index: i for i, b in enumerate(forward_order(flat.buckets))}
    assert len(order) > 2 * cfg.layers
    waits = []
    opt = SimpleNamespace(wait_params=lambda idx: waits.append([order[i] for i in idx]))
    TrainingEngine._install_param_gather_hooks(SimpleNamespace(flat=flat, optimizer=opt, model=m))
    ids = torch.randint(0, cfg.vocab_size, (1, 8))
    m(ids, ids)
    assert len(waits) == cfg.layers + 2  # top-level, every layer, head
    # layer k may only need the buckets issued up to about its own share of the gather
    per_layer = -(-len(order) // cfg.layers)
    seen = -1
    for k, w in enumerate(waits[:-1]):
        seen = max([seen, *w])
        assert seen <= (k + 1) * per_layer + 1, (k, seen, len(order), waits)
    seen = max([seen, *waits[-1]])
    assert seen == len(order) - 1  # everything is waited by the end of the forward


def test_tuning_cache_changes_dispatch(tmp_path, monkeypatch):
    """A tuning cache's winners are applied: TrainingEngine takes the DP bucket size and the
    gemm64 configuration per layout / exact shape, InferenceEngine the decode split count and
    the decode-GEMM table (reference: AutoTuner.load_results filled a dict nothing read)."""
    import json
    import os

    import importlib

    linear = importlib.import_module("llmctl.exec.linear")  # the package re-exports a function named linear
    from llmctl.models import get_model_config
    from llmctl.ops import functional
    from llmctl.runtime.engine import TrainingConfig, TrainingEngine
    from llmctl.serve.engine import InferenceEngine

    cache = {
        "comm_(1024, 1024)_torch.float32": {"best_config": {"bucket_mb": 1, "algorithm": "allreduce"}},
        "gemm64_dgrad_24576x4096x11008": {"best_config": {"config": 108}},
        "gemm64_wgrad_4096x4096x24576": {"best_config": {"config": 204}},
        "decode_splits_16x2048x32": {"best_config": {"splits": 4}},
        "skinny_16x12288x4096": {"best_config": {"config": 0}},
    }
    p = tmp_path / "tuning_cache.json"
    p.write_text(json.dumps(cache))
    monkeypatch.delenv("LLMCTL_KNOBS", raising=False)
    saved = (dict(linear.GEMM64_CONFIGS), dict(linear.GEMM64_SHAPE_CONFIGS), dict(functional.SKINNY_CONFIGS))
    try:
        cfg = TrainingConfig(model_name_or_path="tiny", batch_size=2, seq_len=16, device="cpu", log_level="warning",
                             tuning_cache=str(p))
        eng = TrainingEngine(cfg, get_model_config("tiny"))
        assert eng.config.bucket_mb == 1 and eng.tuned["bucket_mb"] == 1
        assert linear.gemm64_config("dgrad", 24576, 4096, 11008) == 108
        assert linear.gemm64_config("wgrad", 4096, 4096, 24576) == 204
        assert linear.GEMM64_CONFIGS["dgrad"] == 108  # the layout default follows the winner
        eng.shutdown()
        ie = InferenceEngine("tiny", device="cpu", num_kv_blocks=16, block_size=8, max_model_len=64,
                             tuning_cache=str(p))
        from llmctl.config.knobs import knobs

        assert knobs().decode_splits == 4 and ie.tuned["decode_splits"] == 4
        assert functional.SKINNY_CONFIGS[(16, 12288, 4096)] == 0
    finally:
        linear.GEMM64_CONFIGS.clear()
        linear.GEMM64_CONFIGS.update(saved[0])
        linear.GEMM64_SHAPE_CONFIGS.clear()
        linear.GEMM64_SHAPE_CONFIGS.update(saved[1])
        functional.SKINNY_CONFIGS.clear()
        functional.SKINNY_CONFIGS.update(saved[2])


def test_hw_network_benchmark_gloo_rehearsal():
    """``hw benchmark --component network`` measures collectives in-process (here: the gloo
    rehearsal of the RCCL path, 2 ranks, small sizes)."""
    from llmctl.cli.commands.hw import _bench_network

    r = _bench_network(ranks=2, backend="gloo", sizes=(4096,), patterns=("allreduce", "all_gather"), iters=2)
    assert r["status"] == "ok" and len(r["results"]) == 2
    assert all(x["busbw_gbps"] is not None and x["time_ms"] > 0 for x in r["results"])


def test_gemm64_default_config_single_knob(monkeypatch):
    """Without a tuning cache every layout uses knob gemm64_config (default 304, the persistent
    4-wave kernel); an override moves all layouts together."""
    import importlib

    linear = importlib.import_module("llmctl.exec.linear")
    from llmctl.config.knobs import PerfKnobs, override

    monkeypatch.setattr(linear, "GEMM64_CONFIGS", {})
    monkeypatch.setattr(linear, "GEMM64_SHAPE_CONFIGS", {})
    assert PerfKnobs().gemm64_config == 304
    with override(gemm64_config=304):
        assert {linear.gemm64_config(l, 4096, 4096, 4096) for l in ("fwd", "dgrad", "wgrad")} == {304}
    with override(gemm64_config=904):
        assert {linear.gemm64_config(l, 4096, 4096, 4096) for l in ("fwd", "dgrad", "wgrad")} == {904}


def test_checkpoint_commit_ignores_stale_done_markers(tmp_path):
    """A re-save of the same checkpoint (elastic restart after a rank died mid-write) must not
    count the earlier attempt's done-markers: rank 0 clears them (and the old commit record)
    before the pre-write barrier, and only markers carrying this save's id count."""
    from llmctl.io.checkpoint import CheckpointManager
    from llmctl.runtime.engine import TrainingEngine
    from llmctl.testing.workers import _config

    eng = TrainingEngine(_config(output_dir=str(tmp_path)))
    g = torch.Generator().manual_seed(0)
    eng.train_step([(torch.randint(1, 500, (2, 32), generator=g), torch.randint(1, 500, (2, 32), generator=g))])
    mgr = CheckpointManager(eng, str(tmp_path))
    ck = tmp_path / "checkpoint-1"
    (ck / ".done").mkdir(parents=True)
    for r in range(4):  # an interrupted earlier attempt of a 4-rank job
        (ck / ".done" / f"rank_{r:05d}").write_text("stale")
    (ck / "training_state.json").write_text('{"global_step": -1}')
    mgr.save("checkpoint-1", final=True)
    st = json.loads((ck / "training_state.json").read_text())
    assert st["global_step"] == eng.global_step
    assert not (ck / ".done").exists()
    assert (tmp_path / "latest").read_text() == "checkpoint-1"
    # the commit counts only markers of this save: one fresh marker + stale ones of "other ranks"
    (ck / ".done").mkdir()
    (ck / ".done" / "rank_00000").write_text("this-save")
    (ck / ".done" / "rank_00001").write_text("stale")
    with pytest.raises(TimeoutError):
        mgr._commit(ck, st, 1, 2, 0.2, "this-save")


def test_checkpoint_resave_is_staged_and_swapped(tmp_path, caplog):
    """Re-saving an existing checkpoint name writes a sibling staging directory and renames it over
    the target only once complete: an interrupted re-save (a staging directory left behind) never
    touches the committed copy, the next save clears it, and a ``latest`` that names an incomplete
    checkpoint is skipped with a warning."""
    import logging

    from llmctl.io.checkpoint import CheckpointManager
    from llmctl.runtime.engine import TrainingEngine
    from llmctl.testing.workers import _config

    eng = TrainingEngine(_config(output_dir=str(tmp_path)))
    g = torch.Generator().manual_seed(0)
    batch = [(torch.randint(1, 500, (2, 32), generator=g), torch.randint(1, 500, (2, 32), generator=g))]
    eng.train_step(batch)
    mgr = CheckpointManager(eng, str(tmp_path))
    ck = mgr.save("checkpoint-1", final=True)
    assert ck == tmp_path / "checkpoint-1" and (ck / "training_state.json").exists()
    # an interrupted re-save: its staging directory holds partial shards, the committed copy is intact
    st = tmp_path / ".checkpoint-1.staging"
    st.mkdir()
    (st / "model.safetensors").write_bytes(b"partial")
    assert json.loads((ck / "training_state.json").read_text())["global_step"] == 1
    eng.train_step(batch)
    mgr.save("checkpoint-1", final=True)  # the re-save proper
    assert json.loads((ck / "training_state.json").read_text())["global_step"] == 2
    assert not st.exists() and not (tmp_path / ".checkpoint-1.old").exists()
    # ``latest`` naming an incomplete checkpoint: fall back to the newest complete one, with a warning
    (tmp_path / "checkpoint-9").mkdir()
    (tmp_path / "latest").write_text("checkpoint-9")
    eng2 = TrainingEngine(_config(output_dir=str(tmp_path)))
    with caplog.at_level(logging.WARNING, logger="llmctl.io.checkpoint"):
        CheckpointManager(eng2, str(tmp_path)).load(str(tmp_path))
    assert eng2.global_step == 2 and "incomplete" in caplog.text


def test_token_loader_property(tmp_path):
    """Property test (hypothesis) of the native C++ TokenLoader (prefetch thread, seek) and the
    Python fallback of MemmapTokens: every row is one contiguous (S + 1)-token window, the DP
    ranks of an epoch read disjoint samples and each reads per_rank // B full batches, two loaders
    with the same arguments produce the same stream across epoch roll-overs, and seeking to a
    recorded position resumes the stream exactly."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from llmctl import native
    from llmctl.io.dataset import MemmapTokens

    m = native.load()

    @settings(max_examples=40, deadline=None)
    @given(st.integers(2, 9), st.integers(1, 4), st.integers(1, 3), st.integers(0, 2**31), st.integers(1, 5),
           st.integers(0, 40))
    def check(S, B, world, seed, depth, extra):
        n_samples = world * B * 3 + extra
        path = tmp_path / f"t{S}_{B}_{world}_{extra}.bin"
        np.arange(n_samples * S + 1, dtype=np.uint32).tofile(path)
        (tmp_path / (path.stem + ".json")).write_text('{"dtype": "uint32"}')
        per_rank = n_samples // world
        nb = per_rank // B  # full batches per rank per epoch

        def stream(make, n):
            ld = make()
            return [np.asarray(ld()) for _ in range(n)]

        impls = []
        if m is not None:
            impls.append(("native", lambda r: (lambda L: (lambda: L.next()))(
                m.TokenLoader(str(path), 4, S, B, r, world, seed, depth))))

        def py_rows(r):
            ds = MemmapTokens(str(path), S, B, dp_rank=r, dp_size=world, seed=seed)
            ds._native = None

            def nxt():
                x, y = ds.next_batch()
                return torch.cat([x, y[:, -1:]], 1).numpy()
            return nxt

        impls.append(("python", py_rows))
        for name, make in impls:
            seen = []
            for r in range(world):
                rows = np.concatenate(stream(lambda: make(r), nb))
                assert rows.shape == (nb * B, S + 1)
                starts = rows[:, 0]
                assert (starts % S == 0).all() and (rows == starts[:, None] + np.arange(S + 1)).all(), name
                seen.append(set((starts // S).tolist()))
                assert len(seen[-1]) == nb * B, name
            for i in range(world):
                for j in range(i + 1, world):
                    assert not (seen[i] & seen[j]), (name, "ranks overlap")
            a = stream(lambda: make(world - 1), 2 * nb + 1)  # across two epoch roll-overs
            b = stream(lambda: make(world - 1), 2 * nb + 1)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), (name, "not deterministic")
        for use_native in ([True, False] if m is not None else [False]):  # resume through MemmapTokens
            def ds_make(r=0):
                ds = MemmapTokens(str(path), S, B, dp_rank=r, dp_size=world, seed=seed)
                if not use_native:
                    ds._native = None
                return ds
            ref = ds_make()
            want = [torch.cat(ref.next_batch(), 1) for _ in range(2 * nb + 1)]
            k = (seed % (2 * nb)) + 1
            src = ds_make()
            for _ in range(k):
                src.next_batch()
            dst = ds_make()
            dst.load_state_dict(src.state_dict())
            assert torch.equal(torch.cat(dst.next_batch(), 1), want[k]), (use_native, "state_dict resume")
            sk = ds_make()
            sk.skip(k)
            assert torch.equal(torch.cat(sk.next_batch(), 1), want[k]), (use_native, "skip resume")

    check()
