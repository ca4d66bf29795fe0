"""Planner golden values, the MI355X cost model, TOML round-trip, schemas."""

import json
from pathlib import Path

import pytest

from llmctl.config.schemas import resolve_training_config, validate
from llmctl.config.toml_io import dumps_toml, load_toml, loads_toml
from llmctl.models.config import get_model_config
from llmctl.partition.planner import ParallelismPlanner, ReferenceCompatPlanner
from llmctl.partition.shard_map import build_shard_map, split_layers

ROOT = Path(__file__).resolve().parents[2]
LLAMA7B = json.loads((ROOT / "configs/models/llama-7b.json").read_text())
HW8 = {"gpu": {"count": 8}}


# ---------------------------------------------------------------- reference-compatible planner (golden)
def test_reference_param_and_memory_formulas():
    p = ReferenceCompatPlanner(LLAMA7B, HW8)
    assert p.estimate_parameters() == 5_164_761_088
    assert abs(p.estimate_model_memory() - 57.72) < 0.01
    assert abs(p.estimate_activation_memory(1, 2048) - 0.75) < 1e-9


def test_reference_search_golden_plan():
    best = ReferenceCompatPlanner(LLAMA7B, HW8).search_optimal_plan(1e14, 40, 100)
    assert (best["tensor_parallel"], best["pipeline_parallel"], best["data_parallel"], best["zero_stage"],
            best["micro_batch_size"], best["global_batch_size"]) == (8, 1, 1, 0, 1, 4)
    assert abs(best["estimated_memory_gb"] - 7.97) < 0.01


def test_reference_manual_golden_plan():
    m = ReferenceCompatPlanner(LLAMA7B, HW8).manual_plan(2, 2, 3)
    assert abs(m["estimated_memory_gb"] - 5.57) < 0.01
    assert abs(m["estimated_comm_gb"] - 9.62) < 0.01
    assert abs(m["estimated_flops"] - 1.69e14) / 1.69e14 < 0.01


def test_reference_70b_like():
    d = dict(hidden=8192, layers=80, ffn=28672, vocab_size=128256, heads=64)
    p = ReferenceCompatPlanner(d, HW8)
    assert abs(p.estimate_parameters() / 1e9 - 60.1) < 0.05
    assert abs(p.estimate_model_memory() - 671.8) < 0.5
    assert p.search_optimal_plan(1e15, 1000, 100)["tensor_parallel"] == 8


# ---------------------------------------------------------------- MI355X planner
def test_exact_param_count_matches_reference_config():
    cfg = get_model_config(str(ROOT / "configs/models/llama-7b.json"))
    assert cfg.num_parameters() == 6_738_415_616  # the reference's own estimated_params


def _mi355x(n):
    from llmctl.cli.commands.hw import mi355x_preset

    return mi355x_preset(n)


def test_mi355x_plan_7b_single_node_prefers_dp():
    pl = ParallelismPlanner(LLAMA7B, _mi355x(8))
    best = pl.search_optimal_plan(max_memory=259)
    assert best["tensor_parallel"] * best["pipeline_parallel"] * best["data_parallel"] == 8
    # 7B fits one 288 GB GPU with ZeRO: no model parallelism is needed on xGMI
    assert best["tensor_parallel"] == 1 and best["pipeline_parallel"] == 1
    assert best["estimated_memory_gb"] <= 259


def test_mi355x_plan_70b_needs_sharding():
    d = json.loads((ROOT / "configs/models/llama-70b.json").read_text())
    pl = ParallelismPlanner(d, _mi355x(8))
    best = pl.search_optimal_plan(max_memory=259)
    assert best["estimated_memory_gb"] <= 259
    assert best["tensor_parallel"] > 1 or best["pipeline_parallel"] > 1 or best["zero_stage"] >= 1


def test_memory_monotone_in_sharding():
    pl = ParallelismPlanner(LLAMA7B, _mi355x(8))
    m0 = pl.compute_memory_requirement(1, 1, 8, 0, 1)
    m1 = pl.compute_memory_requirement(1, 1, 8, 1, 1)
    m3 = pl.compute_memory_requirement(1, 1, 8, 3, 1)
    mt = pl.compute_memory_requirement(8, 1, 1, 0, 1)
    assert m0 > m1 > m3
    assert mt < m0


def test_shard_map():
    assert split_layers(32, 4) == [(0, 8), (8, 16), (16, 24), (24, 32)]
    sm = build_shard_map(LLAMA7B, tp=2, pp=2, dp=2, zero_stage=1)
    assert sm is not None


# ---------------------------------------------------------------- TOML + schemas
def test_toml_roundtrip_nested():
    d = {"a": 1, "b": {"c": [1, 2, 3], "d": {"e": "x\"y", "f": 1.5e-5, "g": True}},
         "devs": [{"id": 0, "name": "MI355X"}, {"id": 1, "name": "MI355X"}]}
    back = loads_toml(dumps_toml(d))
    assert back == d


def test_reference_presets_parse_and_validate():
    ref = Path("/root/reference/configs/presets")
    files = sorted(ref.glob("*.toml")) if ref.exists() else []
    files += sorted((ROOT / "configs/presets").glob("*.toml"))
    assert files
    for f in files:
        d = load_toml(f)
        kind = "hardware" if "gpu" in d and "system" in d else "train"
        validate(kind, d)


def test_resolve_precedence():
    t = load_toml(ROOT / "configs/presets/llama-7b-mi355x8.toml")
    plan = {"parallelism": {"tensor_parallel": 2, "pipeline_parallel": 1, "data_parallel": 4, "zero_stage": 2,
                            "micro_batch_size": 4, "global_batch_size": 64}}
    out = resolve_training_config(t, plan, {"batch_size": 3, "learning_rate": None})
    assert out["tensor_parallel"] == 2 and out["zero_stage"] == 2
    assert out["batch_size"] == 3  # CLI beats plan
    assert out["learning_rate"] == pytest.approx(2e-4)  # None CLI value does not override the file


def test_model_json_configs_load():
    for f in sorted((ROOT / "configs/models").glob("*.json")):
        cfg = get_model_config(str(f))
        d = json.loads(f.read_text())
        assert cfg.num_parameters() == d["estimated_params"], f.name


def test_planner_virtual_stages_shrink_the_bubble():
    """Interleaved pipeline: the planner's step time falls with virtual stages (bubble
    (pp-1)/(vs*M)), the auto search may pick vs > 1, and the shard map lists each pipeline
    rank's chunks (pp*vs-way layer split, rank p owns chunks p, p+pp, ...)."""
    from llmctl.models import get_model_config
    from llmctl.partition.planner import ParallelismPlanner
    from llmctl.partition.shard_map import build_shard_map

    cfg = get_model_config("llama-70b").to_dict()
    hw = {"gpu": {"count": 8, "memory_gb": 288}}
    pl = ParallelismPlanner(cfg, hw, seq_len=2048)
    t1 = pl.evaluate(1, 4, 2, 1, False, "selective", 1, 64, vs=1)["estimated_step_time_s"]
    t2 = pl.evaluate(1, 4, 2, 1, False, "selective", 1, 64, vs=2)["estimated_step_time_s"]
    assert t2 < t1
    sm = build_shard_map(cfg, 1, 4, 2, 1, virtual_stages=2)
    assert sm["virtual_stages"] == 2 and len(sm["stages"]) == 8
    r0 = [r for r in sm["ranks"] if r["pp_rank"] == 0][0]
    assert r0["layers"] == [sm["stages"][0], sm["stages"][4]]


def test_planner_plan_properties():
    """Property test (hypothesis) of the MI355X planner over model templates, node sizes (including
    non-powers of two), sequence lengths and fixed micro-batches: the chosen layout uses every GPU
    exactly (tp x pp x dp = gpus), divides the heads / KV heads, never has more stages than layers,
    fits the HBM budget whenever any layout does, and reports finite positive estimates."""
    import dataclasses
    import math

    from hypothesis import given, settings
    from hypothesis import strategies as st

    from llmctl.partition.planner import HardwareModel

    models = st.sampled_from(["gpt-7b", "llama-13b", "llama-70b", "tiny", "tiny-wide", "gpt2"])

    @settings(max_examples=60, deadline=None)
    @given(models, st.sampled_from([1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 64]), st.sampled_from([512, 2048, 8192, 32768]),
           st.sampled_from([None, 1, 4, 16]))
    def check(name, gpus, seq, mb):
        cfg = get_model_config(name)
        pl = ParallelismPlanner(dataclasses.asdict(cfg), {}, seq, hw=HardwareModel(gpus=gpus))
        plan = pl.search_optimal_plan(fixed={"mb": mb} if mb else None)
        tp, pp, dp = plan["tensor_parallel"], plan["pipeline_parallel"], plan["data_parallel"]
        assert tp * pp * dp == gpus, plan
        assert cfg.heads % tp == 0 and cfg.kv_heads % tp == 0
        assert 1 <= pp <= cfg.layers
        for k in ("estimated_tokens_per_sec", "estimated_step_time_s", "estimated_memory_gb"):
            assert math.isfinite(plan[k]) and plan[k] > 0, (k, plan)
        feasible = any(pl.evaluate(**c)["estimated_memory_gb"] <= 0.9 * pl.hw.hbm_gb
                       for c in pl.candidates((mb,) if mb else (1, 2, 4, 8, 16)))
        if feasible:
            assert plan["estimated_memory_gb"] <= 0.9 * pl.hw.hbm_gb, plan

    check()


def test_toml_writer_roundtrip_property():
    """Property test (hypothesis): the own TOML emitter round-trips through tomli for nested
    tables of the value kinds the schemas use -- arbitrary unicode keys and strings (quotes,
    backslashes, control characters, newlines), ints, finite / infinite floats, bools, lists of
    scalars, lists of tables; None values are omitted."""
    import math

    from hypothesis import given, settings
    from hypothesis import strategies as st

    keys = st.text(min_size=1, max_size=8)
    scal = st.one_of(st.integers(-2**63, 2**63 - 1), st.booleans(), st.text(max_size=12),
                     st.floats(allow_nan=False))
    lists = st.lists(st.integers(-10**6, 10**6), max_size=4) | st.lists(st.text(max_size=5), max_size=4)
    tables = st.recursive(st.dictionaries(keys, st.one_of(scal, lists, st.none()), max_size=4),
                          lambda inner: st.dictionaries(keys, st.one_of(scal, lists, inner,
                                                                        st.lists(inner, min_size=1, max_size=2)),
                                                        max_size=4), max_leaves=10)

    def strip_none(d):
        if isinstance(d, dict):
            return {k: strip_none(v) for k, v in d.items() if v is not None}
        if isinstance(d, list):
            return [strip_none(x) for x in d]
        return d

    def same(a, b):
        if isinstance(a, dict):
            return isinstance(b, dict) and a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
        if isinstance(a, list):
            return isinstance(b, list) and len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
        if isinstance(a, float):
            return isinstance(b, float) and (a == b or (math.isinf(a) and a == b))
        return type(a) is type(b) and a == b

    @settings(max_examples=300, deadline=None)
    @given(tables)
    def check(d):
        text = dumps_toml(d)
        got = loads_toml(text)
        assert same(strip_none(d), got), text

    check()


def test_shard_map_properties():
    """Property test (hypothesis) of the shard map: pipeline stages are contiguous, cover every
    layer once and differ by at most one layer (the first / last stages never above a middle one);
    every rank has unique (tp, dp, pp) coordinates, the pipeline ranks of each (tp, dp) slice own
    every layer exactly once (virtual chunks included), the TP ranks partition the heads / FFN /
    vocabulary ranges, and only the first / last pipeline rank holds the embedding / LM head."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    @settings(max_examples=400, deadline=None)
    @given(st.integers(1, 96), st.integers(1, 8))
    def stages(L, pp):
        s = split_layers(L, pp)
        assert len(s) == pp and s[0][0] == 0 and s[-1][1] == L
        assert all(a[1] == b[0] for a, b in zip(s, s[1:]))
        sizes = [e - b for b, e in s]
        assert max(sizes) - min(sizes) <= 1
        if pp > 2:
            assert max(sizes[0], sizes[-1]) <= min(sizes[1:-1])

    @settings(max_examples=300, deadline=None)
    @given(st.integers(1, 80), st.sampled_from([1, 2, 4, 8]), st.sampled_from([1, 2, 3, 4]), st.integers(1, 3),
           st.integers(0, 3), st.integers(1, 3), st.integers(1, 64), st.integers(1, 8))
    def shard(L, tp, pp, dp, zero, V, heads, kvdiv):
        kv = max(1, heads // kvdiv)
        model = {"layers": L, "heads": heads, "kv_heads": kv, "hidden": 64 * heads, "ffn": 11008, "vocab_size": 32000}
        sm = build_shard_map(model, tp, pp, dp, zero, virtual_stages=V)
        ranks = sm["ranks"]
        assert len(ranks) == tp * pp * dp
        assert len({(r["tp_rank"], r["dp_rank"], r["pp_rank"]) for r in ranks}) == len(ranks)
        Vr = sm["virtual_stages"]
        assert Vr == (V if pp > 1 else 1)
        for t in range(tp):
            for d in range(dp):
                owned = []
                for r in ranks:
                    if r["tp_rank"] == t and r["dp_rank"] == d:
                        chunks = [r["layers"]] if Vr == 1 else r["layers"]
                        assert len(chunks) == Vr
                        for b, e in chunks:
                            owned.extend(range(b, e))
                        assert r["embedding"] == (r["pp_rank"] == 0) and r["lm_head"] == (r["pp_rank"] == pp - 1)
                        assert r["zero_partition"] == ([d, dp] if zero >= 1 else None)
                assert sorted(owned) == list(range(L))
        for key, total in (("q_heads", heads), ("kv_heads", kv), ("ffn", 11008), ("vocab", 32000)):
            for p in range(pp):
                for d in range(dp):
                    parts = sorted(r[key] for r in ranks if r["pp_rank"] == p and r["dp_rank"] == d)
                    assert parts[0][0] == 0 and parts[-1][1] == total
                    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))

    stages()
    shard()
