"""Serving prefill with the RMSNorm folded into the projections (llmctl/ops/csrc/gemm64.hip row-scaled
epilogue, llmctl/ops/csrc/norm.hip rstd_kernel, llmctl/serve/engine.py ``_prefill_layers_folded``):
each kernel against an fp32 PyTorch oracle of the unfused ops, and the engine's folded prefill
against its norm-kernel prefill (knob ``prefill_norm_fold``)."""

import dataclasses

import pytest
import torch

from llmctl.testing.numerics import row_err

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(*shape, seed=0, scale=1.0):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("T,H", [(256, 256), (300, 4096), (2048, 704)])
def test_rms_rstd_matches_fp32(native_lib, T, H):
    x = _bf(T, H, seed=1, scale=3.0)
    r = native_lib.rms_rstd(x, 1e-5)
    want = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    assert r.dtype == torch.float32 and r.shape == (T,)
    torch.testing.assert_close(r, want, rtol=1e-5, atol=0)


# (2048, 12288, 4096): 384 tiles = a half-full last round -> tail split (scaled in the reduction)
@pytest.mark.parametrize("M,N,K", [(256, 512, 256), (512, 1536, 512), (2048, 12288, 4096), (1024, 768, 1152)])
@pytest.mark.parametrize("config", [304, 1304])
def test_linear_rowscale_matches_fp32(native_lib, M, N, K, config):
    """y = bf16((x W^T) * rstd) == rmsnorm(x) * w_n @ W^T with w_n folded into W, vs fp32."""
    x = _bf(M, K, seed=2)
    w = _bf(N, K, seed=3, scale=K ** -0.5)
    nw = (1.0 + 0.5 * torch.rand(K, device=DEV)).to(torch.bfloat16)
    wf = (w.float() * nw.float()).to(torch.bfloat16)
    r = native_lib.rms_rstd(x, 1e-5)
    y = native_lib.gemm64_rs(x, wf, r, config)
    want = (x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()) @ w.float().t()
    assert y.shape == (M, N)
    assert row_err(y, want) < 1.2e-2
    # the row scale is applied in fp32 before the single bf16 rounding (no double rounding)
    assert row_err(y, (x.float() @ wf.float().t()) * r[:, None]) < 4e-3


def test_linear_rowscale_split_equals_whole(native_lib):
    """Tail split (fp32 partials, scale applied in gemm64_split_reduce) vs whole tiles: within one
    bf16 ulp."""
    M, N, K = 2048, 12288, 4096
    x = _bf(M, K, seed=4)
    w = _bf(N, K, seed=5, scale=K ** -0.5)
    r = (0.5 + torch.rand(M, device=DEV)).float()
    a = native_lib.gemm64_rs(x, w, r, 304)
    b = native_lib.gemm64_rs(x, w, r, 1304)
    assert (a.float() - b.float()).abs().max() <= 8e-3 * b.float().abs().max()


@pytest.mark.parametrize("M,F,K", [(256, 128, 256), (512, 1024, 512), (2048, 11008, 4096)])
def test_up_swiglu_rowscale_matches_fp32(native_lib, M, F, K):
    x = _bf(M, K, seed=6)
    w = _bf(2 * F, K, seed=7, scale=K ** -0.5)
    r = (0.25 + torch.rand(M, device=DEV)).float()
    act = native_lib.gemm64_swiglu_fwd(x, w, 4, r)
    gu = (x.float() @ w.float().t()) * r[:, None]
    want = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert act.shape == (M, F)
    assert row_err(act, want) < 2e-2
    # without rstd the same kernel family gives the unscaled activation
    plain = native_lib.gemm64_swiglu_fwd(x, w, 304)
    assert row_err(plain, torch.nn.functional.silu((x.float() @ w.float().t())[:, :F])
                   * (x.float() @ w.float().t())[:, F:]) < 2e-2


@pytest.mark.parametrize("M,N,K", [(256, 512, 1024), (2048, 4096, 11008)])
def test_linear_acc_matches_fp32(native_lib, M, N, K):
    from llmctl import ops

    x = _bf(M, K, seed=8)
    w = _bf(N, K, seed=9, scale=K ** -0.5)
    h = _bf(M, N, seed=10)
    want = h.float() + x.float() @ w.float().t()
    out = h.clone()
    ops.linear_acc_(x, w, out)
    assert row_err(out, want) < 1.2e-2


def test_engine_prefill_norm_fold_matches_unfused(native_lib):
    """The folded prefill (rstd kernel + row-scaled QKV / gate-up GEMMs, residual adds in the o / down
    GEMM epilogues) gives the norm-kernel prefill's logits and KV cache, for packed fresh prompts
    (flash attention) and through the paged prefill kernel."""
    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import PrefillChunk, SamplingParams, Sequence

    e = InferenceEngine("tiny-wide", device="cuda", max_batch_size=4, num_kv_blocks=128, block_size=16,
                        max_model_len=512, use_graphs=False, perf_knobs={"prefill_norm_fold": True})
    assert e._nf is not None and len(e._nf) == e.cfg.layers
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(0, 512, (n,), generator=g).tolist() for n in (100, 156, 256)]  # 512 tokens
    seqs = [Sequence(prompt_ids=p, params=SamplingParams(max_tokens=1)) for p in prompts]
    for s in seqs:
        assert e.kv.add_sequence_shared(s.seq_id, s.num_tokens, [])
    plan = e.prefill_plan([PrefillChunk(s, 0, s.num_tokens) for s in seqs])
    base = e.knobs
    for fa in (True, False):
        e.knobs = dataclasses.replace(base, prefill_norm_fold=True, prefill_fa=fa)
        assert e._norm_fold_ok(len(plan["ids"]))
        la = e.prefill_exec(plan).float()
        kc_a = [t.clone() for t in e.kv_cache.k]
        e.knobs = dataclasses.replace(base, prefill_norm_fold=False, prefill_fa=fa)
        lb = e.prefill_exec(plan).float()
        assert la.shape == lb.shape == (3, e.cfg.vocab_size)
        assert (la - lb).norm() / lb.norm() < 2e-2
        assert (la.argmax(-1) == lb.argmax(-1)).float().mean() >= 2 / 3
        for a, b in zip(kc_a, e.kv_cache.k):
            assert (a.float() - b.float()).norm() / b.float().norm() < 2e-2
    e.knobs = base
    e.close()


@pytest.mark.parametrize("rs", [False, True])
@pytest.mark.parametrize("config", [304, 404, 104])
def test_swiglu_fwd_tail_split(native_lib, rs, config):
    """4,096 tokens of GPT-7B's gate/up projection: 1,376 paired tiles = 5.375 rounds, so the automatic
    plan splits the last round's K range (fp32 partials, SwiGLU and row scale in gemm64_split_reduce):
    within a bf16 ulp of the whole-tile kernel and vs the fp32 oracle."""
    M, F, K = 4096, 11008, 4096
    x = _bf(M, K, seed=11)
    w = _bf(2 * F, K, seed=12, scale=K ** -0.5)
    r = (0.5 + torch.rand(M, device=DEV)).float() if rs else None
    split = native_lib.gemm64_swiglu_fwd(x, w, config, r)
    whole = native_lib.gemm64_swiglu_fwd(x, w, 1000 + config, r)
    gu = x.float() @ w.float().t()
    if rs:
        gu = gu * r[:, None]
    want = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert row_err(split, want) < 2e-2 and row_err(whole, want) < 2e-2
    assert (split.float() - whole.float()).abs().max() <= 1.6e-2 * whole.float().abs().max()


def test_engine_prefill_norm_fold_gpt7b_layer_dims(native_lib, tmp_path):
    """One decoder layer at GPT-7B's dimensions (hidden 4096, 32 heads, ffn 11008), one 2,048-token
    prompt: the folded prefill (QKV GEMM with the row scale and a tail split, gate/up + SwiGLU with the
    row scale, residual adds in the o / down epilogues) matches the norm-kernel prefill."""
    import json

    from llmctl.serve.engine import InferenceEngine
    from llmctl.serve.scheduler import PrefillChunk, SamplingParams, Sequence

    cfg = {"name": "gpt7b-1l", "arch": "decoder-only", "layers": 1, "hidden": 4096, "ffn": 11008, "heads": 32,
           "vocab_size": 512, "max_position_embeddings": 4096, "rope": {"base": 10000, "scaling": "linear"}}
    path = tmp_path / "gpt7b-1l.json"
    path.write_text(json.dumps(cfg))
    e = InferenceEngine(str(path), device="cuda", max_batch_size=1, num_kv_blocks=160, block_size=16,
                        max_model_len=2560, use_graphs=False, perf_knobs={"prefill_norm_fold": True})
    assert e._nf is not None
    g = torch.Generator().manual_seed(9)
    seq = Sequence(prompt_ids=torch.randint(0, 512, (2048,), generator=g).tolist(), params=SamplingParams(max_tokens=1))
    assert e.kv.add_sequence_shared(seq.seq_id, seq.num_tokens, [])
    plan = e.prefill_plan([PrefillChunk(seq, 0, seq.num_tokens)])
    base = e.knobs
    e.knobs = dataclasses.replace(base, prefill_norm_fold=True)
    la = e.prefill_exec(plan).float()
    ka, va = e.kv_cache.k[0].clone(), e.kv_cache.v[0].clone()
    e.knobs = dataclasses.replace(base, prefill_norm_fold=False)
    lb = e.prefill_exec(plan).float()
    e.knobs = base
    assert (la - lb).norm() / lb.norm() < 2e-2
    for a, b in ((ka, e.kv_cache.k[0]), (va, e.kv_cache.v[0])):
        assert (a.float() - b.float()).norm() / b.float().norm() < 2e-2
    e.close()
