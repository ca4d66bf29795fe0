"""Fused training-forward GEMM epilogues (llmctl/ops/csrc/gemm64.hip EPI_ROPE_QKV / EPI_UP_SWIGLU)
against fp32 references of the unfused ops (F.linear + RoPE / SwiGLU), checked per row, plus
the decoder layer's fused path against the unfused path (knob fused_fwd off) forward and
backward — including the gradients the grad sink writes."""

import pytest
import torch

from llmctl.ops import ref
from llmctl.testing.numerics import row_err

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1.2e-2


def _bf(*shape, seed=0, scale=1.0):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("T,K,nq,nkv", [(512, 256, 4, 2), (1024, 384, 2, 2), (2048, 512, 8, 4)])
@pytest.mark.parametrize("with_pos", [False, True])
@pytest.mark.parametrize("config", [104, 304, 904])
def test_gemm64_qkv_rope_matches_fp32(native_lib, T, K, nq, nkv, with_pos, config):
    D = 128
    x = _bf(T, K, seed=1)
    w = _bf((nq + 2 * nkv) * D, K, seed=2, scale=K ** -0.5)
    S = 256
    cos, sin = ref.rope_tables(4096, D, device=DEV)
    pos = None
    if with_pos:
        pos = torch.randint(0, 4096, (T,), device=DEV, dtype=torch.int32)
    q, k, v = native_lib.gemm64_qkv_rope(x, w, cos, sin, pos, nq, nkv, S, config)
    qkv = (x.float() @ w.float().t())
    rq, rk, rv = ref.rope_qkv_fwd(qkv, cos, sin, nq, nkv, S, pos)
    for got, want in ((q, rq), (k, rk), (v, rv)):
        assert got.shape == want.shape
        assert row_err(got.reshape(T, -1), want.reshape(T, -1)) < TOL
    # bit-exact against the unfused HIP path on the same bf16 projection
    qkv_bf = torch.nn.functional.linear(x, w)
    uq, uk, uv = native_lib.rope_qkv_fwd(qkv_bf, cos, sin, nq, nkv, S, pos)
    for got, want in ((q, uq), (k, uk), (v, uv)):
        assert row_err(got.reshape(T, -1), want.reshape(T, -1)) < 8e-3


@pytest.mark.parametrize("T,K,nq,nkv", [(2048, 4096, 32, 32), (512, 1024, 8, 4)])
def test_gemm64_qkv_rope_tail_split(native_lib, T, K, nq, nkv):
    """Prefill-sized QKV + RoPE with the tail split (partial last round cut into K-ranges, the
    RoPE / head split applied by gemm64_split_reduce) == the same GEMM on whole tiles (config
    1304) up to the order of the split sums, and == the fp32 oracle."""
    D = 128
    x = _bf(T, K, seed=11)
    w = _bf((nq + 2 * nkv) * D, K, seed=12, scale=K ** -0.5)
    cos, sin = ref.rope_tables(4096, D, device=DEV)
    pos = torch.randint(0, 4096, (T,), device=DEV, dtype=torch.int32)
    q, k, v = native_lib.gemm64_qkv_rope(x, w, cos, sin, pos, nq, nkv, T, 304)
    q1, k1, v1 = native_lib.gemm64_qkv_rope(x, w, cos, sin, pos, nq, nkv, T, 1304)
    rq, rk, rv = ref.rope_qkv_fwd(x.float() @ w.float().t(), cos, sin, nq, nkv, T, pos)
    for got, whole, want in ((q, q1, rq), (k, k1, rk), (v, v1, rv)):
        assert row_err(got.reshape(T, -1), whole.reshape(T, -1).float()) < 8e-3  # one bf16 ulp
        assert row_err(got.reshape(T, -1), want.reshape(T, -1)) < TOL


@pytest.mark.parametrize("T,K,F", [(256, 256, 128), (512, 384, 384), (1024, 512, 1024)])
@pytest.mark.parametrize("config", [104, 304, 904])
def test_gemm64_up_swiglu_matches_fp32(native_lib, T, K, F, config):
    x = _bf(T, K, seed=3)
    w = _bf(2 * F, K, seed=4, scale=K ** -0.5)
    gu, act = native_lib.gemm64_up_swiglu(x, w, config)
    act2 = native_lib.gemm64_swiglu_fwd(x, w, config)  # serving prefill form: act only
    assert torch.equal(act2, act)
    gu_ref = x.float() @ w.float().t()
    assert row_err(gu, gu_ref) < TOL
    act_ref = ref.swiglu_fwd(gu_ref)
    assert row_err(act, act_ref) < TOL
    assert row_err(act, ref.swiglu_fwd(gu)) < 8e-3  # act is computed from the stored bf16 gu


def _layer_grads(fused: bool, monkeypatch, sink: bool, extra=None, dims=(512, 4, 2, 1024)):
    from llmctl.config.knobs import configure

    configure({"fused_fwd": fused, **(extra or {})})  # A/B both
    from llmctl.exec.linear import GradSink
    from llmctl.models import ParallelContext, get_model_config
    from llmctl.models.transformer import DecoderLayer

    cfg = get_model_config("tiny")
    cfg.hidden, cfg.heads, cfg.kv_heads, cfg.ffn = dims
    cfg.head_dim = 128
    torch.manual_seed(0)
    layer = DecoderLayer(cfg, ParallelContext(), 0, device=DEV, dtype=torch.bfloat16)
    grads = {}
    if sink:
        s = GradSink()
        for n, p in layer.named_parameters():
            if n in ("wqkv", "wo", "w_up", "w_down"):
                p.grad = torch.zeros_like(p)
                s.attach(p)
    B, S = 2, 256
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    x = (torch.randn(B * S, cfg.hidden, generator=g, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    rope = layer_rope(cfg, S)
    out, res = layer(x, None, B, S, rope)
    loss = (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum() + res.float().sum()
    loss.backward()
    grads["x"] = x.grad.detach().clone()
    for n, p in layer.named_parameters():
        grads[n] = p.grad.detach().clone()
    return out.detach(), grads


def layer_rope(cfg, S):
    return ref.rope_tables(max(S, cfg.max_position_embeddings), cfg.head_dim, device=DEV)


@pytest.mark.parametrize("sink", [False, True])
def test_decoder_layer_fused_forward_matches_unfused(native_lib, monkeypatch, sink):
    out_f, g_f = _layer_grads(True, monkeypatch, sink)
    out_u, g_u = _layer_grads(False, monkeypatch, sink)
    assert row_err(out_f, out_u.float()) < TOL
    for n in g_u:
        a, b = g_f[n].float(), g_u[n].float()
        a2 = a.reshape(a.shape[0], -1) if a.dim() > 1 else a.view(1, -1)
        b2 = b.reshape(b.shape[0], -1) if b.dim() > 1 else b.view(1, -1)
        assert row_err(a2, b2) < 3e-2, n


@pytest.mark.parametrize("config", [104, 304, 904])
def test_decoder_layer_all_gemm64_matches_hipblaslt(native_lib, monkeypatch, config):
    """Every projection of the layer on gemm64 (fused RoPE-QKV / up-SwiGLU forward epilogues,
    forward + data gradients with W read K-major, weight gradients, the SwiGLU backward as the
    down wgrad's side job at hidden 4096 / ffn 1024) against the library path (hipBLASLt
    forward / data gradients, unfused RoPE / SwiGLU), forward and every gradient."""
    knobs = {"gemm64_config": config, "fwd64": "all", "dgrad64": "all"}
    dims = (4096, 32, 8, 1024)
    out_f, g_f = _layer_grads(True, monkeypatch, True, knobs, dims)
    out_u, g_u = _layer_grads(False, monkeypatch, True, {"gemm64": False, "wgrad_kernel": False}, dims)
    assert row_err(out_f, out_u.float()) < TOL
    for n in g_u:
        a, b = g_f[n].float(), g_u[n].float()
        a2 = a.reshape(a.shape[0], -1) if a.dim() > 1 else a.view(1, -1)
        b2 = b.reshape(b.shape[0], -1) if b.dim() > 1 else b.view(1, -1)
        assert row_err(a2, b2) < 3e-2, n
