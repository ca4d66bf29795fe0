"""gemm64_ex (llmctl/ops/csrc/gemm64.hip) vs an fp32 PyTorch reference, every operand layout,
store and accumulate epilogues, every schedule variant; checked per ROW (max error of the row
over the row's max magnitude), so one wrong 16x16 tile fails the test even when a Frobenius
norm over the whole output would hide it (the self-check below proves that)."""

import pytest
import torch

from llmctl.testing.numerics import row_err

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(*shape, seed=0):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return torch.randn(*shape, generator=g, device=DEV).to(torch.bfloat16)



TOL = 1.2e-2  # bf16 output rounding is <= 2^-8 of the row max; fp32 accumulation order adds ~1e-5


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 384), (768, 512, 1024), (2304, 1280, 256)])
@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("split", [0, 1, 2])
@pytest.mark.parametrize("variant", [1, 3, 5, 9])
def test_gemm64_ex(native_lib, M, N, K, at, bt, acc, split, variant):
    A = _bf(M, K, seed=71)
    B = _bf(N, K, seed=72)
    a = A.t().contiguous() if at else A
    b = B.t().contiguous() if bt else B
    c0 = _bf(M, N, seed=73)
    out = c0.clone() if acc else torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    native_lib.gemm64_ex(a, b, out, at, bt, acc, 4 + 100 * variant + 1000 * split)
    want = A.float() @ B.float().t() + (c0.float() if acc else 0.0)
    assert torch.isfinite(out.float()).all()
    assert row_err(out, want) < TOL


@pytest.mark.parametrize("config", [4, 8, 104, 108, 1104, 2104, 4008, 8104, 904, 908, 1904, 2904, 8904,
                                    304, 308, 1304, 2304, 8304])
def test_gemm64_configs(native_lib, config):
    """Every tile-order group / schedule variant / tail split computes the same product (fwd
    and wgrad); 1xxx = no split, Sxxx = S K-ranges (24 tiles < one round: all of them split).
    x0xx-x2xx: 8-wave kernel, x3xx: persistent 4-wave, x4xx-x9xx: one-shot 4-wave."""
    M, N, K = 1536, 1024, 2048  # 24 tiles: more tiles than one group, several K-tile pairs
    A, B = _bf(M, K, seed=3), _bf(N, K, seed=4)
    want = A.float() @ B.float().t()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    native_lib.gemm64_ex(A, B, out, False, False, False, config)
    assert row_err(out, want) < TOL
    native_lib.gemm64_ex(A.t().contiguous(), B.t().contiguous(), out, True, True, False, config)
    assert row_err(out, want) < TOL


def test_gemm64_split_tail_multi_round(native_lib):
    """More tiles than CUs with a partial last round: the main tiles run whole, the tail tiles
    in K-ranges through the workspace; store and accumulate epilogues, wgrad layout."""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    M, N, K = 256 * (n_cu // 8 + 1), 256 * 8, 1024  # n_cu + 8 tiles: 8 tail tiles
    A, B = _bf(K, M, seed=91), _bf(K, N, seed=92)
    c0 = _bf(M, N, seed=93)
    want = A.float().t() @ B.float()
    for cfg in (104, 8104, 904, 8904, 304, 1304, 8304):
        # x1xx: 8-wave; x3xx: 4-wave persistent; x9xx: 4-wave
        out = c0.clone()
        native_lib.gemm64_ex(A, B, out, True, True, True, cfg)
        assert row_err(out, want + c0.float()) < TOL, cfg
        out = torch.full_like(c0, float("nan"))
        native_lib.gemm64_ex(A, B, out, True, True, False, cfg)
        assert row_err(out, want) < TOL, cfg


@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, True)])
@pytest.mark.parametrize("rounds", [3, 8])
def test_gemm64_persistent_many_rounds(native_lib, at, bt, rounds):
    """Persistent kernel over ~3.4 / ~8.3 rounds of items per CU with a split tail: every
    workgroup streams several tiles back to back (the next tile's first K-tiles ride on the
    previous tile's DMA stream, the item-boundary drain is taken repeatedly); fwd / dgrad /
    wgrad layouts vs fp32, NaN-prefilled outputs."""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    tiles = n_cu * rounds + n_cu // 3
    M, N, K = 256 * (tiles // 4 + 1), 256 * 4, 512
    A, B = _bf(M, K, seed=11), _bf(N, K, seed=12)
    a = A.t().contiguous() if at else A
    b = B.t().contiguous() if bt else B
    want = A.float() @ B.float().t()
    for cfg in (304, 1304, 308):
        out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        native_lib.gemm64_ex(a, b, out, at, bt, False, cfg)
        assert torch.isfinite(out.float()).all(), cfg
        assert row_err(out, want) < TOL, cfg


def test_gemm64_strided_views(native_lib):
    """Row-strided operand / output views (flat-buffer gradient views, column slices)."""
    big = _bf(1024, 640, seed=81)
    a = big[:, 64:576]           # K-major A [K=1024][M=512], row stride 640
    b = _bf(1024, 512, seed=82)  # K-major B [K=1024][N=512]
    out_buf = torch.zeros(512, 768, device=DEV, dtype=torch.bfloat16)
    out = out_buf[:, 256:768]
    native_lib.gemm64_ex(a, b, out, True, True, False, 104)
    assert row_err(out, a.float().t() @ b.float()) < TOL
    assert (out_buf[:, :256] == 0).all()


def test_gemm64_rejects_bad_shapes(native_lib):
    a, b = _bf(256, 96, seed=1), _bf(256, 96, seed=2)
    out = torch.empty(256, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="multiples"):
        native_lib.gemm64_ex(a, b, out, False, False, False, 104)


@pytest.mark.parametrize("mode", ["all", "fused"])
def test_linear_backward_on_gemm64(native_lib, mode):
    """exec.linear routes wgrad (into the sink's flat view) through gemm64 at eligible shapes and
    dgrad through gemm64 (knob dgrad64=all: no W^T copy) or, with dgrad64=fused (only the
    SwiGLU-fused down projection on gemm64), hipBLASLt through the W^T copy; all match fp32."""
    from llmctl.config.knobs import configure
    from llmctl.exec.linear import GradSink, dgrad64_ok, linear

    configure({"dgrad64": mode})

    T, inn, out = 512, 768, 1024
    x = _bf(T, inn, seed=5).requires_grad_(True)
    w = torch.nn.Parameter(_bf(out, inn, seed=6))
    w.grad = torch.zeros_like(w)
    sink = GradSink()
    sink.attach(w)
    y = linear(x, w)
    dy = _bf(T, out, seed=7)
    if mode == "all":
        assert getattr(w, "_llmctl_wt", None) is None  # gemm64 dgrad: no transposed copy kept
        assert dgrad64_ok(dy, w)
    else:
        assert getattr(w, "_llmctl_wt", None) is not None and not dgrad64_ok(dy, w)
        assert dgrad64_ok(dy, w, fused=True)
    y.backward(dy)
    assert row_err(x.grad, dy.float() @ w.detach().float()) < TOL
    assert row_err(w.grad, dy.float().t() @ x.detach().float()) < TOL


@pytest.mark.parametrize("M,H,F", [(256, 256, 256), (512, 384, 768), (2304, 1024, 1280)])
@pytest.mark.parametrize("config", [104, 1104, 2104, 904])
def test_gemm64_swiglu_dgrad(native_lib, M, H, F, config):
    """Down-projection data gradient with the SwiGLU backward in the store epilogue (and in the
    tail-split reduction, config 2104): dgu vs fp32 swiglu_bwd(dy @ W, gu)."""
    dy, w, gu = _bf(M, H, seed=81), _bf(H, F, seed=82) * 0.05, _bf(M, 2 * F, seed=83)
    dgu = native_lib.gemm64_swiglu_dgrad(dy, w, gu, config)
    dact = dy.float() @ w.float()
    g, u = gu[:, :F].float(), gu[:, F:].float()
    sg = torch.sigmoid(g)
    want = torch.cat([dact * u * sg * (1 + g * (1 - sg)), dact * g * sg], dim=1)
    assert torch.isfinite(dgu.float()).all()
    assert row_err(dgu[:, :F], want[:, :F]) < TOL and row_err(dgu[:, F:], want[:, F:]) < TOL


def test_swiglu_down_autograd_fused_matches_unfused(native_lib):
    """The MLP's _SwiGLUDown (fused dgrad, saved activation) and its selective-recompute form
    give the gradients of swiglu -> linear through plain autograd (fp32 reference)."""
    from llmctl.models.transformer import _SwiGLUDown

    T, H, F = 512, 512, 768
    gu = (_bf(T, 2 * F, seed=91)).requires_grad_(True)
    w = (_bf(H, F, seed=92) * 0.05).requires_grad_(True)
    dy = _bf(T, H, seed=93)
    g32, w32 = gu.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    f = g32.shape[1] // 2
    ref_out = torch.nn.functional.linear(torch.nn.functional.silu(g32[:, :f]) * g32[:, f:], w32)
    ref_out.backward(dy.float())
    for recompute in (False, True):
        gu.grad = w.grad = None
        out = _SwiGLUDown.apply(gu, w, recompute)
        out.backward(dy)
        assert row_err(out, ref_out.detach()) < 2e-2
        assert row_err(gu.grad, g32.grad) < 2e-2 and row_err(w.grad, w32.grad) < 2e-2


@pytest.mark.parametrize("cfg", [104, 2104, 904, 2904, 1904, 304, 1304, 2304])
def test_gemm64_wgrad_fp32_output(native_lib, cfg):
    """fp32 main gradients: the wgrad layout stores / accumulates an fp32 C (no bf16 rounding of
    the running sum); one-shot and persistent schedules, with and without the split tail."""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    M, N, K = 256 * (n_cu // 8 + 1), 256 * 8, 1024
    A, B = _bf(K, M, seed=31), _bf(K, N, seed=32)
    want = A.float().t() @ B.float()
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float32)
    native_lib.gemm64_ex(A, B, out, True, True, False, cfg)
    assert (out - want).abs().max().item() < 2e-3 * want.abs().max().item()
    c0 = torch.randn(M, N, device=DEV)
    out = c0.clone()
    native_lib.gemm64_ex(A, B, out, True, True, True, cfg)
    assert (out - (want + c0)).abs().max().item() < 2e-3 * want.abs().max().item()


def _swiglu_bwd_ref(dact, gu):
    F = dact.shape[1]
    g, u = gu[:, :F].float(), gu[:, F:].float()
    sg = torch.sigmoid(g)
    return torch.cat([dact.float() * u * sg * (1 + g * (1 - sg)), dact.float() * g * sg], dim=1)


@pytest.mark.parametrize("T,H,F,cfg", [(512, 4096, 1024, 104),   # one chunk per K-tile, exact fit
                                       (512, 2048, 2048, 104),   # two chunks per K-tile
                                       (512, 3072, 2304, 104),   # elements past E (range-checked)
                                       (2048, 4096, 1024, 4104),  # every tile split into 4 K-ranges
                                       (2048, 4096, 1024, 1104),
                                       (512, 4096, 1024, 904),    # 4-wave kernel: one chunk per K-tile
                                       (512, 2048, 2048, 904),    # two chunks
                                       (512, 3072, 2304, 904),    # range-checked tail
                                       (512, 2048, 2048, 304),    # persistent number: one-shot side kernel
                                       (2048, 4096, 1024, 4904)])
@pytest.mark.parametrize("gdt,acc", [(torch.bfloat16, False), (torch.bfloat16, True), (torch.float32, False),
                                     (torch.float32, True)])
def test_gemm64_wgrad_swiglu(native_lib, T, H, F, cfg, gdt, acc):
    """Down-projection weight gradient with the SwiGLU backward as a side job: gw (+)= dy^T act
    and dgu = swiglu_bwd(dact, gu), both against fp32 references."""
    from llmctl.exec.linear import side_chunks

    assert side_chunks(H, F, T, T, F) > 0
    dy, act = _bf(T, H, seed=11), _bf(T, F, seed=12)
    dact, gu = _bf(T, F, seed=13), _bf(T, 2 * F, seed=14)
    g0 = torch.randn(H, F, device=DEV).to(gdt)
    gw = g0.clone() if acc else torch.full((H, F), float("nan"), device=DEV, dtype=gdt)
    dgu = native_lib.gemm64_wgrad_swiglu(dy, act, gw, acc, dact, gu, cfg)
    want = dy.float().t() @ act.float() + (g0.float() if acc else 0.0)
    assert torch.isfinite(gw.float()).all() and torch.isfinite(dgu.float()).all()
    assert row_err(gw, want) < TOL
    ref = _swiglu_bwd_ref(dact, gu)
    assert row_err(dgu[:, :F], ref[:, :F]) < TOL and row_err(dgu[:, F:], ref[:, F:]) < TOL


@pytest.mark.parametrize("main_grad", [False, True])
@pytest.mark.parametrize("dgrad64", ["fused", "all"])
def test_swiglu_down_side_job_autograd(native_lib, main_grad, dgrad64):
    """_SwiGLUDown with a grad-sink weight: plain data gradient (hipBLASLt through W^T, or gemm64
    with dgrad64=all) + weight gradient carrying the SwiGLU backward (swiglu_bwd=side); two
    backward passes accumulate into the sink's view (bf16 .grad or fp32 main_grad); matches fp32
    autograd and the epilogue-fused path."""
    from llmctl.config.knobs import configure
    from llmctl.exec.linear import GradSink, wgrad_swiglu_ok
    from llmctl.models.transformer import _SwiGLUDown

    configure({"dgrad64": dgrad64})
    T, H, F = 512, 4096, 1024
    gu0 = _bf(T, 2 * F, seed=21)
    w = torch.nn.Parameter(_bf(H, F, seed=22) * 0.02)
    dy = _bf(T, H, seed=23)
    sink = GradSink()
    sink.attach(w)
    if main_grad:
        w.main_grad = torch.zeros(H, F, device=DEV)
    else:
        w.grad = torch.zeros_like(w)
    assert wgrad_swiglu_ok(w, T, F)
    g32, w32 = gu0.float().requires_grad_(True), w.detach().float().requires_grad_(True)
    ref_out = torch.nn.functional.linear(torch.nn.functional.silu(g32[:, :F]) * g32[:, F:], w32)
    ref_out.backward(dy.float())
    for step in (1, 2):
        gu = gu0.clone().requires_grad_(True)
        out = _SwiGLUDown.apply(gu, w, False)
        out.backward(dy)
        gw = w.main_grad if main_grad else w.grad
        assert row_err(gu.grad, g32.grad) < 2e-2
        assert row_err(gw, step * w32.grad) < 2e-2
    configure({"dgrad64": dgrad64, "swiglu_bwd": "epilogue"})
    gu = gu0.clone().requires_grad_(True)
    _SwiGLUDown.apply(gu, w, False).backward(dy)
    assert row_err(gu.grad, g32.grad) < 2e-2
