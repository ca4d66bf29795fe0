"""CPU paths of the fused decode / prefill op wrappers (``llmctl.ops``): without the HIP library
they must compose the unfused reference ops exactly, so the serving engine's fused decode body
and the prefill SwiGLU path stay correct on every device."""

import torch

from llmctl import ops
from llmctl.ops import ref


def _x(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def test_decode_up_swiglu_cpu_matches_unfused():
    x, w = _x(5, 64, seed=1), _x(96, 64, seed=2) * 0.1
    assert not ops.decode_fused_ok(x, w)
    torch.testing.assert_close(ops.decode_up_swiglu(x, w), ops.swiglu(x @ w.t()))
    torch.testing.assert_close(ops.up_swiglu(x, w), ops.swiglu(x @ w.t()))


def test_decode_linear_add_rmsnorm_cpu_matches_unfused():
    x, w, res, nw = _x(3, 32, seed=3), _x(48, 32, seed=4) * 0.1, _x(3, 48, seed=5), 1 + 0.1 * _x(48, seed=6)
    y, r = ops.decode_linear_add_rmsnorm(x, w, None, res, nw, 1e-5)
    s = x @ w.t() + res
    torch.testing.assert_close(r, s)
    torch.testing.assert_close(y, s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * nw, rtol=1e-4, atol=1e-5)


def test_decode_qkv_rope_cache_and_attention_cpu():
    nq, nkv, D, bs, nb, M = 4, 2, 16, 4, 8, 2
    x, w = _x(M, 32, seed=7), _x((nq + 2 * nkv) * D, 32, seed=8) * 0.1
    cos, sin = ref.rope_tables(64, D)
    pos = torch.tensor([5, 2], dtype=torch.int32)
    slots = torch.tensor([1 * bs + 1, 3 * bs + 2])
    kc = torch.zeros(nb, bs, nkv, D)
    vc = torch.zeros_like(kc)
    q = ops.decode_qkv_rope_cache(x, w, None, cos, sin, nq, nkv, pos, kc, vc, slots)
    qr, kr, vr = ref.rope_qkv_fwd(x @ w.t(), cos, sin, nq, nkv, 0, pos)
    torch.testing.assert_close(q, qr)
    torch.testing.assert_close(kc.view(-1, nkv, D)[slots], kr)
    torch.testing.assert_close(vc.view(-1, nkv, D)[slots], vr)
    bt = torch.tensor([[0, 1, 2], [3, 4, 5]], dtype=torch.int32)
    ctx = torch.tensor([6, 3], dtype=torch.int32)
    kc2, vc2 = kc.clone(), vc.clone()
    o = ops.decode_attention_qkv(x, w, None, cos, sin, nq, nkv, pos, kc2, vc2, slots, bt, ctx)
    torch.testing.assert_close(o, ref.paged_attention_decode(qr, kc, vc, bt, ctx, D ** -0.5))


def test_fp8_decode_weights_cpu_fallbacks():
    """fp8 (e4m3fn) weights + fp32 row scales: the CPU paths use the dequantised weight."""
    from llmctl.plugins.quantizers import quantize_fp8

    x = _x(3, 64, seed=21)
    qd = quantize_fp8(_x(96, 64, seed=22) * 0.1)
    w8, sc = qd["qweight"], qd["scale"].float()
    wd = w8.float() * sc.unsqueeze(1)
    assert not ops.decode_fused_ok(x, w8)
    torch.testing.assert_close(ops.decode_linear_fp8(x, w8, sc), x @ wd.t())
    torch.testing.assert_close(ops.decode_up_swiglu(x, w8, None, w_scale=sc), ops.swiglu(x @ wd.t()))
    res, nw = _x(3, 96, seed=23), 1 + 0.1 * _x(96, seed=24)
    y, r = ops.decode_linear_add_rmsnorm(x, w8, None, res, nw, 1e-5, w_scale=sc)
    torch.testing.assert_close(r, x @ wd.t() + res)
    # the fp8 image is within e4m3 rounding of the original
    assert ((wd - _x(96, 64, seed=22) * 0.1).abs() <= 0.07 * (_x(96, 64, seed=22) * 0.1).abs() + 1e-6).all()
