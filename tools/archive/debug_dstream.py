import sys
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib, ref
assert _lib.load()
ops = torch.ops.llmctl
DEV = "cuda"
def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV); g.manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)
for (M, K, bias) in [(16, 1024, True), (16, 1024, False), (16, 4096, True), (5, 2048, True)]:
    nq, nkv, D, bs, nb = 8, 2, 128, 16, 8
    N = (nq + 2 * nkv) * D
    x = _bf(M, K, seed=91); w = _bf(N, K, scale=0.05, seed=92); b = _bf(N, seed=93) if bias else None
    cos, sin = ref.rope_tables(256, D, base=10000.0, device=DEV)
    torch.manual_seed(0)
    pos = torch.randint(0, 256, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * bs, device=DEV)[:M]
    if M > 1: slots[1] = -1
    kc = torch.zeros(nb, bs, nkv, D, dtype=torch.bfloat16, device=DEV); vc = torch.zeros_like(kc)
    q = ops.decode_qkv_rope_cache(x, w, b, cos, sin, nq, nkv, pos, kc, vc, slots)
    qkv = ops.skinny_linear_cfg(x, w, b, 25)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(kc)
    q2, _, _ = ops.rope_qkv_cache_fwd(qkv, cos, sin, nq, nkv, 256, pos, kc2, vc2, slots)
    ws = ops.decode_linear_partials(x, w)
    print(M, K, bias, "ws shape", tuple(ws.shape), "q diff", (q.float()-q2.float()).abs().max().item(),
          "kc diff", (kc.float()-kc2.float()).abs().max().item(), "vc diff", (vc.float()-vc2.float()).abs().max().item(),
          "n q mismatch", int((q != q2).sum()), flush=True)
