import sys, os, torch
sys.path.insert(0, os.getcwd())
from llmctl import ops
from llmctl.ops import ref, _lib
from llmctl.testing.numerics import row_err
DEV="cuda"
def bf(*shape, seed=0):
    g = torch.Generator(device=DEV); g.manual_seed(seed)
    return torch.randn(*shape, generator=g, device=DEV).to(torch.bfloat16)
for (B,S,nq,nkv,D) in [(1,2048,8,8,128),(1,1024,8,8,128),(2,256,4,2,128)]:
    T=B*S
    cos, sin = ref.rope_tables(S+40, D, device=DEV)
    base = bf(T,(nq+2*nkv)*D, seed=61); do = bf(B,S,nq,D, seed=62)
    qkv = base.clone().requires_grad_(True)
    o = ops.rope_flash_attention(qkv, cos, sin, nq, nkv, B, S, None); o.backward(do); gf = qkv.grad.clone()
    qkv2 = base.clone().requires_grad_(True)
    q,k,v = ops.rope_qkv(qkv2, cos, sin, nq, nkv, S, None)
    o2 = ops.flash_attention(q.view(B,S,nq,D), k.view(B,S,nkv,D), v.view(B,S,nkv,D), causal=True); o2.backward(do); gu = qkv2.grad.clone()
    q32 = base.float().requires_grad_(True)
    qq,kk,vv = ref.rope_qkv_fwd(q32, cos, sin, nq, nkv, S, None)
    orf,_ = ref.attention_fwd(qq.view(B,S,nq,D), kk.view(B,S,nkv,D), vv.view(B,S,nkv,D), D**-0.5, True); orf.backward(do.float()); gr = q32.grad
    for nm, lo, hi in (("dq",0,nq),("dk",nq,nq+nkv),("dv",nq+nkv,nq+2*nkv)):
        sl = lambda g: g.view(T,-1,D)[:,lo:hi]
        print(B,S,nm, "fused-ref %.4f"%row_err(sl(gf), sl(gr), floor=0.5), "unfused-ref %.4f"%row_err(sl(gu), sl(gr), floor=0.5), "fused-unfused %.4f"%row_err(sl(gf), sl(gu), floor=0.5))
