"""Pure-PyTorch fp32 oracles for every HIP kernel in ``llmctl/ops/csrc``.

These are (a) the numerics reference the kernel tests compare against and (b) the compute
path on CPU (the gloo/CPU distributed tests and the GPT-2-125M CPU plumbing config run
through them).  They are deliberately written in plain fp32 math, not for speed.

Reference parity: the reference runs all of these as stock HF/PyTorch ops
(attention, RMSNorm, RoPE, SwiGLU, AdamW, clip, CE are library calls there).
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- norms
def rmsnorm_fwd(x: torch.Tensor, w: torch.Tensor, eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
    y = (xf * rstd.unsqueeze(-1)) * w.float()
    return y.to(x.dtype), rstd


def rmsnorm_bwd(dy, x, w, rstd, dres: Optional[torch.Tensor] = None):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    r = rstd.unsqueeze(-1)
    xhat = xf * r
    g = dyf * wf
    dx = r * (g - xhat * (g * xhat).mean(-1, keepdim=True))
    if dres is not None:
        dx = dx + dres.float()
    dw = (dyf * xhat).reshape(-1, x.shape[-1]).sum(0)
    return dx.to(x.dtype), dw.to(w.dtype)


def layernorm_fwd(x, w, b, eps):
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = (xf - mu).pow(2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mu) * rstd * w.float() + b.float()
    return y.to(x.dtype), mu.squeeze(-1), rstd.squeeze(-1)


def layernorm_bwd(dy, x, w, mu, rstd, dres=None):
    xf, dyf, wf = x.float(), dy.float(), w.float()
    r = rstd.unsqueeze(-1)
    xhat = (xf - mu.unsqueeze(-1)) * r
    g = dyf * wf
    dx = r * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
    if dres is not None:
        dx = dx + dres.float()
    H = x.shape[-1]
    dw = (dyf * xhat).reshape(-1, H).sum(0)
    db = dyf.reshape(-1, H).sum(0)
    return dx.to(x.dtype), dw.to(w.dtype), db.to(w.dtype)


# ----------------------------------------------------------------------------- rope
def rope_tables(seq_len: int, head_dim: int, base: float = 10000.0, scaling: str = "linear",
                factor: float = 1.0, short_factor=None, long_factor=None,
                original_max_position: Optional[int] = None, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """cos/sin tables [seq_len, head_dim/2] fp32 (host-precomputed, per the CDNA guide's
    'precompute trig tables' rule for RoPE).  ``su`` = LongRoPE-style per-dim rescale."""
    half = head_dim // 2
    inv = 1.0 / (base ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / head_dim))
    pos = torch.arange(seq_len, dtype=torch.float64)
    mscale = 1.0
    if scaling == "linear" and factor and factor != 1.0:
        pos = pos / factor
    elif scaling == "su":
        orig = original_max_position or seq_len
        fac = long_factor if (seq_len > orig and long_factor) else short_factor
        if fac:
            inv = inv / torch.tensor(fac, dtype=torch.float64)
        if seq_len > orig:
            s = seq_len / orig
            mscale = math.sqrt(1 + math.log(s) / math.log(orig))
    ang = torch.outer(pos, inv)
    cos = (torch.cos(ang) * mscale).float()
    sin = (torch.sin(ang) * mscale).float()
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos.contiguous(), sin.contiguous()


def _rot(x, cos, sin):
    # x [..., D] rotate-half convention (Llama/NeoX): (x1, x2) -> (x1 c - x2 s, x2 c + x1 s)
    d = x.shape[-1] // 2
    x1, x2 = x[..., :d], x[..., d:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def rope_qkv_fwd(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, nq: int, nkv: int,
                 seq_len: int, positions: Optional[torch.Tensor] = None):
    """qkv [T, (nq+2nkv)*D] -> q [T, nq, D], k [T, nkv, D], v [T, nkv, D] (q,k rotated)."""
    T = qkv.shape[0]
    D = qkv.shape[1] // (nq + 2 * nkv)
    x = qkv.float().view(T, nq + 2 * nkv, D)
    pos = positions.long() if positions is not None else torch.arange(T, device=qkv.device) % seq_len
    c = cos[pos].unsqueeze(1)
    s = sin[pos].unsqueeze(1)
    q = _rot(x[:, :nq], c, s)
    k = _rot(x[:, nq:nq + nkv], c, s)
    v = x[:, nq + nkv:]
    dt = qkv.dtype
    return q.to(dt).contiguous(), k.to(dt).contiguous(), v.to(dt).contiguous()


def rope_qkv_bwd(dq, dk, dv, cos, sin, seq_len: int, positions=None):
    T = dq.shape[0]
    pos = positions.long() if positions is not None else torch.arange(T, device=dq.device) % seq_len
    c = cos[pos].unsqueeze(1)
    s = sin[pos].unsqueeze(1)
    dqf = _rot(dq.float(), c, -s)  # inverse rotation = transpose
    dkf = _rot(dk.float(), c, -s)
    out = torch.cat([dqf, dkf, dv.float()], dim=1).reshape(T, -1)
    return out.to(dq.dtype)


# ----------------------------------------------------------------------------- attention
def _doc_mask(doc_start, S: int, device):
    """[B,1,S,S] visibility of packed documents: key j visible to query i iff doc_start[i] <= j."""
    j = torch.arange(S, device=device)
    return (j.view(1, 1, 1, S) >= doc_start.to(device).long().view(doc_start.shape[0], 1, S, 1))


def document_starts(input_ids: torch.Tensor, separator: int) -> torch.Tensor:
    """[B,S] position where each token's document begins; a document ends with (includes) the
    ``separator`` token, the next one starts right after it."""
    B, S = input_ids.shape
    pos = torch.arange(S, device=input_ids.device).expand(B, S)
    is_start = torch.zeros_like(input_ids, dtype=torch.bool)
    is_start[:, 0] = True
    is_start[:, 1:] = input_ids[:, :-1] == separator
    starts = torch.where(is_start, pos, torch.zeros_like(pos))
    return torch.cummax(starts, dim=1).values.to(torch.int32).contiguous()


def attention_fwd(q, k, v, scale: float, causal: bool = True, doc_start=None):
    """q [B,S,Hq,D], k/v [B,S,Hkv,D] -> o [B,S,Hq,D], lse [B,Hq,S] (natural log)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    if causal:
        mask = torch.ones(S, Sk, dtype=torch.bool, device=q.device).tril(Sk - S)
        s = s.masked_fill(~mask, float("-inf"))
    if doc_start is not None:
        s = s.masked_fill(~_doc_mask(doc_start, S, q.device), float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse.unsqueeze(-1))
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype).contiguous(), lse


def attention_bwd(do, q, k, v, o, lse, scale: float, causal: bool = True, doc_start=None):
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    dof = do.float().transpose(1, 2)
    of = o.float().transpose(1, 2)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    if causal:
        mask = torch.ones(S, Sk, dtype=torch.bool, device=q.device).tril(Sk - S)
        s = s.masked_fill(~mask, float("-inf"))
    if doc_start is not None:
        s = s.masked_fill(~_doc_mask(doc_start, S, q.device), float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)
    dk = dk.view(B, Hkv, rep, Sk, D).sum(2)
    dv = dv.view(B, Hkv, rep, Sk, D).sum(2)
    return (dq.transpose(1, 2).to(q.dtype).contiguous(), dk.transpose(1, 2).to(k.dtype).contiguous(),
            dv.transpose(1, 2).to(v.dtype).contiguous())


def paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale: float):
    """q [N, Hq, D]; caches [num_blocks, block_size, Hkv, D]; block_tables [N, max_blocks]."""
    N, Hq, D = q.shape
    bs = k_cache.shape[1]
    Hkv = k_cache.shape[2]
    rep = Hq // Hkv
    out = torch.empty_like(q)
    for i in range(N):
        L = int(context_lens[i])
        nb = (L + bs - 1) // bs
        blocks = block_tables[i, :nb].long()
        kk = k_cache[blocks].reshape(nb * bs, Hkv, D)[:L].float()
        vv = v_cache[blocks].reshape(nb * bs, Hkv, D)[:L].float()
        kk = kk.repeat_interleave(rep, dim=1)
        vv = vv.repeat_interleave(rep, dim=1)
        s = torch.einsum("hd,lhd->hl", q[i].float(), kk) * scale
        p = torch.softmax(s, dim=-1)
        out[i] = torch.einsum("hl,lhd->hd", p, vv).to(q.dtype)
    return out


def attn_merge_(o_acc, lse_acc, o_j, lse_j) -> None:
    """In-place log-sum-exp merge: o_acc [B,S,H,D] fp32 / lse_acc [B,H,S] fp32 absorb the
    partial (o_j, lse_j); a fresh accumulator is (0, -inf)."""
    ln = torch.logaddexp(lse_acc, lse_j)
    dead = torch.isinf(ln) & (ln < 0)
    wa = torch.where(dead, torch.zeros_like(ln), torch.exp(lse_acc - ln)).transpose(1, 2).unsqueeze(-1)
    wj = torch.where(dead, torch.zeros_like(ln), torch.exp(lse_j - ln)).transpose(1, 2).unsqueeze(-1)
    o_acc.mul_(wa).add_(o_j.float() * wj)
    lse_acc.copy_(ln)


def paged_prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale: float):
    """Packed new tokens q [T, Hq, D] of N sequences (rows cu_q[n]:cu_q[n+1]) attending, causally,
    every cached key of their sequence: after the chunk's cache write sequence n holds
    ctx_lens[n] tokens and its new tokens sit at positions ctx - qlen .. ctx - 1."""
    T, Hq, D = q.shape
    bs, Hkv = k_cache.shape[1], k_cache.shape[2]
    rep = Hq // Hkv
    out = torch.empty_like(q)
    cu = [int(x) for x in cu_q]
    for n in range(len(cu) - 1):
        q0, q1 = cu[n], cu[n + 1]
        qlen, L = q1 - q0, int(ctx_lens[n])
        if qlen == 0:
            continue
        nb = (L + bs - 1) // bs
        blocks = block_tables[n, :nb].long()
        kk = k_cache[blocks].reshape(nb * bs, Hkv, D)[:L].float().repeat_interleave(rep, dim=1)
        vv = v_cache[blocks].reshape(nb * bs, Hkv, D)[:L].float().repeat_interleave(rep, dim=1)
        s = torch.einsum("qhd,lhd->hql", q[q0:q1].float(), kk) * scale
        pos = torch.arange(L - qlen, L, device=q.device).view(1, qlen, 1)
        keys = torch.arange(L, device=q.device).view(1, 1, L)
        s = s.masked_fill(keys > pos, float("-inf"))
        out[q0:q1] = torch.einsum("hql,lhd->qhd", torch.softmax(s, dim=-1), vv).to(q.dtype)
    return out


def kv_cache_write(k, v, k_cache, v_cache, slot_mapping):
    """k/v [N, Hkv, D] written at flat slots (block*block_size + offset) of the caches."""
    nb, bs = k_cache.shape[:2]
    kc = k_cache.view(nb * bs, *k_cache.shape[2:])
    vc = v_cache.view(nb * bs, *v_cache.shape[2:])
    idx = slot_mapping.long()
    valid = idx >= 0
    if kc.dtype == torch.float8_e4m3fn:  # saturating, like the kernels (torch's cast maps > 448 to NaN)
        k, v = k.float().clamp(-448.0, 448.0), v.float().clamp(-448.0, 448.0)
    kc[idx[valid]] = k[valid].to(kc.dtype)
    vc[idx[valid]] = v[valid].to(vc.dtype)


# ----------------------------------------------------------------------------- MLP
def swiglu_fwd(gu: torch.Tensor) -> torch.Tensor:
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dact: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    d = dact.float()
    sg = torch.sigmoid(g)
    silu = g * sg
    dg = d * u * (sg * (1 + g * (1 - sg)))
    du = d * silu
    return torch.cat([dg, du], dim=-1).to(gu.dtype)


def gelu_fwd(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def gelu_bwd(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    xf = x.float().requires_grad_(True)
    with torch.enable_grad():
        y = F.gelu(xf, approximate="tanh")
        (g,) = torch.autograd.grad(y, xf, dy.float())
    return g.to(x.dtype)


# ----------------------------------------------------------------------------- loss
def cross_entropy_fwd(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100):
    """Per-row loss (fp32, 0 where ignored) and lse (fp32)."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = labels != ignore_index
    tgt = torch.where(valid, labels, torch.zeros_like(labels)).long()
    picked = lf.gather(-1, tgt.unsqueeze(-1)).squeeze(-1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    return loss, lse


def cross_entropy_bwd(dloss: torch.Tensor, logits: torch.Tensor, lse: torch.Tensor, labels: torch.Tensor,
                      ignore_index: int = -100) -> torch.Tensor:
    """dloss per row (fp32) -> dlogits (dtype of logits)."""
    lf = logits.float()
    p = torch.exp(lf - lse.unsqueeze(-1))
    valid = labels != ignore_index
    tgt = torch.where(valid, labels, torch.zeros_like(labels)).long()
    p.scatter_add_(-1, tgt.unsqueeze(-1), -torch.ones_like(p[..., :1]))
    g = p * (dloss * valid.float()).unsqueeze(-1)
    return g.to(logits.dtype)


# ----------------------------------------------------------------------------- optimizer
def adamw_step_(param, master, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step,
                grad_scale: float = 1.0):
    """Decoupled-weight-decay Adam on an fp32 master copy; writes the bf16 param.  A
    non-finite ``grad_scale`` skips the update (same policy as the HIP kernel)."""
    if not math.isfinite(grad_scale):
        return
    g = grad.float() * grad_scale
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    master.mul_(1 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    denom = (exp_avg_sq / bc2).sqrt_().add_(eps)
    master.addcdiv_(exp_avg, denom, value=-lr / bc1)
    param.copy_(master.to(param.dtype))


def l2norm_sq(t: torch.Tensor) -> torch.Tensor:
    return t.float().pow(2).sum()


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
           uniform: torch.Tensor) -> torch.Tensor:
    """Batched temperature / top-k / top-p sampling driven by caller-supplied uniforms
    (so the kernel and this oracle pick the same token).  temperature<=0 => greedy.

    Semantics (shared with ``csrc/sampling.hip``): x = logits / T; the kept set is
    {x >= max(T_k, T_p)} where T_k is the k-th largest x and T_p the smallest value of the
    minimal descending prefix whose softmax mass reaches top_p; the token is drawn by
    inverse CDF over the kept tokens *in vocabulary order* with r = u * kept_mass."""
    N, V = logits.shape
    out = torch.empty(N, dtype=torch.long, device=logits.device)
    for i in range(N):
        l = logits[i].float()
        t = float(temperature[i])
        if t <= 0:
            out[i] = int(torch.argmax(l))
            continue
        x = l / t
        e = torch.exp(x - x.max())
        thr = -float("inf")
        k = int(top_k[i])
        if 0 < k < V:
            thr = float(torch.topk(x, k).values[-1])
        tp = float(top_p[i])
        if tp < 1.0:
            sx, si = torch.sort(x, descending=True)
            cum = torch.cumsum(e[si], 0)
            n = int(torch.searchsorted(cum, torch.tensor([tp * float(e.sum())], device=cum.device), right=False)[0])
            thr = max(thr, float(sx[min(n, V - 1)]))
        keep = x >= thr
        w = torch.where(keep, e, torch.zeros_like(e))
        cum = torch.cumsum(w, 0)
        r = float(uniform[i]) * float(cum[-1])
        j = int(torch.searchsorted(cum, torch.tensor([r], device=cum.device, dtype=cum.dtype), right=True)[0])
        out[i] = min(j, V - 1)
    return out
