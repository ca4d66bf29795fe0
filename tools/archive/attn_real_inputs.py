"""Time the attention forward kernels (knob fa_w64 0 / 3, alternating) on the GPT-7B model's own layer-0
q / k / v (random-init weights, strided views of the packed QKV projection output) instead of gaussian
inputs: the score spread and the data (power) differ from tools/attn_fwd_ab.py's."""
import json, sys, time
import torch
sys.path.insert(0, '.')
from llmctl.ops import _lib
assert _lib.load(), _lib._error
ops = torch.ops.llmctl
from llmctl.models import get_model_config, build_model
cfg = get_model_config("gpt-7b")
cfg.layers = 2
torch.manual_seed(0)
cap = {}
orig = ops.flash_attn_fwd
class Wrap:
    pass
m = build_model(cfg, device="cuda", dtype=torch.bfloat16)
B, S = 16, 2048
ids = torch.randint(0, cfg.vocab_size, (B, S), device="cuda")
import llmctl.ops.functional as T
saved = []
real = T.native
def fake_native():
    n = real()
    class P:
        def __getattr__(self, k):
            if k == "flash_attn_fwd":
                def f(q, k_, v, *a):
                    if not saved:
                        saved.append((q, k_, v, a))
                    return n.flash_attn_fwd(q, k_, v, *a)
                return f
            return getattr(n, k)
    return P()
T.native = fake_native
with torch.no_grad():
    m(ids)
T.native = real
q, k, v, a = saved[0]
print("q", tuple(q.shape), q.stride(), "absmax", q.abs().max().item(), "std", q.float().std().item(), "k std", k.float().std().item(), flush=True)
s = (q[0, :256, 0].float() @ k[0, :256, 0].float().t()) * a[0]
print("score*scale std", s.std().item(), "max", s.max().item(), flush=True)
for var in (0, 3) * 5:
    ops.set_knob("fa_w64", var)
    for _ in range(3):
        ops.flash_attn_fwd(q, k, v, *a)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20):
        ops.flash_attn_fwd(q, k, v, *a)
    torch.cuda.synchronize()
    print(json.dumps({"fa_w64": var, "ms": round((time.perf_counter() - t) / 20 * 1e3, 4)}), flush=True)
