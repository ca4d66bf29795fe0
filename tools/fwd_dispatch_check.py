import os, sys, time, torch
sys.path.insert(0, os.getcwd())
from llmctl.ops import _lib
import importlib
L = importlib.import_module("llmctl.exec.linear")
cnt = {"g64": 0, "pick": []}
orig = L.forward_linear
def wrap(x, w, b=None):
    N, K = w.shape; M = x.numel() // K
    cnt["pick"].append((M, N, K, L.fwd64_pick(M, N, K), L._gemm64_ok(M, N, K, x.reshape(M, K), w) if M % 256 == 0 else None))
    return orig(x, w, b)
L.forward_linear = wrap
from llmctl.serve.engine import InferenceEngine
from llmctl.serve.scheduler import SamplingParams
eng = InferenceEngine("gpt-7b", device="cuda", max_batch_size=1, max_model_len=2048 + 32)
p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
eng.generate([[1] * 32], p)
cnt["pick"].clear()
s = eng.add_request([(7 * i) % 32000 for i in range(2048)], p)
while s.status != "finished":
    eng.step()
print(sorted(set(cnt["pick"]))[:20])
