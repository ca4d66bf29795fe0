#!/usr/bin/env python3
"""Reference-equivalent stack on MI355X: what the reference's engine does (HF transformers
model + torch AdamW, eager PyTorch, ``engine.py:119-140,217-339``), at the SAME config as
bench.py (GPT-7B dims from init.py:18-27, seq 2048, bf16 weights, synthetic tokens).

Differences from the reference run, all in the reference's favour: bf16 weights instead of
fp16 (engine.py:132), fused torch AdamW (foreach) and no double loss scaling.  Prints one
JSON line with tokens/s so BASELINE.md §3 can record the measured baseline.
"""
import argparse, json, time
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--micro-batch", type=int, default=4)
ap.add_argument("--seq-len", type=int, default=2048)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--attn", default="sdpa", help="sdpa | eager")
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--prefill", action="store_true",
                help="serving TTFT as the reference server computes it: one fp16 full-prompt forward "
                     "(server.py:199-206) for a [1, seq_len] prompt, p50 over 10 runs")
a = ap.parse_args()

from transformers import LlamaConfig, LlamaForCausalLM

cfg = LlamaConfig(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=a.layers,
                  num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096,
                  rms_norm_eps=1e-5, tie_word_embeddings=False, attn_implementation=a.attn)
torch.manual_seed(0)
if a.prefill:
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg).to(torch.float16)  # reference loads fp16 (server.py:146-170)
    model.eval()
    ids = torch.randint(0, 32000, (1, a.seq_len), device="cuda")
    ts = []
    with torch.no_grad():
        for i in range(12):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            out = model(input_ids=ids, use_cache=True)
            nxt = out.logits[:, -1].argmax(-1).item()
            ts.append(time.perf_counter() - t0)
    ts = sorted(ts[2:])
    print(json.dumps({"stack": "hf-transformers-fp16-prefill", "attn": a.attn, "prompt_length": a.seq_len,
                      "ttft_forward_p50_ms": round(1000 * ts[len(ts) // 2], 2),
                      "ttft_forward_min_ms": round(1000 * ts[0], 2),
                      "note": "reference server adds up to 10 ms of polling (server.py:345-347) on top"}), flush=True)
    raise SystemExit(0)
with torch.device("cuda"):
    model = LlamaForCausalLM(cfg).to(torch.bfloat16)
model.train()
nparam = sum(p.numel() for p in model.parameters())
opt = torch.optim.AdamW(model.parameters(), lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
g = torch.Generator(device="cuda"); g.manual_seed(0)

def step():
    ids = torch.randint(0, 32000, (a.micro_batch, a.seq_len), device="cuda", generator=g)
    out = model(input_ids=ids, labels=ids)
    out.loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step(); opt.zero_grad(set_to_none=True)
    return out.loss.detach()

for _ in range(a.warmup):
    step()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(a.steps):
    l = step()
torch.cuda.synchronize(); dt = time.perf_counter() - t0
tps = a.micro_batch * a.seq_len * a.steps / dt
print(json.dumps({"stack": "hf-transformers-eager+torch-adamw", "attn": a.attn, "params": nparam,
                  "micro_batch": a.micro_batch, "seq_len": a.seq_len, "layers": a.layers,
                  "tokens_per_sec": round(tps, 1), "ms_per_step": round(1000 * dt / a.steps, 1),
                  "loss": float(l), "max_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}), flush=True)
