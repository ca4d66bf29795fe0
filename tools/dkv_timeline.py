#!/usr/bin/env python3
"""Per-workgroup timeline of the pipelined dK/dV kernel (fa_bwd_ablate abl 5: s_memrealtime stamps,
100 MHz): prologue / tile loop / epilogue durations, per-tile loop time, and the gaps between
consecutive workgroups on one CU (dispatch + launch cost).   dkv_timeline.py [B S H D]"""
import json
import sys
from collections import defaultdict

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from llmctl.ops import _lib  # noqa: E402

ops = _lib.native()
B, S, H, D = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (12, 2048, 32, 128)))
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k, v, do = (torch.randn_like(q) for _ in range(3))
o, lse = ops.flash_attn_fwd(q, k, v, D ** -0.5, True)
delta = (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(5):
    ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, 4)
ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, 5)
torch.cuda.synchronize()
nwg = B * H * ((S + 127) // 128)
st = dq.reshape(-1).view(torch.int64)[: nwg * 8].view(nwg, 8).cpu().tolist()
t0 = min(r[0] for r in st)
us = lambda x: x / 100.0  # 100 MHz ticks -> us
pro = [us(r[2] - r[0]) for r in st]
loop = [us(r[3] - r[2]) for r in st]
epi = [us(r[4] - r[3]) for r in st]
per_tile = [us(r[3] - r[2]) / r[5] for r in st if r[5] > 0]
span = us(max(r[4] for r in st) - t0)
cu = defaultdict(list)
for r in st:
    hw, xcc = r[1] & 0xFFFFFFFF, r[1] >> 32
    cu[(xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)].append((r[0], r[4]))
gaps = []
for v in cu.values():
    v.sort()
    gaps += [us(b[0] - a[1]) for a, b in zip(v, v[1:])]
busy = sum(us(e - s) for v in cu.values() for s, e in v)
mean = lambda x: sum(x) / max(len(x), 1)
pct = lambda x, p: sorted(x)[int(p * (len(x) - 1))] if x else 0
res = {"shape": [B, S, H, D], "workgroups": nwg, "cus_seen": len(cu), "span_us": round(span, 1),
       "busy_fraction": round(busy / (len(cu) * span), 3),
       "prologue_us": [round(mean(pro), 2), round(pct(pro, 0.9), 2)],
       "loop_us_per_tile": [round(mean(per_tile), 3), round(pct(per_tile, 0.1), 3), round(pct(per_tile, 0.9), 3)],
       "epilogue_us": [round(mean(epi), 2), round(pct(epi, 0.9), 2)],
       "gap_between_wgs_us": [round(mean(gaps), 2), round(pct(gaps, 0.5), 2), round(pct(gaps, 0.9), 2)],
       "last_start_us": round(us(max(r[0] for r in st) - t0), 1)}
print(json.dumps(res), flush=True)

# ---- persistent kernel (abl 7): per item [start, loop done, epilogue done, item id], 64 per workgroup
ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, 6)
dq.zero_()
ops.fa_bwd_ablate(do, q, k, v, delta, lse, dq, dk, dv, 7)
torch.cuda.synchronize()
ncu = 256
st = dq.reshape(-1).view(torch.int64)[: ncu * 64 * 4].view(ncu, 64, 4).cpu().tolist()
items = [(w, i, r) for w in range(ncu) for i, r in enumerate(st[w]) if r[0] > 0]
t0 = min(r[0] for _, _, r in items)
loops = [us(r[1] - r[0]) for _, _, r in items]
epis = [us(r[2] - r[1]) for _, _, r in items]
gaps = [us(st[w][i + 1][0] - st[w][i][2]) for w, i, r in items if i + 1 < 64 and st[w][i + 1][0] > 0]
ends = [us(max(r[2] for r in st[w] if r[0] > 0) - t0) for w in range(ncu) if st[w][0][0] > 0]
nkb = S // 128
tiles = [(S // 64 - 2 * (r[3] % nkb)) for _, _, r in items]
print(json.dumps({"persistent": True, "items": len(items), "span_us": round(max(ends), 1),
                  "wg_end_us_min_mean_max": [round(min(ends), 1), round(mean(ends), 1), round(max(ends), 1)],
                  "loop_us_per_tile": round(sum(loops) / sum(tiles), 3), "epilogue_us": [round(mean(epis), 2), round(pct(epis, 0.9), 2)],
                  "gap_between_items_us": [round(mean(gaps), 2), round(pct(gaps, 0.9), 2)]}), flush=True)
