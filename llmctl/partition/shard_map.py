"""Shard maps: which layers / TP shards / ZeRO partitions / process groups each rank owns.

The reference planner emits only degrees (``plan.py:341-358``); SURVEY §2.4 asks for a
``[shard_map]`` section.  :func:`build_shard_map` produces it, and the runtime consumes the
same functions (``split_layers`` is what ``TrainingEngine`` uses to cut pipeline stages), so
a plan file is an exact description of the run.
"""

from __future__ import annotations

from typing import Any, Dict, List, Tuple

from llmctl.parallel.groups import ParallelLayout


def split_layers(num_layers: int, pp: int) -> List[Tuple[int, int]]:
    """Contiguous balanced split; the first/last stages (embedding / lm_head) get the
    remainder last so they are never the heaviest."""
    base, rem = divmod(num_layers, pp)
    sizes = [base] * pp
    # give remainder layers to the middle stages first
    order = list(range(1, pp - 1)) + [0, pp - 1] if pp > 2 else list(range(pp))
    for i in range(rem):
        sizes[order[i % len(order)]] += 1
    out, s = [], 0
    for n in sizes:
        out.append((s, s + n))
        s += n
    return out


def build_shard_map(model: Dict[str, Any], tp: int, pp: int, dp: int, zero_stage: int,
                    virtual_stages: int = 1) -> Dict[str, Any]:
    """Per-rank shard description.  With ``virtual_stages`` V > 1 (interleaved pipeline) the
    layers are cut into pp*V chunks and pipeline rank p owns chunks p, p + pp, ... — its
    ``layers`` entry then lists every [start, end) range it holds."""
    L = int(model.get("layers", 32))
    heads = int(model.get("heads", 32))
    kv = int(model.get("kv_heads", heads) or heads)
    ffn = int(model.get("ffn", 4 * int(model.get("hidden", 4096))))
    vocab = int(model.get("vocab_size", 32000))
    layout = ParallelLayout(tp * pp * dp, tp=tp, pp=pp, dp=dp)
    V = max(int(virtual_stages), 1) if pp > 1 else 1
    stages = split_layers(L, pp * V)
    ranks = []
    for r in range(layout.world_size):
        t, d, p = layout.coords(r)
        mine = [list(stages[v * pp + p]) for v in range(V)]
        ranks.append({
            "rank": r, "tp_rank": t, "dp_rank": d, "pp_rank": p,
            "layers": mine[0] if V == 1 else mine,
            "q_heads": [t * heads // tp, (t + 1) * heads // tp],
            "kv_heads": [t * kv // tp, (t + 1) * kv // tp],
            "ffn": [t * ffn // tp, (t + 1) * ffn // tp],
            "vocab": [t * vocab // tp, (t + 1) * vocab // tp],
            "embedding": p == 0, "lm_head": p == pp - 1,
            "zero_partition": [d, dp] if zero_stage >= 1 else None,
        })
    sm = layout.shard_map()
    sm["stages"] = [list(s) for s in stages]
    sm["virtual_stages"] = V
    sm["ranks"] = ranks
    return sm
