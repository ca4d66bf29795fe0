"""Process-group construction from a parallelism plan (TP × DP × PP [× CP]).

Rank layout (global rank r): TP is the fastest-varying dimension, then DP, then PP:

    r = pp_rank * (dp * tp) + dp_rank * tp + tp_rank

so a TP group is ``tp`` consecutive local ranks — on an 8×MI355X node those GPUs are all
xGMI peers (fully connected K8), which is where the latency-critical per-layer TP
collectives must live.  DP groups stride by ``tp`` and PP groups by ``tp*dp``.  The same
function also produces the explicit rank lists that ``plan compute`` writes into the plan's
``[shard_map]`` section.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch.distributed as dist


@dataclass
class ParallelLayout:
    world_size: int
    tp: int = 1
    pp: int = 1
    dp: int = 1

    def __post_init__(self):
        if self.tp * self.pp * self.dp != self.world_size:
            raise ValueError(f"tp({self.tp})*pp({self.pp})*dp({self.dp}) != world_size({self.world_size})")

    def coords(self, rank: int):
        tp_rank = rank % self.tp
        dp_rank = (rank // self.tp) % self.dp
        pp_rank = rank // (self.tp * self.dp)
        return tp_rank, dp_rank, pp_rank

    def rank_of(self, tp_rank: int, dp_rank: int, pp_rank: int) -> int:
        return pp_rank * (self.dp * self.tp) + dp_rank * self.tp + tp_rank

    def tp_groups(self) -> List[List[int]]:
        return [[self.rank_of(t, d, p) for t in range(self.tp)] for p in range(self.pp) for d in range(self.dp)]

    def dp_groups(self) -> List[List[int]]:
        return [[self.rank_of(t, d, p) for d in range(self.dp)] for p in range(self.pp) for t in range(self.tp)]

    def pp_groups(self) -> List[List[int]]:
        return [[self.rank_of(t, d, p) for p in range(self.pp)] for d in range(self.dp) for t in range(self.tp)]

    def shard_map(self) -> Dict[str, List[List[int]]]:
        return {"tp_groups": self.tp_groups(), "dp_groups": self.dp_groups(), "pp_groups": self.pp_groups()}


@dataclass
class ProcessGroups:
    layout: ParallelLayout
    rank: int
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    pp_group: Optional[object] = None
    pp_ranks: List[int] = field(default_factory=list)

    @property
    def tp_rank(self):
        return self.layout.coords(self.rank)[0]

    @property
    def dp_rank(self):
        return self.layout.coords(self.rank)[1]

    @property
    def pp_rank(self):
        return self.layout.coords(self.rank)[2]


def build_process_groups(tp: int = 1, pp: int = 1, dp: Optional[int] = None) -> ProcessGroups:
    """Create TP/DP/PP groups.  Every rank must call this with identical arguments (group
    creation is collective)."""
    if dist.is_initialized():
        world, rank = dist.get_world_size(), dist.get_rank()
    else:
        world, rank = 1, 0
    if dp is None:
        dp = world // (tp * pp)
    layout = ParallelLayout(world, tp=tp, pp=pp, dp=dp)
    pg = ProcessGroups(layout=layout, rank=rank)
    if world == 1:
        pg.pp_ranks = [0]
        return pg

    def make(groups):
        mine = None
        for ranks in groups:
            g = dist.new_group(ranks) if len(ranks) > 1 else None
            if rank in ranks:
                mine = g
        return mine

    pg.tp_group = make(layout.tp_groups())
    pg.dp_group = make(layout.dp_groups())
    pg.pp_group = make(layout.pp_groups())
    for ranks in layout.pp_groups():
        if rank in ranks:
            pg.pp_ranks = ranks
    return pg
