"""Process-group construction from a parallelism plan (TP × CP × DP × PP).

Rank layout (global rank r): TP is the fastest-varying dimension, then CP (context
parallel), then DP, then PP:

    r = pp_rank * (dp * cp * tp) + dp_rank * (cp * tp) + cp_rank * tp + tp_rank

so a TP group is ``tp`` consecutive local ranks — on an 8×MI355X node those GPUs are all
xGMI peers (fully connected K8), which is where the latency-critical per-layer TP
collectives must live; the per-layer CP all-to-alls come next.  Gradients are reduced over
the combined DP×CP group (``dpcp``: every rank holding the same parameters).  The same
function also produces the explicit rank lists that ``plan compute`` writes into the plan's
``[shard_map]`` section.

Expert parallelism (MoE) lives inside DP: each DP group is cut into blocks of ``ep``
consecutive DP ranks (an *EP group*, the all-to-all domain: on one node these are xGMI peers);
rank ``j`` of every block holds the same expert shard, and those ranks form the *expert-DP*
group over which the experts' gradients are reduced.
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
    cp: int = 1
    ep: int = 1  # expert parallel degree (divides dp)

    def __post_init__(self):
        if self.tp * self.pp * self.dp * self.cp != self.world_size:
            raise ValueError(f"tp({self.tp})*cp({self.cp})*pp({self.pp})*dp({self.dp}) != "
                             f"world_size({self.world_size})")
        if self.ep < 1 or self.dp % self.ep:
            raise ValueError(f"expert_parallel={self.ep} must divide dp={self.dp}")

    def coords4(self, rank: int):
        tp_rank = rank % self.tp
        cp_rank = (rank // self.tp) % self.cp
        dp_rank = (rank // (self.tp * self.cp)) % self.dp
        pp_rank = rank // (self.tp * self.cp * self.dp)
        return tp_rank, cp_rank, dp_rank, pp_rank

    def coords(self, rank: int):
        t, _, d, p = self.coords4(rank)
        return t, d, p

    def rank_of(self, tp_rank: int, dp_rank: int, pp_rank: int, cp_rank: int = 0) -> int:
        return ((pp_rank * self.dp + dp_rank) * self.cp + cp_rank) * self.tp + tp_rank

    def _all(self):
        return [(t, c, d, p) for p in range(self.pp) for d in range(self.dp) for c in range(self.cp)
                for t in range(self.tp)]

    def _groups(self, key):
        out: Dict[tuple, List[int]] = {}
        for t, c, d, p in self._all():
            out.setdefault(key(t, c, d, p), []).append(self.rank_of(t, d, p, c))
        return list(out.values())

    def tp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (c, d, p))

    def cp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, d, p))

    def dp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, c, p))

    def dpcp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, p))

    def pp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, c, d))

    def ep_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, c, p, d // self.ep))

    def edp_groups(self) -> List[List[int]]:
        return self._groups(lambda t, c, d, p: (t, c, p, d % self.ep))

    def shard_map(self) -> Dict[str, List[List[int]]]:
        m = {"tp_groups": self.tp_groups(), "dp_groups": self.dp_groups(), "pp_groups": self.pp_groups()}
        if self.cp > 1:
            m["cp_groups"] = self.cp_groups()
        if self.ep > 1:
            m["ep_groups"] = self.ep_groups()
            m["expert_dp_groups"] = self.edp_groups()
        return m


@dataclass
class ProcessGroups:
    layout: ParallelLayout
    rank: int
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    pp_group: Optional[object] = None
    cp_group: Optional[object] = None
    dpcp_group: Optional[object] = None  # gradient-reduction group (== dp_group when cp == 1)
    ep_group: Optional[object] = None  # MoE all-to-all group
    edp_group: Optional[object] = None  # expert-gradient reduction group
    embed_group: Optional[object] = None  # {first, last} pipeline stage: tied-embedding grads
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

    @property
    def cp_rank(self):
        return self.layout.coords4(self.rank)[1]

    @property
    def ep_rank(self):
        return self.dp_rank % self.layout.ep


def build_process_groups(tp: int = 1, pp: int = 1, dp: Optional[int] = None, cp: int = 1,
                         ep: int = 1) -> ProcessGroups:
    """Create TP/CP/DP/PP groups.  Every rank must call this with identical arguments (group
    creation is collective)."""
    if dist.is_initialized():
        world, rank = dist.get_world_size(), dist.get_rank()
    else:
        world, rank = 1, 0
    if dp is None:
        dp = world // (tp * pp * cp)
    layout = ParallelLayout(world, tp=tp, pp=pp, dp=dp, cp=cp, ep=ep)
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
    if cp > 1:
        pg.cp_group = make(layout.cp_groups())
        pg.dpcp_group = make(layout.dpcp_groups())
    else:
        pg.dpcp_group = pg.dp_group
    if ep > 1:
        pg.ep_group = make(layout.ep_groups())
        pg.edp_group = make(layout.edp_groups())
    for ranks in layout.pp_groups():
        if rank in ranks:
            pg.pp_ranks = ranks
    if pp > 1:
        # Megatron-style embedding group: the first and last stage of each pipeline hold the
        # two copies of a tied embedding / LM-head matrix and sum their gradients here
        pg.embed_group = make([[r[0], r[-1]] for r in layout.pp_groups()])
    return pg
