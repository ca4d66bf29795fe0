"""Collective bandwidth benchmark (``llmctl bench comms``), nccl-tests conventions.

algbw = bytes / time; busbw = algbw × factor (all-reduce 2(n-1)/n, reduce-scatter /
all-gather (n-1)/n, all-to-all (n-1)/n, p2p 1).  Runs inside an existing process group
(torchrun) or spawns ``ranks`` local processes (one per GPU with RCCL over xGMI, or gloo on
CPU).  On an 8×MI355X node the all-reduce busbw is the number the planner's
``intra_node_bw_gbps`` should be calibrated with.
"""

from __future__ import annotations

import os
import re
import time
from typing import Any, Dict


def parse_size(s: str) -> int:
    m = re.fullmatch(r"\s*([\d.]+)\s*([KMGT]?)(i?B)?\s*", s, re.I)
    if not m:
        raise ValueError(f"bad size {s}")
    mult = {"": 1, "K": 2 ** 10, "M": 2 ** 20, "G": 2 ** 30, "T": 2 ** 40}[m.group(2).upper()]
    return int(float(m.group(1)) * mult)


def _factor(pattern: str, n: int) -> float:
    if pattern == "allreduce":
        return 2 * (n - 1) / n
    if pattern in ("reduce_scatter", "all_gather", "alltoall"):
        return (n - 1) / n
    return 1.0


def _bench_in_group(pattern: str, nbytes: int, iters: int) -> Dict[str, Any]:
    import torch
    import torch.distributed as dist

    rank, n = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    numel = max(nbytes // torch.tensor([], dtype=dtype).element_size(), n)
    numel -= numel % n
    x = torch.ones(numel, dtype=dtype, device=dev)
    out = torch.empty(numel // n, dtype=dtype, device=dev)
    full = torch.empty(numel, dtype=dtype, device=dev)

    def op():
        if pattern == "allreduce":
            dist.all_reduce(x)
        elif pattern == "reduce_scatter":
            dist.reduce_scatter_tensor(out, x)
        elif pattern == "all_gather":
            dist.all_gather_into_tensor(full, out)
        elif pattern == "alltoall":
            dist.all_to_all_single(full, x)
        elif pattern == "p2p":
            if rank % 2 == 0 and rank + 1 < n:
                dist.send(x, rank + 1)
            elif rank % 2 == 1:
                dist.recv(x, rank - 1)
        else:
            raise ValueError(pattern)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()

    for _ in range(3):
        op()
    sync()
    t = time.perf_counter()
    for _ in range(iters):
        op()
    sync()
    dt = (time.perf_counter() - t) / iters
    size = numel * x.element_size()
    algbw = size / dt / 1e9
    return {"pattern": pattern, "ranks": n, "bytes": size, "backend": dist.get_backend(), "time_ms": dt * 1e3,
            "algbw_gbps": round(algbw, 2), "busbw_gbps": round(algbw * _factor(pattern, n), 2)}


def _worker(rank, world, pattern, nbytes, iters, backend):
    import torch
    import torch.distributed as dist

    if backend == "nccl":
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group("gloo")
    return _bench_in_group(pattern, nbytes, iters)


def run_comms_benchmark(pattern: str = "allreduce", nbytes: int = 2 ** 30, ranks: int = 2, iters: int = 20,
                        backend: str = "auto") -> Dict[str, Any]:
    import torch
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return _bench_in_group(pattern, nbytes, iters)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        be = "nccl" if torch.cuda.is_available() else "gloo"
        if be == "nccl":
            lr = int(os.environ.get("LOCAL_RANK", 0))
            torch.cuda.set_device(lr)
            dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
        else:
            dist.init_process_group("gloo")
        return _bench_in_group(pattern, nbytes, iters)
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() and torch.cuda.device_count() >= ranks else "gloo"
    if backend == "gloo":
        nbytes = min(nbytes, 64 * 2 ** 20)  # keep CPU runs short
    from llmctl.testing.harness import run_ranks

    res = run_ranks(_worker, ranks, pattern, nbytes, iters, backend, timeout=600)
    return res[0]
