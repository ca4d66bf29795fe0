"""Probe: can two ranks share the one GPU of the test box over RCCL?  (all_reduce,
reduce_scatter_tensor, all_gather_into_tensor, all_to_all_single).

Result on the pool (RCCL 2.26.6): no — "Duplicate GPU detected"; multi-rank paths are
covered by the gloo CPU tests and the custom IPC all-reduce two-process GPU test instead."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(x)
rs = torch.empty(512, device="cuda")
dist.reduce_scatter_tensor(rs, torch.arange(1024, device="cuda", dtype=torch.float32))
ag = torch.empty(2048, device="cuda")
dist.all_gather_into_tensor(ag, x)
a2a = torch.empty(1024, device="cuda")
dist.all_to_all_single(a2a, torch.full((1024,), float(rank), device="cuda"))
torch.cuda.synchronize()
print(f"rank {rank}: allreduce {x[0].item()} rs {rs[0].item()} ag {ag.sum().item()} a2a {a2a[0].item()},{a2a[-1].item()}",
      flush=True)
dist.destroy_process_group()
