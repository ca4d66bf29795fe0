"""Multi-process CPU (gloo) harness: run a function on N ranks and collect results."""

from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "OMP_NUM_THREADS": "1"})
    import torch

    torch.set_num_threads(1)
    from llmctl.utils.env import install_hang_dump

    install_hang_dump()  # debugging aid: LLMCTL_HANG_DUMP=<s> prints every rank's stacks after s seconds
    try:
        out = fn(rank, world, *args)
        import io

        buf = io.BytesIO()  # tensors by value: shared-memory handles die with the child
        torch.save(out, buf)
        q.put((rank, "ok", buf.getvalue()))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def run_ranks(fn, world: int, *args, timeout: float = 240.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    errors = []
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status == "ok":
                import io

                import torch

                results[rank] = torch.load(io.BytesIO(out), weights_only=True)
            else:
                errors.append(f"rank {rank}:\n{out}")
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    if errors:
        raise RuntimeError("\n".join(errors))
    return [results[r] for r in range(world)]
