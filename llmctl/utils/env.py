"""Process / device environment helpers.

One process per GPU: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT come from
torchrun (or our own launcher, ``llmctl.runtime.launcher``).  On ROCm the HIP device is
exposed through the ``torch.cuda`` namespace and the ``"nccl"`` backend is RCCL.
"""

from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass


@dataclass(frozen=True)
class DistEnv:
    rank: int
    local_rank: int
    world_size: int
    master_addr: str
    master_port: int

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


def dist_env() -> DistEnv:
    return DistEnv(
        rank=int(os.environ.get("RANK", "0")),
        local_rank=int(os.environ.get("LOCAL_RANK", "0")),
        world_size=int(os.environ.get("WORLD_SIZE", "1")),
        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
        master_port=int(os.environ.get("MASTER_PORT", "29500")),
    )


def is_rocm_gpu_available() -> bool:
    try:
        import torch
    except Exception:  # pragma: no cover
        return False
    return bool(torch.cuda.is_available() and getattr(torch.version, "hip", None))


def local_device(prefer: str = "auto"):
    """Return the torch.device this process should compute on."""
    import torch

    if prefer == "cpu":
        return torch.device("cpu")
    if torch.cuda.is_available():
        return torch.device("cuda", dist_env().local_rank % max(torch.cuda.device_count(), 1))
    if prefer in ("cuda", "gpu", "hip"):
        raise RuntimeError("a GPU was requested but torch.cuda.is_available() is False")
    return torch.device("cpu")


def init_process_group(backend: str, **kw) -> None:
    """``torch.distributed.init_process_group`` that survives torchrun's elastic restarts.

    Under torchrun's static rendezvous the agent hosts ONE TCPStore for the whole job and hands
    it to every restart attempt unprefixed (``torch/distributed/rendezvous.py``: "We create a new
    TCPStore for every retry" -- not true for the static handler).  The restarted workers then
    read the dead attempt's keys: gloo's full-mesh bootstrap picks up a killed peer's listening
    address ("connectFullMesh failed ... Connection refused") and the store barrier counts stale
    arrivals.  Here every attempt gets its own key space, ``llmctl/attempt_<restart count>/``,
    on a client of the agent's store."""
    import datetime

    import torch.distributed as dist

    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and "store" not in kw:
        from torch.distributed import PrefixStore, TCPStore

        env = dist_env()
        timeout = kw.get("timeout") or datetime.timedelta(seconds=300)
        base = TCPStore(env.master_addr, env.master_port, env.world_size, is_master=False, timeout=timeout)
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        kw.update(store=PrefixStore(f"llmctl/attempt_{attempt}", base), rank=env.rank, world_size=env.world_size)
    dist.init_process_group(backend=backend, **kw)


def install_hang_dump() -> None:
    """``LLMCTL_HANG_DUMP=<seconds>``: every thread's Python stack goes to stderr after that many
    seconds (and again every period), so a hung rank names the call it is stuck in."""
    s = os.environ.get("LLMCTL_HANG_DUMP")
    if s:
        import faulthandler

        faulthandler.dump_traceback_later(float(s), repeat=True, exit=False)


@contextlib.contextmanager
def graph_capture_gc_guard():
    """Collect garbage before a hipGraph capture and keep the cyclic collector off during it.

    A collection inside a capture can run the destructor of an unrelated, unreachable engine
    whose captured graphs then free their executable graphs and pools on a capturing device;
    the runtime refuses that ("operation not permitted when stream is capturing") and the error
    raised inside a destructor aborts the process.  torch's ``torch.cuda.graph`` only collects
    beforehand under ``force_cudagraph_gc``."""
    import gc

    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
