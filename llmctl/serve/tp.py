"""Tensor-parallel serving: one process per GPU, Megatron TP over RCCL (BASELINE config
"``llmctl serve`` GPT-7B paged-attention + dynamic batching, TP=8").

The reference serves from one process with an HF model (``server.py:127-251``) and has no
model parallelism.  Here every rank holds a TP shard of the weights:
  * column-parallel QKV / gate-up, row-parallel o-proj / down-proj (one all-reduce each),
  * a vocab-parallel embedding (all-reduce) and LM head (all-gather of the logits),
  * its own paged KV cache for its ``kv_heads / tp`` heads (the block tables are shared).

Control plane: rank 0 owns the scheduler, the KV block manager, sampling and (for ``llmctl
serve``) the HTTP server.  For every engine step it broadcasts a small host-side *plan*
(token ids, positions, KV slots, block tables) over a gloo group; all ranks then execute the
same step, so every rank posts the identical RCCL sequence.  Ranks != 0 run
:meth:`TPInferenceEngine.worker_loop` until rank 0 broadcasts ``stop``.

Decode-step hipGraph capture stays on for TP (the collectives are captured with the
rest) unless knob ``tp_graphs`` is off.  Decode-sized all-reduces (<= 4 MB) use the one-shot
xGMI peer-memory kernel (:mod:`llmctl.comms.custom_ar`) unless knob ``custom_ar`` is off.
"""

from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from llmctl.models import ParallelContext
from llmctl.utils.env import dist_env

from .engine import InferenceEngine
from .scheduler import PrefillChunk, Sequence

log = logging.getLogger("llmctl.serve.tp")


class TPInferenceEngine(InferenceEngine):
    def __init__(self, model_path: str = "tiny", tp_group=None, control_group=None, **kw):
        if not dist.is_initialized():
            raise RuntimeError("TPInferenceEngine needs torch.distributed (launch with torchrun)")
        self.tp_group = tp_group
        self.tp_size = dist.get_world_size(tp_group)
        self.tp_rank = dist.get_rank(tp_group)
        self._own_control = control_group is None
        self.control = control_group if control_group is not None else dist.new_group(backend="gloo")
        self._closed = False
        self._car_checks = 0
        # plan channel (created on first use by every rank in the same order): "auto" = shm ring
        # on one node, gloo tensors otherwise; "tensor" / "shm" force one
        self.control_kind = kw.pop("control", "auto")
        # liveness deadline of the shm plan ring (a frozen peer; a dead one is seen within ~50 ms)
        self.control_timeout_s = float(kw.pop("control_timeout_s", 600.0))
        self.channel = None
        pc = ParallelContext(tp_group=tp_group, tp_size=self.tp_size, tp_rank=self.tp_rank)
        # this engine's own knobs (perf_knobs + LLMCTL_KNOBS) decide, not whatever is active
        from llmctl.config.knobs import resolve

        if kw.get("use_graphs", True) and not resolve(kw.get("perf_knobs")).tp_graphs:
            kw["use_graphs"] = False
        self.car = None
        super().__init__(model_path, pc=pc, **kw)
        # decode-sized all-reduces go through the one-shot xGMI kernel (llmctl.comms.custom_ar);
        # prefill-sized ones and CPU runs stay on RCCL / gloo
        if (self.device.type == "cuda" and self.tp_size > 1
                and self.knobs.custom_ar):
            from llmctl.comms.custom_ar import CustomAllReduce

            # one-shot up to 4 MB (decode), two-shot up to 32 MB (2k-token prefill chunks at d = 8192)
            self.car = CustomAllReduce(self.tp_group, max_bytes=4 << 20, device=self.device, twoshot_bytes=32 << 20)

    # ------------------------------------------------------------------ TP hooks
    def _load(self, model_path: str, dtype, seed: int):
        """Checkpoints are resharded by ``load_model``; random-init templates are built whole
        (same seed on every rank) and sliced, so TP=N serves exactly the TP=1 model."""
        from llmctl.io.artifact import load_model, resolve_checkpoint_dir
        from llmctl.io.checkpoint import _global_name, shard_tp
        from llmctl.models import build_model, get_model_config

        if resolve_checkpoint_dir(model_path) is not None:
            return load_model(model_path, device=self.device, dtype=dtype, pc=self.pc, seed=seed)
        cfg = get_model_config(model_path)
        full = build_model(cfg, device=self.device, dtype=dtype, seed=seed)
        model = build_model(cfg, device=self.device, dtype=dtype, pc=self.pc, seed=seed)
        src = dict(full.named_parameters())
        with torch.no_grad():
            for n, p in model.named_parameters():
                g = _global_name(n, 0)
                p.copy_(shard_tp(g, src[n].detach(), self.tp_size, self.tp_rank, cfg))
        del full, src
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        return model, cfg, None

    def _agree_min(self, n: int) -> int:
        t = torch.tensor([n], dtype=torch.long)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.control)
        return int(t.item())

    def _reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.car is not None and (self.car.eligible(x) or self.car.twoshot_eligible(x)):
            return self.car.all_reduce(x)
        dist.all_reduce(x, group=self.tp_group)
        return x

    def _fused_reduce_ok(self) -> bool:
        return self.car is not None and self.knobs.tp_fused_decode

    def _reduce_add_rmsnorm(self, part, bias, res, norm_w, eps):
        """One kernel (``car_allreduce_add_rmsnorm``): the row-parallel partials' all-reduce, the
        bias, the residual add and the next sub-layer's RMSNorm; RCCL + add_rmsnorm when the
        message does not fit the one-shot buffer (or under gloo on CPU)."""
        if (self.car is not None and self.car.eligible(part) and part.dim() == 2 and part.shape[1] <= 16384
                and part.numel() * 2 <= self.car.max_bytes):
            return self.car.all_reduce_add_rmsnorm(part, bias, res, norm_w, eps)
        y = self._reduce(part)
        if bias is not None:
            y = y + bias
        from llmctl import ops

        return ops.add_rmsnorm(y, res, norm_w, eps)

    def _gather_vocab(self, logits: torch.Tensor) -> torch.Tensor:
        n, vl = logits.shape
        if self.car is not None and logits.dtype == torch.bfloat16 and self.tp_size * n * vl * 2 <= self.car.max_bytes:
            # all-gather as a sum of zero-padded slots through the one-shot IPC kernel: unlike the
            # RCCL / gloo all-gather it is hipGraph-capturable in every backend configuration
            buf = torch.zeros(self.tp_size, n, vl, dtype=logits.dtype, device=logits.device)
            buf[self.tp_rank].copy_(logits)
            self.car.all_reduce(buf)
            return buf.permute(1, 0, 2).reshape(n, self.tp_size * vl)
        out = torch.empty(self.tp_size * n, vl, dtype=logits.dtype, device=logits.device)
        dist.all_gather_into_tensor(out, logits.contiguous(), group=self.tp_group)
        return out.view(self.tp_size, n, vl).permute(1, 0, 2).reshape(n, self.tp_size * vl)

    # ------------------------------------------------------------------ control plane
    def _bcast(self, plan: Optional[Dict]) -> Dict:
        """Rank 0's plan to every TP rank: packed record through the shared-memory ring
        (``llmctl.serve.control``; gloo tensors across nodes), no pickle on the hot path."""
        if self.channel is None:
            from llmctl.serve.control import make_channel

            self.channel = make_channel(self.control, self.control_kind, timeout_s=self.control_timeout_s)
        if self.tp_rank == 0:
            self.channel.publish(plan)
            return plan
        return self.channel.receive()

    @torch.inference_mode()
    def prefill(self, chunks) -> torch.Tensor:
        if chunks and isinstance(chunks[0], Sequence):
            chunks = [PrefillChunk(s, 0, s.num_tokens) for s in chunks]
        return self.prefill_exec(self._bcast(self.prefill_plan(chunks)))

    @torch.inference_mode()
    def decode(self, seqs: List[Sequence]) -> torch.Tensor:
        out = self.decode_exec(self._bcast(self.decode_plan(seqs)))
        self._car_checks += 1
        if self.car is not None and self._car_checks % self.CAR_CHECK_EVERY == 0:
            self.car.check()  # a peer timed out inside the custom all-reduce: fail loudly, never serve it
        return out

    CAR_CHECK_EVERY = 64  # decode steps between reads of the custom all-reduce's error word (one D2H copy)

    def _publish(self, plan: Dict) -> Dict:
        return self._bcast(plan)

    @torch.inference_mode()
    def _decode_sample_exec(self, plan: Dict) -> torch.Tensor:
        toks = super()._decode_sample_exec(plan)
        self._car_checks += 1
        if self.car is not None and self._car_checks % self.CAR_CHECK_EVERY == 0:
            self.car.check()
        return toks

    @torch.inference_mode()
    def mixed(self, chunks, seqs: List[Sequence]) -> torch.Tensor:
        return self.mixed_exec(self._bcast(self.mixed_plan(chunks, seqs)))

    def stop_workers(self) -> None:
        if self.tp_rank == 0:
            self._bcast({"op": "stop"})
        self.release_graphs()

    def close(self) -> None:
        """Deterministic teardown, never left to garbage collection: drop the captured decode
        graphs (they hold the RCCL communicator's captured work and the custom all-reduce's peer
        pointers), drain the device, check + unmap the custom all-reduce buffers after a barrier
        (no peer may still be reading this rank's IPC memory) and destroy the gloo control group
        this engine created.  Call after :meth:`stop_workers` (rank 0) / :meth:`worker_loop`
        returned (other ranks); the default process group stays the caller's."""
        if self._closed:
            return
        self._closed = True
        self.release_graphs()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        err = None
        if self.car is not None:
            try:
                self.car.check()
            except RuntimeError as e:
                err = e
            dist.barrier(group=self.control)
            self.car.close()
            self.car = None
        if self.channel is not None:
            self.channel.close()
            self.channel = None
        if self._own_control and self.control is not None:
            dist.destroy_process_group(self.control)
        self.control = None
        self._release_resources()
        if err is not None:
            raise err

    @torch.inference_mode()
    def worker_loop(self) -> None:
        """Ranks != 0: execute rank 0's plans until it broadcasts ``stop``."""
        while True:
            plan = self._bcast(None)
            op = plan["op"]
            if op == "stop":
                self.release_graphs()
                return
            if op == "prefill":
                self.prefill_exec(plan)
            elif op == "decode_s":  # async pipeline: decode + in-graph sampling, ids stay on the device
                self._decode_sample_exec(plan)
            elif op == "decode":
                self.decode_exec(plan)
            elif op == "mixed":
                self.mixed_exec(plan)
            else:
                raise RuntimeError(f"unknown TP plan op {op!r}")


def init_tp(backend: str = "auto"):
    """Initialise the default process group from torchrun's env; returns (tp_group, device)."""
    env = dist_env()
    if not dist.is_initialized():
        if backend == "auto":
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(env.local_rank)
        from llmctl.utils.env import init_process_group

        init_process_group(backend)
    dev = f"cuda:{env.local_rank}" if torch.cuda.is_available() else "cpu"
    return None, dev  # the whole world is one TP group (one node, TP <= 8)


def main(argv=None) -> int:
    """``python -m torch.distributed.run --nproc-per-node N -m llmctl.serve.tp --artifact ...``"""
    import argparse

    ap = argparse.ArgumentParser("llmctl.serve.tp")
    ap.add_argument("--artifact", default="gpt-7b")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--max-batch-size", type=int, default=8)
    ap.add_argument("--max-batch-tokens", type=int, default=8192)
    ap.add_argument("--max-concurrent", type=int, default=128)
    ap.add_argument("--kv-cache-fraction", type=float, default=0.85)
    ap.add_argument("--block-size", type=int, default=16)
    ap.add_argument("--scheduler", default="dynamic")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-cache-dtype", default="auto")
    ap.add_argument("--weight-dtype", default="auto")
    ap.add_argument("--control-timeout", type=float, default=600.0,
                    help="seconds a frozen TP peer may stop heart-beating before the others exit")
    a = ap.parse_args(argv)
    group, dev = init_tp()
    eng = TPInferenceEngine(a.artifact, tp_group=group, device=dev, max_batch_size=a.max_batch_size,
                            max_batch_tokens=a.max_batch_tokens, kv_cache_fraction=a.kv_cache_fraction,
                            block_size=a.block_size, scheduler=a.scheduler, use_graphs=not a.no_graphs,
                            kv_cache_dtype=a.kv_cache_dtype, weight_dtype=a.weight_dtype,
                            control_timeout_s=a.control_timeout)
    from .control import PeerLostError

    if eng.tp_rank != 0:
        try:
            eng.worker_loop()
        except PeerLostError as e:
            # a peer is gone: leave non-zero at once (a teardown through the broken group could
            # hang) so torchrun sees the failure and stops the rest of the group
            log.error("%s", e)
            logging.shutdown()
            os._exit(70)
        eng.close()
        dist.destroy_process_group()
        return 0
    from .server import InferenceServer

    try:
        InferenceServer(a.artifact, host=a.host, port=a.port, max_batch_size=a.max_batch_size,
                        max_batch_tokens=a.max_batch_tokens, max_concurrent=a.max_concurrent, engine=eng).run()
    finally:
        eng.stop_workers()
        eng.close()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
