"""Sharded, asynchronous checkpointing with resharding on load.

Reference layout (``engine.py:363-394``) is kept and extended::

    <output_dir>/checkpoint-<step>/ | final/
        model.safetensors                       (tp=pp=1)  or
        model-0000r-of-0000N.safetensors + model.safetensors.index.json   (one per TP×PP shard)
        config.json                             (model JSON; absent in the reference)
        training_state.json                     {"global_step","epoch","config", + scheduler,
                                                 consumed_samples, world_size, layout, data}
        optimizer/rank_XXXXX.pt                 fp32 master + Adam moments (ZeRO shard)
        rng/rank_XXXXX.pt
        plan.toml                               (when a plan drove the run)
    <output_dir>/latest                         name of the newest complete checkpoint

Tensor names are layout-independent: ``layers.<global_idx>.<param>`` with full (unsharded)
shapes recorded in the index, so a checkpoint written at TP=a/PP=b loads at TP=c/PP=d
(:func:`consolidate_tp` / :func:`shard_tp`).  Writes are rank-parallel (each TP×PP shard
owner at DP rank 0 writes its model file, every rank its optimizer shard), done on a
background thread after a device→pinned-host copy, and committed by a barrier + ``latest``
pointer update (``keep_latest`` GC as in the reference config ``checkpoint.keep_latest``).
"""

from __future__ import annotations

import json
import os
import shutil
import threading
import time
from pathlib import Path
from typing import Any, Dict, List, Optional

import logging

import torch
import torch.distributed as dist

log = logging.getLogger("llmctl.io.checkpoint")

# ----------------------------------------------------------------------------- TP (re)sharding
# how each parameter is split across tensor-parallel ranks
#   ("rows", parts)  - dim 0, each rank's block is the concat of `parts` sub-blocks
#   ("cols", 1)      - dim 1
#   None             - replicated


def tp_split_rule(name: str, cfg) -> Optional[tuple]:
    leaf = name.split(".")[-1]
    if leaf in ("wqkv", "bqkv"):
        return ("rows", (cfg.heads, cfg.kv_heads, cfg.kv_heads))
    if leaf in ("w_up", "b_up"):
        return ("rows", (1, 1) if cfg.gated_mlp else (1,))
    if leaf in ("embed", "lm_head"):
        return ("rows", (1,))
    if leaf in ("wo", "w_down"):
        return ("cols", None)
    return None


def consolidate_tp(name: str, shards: List[torch.Tensor], cfg) -> torch.Tensor:
    rule = tp_split_rule(name, cfg)
    if rule is None or len(shards) == 1:
        return shards[0]
    kind, parts = rule
    if kind == "cols":
        return torch.cat(shards, dim=1)
    weights = parts
    tot = sum(weights)
    pieces: List[List[torch.Tensor]] = [[] for _ in weights]
    for s in shards:
        n = s.shape[0]
        unit = n // tot
        o = 0
        for i, w in enumerate(weights):
            pieces[i].append(s[o:o + unit * w])
            o += unit * w
    return torch.cat([torch.cat(p, 0) for p in pieces], 0)


def shard_tp(name: str, full: torch.Tensor, tp: int, rank: int, cfg) -> torch.Tensor:
    rule = tp_split_rule(name, cfg)
    if rule is None or tp == 1:
        return full
    kind, parts = rule
    if kind == "cols":
        n = full.shape[1] // tp
        return full[:, rank * n:(rank + 1) * n]
    tot = sum(parts)
    unit_full = full.shape[0] // tot
    out, o = [], 0
    for w in parts:
        blk = full[o:o + unit_full * w]
        n = blk.shape[0] // tp
        out.append(blk[rank * n:(rank + 1) * n])
        o += unit_full * w
    return torch.cat(out, 0)


def _global_name(name: str, layer_start) -> str:
    """"layers.<local>.x" -> "layers.<global>.x"; ``layer_start`` is the offset of one
    contiguous layer range or the list of global layer ids (``ParallelContext.layer_index``)."""
    if name.startswith("layers."):
        parts = name.split(".")
        i = int(parts[1])
        parts[1] = str(layer_start[i] if isinstance(layer_start, (list, tuple)) else i + layer_start)
        return ".".join(parts)
    return name


def _local_name(name: str, layer_start) -> str:
    if name.startswith("layers."):
        parts = name.split(".")
        g = int(parts[1])
        parts[1] = str(list(layer_start).index(g) if isinstance(layer_start, (list, tuple)) else g - layer_start)
        return ".".join(parts)
    return name


# ----------------------------------------------------------------------------- manager
class CheckpointManager:
    def __init__(self, engine, output_dir: str):
        self.engine = engine
        self.root = Path(output_dir)
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None

    # ------------------------------------------------------------------ save
    def save(self, name: str, final: bool = False) -> Path:
        e = self.engine
        c = e.config
        self.wait()
        path = self.root / name
        pg = e.pg
        rank = pg.rank
        world = pg.layout.world_size
        # save id: markers from an earlier, interrupted save of the same checkpoint (a rank killed
        # mid-write, then an elastic restart that saves this step again) carry another id and are
        # never counted toward this save's commit
        save_id = f"{e.global_step}:{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}:{os.environ.get('TORCHELASTIC_RUN_ID', '')}"
        # every rank writes into a sibling staging directory; rank 0's commit renames it over
        # ``path`` once complete, so re-saving an existing name never leaves it half-overwritten
        final_path = path
        path = self.root / f".{name}.staging"
        if e.is_main:
            # before the barrier, so no rank of this save has written into it yet: the leftovers of
            # an interrupted save (stale shards, markers) must not survive into this one
            shutil.rmtree(path, ignore_errors=True)
            path.mkdir(parents=True, exist_ok=True)
        if dist.is_initialized():
            dist.barrier()
        path.mkdir(parents=True, exist_ok=True)
        # ---- device -> host snapshot (synchronous, so training can continue right away)
        shard_id = pg.pp_rank * pg.layout.tp + pg.tp_rank
        n_shards = pg.layout.tp * pg.layout.pp
        write_model = pg.dp_rank == 0
        e.optimizer.wait_params()  # ZeRO-1/2: parameter all-gathers may still be in flight
        model_sd = {}
        if write_model:
            if getattr(e, "zero3", None) is not None:
                named = e.zero3.full_named_parameters()
            else:
                named = list(e.model.named_parameters())
            for n, p in named:
                model_sd[_global_name(n, e.pc.layer_index)] = p.detach().to("cpu", copy=True).contiguous()
        opt_sd = {k: (v.detach().to("cpu", copy=True) if torch.is_tensor(v) else v)
                  for k, v in e.optimizer.state_dict().items()}
        opt_index = optimizer_index(e)
        rng = {"cpu": torch.get_rng_state(), "cuda": torch.cuda.get_rng_state() if e.device.type == "cuda" else None}
        state = {
            "global_step": e.global_step, "epoch": e.epoch,
            "config": {k: (list(v) if isinstance(v, tuple) else v) for k, v in vars(c).items()},
            "scheduler": e.scheduler.state_dict(), "consumed_samples": e.consumed_samples,
            "world_size": world, "layout": {"tp": pg.layout.tp, "pp": pg.layout.pp, "dp": pg.layout.dp, "cp": pg.layout.cp},
            "zero_stage": c.zero_stage,
            # the resolved performance knobs this run trained under (replay restores them)
            "perf_knobs": e.knobs.as_dict() if getattr(e, "knobs", None) is not None else None,
        }

        timeout = float(getattr(c, "collective_timeout_s", 1800) or 1800)

        def _write():
            try:
                from safetensors.torch import save_file

                if write_model:
                    fname = "model.safetensors" if n_shards == 1 else f"model-{shard_id + 1:05d}-of-{n_shards:05d}.safetensors"
                    meta = {"tp_rank": str(pg.tp_rank), "tp": str(pg.layout.tp), "pp_rank": str(pg.pp_rank),
                            "pp": str(pg.layout.pp), "format": "pt"}
                    save_file(model_sd, str(path / fname), metadata=meta)
                (path / "optimizer").mkdir(exist_ok=True)
                torch.save(opt_sd, path / "optimizer" / f"rank_{rank:05d}.pt")
                if opt_index is not None:
                    (path / "optimizer" / f"rank_{rank:05d}.index.json").write_text(json.dumps(opt_index))
                (path / "rng").mkdir(exist_ok=True)
                torch.save(rng, path / "rng" / f"rank_{rank:05d}.pt")
                (path / ".done").mkdir(exist_ok=True)
                (path / ".done" / f"rank_{rank:05d}").write_text(save_id)
                if e.is_main:
                    self._commit(path, state, n_shards, world, timeout, save_id, final_path)
            except BaseException as ex:  # surfaced by wait()
                self._error = ex

        if c.async_checkpoint and not final:
            self._thread = threading.Thread(target=_write, name=f"llmctl-ckpt-{name}", daemon=True)
            self._thread.start()
        else:
            _write()
            self.wait()
        return final_path

    def _commit(self, path: Path, state: Dict[str, Any], n_shards: int, world: int, timeout: float,
                save_id: str = "", final_path: Optional[Path] = None) -> None:
        """Rank 0, off the training thread: once every rank's done-marker exists (each rank
        writes its marker after its own shards), write the metadata and move ``latest``.

        No collective is involved, so a checkpoint becomes durable as soon as the slowest rank's
        write finishes -- not at the next save -- and a rank killed mid-run never leaves the
        others blocked in a commit barrier.  A checkpoint whose markers never all appear (a rank
        died while writing) stays uncommitted: ``latest`` keeps pointing at the previous one."""
        e = self.engine
        done = path / ".done"
        deadline = time.time() + timeout
        def _ready() -> int:
            n = 0
            for m in done.glob("rank_*"):
                try:
                    n += m.read_text() == save_id
                except OSError:  # being written
                    pass
            return n

        while _ready() < world:
            if time.time() > deadline:
                raise TimeoutError(f"checkpoint {path}: not every rank finished writing within {timeout:.0f} s")
            time.sleep(0.05)
        (path / "config.json").write_text(json.dumps(e.model_config.to_dict(), indent=2))
        if n_shards > 1:
            weight_map = {}
            for f in sorted(path.glob("model-*.safetensors")):
                from safetensors import safe_open

                with safe_open(str(f), "pt") as sf:
                    for k in sf.keys():
                        weight_map.setdefault(k, []).append(f.name)
            (path / "model.safetensors.index.json").write_text(json.dumps(
                {"metadata": {"tp": state["layout"]["tp"], "pp": state["layout"]["pp"]},
                 "weight_map": weight_map}, indent=2))
        if e.config.plan_file and Path(e.config.plan_file).exists():
            shutil.copy(e.config.plan_file, path / "plan.toml")
        # training_state.json last: its presence marks a complete checkpoint (resume keys on it)
        tmp = path / "training_state.json.tmp"
        tmp.write_text(json.dumps(state, indent=2, default=str))
        os.replace(tmp, path / "training_state.json")
        shutil.rmtree(done, ignore_errors=True)
        if final_path is not None and final_path != path:
            # swap the complete staging directory in: the old copy (a re-save of this name) is
            # renamed aside first and deleted only after the new one is in place
            old = self.root / f".{final_path.name}.old"
            shutil.rmtree(old, ignore_errors=True)
            if final_path.exists():
                os.replace(final_path, old)
            os.replace(path, final_path)
            shutil.rmtree(old, ignore_errors=True)
            path = final_path
        lt = self.root / "latest.tmp"
        lt.write_text(path.name)
        os.replace(lt, self.root / "latest")
        self._gc()

    def wait(self) -> None:
        """Join this rank's pending write (rank 0: and its commit); re-raise its error."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            err, self._error = self._error, None
            raise err

    def _gc(self) -> None:
        keep = self.engine.config.keep_latest or self.engine.config.save_total_limit
        if not keep or keep <= 0:
            return
        ckpts = sorted((p for p in self.root.glob("checkpoint-*") if p.is_dir()),
                       key=lambda p: int(p.name.split("-")[-1]))
        for p in ckpts[:-keep]:
            shutil.rmtree(p, ignore_errors=True)

    # ------------------------------------------------------------------ load
    def load(self, path: str) -> None:
        e = self.engine
        p = Path(path)
        if p.is_dir() and (p / "latest").exists() and not (p / "training_state.json").exists():
            root = p
            p = p / (p / "latest").read_text().strip()
            if not (p / "training_state.json").exists():
                # ``latest`` names a checkpoint whose re-save was interrupted (its commit record is
                # removed before the rewrite): fall back to the newest complete one
                done = [d for d in root.iterdir() if d.is_dir() and not d.name.startswith(".")
                        and (d / "training_state.json").exists()]
                if not done:
                    raise FileNotFoundError(f"{root}: no complete checkpoint")
                skipped = p.name
                p = max(done, key=lambda d: json.loads((d / "training_state.json").read_text()).get("global_step", -1))
                log.warning("checkpoint: 'latest' names %s, which is incomplete (an interrupted save); "
                            "resuming from %s instead", skipped, p.name)
        state = json.loads((p / "training_state.json").read_text())
        e.optimizer.wait_params()
        full = load_full_state_dict(p, e.model_config)
        # re-shard for this rank's layout
        named = (e.zero3.full_named_parameters() if getattr(e, "zero3", None) is not None
                 else list(e.model.named_parameters()))
        with torch.no_grad():
            for n, prm in named:
                g = _global_name(n, e.pc.layer_index)
                if hasattr(e, "_expert_global"):
                    g = e._expert_global(g)
                if g == "lm_head" and g not in full and e.model_config.tie_word_embeddings:
                    g = "embed"  # PP>1 last-stage copy of a tied matrix saved under PP=1 / HF
                if g not in full:
                    raise KeyError(f"checkpoint {p} lacks tensor {g}")
                t = shard_tp(g, full[g], e.pg.layout.tp, e.pg.tp_rank, e.model_config)
                prm.copy_(t.to(prm.dtype))
        if getattr(e, "zero3", None) is not None:
            e.zero3.reload_shards_from_full()
        old_layout = dict(state.get("layout", {}))
        old_layout.setdefault("cp", 1)
        same_layout = (old_layout == {"tp": e.pg.layout.tp, "pp": e.pg.layout.pp, "dp": e.pg.layout.dp,
                                      "cp": e.pg.layout.cp}
                       and state.get("zero_stage", 0) == e.config.zero_stage)
        opt_file = p / "optimizer" / f"rank_{e.pg.rank:05d}.pt"
        if same_layout and opt_file.exists():
            e.optimizer.load_state_dict(torch.load(opt_file, map_location=e.device, weights_only=True))
        elif getattr(e, "zero3", None) is None and list((p / "optimizer").glob("rank_*.index.json")):
            # layout changed: fp32 master + Adam moments are resharded from the saved
            # layout-independent index (TP consolidate -> re-split -> new ZeRO shard)
            reshard_optimizer(e, p, state)
        else:
            # no index (older checkpoint / ZeRO-3): masters restart from the resharded weights
            _reinit_master_from_params(e)
            e.optimizer.step_count = int(state.get("global_step", 0))
        rng_file = p / "rng" / f"rank_{e.pg.rank:05d}.pt"
        if rng_file.exists():
            rng = torch.load(rng_file, weights_only=True)
            torch.set_rng_state(rng["cpu"])
            if rng.get("cuda") is not None and e.device.type == "cuda":
                torch.cuda.set_rng_state(rng["cuda"])
        e.global_step = int(state["global_step"])
        e.epoch = int(state.get("epoch", 0))
        e.consumed_samples = int(state.get("consumed_samples", 0))
        if hasattr(e, "_weights_changed"):
            e._weights_changed()


def optimizer_index(e) -> Optional[Dict[str, Any]]:
    """Map this rank's optimizer-state vector onto (global parameter, element range) pairs:
    ``segments`` = [global_name, offset_in_local_param, offset_in_state, length] plus the
    TP-local shape of every parameter, so the state can be re-split for any other layout.
    ZeRO-3 (per-unit shard flats) is not indexed."""
    if getattr(e, "zero3", None) is not None:
        return None
    opt, flat = e.optimizer, e.flat
    start = e.pc.layer_index
    params = [(flat.offsets[id(q)], q.numel(), _global_name(flat.names[id(q)], start), list(q.shape))
              for q in flat.params]
    segs = []
    if opt.zero_stage == 0:
        for off, n, g, _ in params:
            segs.append([g, 0, off, n])
    else:
        for b in flat.buckets:
            soff, c = opt.shard_offsets[b.index]
            r0 = b.start + opt.dp_rank * c
            r1 = r0 + c
            for off, n, g, _ in params:
                lo, hi = max(off, r0), min(off + n, r1)
                if lo < hi:
                    segs.append([g, lo - off, soff + lo - r0, hi - lo])
    pg = e.pg
    return {"tp_rank": pg.tp_rank, "pp_rank": pg.pp_rank, "dp_rank": pg.dp_rank, "zero": opt.zero_stage,
            "shapes": {g: shp for _, _, g, shp in params}, "segments": segs}


def reshard_optimizer(e, path: Path, state: Dict[str, Any]) -> None:
    """Rebuild this rank's fp32 master / exp_avg / exp_avg_sq from a checkpoint written under
    a different TP / PP / DP / ZeRO layout.  Old shards are memory-mapped, so a rank reads only
    the byte ranges of the parameters it now owns."""
    opt, flat, cfg = e.optimizer, e.flat, e.model_config
    old: Dict[tuple, List] = {}  # (tp_rank, pp_rank) -> [(index, state_dict)]
    for f in sorted((path / "optimizer").glob("rank_*.index.json")):
        idx = json.loads(f.read_text())
        sd = torch.load(f.with_name(f.name.replace(".index.json", ".pt")), map_location="cpu", weights_only=True,
                        mmap=True)
        old.setdefault((idx["tp_rank"], idx["pp_rank"]), []).append((idx, sd))
    old_tp = int(state.get("layout", {}).get("tp", 1))
    # global name -> (pp_rank, {tp_rank: [(index, sd, segments of that name)]})
    where: Dict[str, Dict[int, list]] = {}
    for (tr, pr), items in old.items():
        for idx, sd in items:
            for seg in idx["segments"]:
                where.setdefault(seg[0], {}).setdefault(tr, []).append((idx, sd, seg))
    keys = ("master", "exp_avg", "exp_avg_sq")
    start = e.pc.layer_index
    new_tp, new_tr = e.pg.layout.tp, e.pg.tp_rank
    for q in flat.params:
        g = _global_name(flat.names[id(q)], start)
        if g == "lm_head" and g not in where and cfg.tie_word_embeddings:
            g = "embed"  # tied matrix: the PP>1 last-stage copy restarts from embed's state
        if g not in where:
            raise KeyError(f"optimizer state for {g} missing in {path}")
        per_tp = where[g]
        full = {}
        for k in keys:
            parts = []
            for tr in range(old_tp if tp_split_rule(g, cfg) is not None else 1):
                items = per_tp[tr]
                shape = items[0][0]["shapes"][g]
                buf = torch.zeros(int(torch.tensor(shape).prod().item()) if shape else 1, dtype=torch.float32)
                for idx, sd, (_, poff, soff, n) in items:
                    buf[poff:poff + n] = sd[k][soff:soff + n].float()
                parts.append(buf.view(shape))
            t = consolidate_tp(g, parts, cfg) if len(parts) > 1 else parts[0]
            full[k] = shard_tp(g, t, new_tp, new_tr, cfg).reshape(-1)
        off, n = flat.offsets[id(q)], q.numel()
        with torch.no_grad():
            if opt.zero_stage == 0:
                for k in keys:
                    getattr(opt, k)[off:off + n].copy_(full[k].to(opt.master.device))
            else:
                for b in flat.buckets:
                    soff, c = opt.shard_offsets[b.index]
                    r0 = b.start + opt.dp_rank * c
                    lo, hi = max(off, r0), min(off + n, r0 + c)
                    if lo < hi:
                        for k in keys:
                            getattr(opt, k)[soff + lo - r0:soff + hi - r0].copy_(
                                full[k][lo - off:hi - off].to(opt.master.device))
    opt.step_count = int(state.get("global_step", 0))


def _reinit_master_from_params(e) -> None:
    opt = e.optimizer
    f = e.flat
    with torch.no_grad():
        if opt.zero_stage == 0:
            opt.master.copy_(f.data.float())
        else:
            for b in f.buckets:
                off, c = opt.shard_offsets[b.index]
                s = b.start + opt.dp_rank * c
                opt.master[off:off + c].copy_(f.data[s:s + c].float())
        opt.exp_avg.zero_()
        opt.exp_avg_sq.zero_()


def load_full_state_dict(path, model_cfg) -> Dict[str, torch.Tensor]:
    """Load a (possibly TP/PP-sharded) checkpoint directory into full, unsharded tensors."""
    from safetensors import safe_open

    p = Path(path)
    single = p / "model.safetensors"
    if single.exists():
        out = {}
        with safe_open(str(single), "pt") as sf:
            for k in sf.keys():
                out[k] = sf.get_tensor(k)
        return out
    files = sorted(p.glob("model-*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no model weights in {p}")
    by_name: Dict[str, Dict[int, torch.Tensor]] = {}
    for f in files:
        with safe_open(str(f), "pt") as sf:
            meta = sf.metadata() or {}
            tr = int(meta.get("tp_rank", 0))
            for k in sf.keys():
                by_name.setdefault(k, {})[tr] = sf.get_tensor(k)
    out = {}
    for k, shards in by_name.items():
        out[k] = consolidate_tp(k, [shards[i] for i in sorted(shards)], model_cfg)
    return out
