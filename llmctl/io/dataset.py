"""Datasets: synthetic tokens, memory-mapped token files, sequence packing, DP sharding.

Reference: a hard-coded 3-sentence × 100 dummy text list tokenized with HF
(``engine.py:142-204``) and a declared-but-absent streaming/memmap layer
(``README.md:21``).  Here:

* ``synthetic`` — :class:`llmctl.io.synthetic.SyntheticTokens` (benchmarks / no data);
* ``*.bin`` (+ optional ``.idx``) — flat uint16/uint32 token file, memory-mapped and read by
  the native C++ loader (``llmctl.native``: background prefetch thread, packing,
  DP-strided sampling) when built, else by numpy memmap;
* ``*.jsonl`` / ``*.txt`` — tokenized once with the byte-level tokenizer into a ``.bin``.
"""

from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .synthetic import SyntheticTokens


class MemmapTokens:
    """Packed next-token-prediction samples from a flat token file.

    Sample ``i`` covers tokens ``[i*S, i*S + S + 1)``; DP rank ``r`` of ``n`` visits samples
    ``perm[r::n]`` of an epoch permutation seeded by (seed, epoch) — the same order on every
    restart, so resume/replay is exact given ``consumed`` samples.
    """

    def __init__(self, path: str, seq_len: int, micro_batch: int, *, dp_rank: int = 0, dp_size: int = 1,
                 seed: int = 0, dtype: Optional[str] = None, device=None):
        self.path = Path(path)
        meta = self.path.with_suffix(".json")
        if dtype is None:
            dtype = json.loads(meta.read_text()).get("dtype", "uint16") if meta.exists() else "uint16"
        self.tokens = np.memmap(self.path, dtype=np.dtype(dtype), mode="r")
        self.S, self.B = seq_len, micro_batch
        self.rank, self.world, self.seed = dp_rank, dp_size, seed
        self.n_samples = (len(self.tokens) - 1) // seq_len
        if self.n_samples < dp_size * micro_batch:
            raise ValueError(f"{path}: only {self.n_samples} samples of length {seq_len}")
        self.device = device
        self.epoch = 0
        self.pos = 0  # samples consumed by this rank in the current epoch
        self._native = None
        try:
            from llmctl.native import loader as native_loader

            self._native = native_loader.TokenLoader(str(self.path), np.dtype(dtype).itemsize, seq_len,
                                                     micro_batch, dp_rank, dp_size, seed)
        except Exception:
            self._native = None
        self._perm = None

    def _epoch_perm(self):
        if self._perm is None or self._perm[0] != self.epoch:
            g = np.random.default_rng(self.seed + 7919 * self.epoch)
            self._perm = (self.epoch, g.permutation(self.n_samples))
        return self._perm[1]

    def next_batch(self) -> Tuple[torch.Tensor, torch.Tensor]:
        if self._native is not None:
            arr = self._native.next()  # int64 [B, S+1]
        else:
            perm = self._epoch_perm()
            per_rank = len(perm) // self.world
            if self.pos + self.B > per_rank:
                self.epoch += 1
                self.pos = 0
                perm = self._epoch_perm()
            idx = perm[self.rank::self.world][self.pos:self.pos + self.B]
            self.pos += self.B
            arr = np.stack([np.asarray(self.tokens[i * self.S:i * self.S + self.S + 1], dtype=np.int64)
                            for i in idx])
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if self.device is not None and torch.device(self.device).type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t[:, :-1], t[:, 1:]

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            yield self.next_batch()

    def skip(self, n_batches: int) -> None:
        """Resume: position after ``n_batches`` micro-batches of this rank (same epoch
        roll-over rule as :meth:`next_batch`)."""
        per_epoch = max((self.n_samples // self.world) // self.B, 1)
        self.load_state_dict({"epoch": n_batches // per_epoch, "pos": (n_batches % per_epoch) * self.B})

    def state_dict(self):
        if self._native is not None:
            e, p = self._native.position()
            return {"epoch": e, "pos": p}
        return {"epoch": self.epoch, "pos": self.pos}

    def load_state_dict(self, sd):
        self.epoch, self.pos = int(sd.get("epoch", 0)), int(sd.get("pos", 0))
        if self._native is not None:
            self._native.seek(self.epoch, self.pos)


def tokenize_to_bin(src: str, dst: str, vocab_size: int = 256) -> int:
    """Byte-level tokenization (no tokenizer download is possible offline) of a .txt or
    .jsonl (``{"text": ...}`` per line) file into a uint16 token file."""
    src_p = Path(src)
    out = []
    with open(src_p, "r", encoding="utf-8", errors="replace") as f:
        for line in f:
            text = line.rstrip("\n")
            if not text:
                continue  # same document split as the native indexer: one non-empty line per doc
            if src_p.suffix == ".jsonl":
                try:
                    text = json.loads(line).get("text", "")
                except json.JSONDecodeError:
                    continue
            out.append(np.frombuffer(text.encode("utf-8"), dtype=np.uint8).astype(np.uint16))
            out.append(np.array([0], dtype=np.uint16))  # document separator
    arr = np.concatenate(out) if out else np.zeros(0, dtype=np.uint16)
    arr.tofile(dst)
    Path(dst).with_suffix(".json").write_text(json.dumps({"dtype": "uint16", "tokens": int(arr.size),
                                                          "tokenizer": "bytes"}))
    return int(arr.size)


def build_dataset(cfg, model_cfg, *, dp_rank: int = 0, dp_size: int = 1, device=None):
    path = cfg.dataset_path
    if path in (None, "", "synthetic") or str(path).startswith("synthetic"):
        return SyntheticTokens(model_cfg.vocab_size, cfg.seq_len, cfg.batch_size, seed=cfg.seed, rank=dp_rank,
                               device=device)
    p = Path(path)
    if p.suffix in (".toml",):
        from llmctl.config.toml_io import load_toml

        d = load_toml(p)
        srcs = d.get("sources") or []
        train = [s["path"] for s in srcs if s.get("split", "train") == "train"]
        if not train:
            return SyntheticTokens(model_cfg.vocab_size, cfg.seq_len, cfg.batch_size, seed=cfg.seed, rank=dp_rank,
                                   device=device)
        p = (p.parent / train[0]) if not Path(train[0]).is_absolute() else Path(train[0])
        if not p.exists():
            p = Path(train[0])
    if p.suffix in (".txt", ".jsonl"):
        dst = p.with_suffix(".bin")
        if not dst.exists():
            tokenize_to_bin(str(p), str(dst))
        p = dst
    if p.is_dir():
        bins = sorted(p.glob("*.bin"))
        if not bins:
            raise FileNotFoundError(f"no .bin token files in {p}")
        p = bins[0]
    return MemmapTokens(str(p), cfg.seq_len, cfg.batch_size, dp_rank=dp_rank, dp_size=dp_size, seed=cfg.seed,
                        device=device)
