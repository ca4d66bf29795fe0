"""Synthetic token streams (benchmarks / tests; the GPU box has no datasets or network).

Tokens are drawn on the compute device with a per-(seed, rank, step) generator so every
run is reproducible and no host→device copy sits in the timed loop.  ``labels`` are the
inputs shifted by one (the last position is the next token of the stream), like a packed
pre-training corpus.
"""

from __future__ import annotations

from typing import Iterator, Tuple

import torch


class SyntheticTokens:
    def __init__(self, vocab_size: int, seq_len: int, micro_batch: int, *, seed: int = 1234, rank: int = 0,
                 device=None):
        self.vocab, self.S, self.B = vocab_size, seq_len, micro_batch
        self.seed, self.rank = seed, rank
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.step = 0

    def batch(self, step: int) -> Tuple[torch.Tensor, torch.Tensor]:
        g = torch.Generator(device=self.device)
        g.manual_seed((self.seed * 1000003 + self.rank * 7919 + step) % (2**63 - 1))
        toks = torch.randint(0, self.vocab, (self.B, self.S + 1), generator=g, device=self.device)
        return toks[:, :-1].contiguous(), toks[:, 1:].contiguous()

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            yield self.batch(self.step)
            self.step += 1

    def skip(self, n_batches: int) -> None:
        """Resume: continue after ``n_batches`` already-consumed micro-batches."""
        self.step += n_batches

    def state_dict(self):
        return {"step": self.step, "seed": self.seed, "rank": self.rank}

    def load_state_dict(self, sd):
        self.step = int(sd.get("step", 0))
