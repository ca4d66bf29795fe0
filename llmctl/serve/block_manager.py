"""Paged KV-cache block manager.

Replaces the reference's ``KVCacheManager`` (a dict of per-request (k, v) tensors with an
LRU cap that was never written to, ``server.py:57-87``).  The KV cache is ONE preallocated
HBM pool per layer, ``[num_blocks, block_size, Hkv, D]`` bf16 for K and V, sized from free
HBM (288 GB on MI355X holds ~500k tokens of GPT-7B KV at 85 %).  Sequences own block
tables; blocks are ref-counted (fork = prefix sharing).  Bookkeeping runs in the native C++
``KVManager`` (``llmctl/native``); :class:`PyKVManager` is a same-semantics fallback.
"""

from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch


class PyKVManager:
    def __init__(self, num_blocks: int, block_size: int):
        self.bs = block_size
        self._num_blocks = num_blocks
        self.free_list = list(range(num_blocks - 1, -1, -1))
        self.ref = [0] * num_blocks
        self.tables: Dict[int, List[int]] = {}
        self.tokens: Dict[int, int] = {}

    def blocks_needed(self, tokens: int) -> int:
        return (tokens + self.bs - 1) // self.bs

    def can_allocate(self, tokens: int) -> bool:
        return self.blocks_needed(tokens) <= len(self.free_list)

    def _alloc(self) -> int:
        if not self.free_list:
            return -1
        b = self.free_list.pop()
        self.ref[b] = 1
        return b

    def _new(self, seq: int) -> None:
        if seq in self.tables:
            raise RuntimeError("sequence already registered")

    def add_sequence(self, seq: int, tokens: int) -> bool:
        self._new(seq)
        n = self.blocks_needed(max(tokens, 1))
        if n > len(self.free_list):
            return False
        self.tables[seq] = [self._alloc() for _ in range(n)]
        self.tokens[seq] = tokens
        return True

    def add_sequence_shared(self, seq: int, tokens: int, prefix: List[int]) -> bool:
        self._new(seq)
        need = self.blocks_needed(max(tokens, 1))
        if len(prefix) > need:
            raise ValueError("prefix longer than the sequence")
        if need - len(prefix) > len(self.free_list):
            return False
        for b in prefix:
            self.incref_block(b)
        self.tables[seq] = list(prefix) + [self._alloc() for _ in range(need - len(prefix))]
        self.tokens[seq] = tokens
        return True

    def incref_block(self, b: int) -> None:
        if self.ref[b] <= 0:
            raise RuntimeError("incref of a free block")
        self.ref[b] += 1

    def decref_block(self, b: int) -> bool:
        if self.ref[b] <= 0:
            raise RuntimeError(f"double free of KV block {b}")
        self.ref[b] -= 1
        if self.ref[b] == 0:
            self.free_list.append(b)
            return True
        return False

    def refcount(self, b: int) -> int:
        return self.ref[b]

    def append_token(self, seq: int) -> int:
        t = self.tables[seq]
        pos = self.tokens[seq]
        if pos // self.bs >= len(t):
            b = self._alloc()
            if b < 0:
                return -1
            t.append(b)
        self.tokens[seq] = pos + 1
        return t[pos // self.bs] * self.bs + pos % self.bs

    def slot(self, seq: int, pos: int) -> int:
        return self.tables[seq][pos // self.bs] * self.bs + pos % self.bs

    def fork(self, src: int, dst: int) -> None:
        self._new(dst)
        for b in self.tables[src]:
            self.ref[b] += 1
        self.tables[dst] = list(self.tables[src])
        self.tokens[dst] = self.tokens[src]

    def free_sequence(self, seq: int) -> None:
        for b in self.tables.pop(seq, []):
            self.decref_block(b)
        self.tokens.pop(seq, None)

    def num_tokens(self, seq: int) -> int:
        return self.tokens[seq]

    def block_table(self, seq: int) -> List[int]:
        return list(self.tables[seq])

    def block_tables(self, seqs: List[int], max_blocks: int) -> np.ndarray:
        out = np.zeros((len(seqs), max_blocks), dtype=np.int32)
        for i, s in enumerate(seqs):
            t = self.tables[s]
            out[i, :len(t)] = t
        return out

    def slots(self, seq: int, start: int, count: int) -> np.ndarray:
        return np.array([self.slot(seq, start + i) for i in range(count)], dtype=np.int64)

    @property
    def num_free_blocks(self) -> int:
        return len(self.free_list)

    @property
    def num_blocks(self) -> int:
        return self._num_blocks

    @property
    def num_sequences(self) -> int:
        return len(self.tables)

    def usage(self) -> float:
        return 1.0 - len(self.free_list) / self._num_blocks


def make_kv_manager(num_blocks: int, block_size: int, prefer_native: bool = True):
    if prefer_native:
        from llmctl import native

        m = native.load()
        if m is not None:
            return m.KVManager(num_blocks, block_size)
    return PyKVManager(num_blocks, block_size)


class PagedKVCache:
    """Per-layer K/V block pools on the device."""

    def __init__(self, layers: int, num_blocks: int, block_size: int, kv_heads: int, head_dim: int,
                 dtype=torch.bfloat16, device=None):
        self.layers, self.num_blocks, self.block_size = layers, num_blocks, block_size
        shape = (layers, num_blocks, block_size, kv_heads, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)

    @staticmethod
    def blocks_for_memory(bytes_available: float, layers: int, block_size: int, kv_heads: int, head_dim: int,
                          dtype_bytes: int = 2) -> int:
        per_block = 2 * layers * block_size * kv_heads * head_dim * dtype_bytes
        return max(int(bytes_available // per_block), 1)

    @property
    def nbytes(self) -> int:
        return self.k.numel() * self.k.element_size() * 2
