"""Prefix cache: full KV blocks indexed by the token prefix they hold.

The reference's ``KVCacheManager`` (``llmctl/serve/server.py:57-87``) stored per-request tensors
that were never read back; every request (and every generated token) re-ran its whole prefix.
Here a KV block becomes reusable once all of its ``block_size`` positions are computed: its key
is a hash chained over the token ids of every block up to and including it, so two sequences
share a block only if their whole prefixes match.  The cache holds ONE reference on every block
it indexes (through the KV manager's ``incref_block``), so a finished or preempted sequence's
blocks stay resident until space is needed; eviction is LRU over blocks that nothing but the
cache still references.

Used for (a) requests that share a system prompt / few-shot prefix and (b) sequences resumed
after preemption, which re-attach their computed blocks instead of recomputing them.
"""

from __future__ import annotations

import hashlib
import os
from array import array
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence

# Block keys are keyed BLAKE2b digests chained over the parent key and the block's token bytes:
# Python's ``hash`` of an int tuple is unkeyed and cheap to collide on purpose, and a collision
# would re-attach another request's KV blocks (wrong outputs, cross-request data exposure).
# The per-process key makes digests unpredictable to clients.
_KEY = os.urandom(16)


def _block_hash(parent: bytes, tokens: Sequence[int]) -> bytes:
    h = hashlib.blake2b(parent, digest_size=16, key=_KEY)
    h.update(array("q", tokens).tobytes())
    return h.digest()


class PrefixCache:
    def __init__(self, kv, block_size: int):
        self.kv = kv
        self.bs = block_size
        self._blocks: "OrderedDict[bytes, int]" = OrderedDict()  # chain key -> block id (LRU order)
        self._owner: Dict[int, bytes] = {}  # block id -> chain key
        self.stats = {"lookups": 0, "hit_tokens": 0, "inserted": 0, "evicted": 0}

    def __len__(self) -> int:
        return len(self._blocks)

    def _hashes(self, ids: Sequence[int], nblocks: int) -> List[bytes]:
        out, h = [], b""
        for i in range(nblocks):
            h = _block_hash(h, ids[i * self.bs:(i + 1) * self.bs])
            out.append(h)
        return out

    def match(self, ids: Sequence[int]) -> List[int]:
        """Block ids of the longest cached prefix of ``ids`` in whole blocks, leaving at least one
        token of ``ids`` uncached (its logits are what the prefill must produce)."""
        self.stats["lookups"] += 1
        nfull = (len(ids) - 1) // self.bs
        blocks: List[int] = []
        for h in self._hashes(ids, nfull):
            b = self._blocks.get(h)
            if b is None:
                break
            self._blocks.move_to_end(h)
            blocks.append(b)
        self.stats["hit_tokens"] += len(blocks) * self.bs
        return blocks

    def insert(self, ids: Sequence[int], table: Sequence[int], num_computed: int,
               hashes: Optional[List[bytes]] = None, start: int = 0) -> None:
        """Index every fully computed block of a sequence (``ids`` its tokens, ``table`` its block
        table, ``num_computed`` the positions whose K/V are in the cache).  ``hashes``: the
        sequence's chain-hash list, extended in place (only new blocks are hashed); ``start``:
        blocks before it are already indexed (a live sequence's blocks cannot be evicted)."""
        nfull = min(num_computed // self.bs, len(table))
        if hashes is None:
            hashes = []
        h = hashes[-1] if hashes else b""
        for i in range(len(hashes), nfull):
            h = _block_hash(h, ids[i * self.bs:(i + 1) * self.bs])
            hashes.append(h)
        for i in range(start, nfull):
            h = hashes[i]
            b = table[i]
            if h in self._blocks:
                self._blocks.move_to_end(h)
                continue
            if b in self._owner:  # block already indexed under another chain (cannot happen
                continue           # for blocks shared through match(); kept as a guard)
            self.kv.incref_block(b)
            self._blocks[h] = b
            self._owner[b] = h
            self.stats["inserted"] += 1

    def evict(self, blocks_needed: int, protect: Iterable[int] = ()) -> int:
        """Release LRU cached blocks that no sequence uses until ``blocks_needed`` free blocks
        exist (or nothing evictable is left); returns how many blocks were freed.  Blocks in
        ``protect`` are kept (a prefix that ``match`` just returned to an admission that is
        still reserving the rest of its blocks)."""
        freed = 0
        keep = set(protect)
        for h in list(self._blocks):
            if self.kv.num_free_blocks >= blocks_needed:
                break
            b = self._blocks[h]
            if b in keep or self.kv.refcount(b) > 1:  # protected / still part of a live sequence
                continue
            del self._blocks[h]
            del self._owner[b]
            if self.kv.decref_block(b):
                freed += 1
            self.stats["evicted"] += 1
        return freed

    def num_evictable(self) -> int:
        """Cached blocks that nothing but the cache references (what ``evict`` could free)."""
        return sum(1 for b in self._blocks.values() if self.kv.refcount(b) == 1)

    def clear(self) -> None:
        for h, b in list(self._blocks.items()):
            self.kv.decref_block(b)
        self._blocks.clear()
        self._owner.clear()
