"""Continuous-batching scheduler (and a static batcher for comparison).

Reference ``DynamicBatchScheduler`` (``server.py:89-125``): FIFO admission up to 8 requests
/ 8192 tokens, head-of-line blocking, and — the fatal bug — unfinished requests were never
re-queued, so any ``max_tokens > 1`` request hung.

Here (``scheduler="dynamic"``), every engine step:
1. all RUNNING sequences decode one token (up to ``max_batch_size``); each first gets a KV
   slot — if the pool is exhausted the most recently admitted sequence is preempted (its
   blocks freed, it returns to the front of the queue and is recomputed later);
2. WAITING sequences are admitted FIFO for prefill while the step's token budget
   (``max_batch_tokens`` minus the decode tokens), the batch-size cap and the free KV
   blocks (prompt + one block headroom) allow.
Prefills are CHUNKED: a sequence whose known tokens are not all in the KV cache gets a chunk
of them per step (at most the step's remaining token budget), so a long prompt no longer
stalls the decodes of the running batch for a whole prefill, and prefill chunks of several
sequences pack into one varlen batch with no padding.  With a :class:`PrefixCache`, admission
first re-attaches the longest cached block prefix of the prompt (shared system prompts; a
sequence resumed after preemption gets its own computed blocks back) and only the rest is
computed.
``scheduler="static"`` admits a new group only when the running group has fully finished.
``scheduler="prefill_first"`` (TTFT-oriented): a step that can admit a waiting request runs
only prefills — running sequences pause for that step — so a burst of arrivals gets its first
tokens back-to-back; with a one-prompt token budget the i-th request's TTFT is about i prefill
times instead of i x (prefill + decode step).
"""

from __future__ import annotations

import itertools
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, List, Optional, Tuple


@dataclass
class SamplingParams:
    max_tokens: int = 100
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    stop: List[str] = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None


_ids = itertools.count(1)


@dataclass
class Sequence:
    prompt_ids: List[int]
    params: SamplingParams
    request_id: str = ""
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: List[int] = field(default_factory=list)
    status: str = "waiting"  # waiting | running | finished
    finish_reason: Optional[str] = None
    arrival_time: float = field(default_factory=time.time)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    preemptions: int = 0
    on_token: Optional[Callable[["Sequence", int], None]] = None
    on_finish: Optional[Callable[["Sequence"], None]] = None
    num_computed: int = 0  # leading positions whose K/V are in the paged cache
    cached_tokens: int = 0  # of those, re-attached from the prefix cache (not computed)
    kv_len: int = 0  # positions reserved in the block table (prefill target; +1 per decode)
    # prefix-cache bookkeeping: chain hashes of this sequence's full token blocks (tokens only
    # ever append, so they stay valid) and how many of its current blocks are indexed
    block_hashes: List[bytes] = field(default_factory=list, repr=False)
    indexed_blocks: int = 0

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def last_id(self) -> int:
        return self.output_ids[-1] if self.output_ids else self.prompt_ids[-1]

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)


@dataclass
class PrefillChunk:
    """Positions [start, start + count) of ``seq`` computed in this step."""
    seq: Sequence
    start: int
    count: int

    @property
    def final(self) -> bool:  # the chunk reaches the sequence's last known token: sample after it
        return self.start + self.count == self.seq.num_tokens


@dataclass
class SchedulerOutput:
    prefill: List[PrefillChunk]
    decode: List[Sequence]
    preempted: List[Sequence]


class ContinuousBatchScheduler:
    def __init__(self, kv, max_batch_size: int = 8, max_batch_tokens: int = 8192, max_model_len: int = 4096,
                 policy: str = "dynamic", block_size: int = 16, prefix_cache=None):
        self.kv = kv
        self.prefix_cache = prefix_cache
        self.block_size = block_size
        self.max_batch_size = max_batch_size
        self.max_batch_tokens = max_batch_tokens
        self.max_model_len = max_model_len
        self.policy = policy
        self.waiting: Deque[Sequence] = deque()
        self.running: List[Sequence] = []

    # ------------------------------------------------------------------ queue
    def add(self, seq: Sequence) -> None:
        if len(seq.prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(seq.prompt_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(seq.prompt_ids)} tokens exceeds max_model_len {self.max_model_len}")
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    @property
    def num_waiting(self) -> int:
        return len(self.waiting)

    @property
    def num_running(self) -> int:
        return len(self.running)

    # ------------------------------------------------------------------ step
    def _can_admit(self) -> bool:
        if not self.waiting or len(self.running) >= self.max_batch_size:
            return False
        n = self.waiting[0].num_tokens + self.kv_block_size()
        if self.kv.can_allocate(n):
            return True
        # blocks held only by the prefix cache are free for admission purposes (_admit evicts
        # them); without this a full cache would make prefill_first never pause the decodes
        if self.prefix_cache is None:
            return False
        return self.kv.num_free_blocks + self.prefix_cache.num_evictable() >= self.kv.blocks_needed(n)

    def _reserve(self, blocks: int, protect=()) -> bool:
        """``blocks`` free KV blocks, evicting unused prefix-cache blocks (never those in
        ``protect``) if needed."""
        if self.kv.num_free_blocks >= blocks:
            return True
        if self.prefix_cache is not None:
            self.prefix_cache.evict(blocks, protect)
        return self.kv.num_free_blocks >= blocks

    def _admit(self, seq: Sequence) -> bool:
        """Reserve blocks for all known tokens of ``seq`` (re-attaching its cached prefix).
        The matched prefix blocks are held only by the cache until ``add_sequence_shared``
        takes its references, so the reservation must not evict them."""
        n = seq.num_tokens  # a resumed sequence also re-covers its generated tokens
        prefix = self.prefix_cache.match(seq.all_ids) if self.prefix_cache is not None else []
        need = self.kv.blocks_needed(n + self.kv_block_size()) - len(prefix)
        if not self._reserve(need, protect=prefix):
            return False
        if not self.kv.add_sequence_shared(seq.seq_id, n, prefix):
            return False
        seq.num_computed = seq.cached_tokens = len(prefix) * self.block_size
        seq.kv_len = n
        return True

    def schedule(self) -> SchedulerOutput:
        preempted: List[Sequence] = []
        decode: List[Sequence] = []
        # 1) decodes: running sequences whose known tokens are all cached but the newest (each
        #    needs one more KV slot); prefill_first skips them while a request can be admitted
        running = [] if self.policy == "prefill_first" and self._can_admit() else list(self.running)
        for seq in running:
            if len(decode) >= self.max_batch_size:
                break
            if seq.status != "running" or seq.num_computed < seq.kv_len:  # preempted / still prefilling
                continue
            slot = self.kv.append_token(seq.seq_id)
            while slot < 0:
                if self.prefix_cache is not None and self._reserve(1):
                    slot = self.kv.append_token(seq.seq_id)
                    continue
                victim = self._preempt_newest(exclude=seq)
                if victim is None:
                    break
                preempted.append(victim)
                slot = self.kv.append_token(seq.seq_id)
            if slot < 0:  # cannot even fit this one: preempt it
                self._preempt(seq)
                preempted.append(seq)
                continue
            seq._decode_slot = slot
            seq.kv_len += 1
            decode.append(seq)
        decode = [s for s in decode if s.status == "running"]  # a later victim may have been listed
        # 2) prefill chunks: sequences already admitted but not fully computed, then admissions
        prefill: List[PrefillChunk] = []
        budget = self.max_batch_tokens - len(decode)
        decoding = {id(q) for q in decode}
        for seq in self.running:
            if budget <= 0:
                break
            if seq.status == "running" and id(seq) not in decoding and seq.num_computed < seq.kv_len:
                c = min(seq.kv_len - seq.num_computed, budget)
                prefill.append(PrefillChunk(seq, seq.num_computed, c))
                budget -= c
        if self.policy == "static" and self.running:
            return SchedulerOutput(prefill, decode, preempted)
        admitted: List[Sequence] = []
        while self.waiting and budget > 0 and len(self.running) + len(admitted) < self.max_batch_size:
            seq = self.waiting[0]
            if not self._admit(seq):
                break
            self.waiting.popleft()
            seq.status = "running"
            admitted.append(seq)
            c = min(seq.kv_len - seq.num_computed, budget)
            prefill.append(PrefillChunk(seq, seq.num_computed, c))
            budget -= c
        self.running.extend(admitted)
        return SchedulerOutput(prefill, decode, preempted)

    def computed(self, seq: Sequence, count: int) -> None:
        """The engine ran ``count`` more positions of ``seq``: index its newly full blocks."""
        seq.num_computed += count
        # index newly completed blocks only (a decode step completes one every block_size steps;
        # re-hashing the whole prefix every step cost ~0.5 ms per 16 x 2k decode step)
        if (self.prefix_cache is not None and seq.status == "running"
                and seq.num_computed // self.block_size > seq.indexed_blocks):
            self.prefix_cache.insert(seq.all_ids, self.kv.block_table(seq.seq_id), seq.num_computed,
                                     hashes=seq.block_hashes, start=seq.indexed_blocks)
            seq.indexed_blocks = seq.num_computed // self.block_size

    def kv_block_size(self) -> int:
        return self.block_size

    def _preempt_newest(self, exclude: Sequence) -> Optional[Sequence]:
        for seq in reversed(self.running):
            if seq is not exclude:
                self._preempt(seq)
                return seq
        return None

    def _preempt(self, seq: Sequence) -> None:
        self._release(seq)
        if seq in self.running:
            self.running.remove(seq)
        seq.status = "waiting"
        seq.num_computed = seq.kv_len = 0
        seq.indexed_blocks = 0  # its blocks were released: re-index against the next block table
        seq.preemptions += 1
        self.waiting.appendleft(seq)

    def _release(self, seq: Sequence) -> None:
        """Free a sequence's blocks; with a prefix cache its computed full blocks stay indexed
        (resumption after preemption and requests sharing the prefix re-attach them)."""
        if self.prefix_cache is not None and seq.num_computed > 0:
            try:
                table = self.kv.block_table(seq.seq_id)
            except (KeyError, IndexError, RuntimeError):
                table = []
            if table:
                self.prefix_cache.insert(seq.all_ids, table, seq.num_computed, hashes=seq.block_hashes)
        self.kv.free_sequence(seq.seq_id)

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = "finished"
        seq.finish_reason = reason
        seq.finish_time = time.time()
        self._release(seq)
        if seq in self.running:
            self.running.remove(seq)
        if seq.on_finish:
            seq.on_finish(seq)

    def abort(self, request_id: str) -> None:
        for seq in list(self.running) + list(self.waiting):
            if seq.request_id == request_id:
                if seq in self.waiting:
                    self.waiting.remove(seq)
                    seq.status = "finished"
                    seq.finish_reason = "abort"
                else:
                    self.finish(seq, "abort")
