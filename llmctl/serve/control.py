"""TP serving control plane: rank 0's per-step plan to the other TP ranks without pickling.

Every engine step of :class:`llmctl.serve.tp.TPInferenceEngine` ships a plan (token ids,
positions, KV slots, block tables, ...) from rank 0 to the other ranks.  Round 4 sent it with
``dist.broadcast_object_list`` over gloo: a pickle on rank 0, a size broadcast plus a payload
broadcast through TCP, an unpickle on every rank -- per decode step, on every rank.

Here a plan is packed into a fixed-layout byte record (:func:`pack` / :func:`unpack`: a small
header per field -- key, kind, dtype, shape -- and the raw array bytes; nested dicts are
flattened to ``a/b`` keys) and moved through one of two channels:

* :class:`ShmChannel` (one node, the TP serving case): a ring of slots in a ``/dev/shm`` file
  mapped by every rank.  Rank 0 writes the record into slot ``seq % SLOTS`` and publishes
  ``seq`` in the slot header last; readers poll that word (spin, then back off to short
  sleeps when idle) and acknowledge ``seq`` in their own header word, which rank 0 checks
  before it reuses a slot.  No syscall or socket on the hot path: a decode step's plan costs a
  few microseconds per rank (``tools/tp_control_bench.py``, ``profiles/tp_control_r5.txt``).
* :class:`TensorChannel` (fallback: multi-node groups, or a plan larger than a slot): two gloo
  broadcasts of uint8 tensors (length, then bytes) -- still no pickle.

Reference: the reference server runs one process and has no TP control plane
(``/root/reference/llmctl/serve/server.py:372-386``).
"""

from __future__ import annotations

import math
import os
import struct
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

# ---------------------------------------------------------------------------- record codec
_KIND_NONE, _KIND_ARRAY, _KIND_LIST, _KIND_INT, _KIND_STR, _KIND_BOOL, _KIND_FLOAT, _KIND_DICT = range(8)
_DTYPES = [np.dtype(t) for t in ("int64", "int32", "int16", "int8", "uint8", "bool", "float32", "float64", "uint32")]
_DT_CODE = {d: i for i, d in enumerate(_DTYPES)}
_HDR = struct.Struct("<HBBBxxx")  # key length, kind, dtype code, ndim


def _flatten(d: Dict[str, Any], prefix: str, out: List[Tuple[str, Any]]) -> None:
    for k, v in d.items():
        key = prefix + k
        if isinstance(v, dict):
            out.append((key, _KIND_DICT))
            _flatten(v, key + "/", out)
        else:
            out.append((key, v))


# decode steps (the per-token hot path) have a fixed layout: [magic, n, mb, stamp] then ids /
# positions / slots / ctx as int64 rows and the [n, mb] int32 block table -- one conversion, one
# copy.  Sampling decode steps (``decode_s``: the TP async pipeline) add [cont] to the head and the
# uniforms, temperatures, top-k and top-p rows (fp32 / int32) after the block table.
_DECODE_MAGIC = 0x0DEC0DE1
_DECODE_S_MAGIC = 0x0DEC0DE2
_DECODE_KEYS = {"op", "ids", "positions", "slots", "ctx", "bt"}
_DECODE_KEYS_STAMPED = _DECODE_KEYS | {"stamp"}  # + a float timestamp (tools/tp_control_bench.py)
_DECODE_S_KEYS = _DECODE_KEYS | {"cont", "u", "temp", "topk", "topp"}


def _pack_decode(plan: Dict[str, Any]) -> bytes:
    bt = np.ascontiguousarray(plan["bt"], dtype=np.int32)
    n = len(plan["positions"])
    samp = plan["op"] == "decode_s"
    head = np.empty(5 + 4 * n, dtype=np.int64)
    head[0], head[1], head[2] = _DECODE_S_MAGIC if samp else _DECODE_MAGIC, n, bt.shape[1] if bt.ndim == 2 else 0
    head[3:4].view(np.float64)[0] = plan.get("stamp", float("nan"))
    head[4] = int(plan.get("cont", 0))
    for i, k in enumerate(("ids", "positions", "slots", "ctx")):
        head[5 + i * n: 5 + (i + 1) * n] = plan[k]
    parts = [head.tobytes(), bt.tobytes()]
    if samp:
        parts += [np.ascontiguousarray(plan["u"], dtype=np.float32).tobytes(),
                  np.ascontiguousarray(plan["temp"], dtype=np.float32).tobytes(),
                  np.ascontiguousarray(plan["topk"], dtype=np.int32).tobytes(),
                  np.ascontiguousarray(plan["topp"], dtype=np.float32).tobytes()]
    return b"".join(parts)


def _unpack_decode(buf) -> Dict[str, Any]:
    a = np.frombuffer(buf, dtype=np.int64, count=5)
    samp = int(a[0]) == _DECODE_S_MAGIC
    n, mb = int(a[1]), int(a[2])
    rows = np.frombuffer(buf, dtype=np.int64, count=4 * n, offset=40).reshape(4, n).copy()
    off = 40 + 32 * n
    bt = np.frombuffer(buf, dtype=np.int32, count=n * mb, offset=off).reshape(n, mb).copy()
    off += 4 * n * mb
    out = {"op": "decode_s" if samp else "decode", "ids": rows[0], "positions": rows[1], "slots": rows[2],
           "ctx": rows[3], "bt": bt}
    if samp:
        out["cont"] = bool(a[4])
        for k, dt in (("u", np.float32), ("temp", np.float32), ("topk", np.int32), ("topp", np.float32)):
            out[k] = np.frombuffer(buf, dtype=dt, count=n, offset=off).copy()
            off += 4 * n
    stamp = float(a[3:4].view(np.float64)[0])
    if stamp == stamp:
        out["stamp"] = stamp
    return out


def pack(plan: Dict[str, Any]) -> bytes:
    """Plan dict -> bytes.  Values: None, bool, int, float, str, list of ints (round-trips as a
    list), numpy arrays (int / bool / float dtypes, any shape), nested dicts.  Decode plans use a
    fixed layout (their lists come back as int64 arrays)."""
    op = plan.get("op")
    if ((op == "decode" and (plan.keys() == _DECODE_KEYS or plan.keys() == _DECODE_KEYS_STAMPED))
            or (op == "decode_s" and plan.keys() - {"stamp"} == _DECODE_S_KEYS)):
        return _pack_decode(plan)
    items: List[Tuple[str, Any]] = []
    _flatten(plan, "", items)
    parts: List[bytes] = [struct.pack("<I", len(items))]
    for key, v in items:
        kb = key.encode()
        if v is _KIND_DICT:
            parts += [_HDR.pack(len(kb), _KIND_DICT, 0, 0), kb]
            continue
        if v is None:
            parts += [_HDR.pack(len(kb), _KIND_NONE, 0, 0), kb]
        elif isinstance(v, (bool, np.bool_)):
            parts += [_HDR.pack(len(kb), _KIND_BOOL, 0, 0), kb, struct.pack("<q", int(v))]
        elif isinstance(v, (int, np.integer)):
            parts += [_HDR.pack(len(kb), _KIND_INT, 0, 0), kb, struct.pack("<q", int(v))]
        elif isinstance(v, (float, np.floating)):
            parts += [_HDR.pack(len(kb), _KIND_FLOAT, 0, 0), kb, struct.pack("<d", float(v))]
        elif isinstance(v, str):
            sb = v.encode()
            parts += [_HDR.pack(len(kb), _KIND_STR, 0, 0), kb, struct.pack("<q", len(sb)), sb]
        else:
            kind = _KIND_ARRAY if isinstance(v, np.ndarray) else _KIND_LIST
            a = v if kind == _KIND_ARRAY else np.asarray(v, dtype=np.int64)
            a = np.ascontiguousarray(a).reshape(a.shape)  # (ascontiguousarray alone turns 0-d into 1-d)
            if a.dtype not in _DT_CODE:
                raise TypeError(f"plan field {key!r}: unsupported dtype {a.dtype}")
            parts += [_HDR.pack(len(kb), kind, _DT_CODE[a.dtype], a.ndim), kb,
                      struct.pack(f"<{a.ndim}q", *a.shape), a.tobytes()]
    return b"".join(parts)


def unpack(buf) -> Dict[str, Any]:
    """bytes / uint8 view -> plan dict (arrays are copies, safe after the slot is reused)."""
    mv = memoryview(buf)
    if len(mv) >= 40 and struct.unpack_from("<q", mv, 0)[0] in (_DECODE_MAGIC, _DECODE_S_MAGIC):
        return _unpack_decode(mv)
    (n,) = struct.unpack_from("<I", mv, 0)
    off = 4
    out: Dict[str, Any] = {}
    for _ in range(n):
        klen, kind, dt, ndim = _HDR.unpack_from(mv, off)
        off += _HDR.size
        key = bytes(mv[off:off + klen]).decode()
        off += klen
        *path, leaf = key.split("/")
        d = out
        for p in path:
            d = d[p]
        if kind == _KIND_DICT:
            d[leaf] = {}
        elif kind == _KIND_NONE:
            d[leaf] = None
        elif kind in (_KIND_INT, _KIND_BOOL):
            (x,) = struct.unpack_from("<q", mv, off)
            off += 8
            d[leaf] = bool(x) if kind == _KIND_BOOL else x
        elif kind == _KIND_FLOAT:
            (x,) = struct.unpack_from("<d", mv, off)
            off += 8
            d[leaf] = x
        elif kind == _KIND_STR:
            (ln,) = struct.unpack_from("<q", mv, off)
            off += 8
            d[leaf] = bytes(mv[off:off + ln]).decode()
            off += ln
        else:
            shape = struct.unpack_from(f"<{ndim}q", mv, off)
            off += 8 * ndim
            dtype = _DTYPES[dt]
            nb = math.prod(shape) * dtype.itemsize
            a = np.frombuffer(mv[off:off + nb], dtype=dtype).reshape(shape).copy()
            off += nb
            d[leaf] = a.tolist() if kind == _KIND_LIST else a
    return out


# ---------------------------------------------------------------------------- channels
class TensorChannel:
    """Packed plans over two gloo broadcasts (length, bytes); any group, any node count."""

    def __init__(self, group, src_rank: int = 0):
        self.group = group
        self.src = dist.get_global_rank(group, src_rank) if group is not None else src_rank
        self.rank = dist.get_rank(group)

    def publish(self, plan: Dict[str, Any]) -> None:
        b = pack(plan)
        n = torch.tensor([len(b)], dtype=torch.int64)
        dist.broadcast(n, self.src, group=self.group)
        dist.broadcast(torch.frombuffer(bytearray(b), dtype=torch.uint8), self.src, group=self.group)

    def publish_bytes(self, b: bytes) -> None:
        n = torch.tensor([len(b)], dtype=torch.int64)
        dist.broadcast(n, self.src, group=self.group)
        dist.broadcast(torch.frombuffer(bytearray(b), dtype=torch.uint8), self.src, group=self.group)

    def receive(self) -> Dict[str, Any]:
        n = torch.zeros(1, dtype=torch.int64)
        dist.broadcast(n, self.src, group=self.group)
        buf = torch.empty(int(n.item()), dtype=torch.uint8)
        dist.broadcast(buf, self.src, group=self.group)
        return unpack(buf.numpy().tobytes())

    def close(self) -> None:
        pass


class PeerLostError(RuntimeError):
    """A TP control-plane peer died, closed its end or stopped heart-beating past the deadline."""


def _pid_alive(pid: int) -> bool:
    if pid <= 0:
        return True  # not registered yet
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


class ShmChannel:
    """Single-writer ring in a ``/dev/shm`` file (one node).  Layout (bytes):

    ``[0, 64 * 32)``        one 64-B line per rank (index = group rank), u64 words:
                            [0] ack (last seq read; readers), [1] pid, [2] heartbeat
                            (CLOCK_MONOTONIC ns, node-wide), [3] closed flag
    ``[2048, ...)``         SLOTS slots of ``slot_bytes``: [u64 seq][u64 nbytes][u64 spill][pad
                            to 64][record]

    A plan that does not fit a slot is published with ``spill = 1`` and its bytes follow through
    the gloo :class:`TensorChannel` (same order on every rank).

    Liveness (the gloo path it replaced raised on the process-group timeout): every
    rank writes its pid at setup and a heartbeat word from a daemon thread every
    ``timeout_s / 8`` (at most 1 s).  A reader waiting for a plan and rank 0 waiting for a reader's
    ack check the peer they wait on about every 50 ms and raise :class:`PeerLostError` when its
    process is gone, it closed the channel, or its heartbeat is older than ``timeout_s`` (a frozen
    process).  An idle server is not a failure: rank 0's heartbeat keeps its readers waiting.  The
    TP worker then exits non-zero and torchrun tears the group down
    (``/root/reference/llmctl/runtime/launcher.py:283-312`` watches exit codes the same way)."""

    SLOTS = 4
    HDR = 2048
    SLOT_HDR = 64
    CHECK_S = 0.05  # liveness check period while blocked

    def __init__(self, group, slot_bytes: int = 8 << 20, path: Optional[str] = None, poll_spin_s: float = 2e-3,
                 timeout_s: float = 600.0):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 32:
            raise ValueError("ShmChannel: at most 32 ranks")
        self.slot_bytes = slot_bytes
        self.poll_spin_s = poll_spin_s
        self.timeout_s = float(timeout_s)
        self.fallback = TensorChannel(group)
        box = [None]
        if self.rank == 0:
            path = path or f"/dev/shm/llmctl-tp-{uuid.uuid4().hex[:16]}"
            size = self.HDR + self.SLOTS * slot_bytes
            with open(path, "wb") as f:
                f.truncate(size)
            box[0] = path
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        self.path = box[0]
        import mmap

        with open(self.path, "r+b") as f:
            self._mmap = mmap.mmap(f.fileno(), self.HDR + self.SLOTS * slot_bytes)
        self.mm = np.frombuffer(self._mmap, dtype=np.uint8)  # plain ndarray views: no memmap overhead
        self.u64 = self.mm.view(np.uint64)
        self._ack_idx = np.arange(1, self.world, dtype=np.int64) * 8
        self.seq = 0
        me = 8 * self.rank
        self.u64[me + 1] = os.getpid()
        self.u64[me + 2] = time.monotonic_ns()
        self._hb_stop = None
        self._start_heartbeat()
        dist.barrier(group=group)  # every rank mapped the file (and wrote its pid) before rank 0 unlinks it
        if self.rank == 0:
            os.unlink(self.path)  # the mappings keep it alive; nothing leaks if a rank dies
        self.stats = {"published": 0, "spilled": 0}

    # ------------------------------------------------------------------ liveness
    def _start_heartbeat(self) -> None:
        import threading

        stop = threading.Event()
        period = min(1.0, max(0.01, self.timeout_s / 8))
        u64, word = self.u64, 8 * self.rank + 2

        def beat():
            while not stop.wait(period):
                u64[word] = time.monotonic_ns()

        self._hb_stop = stop
        self._hb_thread = threading.Thread(target=beat, name=f"llmctl-shm-hb{self.rank}", daemon=True)
        self._hb_thread.start()

    def _check_peer(self, r: int, waited_s: float) -> None:
        line = 8 * r
        pid = int(self.u64[line + 1])
        if int(self.u64[line + 3]):
            raise PeerLostError(f"TP control plane: rank {r} closed the channel while rank {self.rank} waited on it")
        if not _pid_alive(pid):
            raise PeerLostError(f"TP control plane: rank {r} (pid {pid}) is gone; rank {self.rank} gives up")
        age = (time.monotonic_ns() - int(self.u64[line + 2])) / 1e9
        if age > self.timeout_s:
            raise PeerLostError(f"TP control plane: rank {r} (pid {pid}) has not heart-beaten for {age:.1f} s "
                                f"(deadline {self.timeout_s:.1f} s; rank {self.rank} waited {waited_s:.1f} s)")

    def _slot(self, seq: int) -> int:
        return self.HDR + (seq % self.SLOTS) * self.slot_bytes

    def _ack_min(self) -> int:
        return int(self.u64[self._ack_idx].min()) if self.world > 1 else self.seq

    def publish(self, plan: Dict[str, Any]) -> None:
        b = pack(plan)
        self.seq += 1
        s = self.seq
        base = self._slot(s)
        t0 = time.perf_counter()
        next_check = t0 + self.CHECK_S
        while s - self._ack_min() > self.SLOTS:  # slot still unread by some rank
            now = time.perf_counter()
            if now - t0 > self.poll_spin_s:
                time.sleep(1e-5)
            if now > next_check:
                next_check = now + self.CHECK_S
                for r in range(1, self.world):
                    if s - int(self.u64[8 * r]) > self.SLOTS:  # only the laggards
                        self._check_peer(r, now - t0)
                if now - t0 > self.timeout_s:
                    raise PeerLostError(f"TP control plane: no ack within {self.timeout_s:.1f} s")
        spill = len(b) > self.slot_bytes - self.SLOT_HDR
        w = base // 8
        if not spill:
            self.mm[base + self.SLOT_HDR: base + self.SLOT_HDR + len(b)] = np.frombuffer(b, dtype=np.uint8)
        self.u64[w + 1] = len(b)
        self.u64[w + 2] = 1 if spill else 0
        self.u64[w] = s  # published last (x86-64 keeps store order)
        self.stats["published"] += 1
        if spill:
            self.stats["spilled"] += 1
            self.fallback.publish_bytes(b)

    def receive(self) -> Dict[str, Any]:
        self.seq += 1
        s = self.seq
        base = self._slot(s)
        w = base // 8
        t0 = time.perf_counter()
        next_check = t0 + self.CHECK_S
        while int(self.u64[w]) != s:
            now = time.perf_counter()
            el = now - t0
            if el > self.poll_spin_s:  # idle server: back off (50 us, then 1 ms sleeps)
                time.sleep(1e-3 if el > 0.5 else 5e-5)
            else:
                os.sched_yield()  # spinning, but never starve the ranks that share this CPU
            if now > next_check:
                next_check = now + self.CHECK_S
                try:
                    self._check_peer(0, el)
                except PeerLostError:
                    if int(self.u64[w]) != s:  # rank 0 may publish its last plan (stop) and close at once
                        raise
        n = int(self.u64[w + 1])
        if int(self.u64[w + 2]):
            plan = self.fallback.receive()
        else:
            plan = unpack(self.mm[base + self.SLOT_HDR: base + self.SLOT_HDR + n].tobytes())
        self.u64[8 * self.rank] = s  # ack: the slot may be reused
        return plan

    def close(self) -> None:
        if self._hb_stop is not None:
            self._hb_stop.set()
            self._hb_thread.join(timeout=2.0)  # it holds a view of the mapping
            self._hb_stop = self._hb_thread = None
        if self.mm is not None:
            self.u64[8 * self.rank + 3] = 1  # a clean close: peers still waiting on this rank raise
            del self.u64
            self.mm = None
            try:
                self._mmap.close()
            except BufferError:  # an unpacked view still alive somewhere: the mapping dies with it
                pass


def _node_id() -> str:
    import socket

    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    return f"{socket.gethostname()}/{boot}"


def make_channel(group, kind: str = "auto", timeout_s: float = 600.0):
    """``shm`` when every rank of ``group`` is on this node (TP serving), else gloo tensors.

    ``auto`` decides from the node ids (hostname + boot id) all-gathered over ``group``: every rank
    sees the same list, so every rank picks the same channel -- a group that spans nodes (or ranks
    with inconsistent ``LOCAL_WORLD_SIZE``) falls back to gloo instead of half the ranks opening a
    file the other node holds."""
    if kind == "auto":
        ids: List[Optional[str]] = [None] * dist.get_world_size(group)
        dist.all_gather_object(ids, _node_id(), group=group)
        kind = "shm" if len(set(ids)) == 1 and os.path.isdir("/dev/shm") else "tensor"
    return ShmChannel(group, timeout_s=timeout_s) if kind == "shm" else TensorChannel(group)
