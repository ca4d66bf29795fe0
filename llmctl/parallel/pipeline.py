"""Pipeline parallelism: non-interleaved 1F1B schedule over RCCL point-to-point.

The reference only models PP in its planner (``plan.py:92-93,116-118,140``); nothing runs.
Here a stage owns a contiguous slice of decoder layers (``partition.shard_map.split_layers``)
plus the embedding (first stage) and final norm + lm_head + loss (last stage).  Between
stages the residual stream ``[tokens, hidden]`` travels as one bf16 tensor (the deferred
residual add is materialised at the stage boundary), ``batch_isend_irecv`` pairs every send
with the opposite recv so the schedule is deadlock-free, and DP gradient sync is enabled
only for the last micro-batch's backward (so the overlap engine still hides it under the
cool-down backwards of earlier stages).

Schedule per stage s of P with M micro-batches (Megatron 1F1B):
  warm-up   min(P-s-1, M) forwards
  steady    M - warmup  (forward, backward) pairs
  cool-down warmup backwards
Activation memory is bounded by P in-flight micro-batches on stage 0.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def interleaved_order(P: int, V: int, M: int, s: int) -> List[Tuple[str, int, int]]:
    """Megatron's interleaved 1F1B order on rank ``s``: (kind, model chunk, micro-batch).
    Forward k runs chunk (k // P) % V on micro-batch (k // PV) * P + k % P (groups of P
    micro-batches sweep the chunks), backward k the mirrored chunk V-1-(k // P) % V; warm-up
    (P - s - 1) * 2 + (V - 1) * P forwards (all of them when M == P), then 1F1B, then cool-down."""
    total = M * V

    def mb(k):
        return (k // (P * V)) * P + k % P

    warm = total if M == P else min((P - s - 1) * 2 + (V - 1) * P, total)
    order = [("F", (k // P) % V, mb(k)) for k in range(warm)]
    f, b = warm, 0
    while f < total:
        order.append(("F", (f // P) % V, mb(f)))
        order.append(("B", V - 1 - (b // P) % V, mb(b)))
        f, b = f + 1, b + 1
    while b < total:
        order.append(("B", V - 1 - (b // P) % V, mb(b)))
        b += 1
    return order


def build_interleaved_rounds(P: int, V: int, M: int):
    """Lock-step execution table of the interleaved schedule, computed identically on every
    rank: ``[(actions, messages)]`` per round, ``actions[s]`` = the (kind, chunk, mb) rank s
    runs (or None: its next action's input has not arrived), ``messages`` =
    (kind, src, dst, dst virtual stage, mb) sent after the round, in canonical order.  A message
    sent in round r is consumed in a later round.  Raises if the order deadlocks."""
    orders = [interleaved_order(P, V, M, s) for s in range(P)]
    ptr = [0] * P
    have = [set() for _ in range(P)]  # ("act" | "grad", virtual stage, mb) received
    last = P * V - 1
    rounds = []
    while any(ptr[s] < len(orders[s]) for s in range(P)):
        acts = [None] * P
        for s in range(P):
            if ptr[s] >= len(orders[s]):
                continue
            kind, c, m = orders[s][ptr[s]]
            vs = c * P + s
            need = (None if vs == 0 else ("act", vs, m)) if kind == "F" else (None if vs == last else ("grad", vs, m))
            if need is None or need in have[s]:
                acts[s] = (kind, c, m)
                ptr[s] += 1
        if all(a is None for a in acts):
            raise RuntimeError(f"interleaved pipeline schedule deadlocks (P={P}, V={V}, M={M})")
        msgs = []
        for s, a in enumerate(acts):
            if a is None:
                continue
            kind, c, m = a
            vs = c * P + s
            if kind == "F" and vs < last:
                msgs.append(("act", s, (vs + 1) % P, vs + 1, m))
            elif kind == "B" and vs > 0:
                msgs.append(("grad", s, (vs - 1) % P, vs - 1, m))
        msgs.sort()
        for kind, src, dst, vs, m in msgs:
            have[dst].add((kind, vs, m))
        rounds.append((acts, msgs))
    return rounds


class _Once:
    """Works of one batch_isend_irecv group, waited for at most once (a second ``wait`` on a
    completed gloo receive blocks forever)."""

    def __init__(self, works):
        self.works = works

    def wait(self) -> None:
        for w in self.works or ():
            w.wait()
        self.works = None


@torch.no_grad()
def broadcast_tied_embedding(model, pg) -> None:
    """Copy stage 0's ``embed`` into the last stage's ``lm_head`` (tied word embeddings).
    Must run before the optimizer is built: ``FlatAdamW`` snapshots the fp32 master weights
    from the parameters at construction, and the first update writes ``param = master``."""
    if pg.layout.pp <= 1 or pg.embed_group is None:
        return
    p = model.embed if pg.pp_rank == 0 else (model.lm_head if pg.pp_rank == pg.layout.pp - 1 else None)
    if p is not None:
        dist.broadcast(p.data, src=pg.pp_ranks[0], group=pg.embed_group)


class PipelineSchedule:
    def __init__(self, engine, num_microbatches: int):
        self.e = engine
        pg = engine.pg
        self.P = pg.layout.pp
        self.s = pg.pp_rank
        self.ranks = pg.pp_ranks
        self.num_microbatches = max(int(num_microbatches), 1)
        self.V = max(int(getattr(engine.config, "virtual_stages", 1) or 1), 1)
        if self.V > 1 and self.num_microbatches % self.P:
            raise ValueError(f"interleaved pipeline: micro-batches ({self.num_microbatches}) must be a multiple of "
                             f"pipeline_parallel ({self.P})")
        self._rounds = build_interleaved_rounds(self.P, self.V, self.num_microbatches) if self.V > 1 else None
        self.prev = self.ranks[self.s - 1] if self.s > 0 else None
        self.next = self.ranks[self.s + 1] if self.s < self.P - 1 else None
        # tied word embeddings: stage 0 owns ``embed``, stage P-1 an ``lm_head`` copy.  The copy
        # starts equal (``broadcast_tied_embedding``, called by the engine BEFORE the optimizer
        # snapshots its fp32 master weights) and stays equal because both receive the SUM of
        # the two stages' gradients (``sync_tied_grads``) before identical optimizer updates.
        self.tied = bool(engine.model_config.tie_word_embeddings and self.P > 1)
        if self.tied and self.is_last:
            engine.optimizer.norm_exclude.append(self._tied_grad)
        self.last_loss: Optional[torch.Tensor] = None
        self._pending_sends: List = []

    # ------------------------------------------------------------------ tied embeddings
    def _tied_param(self):
        m = self.e.model
        return m.embed if self.is_first else (m.lm_head if self.is_last else None)

    def _tied_grad(self) -> Optional[torch.Tensor]:
        """The DP-reduced gradient of the tied copy this rank holds: the whole ``p.grad`` under
        ZeRO-0, else this DP rank's shard of its solo bucket (the same element range on both
        stages: the engine gives each copy an equal-sized bucket of its own)."""
        p = self._tied_param()
        if p is None:
            return None
        opt = self.e.optimizer
        if opt.zero_stage == 0:
            from llmctl.runtime.flat import grad_view

            return grad_view(p)
        b = self.e.flat.param_bucket[id(p)]
        assert b.params == [p], "tied embedding copy must own its bucket"
        off, c = opt.shard_offsets[b.index]
        return opt.grad_shard[off:off + c]

    @torch.no_grad()
    def sync_tied_grads(self):
        """Sum the tied matrix's gradient over the first and last stage (after DP reduction:
        both are linear, so the order does not matter)."""
        if not self.tied:
            return
        g = self._tied_grad()
        if g is not None:
            dist.all_reduce(g, group=self.e.pg.embed_group)

    # ------------------------------------------------------------------ helpers
    @property
    def is_first(self):
        return self.s == 0

    @property
    def is_last(self):
        return self.s == self.P - 1

    def _act_shape(self, B: int, S: int) -> Tuple[int, int]:
        pc = self.e.pc
        T = B * S
        if pc.sequence_parallel and pc.tp_size > 1:
            T //= pc.tp_size
        return (T, self.e.model_config.hidden)

    def _p2p(self, send: Optional[Tuple[torch.Tensor, int]] = None,
             recv: Optional[Tuple[torch.Tensor, int]] = None) -> None:
        """One matched send/recv group.  A group with a receive is waited for (its data is used
        next).  A SEND-ONLY group (warm-up forwards, cool-down backwards) completes in the
        background: its work handles and tensor are kept until ``_drain_sends`` (end of the
        schedule), so the next micro-batch's compute starts while the activation / gradient is
        still on the wire (no compute-stream wait on the send)."""
        ops = []
        if send is not None:
            t = send[0].contiguous()
            ops.append(dist.P2POp(dist.isend, t, send[1]))
        if recv is not None:
            ops.append(dist.P2POp(dist.irecv, recv[0], recv[1]))
        if not ops:
            return
        works = dist.batch_isend_irecv(ops)
        if recv is None:  # send-only group (warm-up / cool-down): completes in the background
            self._pending_sends.extend((w, t) for w in works)
        else:
            # with a receive in the group, wait for the group (NCCL returns ONE work for a
            # coalesced send+recv group, so the two cannot be waited for separately)
            for w in works:
                w.wait()

    def _post_recv(self, buf: torch.Tensor, peer: int) -> List:
        """Post a receive and return its works: the caller waits for them only when the data is
        needed, so the transfer overlaps the compute in between.  Used only where every op
        posted on that peer pair in the meantime is also a receive (warm-up activations from the
        previous stage, cool-down gradients from the next), so the per-pair order of operations
        — all NCCL matches point-to-point by — is exactly that of the un-prefetched schedule."""
        return dist.batch_isend_irecv([dist.P2POp(dist.irecv, buf, peer)])

    @staticmethod
    def _wait(works: Optional[List]) -> None:
        for w in works or ():
            w.wait()

    def _drain_sends(self) -> None:
        for w, _ in self._pending_sends:
            w.wait()
        self._pending_sends.clear()

    def _empty(self, B, S):
        return torch.empty(self._act_shape(B, S), dtype=self.e.config.dtype, device=self.e.device)

    # ------------------------------------------------------------------ stage compute
    def _forward(self, x_in: Optional[torch.Tensor], ids: torch.Tensor, labels: torch.Tensor, denom: float,
                 chunk: Optional[int] = None, first: Optional[bool] = None, last: Optional[bool] = None):
        """One stage's (or, under virtual stages, one model chunk's) forward: embedding on the
        first, loss on the last."""
        first = self.is_first if first is None else first
        last = self.is_last if last is None else last
        m = self.e.model
        B, S = ids.shape
        positions = doc_start = None
        c = self.e.config
        if c.pack_sequences:  # every stage rebuilds the document map from the (shared) token ids
            from llmctl.ops.ref import document_starts

            doc_start = document_starts(ids, c.doc_separator)
            labels = labels.masked_fill(ids == c.doc_separator, -100)
            positions = (torch.arange(S, device=ids.device, dtype=torch.int32).view(1, S) - doc_start).reshape(-1)
        x = m.embed_tokens(ids, positions) if first else x_in
        x, res = m.run_layers(x, B, S, positions=positions, doc_start=doc_start, chunk=chunk)
        if last:
            logits = m.head(x, res)
            return m.loss(logits, labels, denom)
        return x + res if res is not None else x

    def _set_sync(self, enabled: bool):
        e = self.e
        if e.zero3 is not None:
            e.zero3.set_sync(enabled)
        elif e.sync is not None:
            e.sync.enabled = enabled

    # ------------------------------------------------------------------ 1F1B
    def run(self, batches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        if self.V > 1:
            return self._run_interleaved(batches)
        M = len(batches)
        P, s = self.P, self.s
        B, S = batches[0][0].shape
        # loss = per-token mean over the whole micro-batch set; CP ranks hold 1/cp of each sequence
        denom = float(batches[0][1].numel() * M * self.e.pg.layout.cp)
        warm = min(P - s - 1, M)
        inputs: List[Optional[torch.Tensor]] = []
        outputs: List[torch.Tensor] = []
        losses: List[torch.Tensor] = []
        fwd_i = 0
        bwd_i = 0

        def do_forward(x_in):
            nonlocal fwd_i
            ids, labels = batches[fwd_i]
            if x_in is not None:
                x_in.requires_grad_(True)
            out = self._forward(x_in, ids, labels, denom)
            inputs.append(x_in)
            outputs.append(out)
            if self.is_last:
                losses.append(out.detach())
            fwd_i += 1
            return out

        def do_backward(grad_out):
            nonlocal bwd_i
            self._set_sync(bwd_i == M - 1)
            out = outputs[bwd_i]
            if self.is_last:
                out.backward()
            else:
                torch.autograd.backward(out, grad_out)
            x_in = inputs[bwd_i]
            g = x_in.grad if x_in is not None else None
            outputs[bwd_i] = None  # free activations
            inputs[bwd_i] = None
            bwd_i += 1
            return g

        remaining = M - warm
        # warm-up forwards: the receive of the NEXT activation is posted before this forward's
        # compute (receive-ahead), so it lands while the stage computes
        x_next, rw = None, None
        if not self.is_first and M > 0:
            x_next = self._empty(B, S)
            rw = self._post_recv(x_next, self.prev)
        for j in range(warm):
            self._wait(rw)
            x_in, rw = x_next, None
            if not self.is_first and j + 1 < M:  # the next forward's input (warm-up or steady)
                x_next = self._empty(B, S)
                rw = self._post_recv(x_next, self.prev)
            out = do_forward(x_in)
            if not self.is_last:
                self._p2p(send=(out.detach(), self.next))
        self._wait(rw)
        x_in = x_next if remaining > 0 else None
        for i in range(remaining):
            out = do_forward(x_in)
            grad_out = None
            if not self.is_last:
                grad_out = self._empty(B, S)
                self._p2p(send=(out.detach(), self.next), recv=(grad_out, self.next))
            g = do_backward(grad_out)
            last_iter = i == remaining - 1
            if not self.is_first:
                if not last_iter:
                    x_in = self._empty(B, S)
                    self._p2p(send=(g, self.prev), recv=(x_in, self.prev))
                else:
                    self._p2p(send=(g, self.prev))
        # cool-down backwards: the next gradient's receive is posted before this backward
        g_next, gw = None, None
        if warm > 0 and not self.is_last:
            g_next = self._empty(B, S)
            gw = self._post_recv(g_next, self.next)
        for j in range(warm):
            self._wait(gw)
            grad_out, gw = g_next, None
            if not self.is_last and j + 1 < warm:
                g_next = self._empty(B, S)
                gw = self._post_recv(g_next, self.next)
            g = do_backward(grad_out)
            if not self.is_first:
                self._p2p(send=(g, self.prev))
        self._set_sync(True)
        self._drain_sends()
        if self.is_last:
            loss = torch.stack(losses).sum()
        else:
            loss = torch.zeros((), device=self.e.device)
        self.last_loss = loss
        return loss

    # ------------------------------------------------------------------ interleaved 1F1B
    INFLIGHT_ROUNDS = 2  # interleaved schedule: send/recv groups kept un-waited behind the current round

    def _run_interleaved(self, batches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """Virtual-stage schedule: rank s owns model chunks c = 0..V-1 = virtual stages
        c*P + s; activations go to virtual stage +1 (rank s+1, or rank 0's next chunk after
        the last rank), gradients back.  Each rank follows Megatron's interleaved order
        (:func:`interleaved_order`); the lock-step round table from
        :func:`build_interleaved_rounds` (identical on every rank) says which messages cross
        the wire after each round, so both ends of every send/recv pair issue it in the same
        round and in the same canonical order (NCCL matches point-to-point by order only)."""
        M = len(batches)
        if M != self.num_microbatches:
            raise ValueError(f"interleaved pipeline was built for {self.num_microbatches} micro-batches, got {M}")
        P, V, s = self.P, self.V, self.s
        B, S = batches[0][0].shape
        denom = float(batches[0][1].numel() * M * self.e.pg.layout.cp)
        last_vs = P * V - 1
        inputs: dict = {}
        grads: dict = {}
        stash: dict = {}
        losses: List[torch.Tensor] = []
        # a round's send/recv group is NOT waited at the end of the round: every received buffer
        # remembers its group's works and is waited for when a later round consumes it, so the
        # transfers overlap the next rounds' compute (the group stays one batch_isend_irecv:
        # opposite-direction messages on one peer pair must be posted together)
        arrive: dict = {}
        inflight: List = []
        for acts, msgs in self._rounds:
            a = acts[s]
            out_msg: dict = {}
            if a is not None:
                kind, c, mb = a
                vs = c * P + s
                if kind == "F":
                    x_in = None
                    if vs > 0:
                        arrive.pop(("act", vs, mb)).wait()
                        x_in = inputs.pop((vs, mb))
                        x_in.requires_grad_(True)
                    ids, labels = batches[mb]
                    out = self._forward(x_in, ids, labels, denom, chunk=c, first=vs == 0, last=vs == last_vs)
                    stash[(vs, mb)] = (x_in, out)
                    if vs == last_vs:
                        losses.append(out.detach())
                    else:
                        out_msg[("act", vs + 1, mb)] = out.detach()
                else:
                    x_in, out = stash.pop((vs, mb))
                    self._set_sync(mb == M - 1)  # the chunk's last micro-batch: its grads are final
                    if vs == last_vs:
                        out.backward()
                    else:
                        arrive.pop(("grad", vs, mb)).wait()
                        torch.autograd.backward(out, grads.pop((vs, mb)))
                    if vs > 0:
                        out_msg[("grad", vs - 1, mb)] = x_in.grad
            ops, keys, sent = [], [], []
            for kind, src, dst, vs_dst, mb in msgs:
                if src == s:
                    t = out_msg[(kind, vs_dst, mb)].contiguous()
                    sent.append(t)
                    ops.append(dist.P2POp(dist.isend, t, self.ranks[dst]))
                elif dst == s:
                    buf = self._empty(B, S)
                    (inputs if kind == "act" else grads)[(vs_dst, mb)] = buf
                    keys.append((kind, vs_dst, mb))
                    ops.append(dist.P2POp(dist.irecv, buf, self.ranks[src]))
            if ops:
                works = _Once(dist.batch_isend_irecv(ops))
                for k in keys:
                    arrive[k] = works
                inflight.append((works, sent))
                # bounded backlog: a round's sends are retired two rounds later, so the sent
                # activations / input gradients (and their irecv twins) are freed as the schedule
                # goes instead of all M*V of them living until the end of the step.  Both ends
                # posted round r-2's group in round r-2, so this wait never blocks on the future
                while len(inflight) > self.INFLIGHT_ROUNDS:
                    inflight.pop(0)[0].wait()
                self.peak_inflight_tensors = max(getattr(self, "peak_inflight_tensors", 0),
                                                 sum(len(t) for _, t in inflight))
        for works, _ in inflight:
            works.wait()
        self._set_sync(True)
        loss = torch.stack(losses).sum() if losses else torch.zeros((), device=self.e.device)
        self.last_loss = loss
        return loss

    # ------------------------------------------------------------------ loss / eval
    def broadcast_loss(self, loss: torch.Tensor) -> float:
        t = loss.detach().float().reshape(1).clone()
        if not self.is_last:
            t.zero_()
        dist.all_reduce(t, group=self.e.pg.pp_group)
        if self.e.pg.cp_group is not None:  # CP ranks hold partial sums of one loss
            dist.all_reduce(t, group=self.e.pg.cp_group)
        if self.e.pg.dp_group is not None:
            dist.all_reduce(t, group=self.e.pg.dp_group)
            t /= self.e.pg.layout.dp
        return float(t)

    @torch.no_grad()
    def eval_loss(self, ids: torch.Tensor, labels: torch.Tensor, denom: Optional[float] = None) -> torch.Tensor:
        B, S = ids.shape
        if self.V > 1:  # walk the virtual stages in order: 0..P-1 on chunk 0, then chunk 1, ...
            P, last_vs = self.P, self.P * self.V - 1
            d = float(denom if denom is not None else labels.numel())
            x, out = None, torch.zeros((), device=self.e.device)
            for vs in range(last_vs + 1):
                owner, c = vs % P, vs // P
                if owner == self.s:
                    if vs > 0:
                        x = self._empty(B, S)
                        self._p2p(recv=(x, self.ranks[(vs - 1) % P]))
                    y = self._forward(x, ids, labels, d, chunk=c, first=vs == 0, last=vs == last_vs)
                    if vs == last_vs:
                        out = y
                    else:
                        self._p2p(send=(y, self.ranks[(vs + 1) % P]))
                        self._drain_sends()
            t = out.float().reshape(1).clone()
            dist.all_reduce(t, group=self.e.pg.pp_group)
            if self.e.pg.cp_group is not None:
                dist.all_reduce(t, group=self.e.pg.cp_group)
            return t[0]
        x_in = None
        if not self.is_first:
            x_in = self._empty(B, S)
            self._p2p(recv=(x_in, self.prev))
        out = self._forward(x_in, ids, labels, float(denom if denom is not None else labels.numel()))
        if not self.is_last:
            self._p2p(send=(out, self.next))
            self._drain_sends()
            out = torch.zeros((), device=self.e.device)
        t = out.float().reshape(1).clone()
        dist.all_reduce(t, group=self.e.pg.pp_group)
        if self.e.pg.cp_group is not None:
            dist.all_reduce(t, group=self.e.pg.cp_group)
        return t[0]
