"""Row-sharded multi-GPU training step — one process per GPU, RCCL over xGMI.

Partitioning: every embedding table is row-sharded by ``owner(id) = id mod W``, local row
``id div W`` (each rank holds ``R = ceil(rows / W)`` rows of each of the four tables, their Adam
moments and deferred-Adam stamps).  Dense parameters are replicated.  Each rank trains on its own
batch of B groups (weak scaling); the W local batches form one global batch whose loss is the mean
over all W*N samples — a W-rank step equals the 1-rank step on the concatenated batch.

A step has a PLAN and a RUN:
  plan  (requester)  re-key ids as (owner, local row), dedup (radix sort): the compact order of
                     the unique rows is the owner order, so the all-to-all send buffer comes
                     straight out of the dedup; all_to_all of the per-destination counts and ONE
                     device-to-host copy of them (RCCL needs the split sizes on the host)
  run   1. all_to_all of the local rows (users then items per destination)          [RCCL]
        2. owners dedup what they received without a sort (per-row claim tokens), bring
           those rows current (deferred dense-exact Adam catch-up), gather GMF+MLP rows
        3. all_to_all of the rows back; requesters unpack them into mini tables        [RCCL]
        4. forward + backward on the mini tables (the 1-GPU kernels; the dedup's segments
           drive the backward's segment reduce)
        5. all_to_all of the compact row gradients to the owners, who sum them per row in
           rank order (deterministic) and apply the step; rolling sweep                [RCCL]
        6. one all_reduce of the flat dense-gradient buffer (on the second communicator,
           beside step 5), replicated dense Adam                                       [RCCL]
The plan of step t+1 is pipelined under the run of step t (``step(u, i, t, next=(u', i'))``, the
role of torchrec's TrainPipelineSparseDist): its kernels run on a side stream and its count
exchange on a second communicator, so the host-side wait for the split sizes overlaps the GPU
work of step t instead of draining the GPU every step.

The protocol (``ShardExchange`` + ``ShardedTrainStep``) is device-agnostic; the ops backend does
the per-rank work: ``HipShardOps`` (this file, the product path) or, in the CPU ``gloo`` tests, a
torch reference backend.
"""
import ctypes
import math
import random
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import ptr


# launch-tape slots of the row-sharded step (tapes.py): pointer ranges first (the next batch's
# ids, the targets, the compute stream), then the per-step scalars
SLOT_NEXT_U, SLOT_NEXT_I, SLOT_TARGETS, SLOT_STREAM = 0, 1, 2, 3
SLOT_TOKEN, SLOT_NMAX, SLOT_NUNI, SLOT_TOKEN_NEXT = 4, 5, 6, 7
TAPE_SHARDED = True
# The next step's rows sent to their owners during this step (on the side communicator)
SHARD_AHEAD = True
# The owner's rolling sweep overlapped on a side stream, and queued on the plan stream
SHARD_OVERLAP_SWEEP = True
SWEEP_ON_PLAN = True
# The exchange implementation (None: RCCL through the C-ABI on the nccl backend, torch
# collectives otherwise; "rccl" / "torch" force one)
EXCHANGE = None
# The owner's rank-order gradient sum inside the table Adam's apply (ncf_adam_pairs_apply_gsum_clock,
# one launch and no compact gradient round trip; False: ncf_shard_owner_gradsum + the apply)
GSUM_APPLY = True
# rolling-sweep period of the row-sharded step's deferred table Adam.  Its catch-up runs on the
# owner's critical path, so FusedTrainStep's longer period was measured here separately: world 1,
# 2 interleaved runs each, 0.3255 / 0.3268 ms/step at 128 against 0.3301 / 0.3302 at 64 (r5zo)
SWEEP_EVERY = 128
# The requester's table gradients written by the embedding backward straight into its send
# buffer (ncf_embedding_bwd_reduce_rows; False: compact rows, then ncf_shard_rows)
GRAD_ROWS = True
# The requester's forward gather and embedding backward read the received rows in place (each
# batch row at its send position; ncf_gather_ln_gmf_ld_fwd, table_ld = 2 D) instead of copying
# them into compact mini tables first (ncf_shard_rows); needs GRAD_ROWS
BACK_ROWS = True
# The owner's claim of the next step's rows (dedup + positions, ncf_shard_owner_prepare) run a
# step ahead on the plan stream, right behind the exchange that sends them (ahead mode); the step
# itself then only catches those rows up.  Same bits (tools/shard_bisect.py).  Off: measured at
# world 1 (2 interleaved runs each) 0.3292 / 0.3638 ms/step against 0.3305 / 0.3282 without —
# the claim leaves the critical path (17.7 -> 5.7 us) but the plan stream's extra work beside
# the fused backward slows it by as much (110 -> 122 us)
CLAIM_AHEAD = False


class ShardExchange:
    """The collectives of the sharded step (torch.distributed: RCCL on GPU, gloo on CPU).
    ``plan_group`` (a second communicator) carries the count exchange of the pipelined plan so
    it never queues behind the run's collectives."""

    def __init__(self, group=None, device=None, plan_group=None):
        self.group = group
        self.plan_group = plan_group if plan_group is not None else group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device

    def counts_issue(self, plan):
        """Start the exchange of plan.counts ([W][2] per destination: users, items; device
        tensor or host lists).  On the GPU the all_to_all runs on the plan's side stream and
        communicator and the result lands in pinned host memory with an event: nothing waits."""
        W = self.world
        if plan.stream is None:                      # CPU (gloo): synchronous
            send = torch.tensor(plan.counts, dtype=torch.int64, device=self.device).view(W, 2)
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.plan_group)
            both = torch.cat([send, recv]).tolist()
            plan.send_counts, plan.recv_counts = both[:W], both[W:]
            return
        with torch.cuda.stream(plan.stream):
            send = plan.counts.view(W, 2)
            both = plan.extra["counts_both"]          # device [2W, 2]: send rows, then recv rows
            dist.all_to_all_single(both[W:], send, group=self.plan_group)
            both[:W].copy_(send)
            plan.extra["counts_host"].copy_(both, non_blocking=True)
            plan.extra["counts_ev"].record(plan.stream.cuda_stream)

    def counts_wait(self, plan):
        """plan.send_counts / plan.recv_counts as host lists [W][2] (the step's only host
        wait: for a plan issued a step ahead it has long completed)."""
        if plan.send_counts is not None:
            return
        W = self.world
        plan.extra["counts_ev"].synchronize()
        both = plan.extra["counts_host"].tolist()
        plan.send_counts, plan.recv_counts = both[:W], both[W:]

    def exchange_counts(self, plan):
        self.counts_issue(plan)
        self.counts_wait(plan)

    def exchange(self, t: torch.Tensor, send_splits: List[int], recv_splits: List[int],
                 side: bool = False, slot: Optional[str] = None):
        out = torch.empty((sum(recv_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t[:sum(send_splits)], recv_splits, send_splits,
                               group=self.plan_group if side else self.group)
        return out

    def exchange_ahead(self, plan):
        """The first exchange of a plan issued a step ahead (its local rows to their owners), run
        on the plan's side stream and communicator as soon as its counts are home, so the next
        step starts with its rows already at the owners.  Returns (recv, event)."""
        send_splits, recv_splits = plan.splits()
        if plan.stream is None:
            return self.exchange(plan.send, send_splits, recv_splits, side=True), None
        with torch.cuda.stream(plan.stream):
            out = self.exchange(plan.send, send_splits, recv_splits, side=True)
            ev = torch.cuda.Event()
            ev.record()
        return out, ev

    def wait_ahead(self, out, ev):
        if ev is not None:
            cur = torch.cuda.current_stream(out.device)
            cur.wait_event(ev)
            out.record_stream(cur)

    def all_reduce_(self, t: torch.Tensor):
        dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_start(self, t: torch.Tensor):
        """Start the dense-gradient all-reduce on the plan communicator: its RCCL kernel runs
        beside the row-gradient all-to-all and the owners' table update on the main one."""
        return dist.all_reduce(t, group=self.plan_group, async_op=True)

    def all_reduce_wait(self, work):
        if work is not None:
            work.wait()


class RcclExchange(ShardExchange):
    """The same collectives issued through the C-ABI (``ncf_comm_*``: grouped ncclSend/ncclRecv
    and ncclAllReduce on the step's own HIP streams) on two RCCL communicators of this library,
    one per stream: ``main`` for the run's exchanges on the step's stream, ``side`` for the
    pipelined count exchange, the rows sent ahead and the dense all-reduce on the plan stream
    (the roles of ``group`` / ``plan_group``).  The communicators are created over
    ``group`` (unique ids broadcast by its rank 0).  Same results as ``ShardExchange``; none of
    the c10d per-call work (Work objects, stream-sync events, allocator bookkeeping)."""

    def __init__(self, group=None, device=None, plan_group=None):
        super().__init__(group, device, plan_group)
        if not _lib.query("ncf_comm_available"):
            raise RuntimeError("RcclExchange: librccl is not loaded in this process")
        # Two communicators, each used from ONE stream only: ``main`` on the step's stream (the
        # row exchanges), ``side`` on the plan stream (the pipelined count exchange, the rows sent
        # ahead, the dense all-reduce).  Every rank issues the same host program, so each stream
        # — and each hardware queue two streams may share (4 per process) — receives
        # the collectives in the same order on every rank: no rank can hold one communicator's
        # collective in a queue ahead of another's that its peer runs first.  (One communicator
        # for both roles, measured in round 4, makes RCCL order each collective behind the
        # communicator's previous one across the two streams, which ties the plan stream — the
        # next batch's sort, the overlapped sweep — to the step's: world 1, 0.48 against 0.35
        # ms/step)
        self.main = self._comm()
        self.side = self._comm()
        W = self.world
        # host split arrays, one pair per call site: the collective reads them when it is
        # called, so a launch tape replays each site with the sizes written there for the step
        self._sites = {}
        self._one = (ctypes.c_int64 * W)(*([1] * W))
        self._one_addr = ctypes.addressof(self._one)
        self._side_stream = None
        self._ev_in, self._ev_out = _lib.RawEvent(), _lib.RawEvent()
        self._ahead_ev = [_lib.RawEvent(), _lib.RawEvent()]
        self._slots = {}

    def site(self, name: str, send_splits=None, recv_splits=None):
        """(send, recv) host split arrays of call site `name` (addresses), filled when given."""
        a = self._sites.get(name)
        if a is None:
            W = self.world
            sr, rr = (ctypes.c_int64 * W)(), (ctypes.c_int64 * W)()
            a = self._sites[name] = (sr, rr, ctypes.addressof(sr), ctypes.addressof(rr))
        if send_splits is not None:
            sr, rr = a[0], a[1]
            for p in range(self.world):
                sr[p], rr[p] = send_splits[p], recv_splits[p]
        return a[2], a[3]

    def _comm(self):
        uid = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            _lib.call("ncf_comm_unique_id", uid.data_ptr(), 128)
        t = uid.to(self.device)
        dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                       group=self.group)
        uid = t.cpu()
        c = ctypes.c_void_p()
        _lib.call("ncf_comm_init", uid.data_ptr(), 128, self.world, self.rank, ctypes.byref(c))
        return c.value

    def close(self):
        c = getattr(self, "main", None)
        if c is not None:
            _lib.call("ncf_comm_destroy", c)
        c2 = getattr(self, "side", None)
        if c2 is not None and c2 != c:
            _lib.call("ncf_comm_destroy", c2)
        self.main = self.side = None

    def counts_issue(self, plan):
        if plan.stream is None:
            raise RuntimeError("RcclExchange needs a plan on a GPU side stream")
        W = self.world
        both = plan.extra["counts_both"]              # device [2W, 2] int64: send rows, recv rows
        ps = plan.stream.cuda_stream
        send = plan.counts
        # (C-ABI copies and event: the step's launch tape holds them in order)
        _lib.call("ncf_comm_alltoallv", self.side, ptr(send), self._one_addr, ptr(both) + 16 * W,
                  self._one_addr, 16, ps)
        _lib.call("ncf_memcpy_async", ptr(both), ptr(send), 16 * W, ps)
        _lib.call("ncf_memcpy_async", ptr(plan.extra["counts_host"]), ptr(both), 32 * W, ps)
        plan.extra["counts_ev"].record(ps)
        self._side_stream = plan.stream

    def exchange(self, t: torch.Tensor, send_splits: List[int], recv_splits: List[int],
                 side: bool = False, slot: Optional[str] = None, stream: Optional[int] = None):
        """``slot``: a grow-only output buffer reused by every call with that name (the caller
        consumes it in stream order before the next such call), else a fresh tensor; it also
        names the call site's split arrays.  Over one rank the all-to-all is the identity: the
        input itself is returned (no copy; every caller consumes the output in stream order
        before it next writes the input)."""
        if self.world == 1:
            return t[:send_splits[0]]
        sr, rr = self.site(slot or ("side" if side else "main"), send_splits, recv_splits)
        out = self.exchange_out(t, recv_splits, slot)
        row = t.element_size() * (math.prod(t.shape[1:]) if t.dim() > 1 else 1)
        _lib.call("ncf_comm_alltoallv", self.side if side else self.main, ptr(t), sr, ptr(out),
                  rr, row, stream if stream is not None else _lib.stream_ptr(t.device))
        return out

    def exchange_out(self, t: torch.Tensor, recv_splits: List[int], slot: Optional[str] = None):
        """The output of an exchange of `t` (host side only): a view of slot buffer `slot`
        (grow-only), or a fresh tensor; over one rank the input itself."""
        if self.world == 1:
            return t[:recv_splits[0]]
        shape = (sum(recv_splits),) + tuple(t.shape[1:])
        if slot is None:
            return torch.empty(shape, dtype=t.dtype, device=t.device)
        buf = self._slots.get(slot)
        n = math.prod(shape)
        if buf is None or buf.numel() < n or buf.dtype != t.dtype:
            buf = self._slots[slot] = torch.empty(max(n, 1) * 5 // 4, dtype=t.dtype,
                                                  device=t.device)
        return buf[:n].view(shape)

    def exchange_ahead(self, plan):
        """ShardExchange.exchange_ahead on the C-ABI: output slot and event per plan-buffer set
        (two alternate), so consecutive steps never share them."""
        send_splits, recv_splits = plan.splits()
        k = plan.extra["set"]["k"]
        ps = plan.stream.cuda_stream
        out = self.exchange(plan.send, send_splits, recv_splits, side=True, slot=f"ahead{k}",
                            stream=ps)
        ev = self._ahead_ev[k]
        ev.record(ps)
        return out, ev

    def wait_ahead(self, out, ev):
        if ev is not None:
            ev.wait(_lib.stream_ptr(out.device))

    def all_reduce_(self, t: torch.Tensor):
        _lib.call("ncf_comm_allreduce_sum_f32", self.main, ptr(t), t.numel(),
                  _lib.stream_ptr(t.device))
        return t

    def all_reduce_start(self, t: torch.Tensor):
        """The dense all-reduce on the side communicator and stream (behind the next plan's
        count exchange there), beside the row-gradient exchange on the main one."""
        ss = self._side_stream
        if ss is None:
            return self.all_reduce_(t)
        self._ev_in.record(_lib.stream_ptr(t.device))
        self._ev_in.wait(ss.cuda_stream)
        _lib.call("ncf_comm_allreduce_sum_f32", self.side, ptr(t), t.numel(), ss.cuda_stream)
        self._ev_out.record(ss.cuda_stream)
        return self._ev_out

    def all_reduce_wait(self, work):
        if isinstance(work, _lib.RawEvent):
            work.wait(_lib.stream_ptr(self.device))


@dataclass
class Plan:
    """One step's requester-side plan.  ``send`` holds the local rows in destination-major order
    (per destination: users then items); ``counts`` the per-destination row counts [W][2]."""
    send: object
    counts: object
    stream: Optional[object] = None
    send_counts: Optional[list] = None     # host [W][2], after ShardExchange.exchange_counts
    recv_counts: Optional[list] = None
    extra: dict = field(default_factory=dict)

    def splits(self):
        return ([a + b for a, b in self.send_counts], [a + b for a, b in self.recv_counts])

    def totals(self):
        return (sum(c[0] for c in self.send_counts), sum(c[1] for c in self.send_counts))


class ShardedTrainStep:
    """One data-parallel + row-sharded training step: the protocol above over an ops backend.
    ``step(u, i, t, next=(u2, i2))`` also plans the following step (pipelined)."""

    def __init__(self, ops, exchange: ShardExchange, ahead: Optional[bool] = None):
        self.ops, self.x = ops, exchange
        self._pending = None      # [user_ids, item_ids, Plan, (recv, event) | None] planned ahead
        # send the next step's rows to their owners during this step (SHARD_AHEAD)
        self.ahead = ahead if ahead is not None else bool(SHARD_AHEAD)
        # launch tapes (HIP ops + C-ABI collectives): the two launch segments of a step (split
        # at the host wait for the next plan's sizes) recorded once per geometry and replayed.
        # World 1 only: a replay of recorded RCCL collectives at world > 1 has not run on
        # hardware (no multi-GPU box here), so that path stays eager until one covers it
        from .tapes import SegmentTapes
        self.tapes = SegmentTapes() if (TAPE_SHARDED and isinstance(ops, HipShardOps)
                                        and isinstance(exchange, RcclExchange)
                                        and exchange.world == 1) else None

    def plan(self, user_ids, item_ids):
        p = self.ops.plan(user_ids, item_ids, self.x.world)
        self.x.counts_issue(p)
        return p

    def _claims_ahead(self):
        return CLAIM_AHEAD and hasattr(self.ops, "owner_claim")

    def _claim_ahead(self, nxt, ahead, token_slot=SLOT_TOKEN):
        """Step t+1's owner claim (dedup + positions of the rows it was just sent) on the plan
        stream behind their exchange; the ahead event is recorded again behind it, so the step
        that uses it waits for both.  Returns its owner state (owner_host)."""
        ops = self.ops
        own = ops.owner_host(nxt)
        ps = nxt.stream
        ops.owner_claim(ahead[0], own, ps.cuda_stream, token_slot)
        ev = ahead[1]
        if isinstance(ev, _lib.RawEvent):
            ev.record(ps.cuda_stream)
        elif ev is not None:
            ev.record(ps)
        return own

    def _settle_pending(self, pend):
        """A pending next-step plan that is not used (other ids came): its launches on the plan
        stream must be behind the step before the buffers of its set are written again."""
        if pend is not None and pend[3] is not None:
            self.x.wait_ahead(*pend[3])

    def __call__(self, user_ids, item_ids, targets, next=None):
        if self.tapes is not None and self.tapes.usable(self.ops.deferred, self.ops.eng):
            return self._call_taped(user_ids, item_ids, targets, next)
        ops, X = self.ops, self.x
        ops.mark_entry()          # ids of this call and of `next` exist from here on
        pend, self._pending = self._pending, None
        ahead = own = None
        if pend is not None and pend[0] is user_ids and pend[1] is item_ids:
            plan, ahead = pend[2], pend[3]   # planned (and its rows sent) one call ago
            own = pend[4]                    # (and claimed by their owners, CLAIM_AHEAD)
        else:
            self._settle_pending(pend)
            plan = self.plan(user_ids, item_ids)
        X.counts_wait(plan)
        if next is not None:      # plan step t+1 now: it runs under this step's GPU work
            self._pending = [next[0], next[1], self.plan(next[0], next[1]), None, None]
        ops.begin(plan)
        send_splits, recv_splits = plan.splits()
        if ahead is not None:
            recv = ahead[0]
            X.wait_ahead(*ahead)
        else:
            recv = X.exchange(plan.send, send_splits, recv_splits)
        if own is not None:       # claimed a step ahead: its rows only need catching up
            ops.owner_catchup(own)
        else:
            own = ops.owner_prepare(recv, plan)
        rows = ops.owner_gather(own, recv)
        back = X.exchange(rows, recv_splits, send_splits, slot="rows")
        grads, loss = ops.compute(plan, back, user_ids, item_ids, targets,
                                  loss_denominator=user_ids.numel() * X.world)
        if self.ahead and self._pending is not None:   # step t+1's rows to their owners now
            nxt = self._pending[2]
            X.counts_wait(nxt)
            self._pending[3] = X.exchange_ahead(nxt)
            if self._claims_ahead():
                self._pending[4] = self._claim_ahead(nxt, self._pending[3])
        ar = X.all_reduce_start(ops.dense_grad())
        got = X.exchange(grads, send_splits, recv_splits, slot="grads")
        ops.owner_apply(own, got)
        X.all_reduce_wait(ar)
        ops.dense_step()
        return loss

    # ---- the same step with its launches recorded / replayed (tapes.SegmentTapes)
    def _signature(self):
        ops, X = self.ops, self.x
        d = ops.deferred
        eng = ops.eng
        return (id(d), d._consts(), d._table.data_ptr(), tuple(d.fork_points), d.overlap,
                eng.flat.data_ptr(), eng.flat_grad.data_ptr(),
                tuple(p.data_ptr() for p in eng.table_params().values()),
                tuple(b.data_ptr() for b in ops._bufs.values() if torch.is_tensor(b)),
                tuple(b.data_ptr() for b in X._slots.values()),
                tuple((k, id(v)) for k, v in eng.ws.items()))

    def _call_taped(self, user_ids, item_ids, targets, next=None):
        ops, X, T = self.ops, self.x, self.tapes
        d = ops.deferred
        st = ops._st()
        ops.eng.ensure_layout()   # (as eng.forward would; a re-pack moves the signature)
        ops.mark_entry()
        pend, self._pending = self._pending, None
        ahead = own_ahead = None
        if pend is not None and pend[0] is user_ids and pend[1] is item_ids:
            plan, ahead, own_ahead = pend[2], pend[3], pend[4]
        else:
            self._settle_pending(pend)
            plan = self.plan(user_ids, item_ids)
        X.counts_wait(plan)
        n = plan.extra["n"]
        nplan = None
        if next is not None:
            nu_, ni_ = next[0].reshape(-1), next[1].reshape(-1)
            nplan = ops.plan_host(nu_, ni_)
            self._pending = [next[0], next[1], nplan, None, None]
        targets = targets.reshape(-1).to(device=ops.dev, dtype=torch.float32).contiguous()
        send_splits, recv_splits = plan.splits()
        own = own_ahead if own_ahead is not None else ops.owner_host(plan)
        nu, ni = plan.totals()
        X.site("recv", send_splits, recv_splits)
        X.site("rows", recv_splits, send_splits)
        X.site("grads", send_splits, recv_splits)
        T.horizon(d)
        k_set = plan.extra["set"]["k"]
        key_a = ("a", n, k_set, None if nplan is None else nplan.extra["set"]["k"],
                 ahead is not None, own["nmax"] > 0, own_ahead is not None)
        nn_ = 8 * n if next is not None else 0
        ranges = (ptr(next[0]) if next is not None else 0, nn_,
                  ptr(next[1]) if next is not None else 0, nn_, ptr(targets), 4 * n, st, 1)
        # buffers the segments write, at this step's sizes before the signature (grow-only)
        X.exchange_out(own["rows"], send_splits, "rows")
        if ahead is None:
            X.exchange_out(plan.send, recv_splits, "recv")
        sig = self._signature()
        w = ops.eng.ws.get((n, ops.M, True))
        if w is not None:
            # host-side state the recorded launches read back at replay: the descriptor list
            # the backward fills, the targets' address in the tower's head arguments
            w.red_list.count = 0
            w.wgrads = []
            h = w.cache.get("head_args")
            if h is not None:
                h.targets, h.grad_prob = ptr(targets), None
                # (this step's user row ids: send positions read in place, or mini-table ids)
                h.user_ids = ptr(plan.extra["set"]["rowpos" if BACK_ROWS and GRAD_ROWS
                                                  else "inv"][0])
        scalars = (own["token"], own["nmax"], max(nu, ni))
        if next is not None and (not next[0].is_contiguous() or not next[1].is_contiguous()
                                 or next[0].dtype != torch.int64 or next[1].dtype != torch.int64):
            T.skip()      # (the plan converts such ids into temporaries: not replayable)
        res = {}

        def seg_a():
            if nplan is not None:
                ops.plan_launch(nplan, next[0].reshape(-1), next[1].reshape(-1))
                X.counts_issue(nplan)
            ops.begin(plan)
            if ahead is not None:
                recv = ahead[0]
                X.wait_ahead(*ahead)
            else:
                recv = X.exchange(plan.send, send_splits, recv_splits, slot="recv")
            if own_ahead is not None:
                ops.owner_catchup(own)
            else:
                ops.owner_prepare(recv, plan, own)
            rows = ops.owner_gather(own, recv)
            back = X.exchange(rows, recv_splits, send_splits, slot="rows")
            res["grads"], res["loss"] = ops.compute(plan, back, user_ids, item_ids, targets,
                                                   loss_denominator=user_ids.numel() * X.world)
        T.run(key_a, sig, self._pre(), ranges, scalars, seg_a, self._post_a)
        if "grads" not in res:       # replayed: the same buffers as recorded
            w = ops.eng.ws[(n, ops.M, True)]
            w.red_list.count = 0
            res["grads"] = ops._bufs["send_grads"][:(nu + ni) * 2 * ops.D].view(nu + ni, 2 * ops.D)
            res["loss"] = w.loss
            ops.last_loss = res["loss"]
        # the next plan's sizes (for its rows' exchange ahead), then the rest of the step
        nahead = None
        own_next = None
        if self.ahead and self._pending is not None:
            nxt = self._pending[2]
            X.counts_wait(nxt)
            s_, r_ = nxt.splits()
            nahead = nxt.extra["set"]["k"]
            X.site(f"ahead{nahead}", s_, r_)
            ahead_out = X.exchange_out(nxt.send, r_, f"ahead{nahead}")
            if self._claims_ahead():
                own_next = ops.owner_host(nxt)      # (host side; its claim is in segment B)
        grads = res["grads"]
        X.exchange_out(grads, recv_splits, "grads")
        key_b = ("b", n, k_set, nahead, own["nmax"] > 0, own_next is not None)
        sig = self._signature()
        scalars_b = scalars + ((own_next["token"],) if own_next is not None else (0,))

        def seg_b():
            if nahead is not None:
                self._pending[3] = X.exchange_ahead(self._pending[2])
                if own_next is not None:
                    ops.owner_claim(self._pending[3][0], own_next,
                                    self._pending[2].stream.cuda_stream, SLOT_TOKEN_NEXT)
                    self._pending[3][1].record(self._pending[2].stream.cuda_stream)
            ar = X.all_reduce_start(ops.dense_grad())
            got = X.exchange(grads, send_splits, recv_splits, slot="grads")
            ops.owner_apply(own, got)
            X.all_reduce_wait(ar)
            ops.dense_step()
        replayed = T.run(key_b, sig, self._pre(), (0, 0, 0, 0, 0, 0, st, 1), scalars_b, seg_b,
                         self._post_b)
        if own_next is not None:
            self._pending[4] = own_next
        if replayed:
            if nahead is not None:
                self._pending[3] = (ahead_out, X._ahead_ev[nahead])
            ops.step_count += 1
            ops.eng.updates += 1
        return res["loss"]

    def _pre(self):
        ops = self.ops
        d = ops.deferred
        return (tuple(d._owed), d._joined, ops.eng.pending is None)

    def _post_a(self, state):
        """Host state segment A leaves: the deferred sweep's fork (None: capture it)."""
        d = self.ops.deferred
        if state is None:
            return (tuple(d._owed), d._joined)
        d._owed, d._joined = list(state[0]), state[1]

    def _post_b(self, state):
        """Segment B closes the step: the deferred schedule's step and sweep state."""
        d = self.ops.deferred
        if state is None:
            return (tuple(d._owed), d._joined)
        d.t += 1                              # DeferredTableAdam.advance
        d._owed, d._joined = list(state[0]), state[1]
        d.engine.pending = None


class HipShardOps:
    """Per-rank work of the sharded step on the MI355X (HIP kernels through the C-ABI)."""

    def __init__(self, model, num_users: int, num_items: int, world: int, lr=1e-3,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, sweep_every=None):
        sweep_every = SWEEP_EVERY if sweep_every is None else sweep_every
        from .deferred import DeferredTableAdam
        if world > _lib.SHARD_MAX_WORLD:
            raise ValueError(f"world size {world} > {_lib.SHARD_MAX_WORLD}")
        self.model, self.U, self.I, self.W = model, num_users, num_items, world
        self.Ru, self.Ri = math.ceil(num_users / world), math.ceil(num_items / world)
        if model.num_users < self.Ru or model.num_products < self.Ri:
            raise ValueError("shard model too small for the global tables")
        self.eng = model.engine
        self.eng.ensure_layout()
        self.D = model.mlp_embedding_dim
        self.M = 1 + model.negative_samples
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.dev = self.eng.flat.device
        # device step clock: the table Adam launches read their step on the device (both kinds
        # per launch), the host never waits for it
        self.base_seed = random.getrandbits(62)
        self.clock = torch.tensor([0, self.base_seed], dtype=torch.int64, device=self.dev)
        self.deferred = DeferredTableAdam(self.eng, lr, betas, eps, weight_decay, sweep_every,
                                          clock=self.clock,
                                          overlap_sweep=bool(SHARD_OVERLAP_SWEEP))
        self.m_flat = torch.zeros_like(self.eng.flat)
        self.v_flat = torch.zeros_like(self.eng.flat)
        self.step_count = 0
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.last_loss = None
        # owner side: claim tokens and row -> unique index, one int32 per local row and kind
        ru, ri = model.num_users, model.num_products
        # (one set per plan-buffer set: a step's owner claim may run a step ahead, on the plan
        # stream, while the previous step still reads its own)
        self.marks = [[torch.zeros(ru, dtype=torch.int32, device=self.dev),
                       torch.zeros(ri, dtype=torch.int32, device=self.dev)] for _ in range(2)]
        self.uidxs = [[torch.zeros(ru, dtype=torch.int32, device=self.dev),
                       torch.zeros(ri, dtype=torch.int32, device=self.dev)] for _ in range(2)]
        self.mark, self.uidx = self.marks[0], self.uidxs[0]
        self.token = 0
        self.cnts = [torch.zeros(2, dtype=torch.int32, device=self.dev) for _ in range(2)]
        self.cnt = self.cnts[0]
        # (one that runs beside the step's stream: _lib.side_stream probes the pool's streams
        # for a hardware queue of their own — with the plan on the step's queue the world-1
        # step took 0.453-0.461 ms instead of 0.33, run r06q)
        self.plan_stream = _lib.side_stream(self.dev)
        if self.deferred.overlap and SWEEP_ON_PLAN:
            # the overlapped sweep on the plan's stream, not a stream of its own: world 1,
            # ms/step (interleaved, 3 runs each): sweep serial 0.378-0.385, overlapped on its
            # own stream 0.40-0.43, overlapped on the plan stream 0.361-0.365 (hardware queues
            # are few: GPU_MAX_HW_QUEUES=4, and RCCL's communicators hold streams of their own;
            # with 8 queues the step took 0.70 ms)
            self.deferred._side = self.plan_stream
            self.deferred._ev = (_lib.RawEvent(), _lib.RawEvent())
        self._sets = [None, None]     # double-buffered plan buffers (plan t+1 while t runs)
        self._k = 0
        self._bufs = {}

    def _st(self):
        return _lib.stream_ptr(self.dev)

    def _buf(self, name, shape, dtype=torch.float32):
        """Grow-only scratch buffer (no allocator traffic in the steady state)."""
        n = math.prod(shape)
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = self._bufs[name] = torch.empty(max(n, 1), dtype=dtype, device=self.dev)
        return b[:n].view(*shape)

    def _plan_set(self, n):
        k = self._k % 2
        self._k += 1
        s = self._sets[k]
        if s is None or s["n"] < n:
            old = s
            i64 = dict(dtype=torch.int64, device=self.dev)
            i32 = dict(dtype=torch.int32, device=self.dev)
            cap = max(n, 1)
            s = self._sets[k] = dict(
                n=n, keys=[torch.empty(cap, **i64) for _ in range(2)],
                uniq=[torch.empty(cap, **i64) for _ in range(2)],
                num_unique=torch.zeros(2, dtype=torch.int32, device=self.dev),
                inv=[torch.empty(cap, **i64) for _ in range(2)],
                counts=torch.zeros(self.W, 2, **i64), send=torch.empty(2 * cap, **i32),
                spos=[torch.empty(cap, **i32) for _ in range(2)],
                spos64=[torch.empty(cap, **i64) for _ in range(2)],
                rowpos=[torch.empty(cap, **i64) for _ in range(2)],
                bounds=torch.empty(3 * (self.W + 1), **i32),
                counts_both=torch.zeros(2 * self.W, 2, **i64),
                counts_host=torch.zeros(2 * self.W, 2, dtype=torch.int64, pin_memory=True),
                counts_ev=old["counts_ev"] if old else _lib.RawEvent(),
                ws=torch.empty(_lib.query("ncf_embedding_bwd_workspace", cap, self.D),
                               dtype=torch.uint8, device=self.dev),
                ready=old["ready"] if old else _lib.RawEvent(), k=k)
            o = s["out"] = _lib.ShardPlanOut()
            o.keys0, o.keys1 = ptr(s["keys"][0]), ptr(s["keys"][1])
            o.uniq0, o.uniq1 = ptr(s["uniq"][0]), ptr(s["uniq"][1])
            o.num_unique = ptr(s["num_unique"])
            o.inv0, o.inv1 = ptr(s["inv"][0]), ptr(s["inv"][1])
            o.counts, o.send = ptr(s["counts"]), ptr(s["send"])
            o.spos0, o.spos1 = ptr(s["spos"][0]), ptr(s["spos"][1])
            o.bounds = ptr(s["bounds"])
            o.spos64_0, o.spos64_1 = ptr(s["spos64"][0]), ptr(s["spos64"][1])
            o.rows0, o.rows1 = ptr(s["rowpos"][0]), ptr(s["rowpos"][1])
        return s

    def mark_entry(self):
        """Event on the compute stream at the start of a step call: the step's ids and the
        next step's ids are complete there, and so is the run that last used the plan buffer
        set the next plan will fill (two sets alternate).  A plan waits for this event only,
        not for the run enqueued after it, so it overlaps that run."""
        if getattr(self, "_entry", None) is None:
            self._entry = _lib.RawEvent()
        self._entry.record(self._st())

    # plan: requester-side dedup in owner order (side stream)
    def plan_host(self, uid, iid):
        """The host side of a plan: its buffer set (two alternate) and the Plan object."""
        n = uid.numel()
        s = self._plan_set(n)
        return Plan(send=s["send"], counts=s["counts"], stream=self.plan_stream,
                    extra={"set": s, "n": n, "counts_both": s["counts_both"],
                           "counts_host": s["counts_host"], "counts_ev": s["counts_ev"]})

    def plan_launch(self, plan, uid, iid):
        """The plan's launches on the side stream, after the step entry."""
        s, n = plan.extra["set"], plan.extra["n"]
        if getattr(self, "_entry", None) is None:
            self.mark_entry()
        ps = self.plan_stream.cuda_stream
        self._entry.wait(ps)
        _lib.call("ncf_shard_plan", ptr(uid), ptr(iid), n, self.W, self.U, self.I, self.D,
                  ctypes.addressof(s["out"]), ptr(s["ws"]), s["ws"].numel(), ptr(self.err), ps)
        s["ready"].record(ps)

    def plan(self, uid, iid, world):
        p = self.plan_host(uid, iid)
        self.plan_launch(p, uid, iid)
        return p

    def begin(self, plan):
        plan.extra["set"]["ready"].wait(self._st())

    # 2. owner side: sort-free dedup of the received rows, catch-up, gather
    def _layout(self, counts, par=0):
        ls = self.__dict__.setdefault("_recv_layouts", [None, None])
        L = ls[par] = ls[par] or _lib.ShardRecv()
        L.world = self.W
        off = 0
        for s in range(self.W):
            L.start[s] = off
            L.n0[s] = counts[s][0]
            off += counts[s][0] + counts[s][1]
        L.start[self.W] = off
        return L

    def owner_host(self, plan):
        """Host side of the owner phase of a step: the receive layout (one persistent host
        struct per plan-buffer set), the claim token and the sizes; the buffers sized for them
        (the per-step ones of the plan's set: its claim may run a step ahead)."""
        par = plan.extra["set"]["k"]
        L = self._layout(plan.recv_counts, par)
        tu = sum(c[0] for c in plan.recv_counts)
        ti = sum(c[1] for c in plan.recv_counts)
        nmax = max(tu, ti)
        # (both sets' buffers grown together: a launch tape's signature holds their addresses,
        # and a set first allocated a few steps in would drop the tapes recorded before)
        for q in (1 - par, par):       # (par last: its buffers are the ones returned)
            uq = [self._buf(f"own_uq0_{q}", (max(tu, 1),), torch.int64),
                  self._buf(f"own_uq1_{q}", (max(ti, 1),), torch.int64)]
            pos = [self._buf(f"own_pos0_{q}", (max(tu, 1), self.W), torch.int32),
                   self._buf(f"own_pos1_{q}", (max(ti, 1), self.W), torch.int32)]
        self.token += 1
        total = L.start[self.W]
        rows = self._buf("own_rows", (max(total, 1), 2 * self.D))[:total]
        G = [self._buf(f"own_g{j}", (max(nmax, 1), self.D)) for j in range(4)]
        return {"layout": L, "uniq": uq, "pos": pos, "nmax": nmax, "token": self.token,
                "rows": rows, "G": G, "par": par, "cnt": self.cnts[par]}

    def owner_claim(self, recv, own, st, token_slot=SLOT_TOKEN):
        """The owner's sort-free dedup of the received rows (claim + positions) on stream st."""
        L, uq, pos, par = own["layout"], own["uniq"], own["pos"], own["par"]
        mk, ux = self.marks[par], self.uidxs[par]
        _lib.call_tagged("ncf_shard_owner_prepare", {2: token_slot}, ptr(recv), ctypes.addressof(L),
                         own["token"], ptr(mk[0]), ptr(mk[1]), ptr(ux[0]), ptr(ux[1]),
                         mk[0].numel(), mk[1].numel(), ptr(uq[0]), ptr(uq[1]), ptr(own["cnt"]),
                         ptr(pos[0]), ptr(pos[1]), ptr(self.err), st)

    def owner_catchup(self, own):
        """The claimed rows caught up through the current step (on the step's stream)."""
        d = self.deferred
        if own["nmax"] > 0:
            d._ensure(d.t + 1)
            pairs = self._pairs(own["uniq"])
            _lib.call_tagged("ncf_adam_pairs_catchup_clock", {4: SLOT_NMAX},
                             ctypes.addressof(pairs), 2, self.D, ptr(own["cnt"]), own["nmax"], 0,
                             ptr(self.clock), ptr(d._table), *d._consts(), self._st())

    def owner_prepare(self, recv, plan, own=None):
        own = own or self.owner_host(plan)
        self.owner_claim(recv, own, self._st())
        self.owner_catchup(own)
        return own

    def _pairs(self, uq, G=None):
        """ncf_table_pair[2] for the owner's unique rows (cached: the buffers are stable)."""
        key = (ptr(uq[0]), ptr(uq[1])) + (tuple(ptr(g) for g in G) if G is not None else ())
        cache = self.__dict__.setdefault("_pairs_cache", {})
        pairs = cache.get(key)
        if pairs is None:
            pairs = cache[key] = self.deferred._pairs()
            for k in (0, 1):
                pairs[k].row_ids = ptr(uq[k])
                if G is not None:
                    pairs[k].g0, pairs[k].g1 = ptr(G[2 * k]), ptr(G[2 * k + 1])
        return pairs

    def owner_gather(self, own, recv):
        L = own["layout"]
        out = own["rows"]
        tb = self.eng.table_params()
        _lib.call("ncf_shard_owner_gather", ptr(recv), ctypes.addressof(L), ptr(tb["mf_user"]),
                  ptr(tb["mlp_user"]), self.mark[0].numel(), ptr(tb["mf_item"]),
                  ptr(tb["mlp_item"]), self.mark[1].numel(), self.D, ptr(out), self._st())
        return out

    # 3.-4. forward + backward on the mini tables
    def compute(self, plan, back, uid, iid, targets, loss_denominator):
        st = self._st()
        eng, s = self.eng, plan.extra["set"]
        n = plan.extra["n"]
        nu, ni = plan.totals()
        D = self.D
        back_rows = BACK_ROWS and GRAD_ROWS
        if back_rows:
            # the received rows read in place: [mf | mlp] halves, 2 D floats a row, each batch row
            # at its send position (the plan's rowpos)
            bp = ptr(back)
            mini = {"mf_user": bp, "mlp_user": bp + 4 * D, "mf_item": bp, "mlp_item": bp + 4 * D}
        else:
            # mini tables: four [n][D] slabs of one buffer sized for the batch (unique rows <= n)
            base = ptr(self._buf("mini", (4, max(n, 1), D)))
            slab = 4 * max(n, 1) * D
            mini = {"mf_user": base, "mlp_user": base + slab, "mf_item": base + 2 * slab,
                    "mlp_item": base + 3 * slab}
            _lib.call_tagged("ncf_shard_rows", {4: SLOT_NUNI}, ptr(back), ptr(s["spos"][0]),
                             ptr(s["spos"][1]), ptr(s["num_unique"]), max(nu, ni), D,
                             mini["mf_user"], mini["mlp_user"], mini["mf_item"],
                             mini["mlp_item"], 0, st)
        m = self.model
        drop_p = float(m.dropout)
        seed = 0      # the dropout stream comes from the device clock's per-step seed
        if back_rows:
            inv_u, inv_i = s["rowpos"][0][:n], s["rowpos"][1][:n]
            # (bound of the send positions: 2 n >= nu + ni, fixed per batch size — a launch tape
            # replays this call's scalars, so a per-step count would go stale)
            rb = max(2 * n, 1)
            bounds, ld = (rb, rb), 2 * D
            uq = (s["spos64"][0], s["spos64"][1])
        else:
            inv_u, inv_i = s["inv"][0][:n], s["inv"][1][:n]
            # (mini-table bounds: the batch size, a bound of the unique-row counts that does not
            # change per step; the plan's inverse ids are always in range)
            bounds, ld = (max(n, 1), max(n, 1)), None
            ar = self._buf("arange", (max(n, 1),), torch.int64)
            if self._bufs.get("arange_n") != ar.numel():
                torch.arange(ar.numel(), out=ar)
                self._bufs["arange_n"] = ar.numel()
            uq = (ar, ar)
        w = eng.workspace(n, self.M, True)
        w.emb_ws = s["ws"]            # the plan's dedup segments drive the segment reduce

        def mark(wk, u, i, st_):
            wk.deduped = True
        eng.forward(inv_u, inv_i, self.M, True, drop_p, seed, prepare=mark, tables=mini,
                    rows=bounds, table_ld=ld)
        g = self._buf("send_grads", (max(2 * n, 1), 2 * D))      # (nu + ni <= 2 n rows)
        # the table gradients straight into the send buffer at their send positions
        # (GRAD_ROWS; else compact rows, then ncf_shard_rows re-orders them)
        eng.backward(w, inv_u, inv_i, None, targets, drop_p, seed,
                     loss_denominator=loss_denominator, tables=mini,
                     rows=(self.W * self.Ru, self.W * self.Ri), uniq=uq,
                     grad_rows=(g, s["spos"][0], s["spos"][1]) if GRAD_ROWS else None,
                     table_ld=ld)
        eng.pending = None
        if not GRAD_ROWS:
            _lib.call_tagged("ncf_shard_rows", {4: SLOT_NUNI}, ptr(g), ptr(s["spos"][0]),
                             ptr(s["spos"][1]), ptr(s["num_unique"]), max(nu, ni), D,
                             ptr(w.G["mf_user"]), ptr(w.G["mlp_user"]), ptr(w.G["mf_item"]),
                             ptr(w.G["mlp_item"]), 1, st)
        self.last_loss = w.loss
        return g[:nu + ni], w.loss

    # 5. owner side: sum received gradients per unique row (rank order), apply the step
    def owner_apply(self, own, got):
        st = self._st()
        uq, pos, nmax, G, cnt = own["uniq"], own["pos"], own["nmax"], own["G"], own["cnt"]
        d = self.deferred
        if not GSUM_APPLY:
            _lib.call_tagged("ncf_shard_owner_gradsum", {4: SLOT_NMAX}, ptr(got), ptr(pos[0]),
                             ptr(pos[1]), ptr(cnt), nmax, self.W, self.D, ptr(G[0]),
                             ptr(G[1]), ptr(G[2]), ptr(G[3]), st)
        d._ensure(d.t + 1)
        d.sweep_join()
        d._settle(st)
        if nmax > 0 and GSUM_APPLY:
            # the rank-order gradient sum inside the apply (one launch, the same bits)
            pairs = self._pairs(uq)
            _lib.call_tagged("ncf_adam_pairs_apply_gsum_clock", {4: SLOT_NMAX},
                             ctypes.addressof(pairs), 2, self.D, ptr(cnt), nmax, 1, ptr(got),
                             ptr(pos[0]), ptr(pos[1]), self.W, ptr(self.clock), ptr(d._table),
                             *d._consts(), st)
        elif nmax > 0:
            pairs = self._pairs(uq, G)
            _lib.call_tagged("ncf_adam_pairs_apply_clock", {4: SLOT_NMAX}, ctypes.addressof(pairs),
                             2, self.D, ptr(cnt), nmax, 1, ptr(self.clock), ptr(d._table),
                             *d._consts(), st)
        d.advance(st)                               # rolling sweep of step t + 1 (clock)

    def dense_grad(self):
        self.eng.join_reductions()
        return self.eng.flat_grad

    def dense_step(self):
        self.step_count += 1
        self.eng.updates += 1
        b1, b2 = self.betas
        st = self._st()
        _lib.call("ncf_adam_flat_clock_close", ptr(self.eng.flat), ptr(self.eng.flat_grad),
                  ptr(self.m_flat), ptr(self.v_flat), self.eng.flat.numel(),
                  ptr(self.deferred._table), 1, ptr(self.clock), b1, b2, self.eps, self.wd,
                  self.base_seed, st)

    def check(self):
        """Raise IndexError if any step saw an out-of-range id (one host sync)."""
        e = int(self.err.item())
        if e:
            raise IndexError(f"row-sharded step: out-of-range ids (flags {e:#x})")


def shard_rows(rows: int, world: int) -> int:
    return (rows + world - 1) // world


def make_sharded_step(model_factory, num_users, num_items, group=None, plan_group=None,
                      exchange=None, **adam):
    """Build the local shard model (tables of ceil(rows / W) rows) and its sharded step.
    Dense parameters are broadcast from rank 0 so every replica starts identical.  A second
    communicator for the pipelined plan's count exchange is created unless given.
    ``exchange``: "rccl" (the C-ABI collectives, default on the nccl backend) or "torch"
    (torch.distributed collectives); the module's EXCHANGE overrides the default."""
    world = dist.get_world_size(group)
    model = model_factory(shard_rows(num_users, world), shard_rows(num_items, world))
    dev = model.mf_norm.weight.device
    eng = model.engine
    eng.ensure_layout()
    dist.broadcast(eng.flat, src=0, group=group)
    if plan_group is None:
        ranks = list(range(world)) if group is None else dist.get_process_group_ranks(group)
        plan_group = dist.new_group(ranks)
    ops = HipShardOps(model, num_users, num_items, world, **adam)
    kind = exchange or EXCHANGE or (
        "rccl" if dist.get_backend(group) == "nccl" else "torch")
    if kind not in ("rccl", "torch"):
        raise ValueError(f"exchange must be 'rccl' or 'torch', not {kind!r}")
    X = (RcclExchange if kind == "rccl" else ShardExchange)(group, dev, plan_group)
    return model, ShardedTrainStep(ops, X)
