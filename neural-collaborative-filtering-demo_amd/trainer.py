"""Training loop for AdvancedNCF on MI355X.

``ModelTrainer.train_epoch`` mirrors the reference loop (src/model/trainer.py:216-337): per batch
``model(features)`` -> ``nn.BCELoss`` -> ``zero_grad`` -> ``backward`` -> no clipping (the
reference's ``hasattr(dict, 'gradient_clipping')`` guard at :279 is always False) ->
``Adam.step`` with lr / weight_decay from the config (:54-75).  The BigQuery / DataLoader side of
the reference trainer is out of scope; batches are (KeyedJaggedTensor, targets[N, 1]) exactly as
``collate_recommender_batch`` builds them (src/model/data_prep.py:230-320).

``FusedTrainStep`` is the same step without autograd or host syncs: forward kernels, fused
BCE + backward kernels, fused Adam — identical math, one kernel sequence on one stream.  It is
what the benchmark times (and what a production trainer uses).
"""
import logging
import weakref
from typing import Any, Dict, Optional  # noqa: F401

import torch
import torch.nn as nn

from . import _lib
from . import deferred as deferred_mod
from ._lib import ptr

log = logging.getLogger(__name__)


# Where the next batch's id sort is launched on the side stream: "entry" (the step's start) or
# one of the engine's fork points ("tower", "mlp_bwd", "attn_bwd", "emb_bwd", "reduce").
# Measured at C2 with the rolling sweep forked at mlp_bwd (ms/step): entry 0.319-0.321, tower
# 0.325, mlp_bwd 0.341, attn_bwd 0.312-0.314, emb_bwd 0.318-0.319, reduce 0.332-0.334: beside the
# attention / embedding backward, after the sweep has taken the tower backward's idle slots.
# "sweep" (the default): queued behind the overlapped sweep on its stream when the sweep forks
# this step (else at attn_bwd), joined by the sweep's own join: no event record or wait of its
# own on the step's queue, where each costs ~5 us (0.2986-0.2992 against 0.3020-0.3040 ms/step
# at attn_bwd, r3ax_*).
DEDUP_FORK = "sweep"
# Steps of per-step Adam scalars a captured step graph is given before it must be re-captured
# (the scalar table cannot grow from inside a replay); tests shrink it to force re-captures.
GRAPH_HORIZON = 1 << 16
# The dense-gradient reductions on a side stream beside the table Adam's apply (engine.backward
# reduce_async, a stream of its own; joined before the flat Adam close): measured slower (0.379
# against 0.288 ms/step: a third stream shares a hardware queue)
REDUCE_ASYNC = False
# The fused tower/attention backward's reductions queued on the overlapped sweep's side stream
# right after that kernel (engine.backward reduce_side), beside the embedding backward and the
# table Adam; joined before the flat Adam close.  Same bits (the bitwise suite runs it).  Off:
# measured slower (3 interleaved runs each: 0.3028 / 0.3033 against 0.2866 / 0.2888 ms/step —
# the 105 MB of partials read beside the embedding backward and the apply slow both)
EARLY_REDUCE = False
# The deferred table Adam's apply of the step fused into the embedding backward
# (ncf_embedding_bwd_reduce_apply_clock: a row steps where its gradient rows complete; the same
# bits as the separate apply)
FUSE_APPLY = True
# The rolling sweep's period (every row current at least every SWEEP_EVERY steps).  A longer
# period halves the sweep's HBM traffic beside the forward; the replayed element-steps are the
# same in total (moved from the sweep to the catch-up, which now runs beside the reductions:
# deferred.LATE_CATCHUP).  At C2 steady state, 3 interleaved runs each: 0.2703 / 0.2709 ms/step
# at 128 against 0.2769-0.2794 at 64 (tools/step_ab.py, primed 2 x the period); round 6 (run
# r06zx, min of 3): 128 0.2653, 192 0.2632, 256 0.2669 — within the runs' spread, 128 stays.
SWEEP_EVERY = 128
# The step's join of the side stream (sweep, next sort, late catch-up) after the dense Adam
# rather than before it: the flat Adam (ncf_adam_flat_clock) runs first, then the join, then the
# clock advance (ncf_step_clock_advance) that the side kernels must not see early.  A join whose
# event is still pending costs the queue ~10 us after the signal (tools/event_cost.py); placed
# later, the side work is usually complete when the queue reaches it.  Off: measured neutral
# (3 interleaved runs each, 0.2706 / 0.2714 against 0.2706 / 0.2707 ms/step: the separate
# clock-advance launch costs what the later join saves)
SPLIT_CLOSE = False
# Trainer.train_epoch runs loss.backward() on the calling thread (torch's autograd otherwise hands
# every backward of CUDA tensors to a per-device worker thread and waits for it: two thread
# wake-ups per step, on a host that is the bottleneck of this loop).  The reference loop at C2
# (tools/dropin_host.py, run r06p): 0.368 -> 0.317 ms/step.  Scoped to the epoch (the
# torch.autograd.set_multithreading_enabled context manager); the numbers are the same bits.
CALLING_THREAD_BACKWARD = True
# The late catch-up of the next batch's rows (deferred.LATE_CATCHUP) left running past the step:
# the step's join before the clock advance waits for the sweep and the sort only, the late
# catch-up reads its target from a copy of the clock taken before that join, and the next user
# of the tables waits for it (deferred.late_join: the next prepare, a flush, a sync).  Without
# it the step's stream reached that join before the catch-up (~30 us, queued behind the apply)
# was done and resumed ~10 us after it (rocprof r06k: an 11.5 us gap before the flat Adam).
# Off: measured neutral (run r06zf, 3 interleaved runs each: min 0.2726 ms/step on, 0.2713 off;
# the gap moves to the next step's prepare, where the catch-up is still running beside the
# forward's head).  Bitwise-green either way (the late catch-up / early catch-up tests).
LATE_DETACHED = False
# The side stream's work of a step queued at the step's entry, off the step's queue: the next
# batch's id sort, then the rolling sweep owed by the closed step, their step targets read from a
# side copy of the clock set from the host's counter (deferred.side_clock), and the late catch-up
# at the table apply as before, from the same copy.  The step's stream records one event (the
# table apply done) and waits once (for the late catch-up, before the next gather): no fork
# event at the tower, no join before the clock advance.  Three dedup sets (the sort at the entry
# of step T + 1 writes the set of step T - 1, whose reductions are queued before the event the
# side stream waited for in step T).  Off: measured slower (run r06zj, tools/step_ab.py, 3
# interleaved runs each: C2 min 0.2795 against 0.2698 ms/step, B = 256 0.1669 against 0.1637 —
# the sweep beside the reductions and the next gather runs longer than beside the fused forward
# (64 against 50 us), more than the fork event it saves); bit-identical (its tests run it).
SIDE_AHEAD = False


def _join_side_streams(dev, streams):
    """FusedTrainStep finalizer: the current stream of `dev` waits for each side stream."""
    try:
        if torch.cuda.is_current_stream_capturing():
            return          # (not inside another step's graph capture: nothing may join it)
        cur = torch.cuda.current_stream(dev)
        for s in streams:
            cur.wait_stream(s)
    except Exception:       # (interpreter shutdown: the runtime may be gone already)
        pass


class FusedTrainStep:
    """forward + BCE + backward + Adam for one batch, on the current HIP stream, no host sync.

    ``deferred=True`` (default) updates the embedding tables with the deferred dense-exact
    schedule (deferred.py: bit-identical to the dense sweep, without streaming untouched rows);
    ``deferred=False`` sweeps every table every step (ncf_adam_table).  Adam state lives in
    ``self.state`` with torch's keys; ``export_optimizer_state`` copies it into a
    torch.optim.Adam's ``state`` for checkpointing in torch's format.

    ``graph=True`` captures the whole step once as a hipGraph (torch.cuda.CUDAGraph) and replays
    it: ~50 launches for the price of one, no per-step host work.  Every step-dependent value
    (Adam step, rolling-sweep slice, dropout stream) then lives in a device ``ncf_step_clock``
    that the last kernel of the step advances (``clock=True`` uses the clock without capture;
    the two are bit-identical).  Inputs are copied into static buffers before each replay."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5,
                 deferred: bool = True, sweep_every: int = SWEEP_EVERY, graph: bool = False,
                 clock: Optional[bool] = None, warmup: int = 2, concurrent: Optional[bool] = None,
                 overlap_sweep: Optional[bool] = None, table_dtype: torch.dtype = torch.float32):
        self.model = model
        self.deferred = None
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        if model.mf_embedding_dim != model.mlp_embedding_dim:
            # the deferred schedule steps an MF and an MLP table as one pair of one width: the
            # dense per-step sweep (the same values) when the collections differ
            if graph or clock or table_dtype != torch.float32:
                raise ValueError("mf_embedding_dim != mlp_embedding_dim: fp32 tables, eager, "
                                 "the dense table schedule")
            deferred, clock = False, False
        self.step_count = 0
        eng = model.engine
        eng.ensure_layout()
        dev = eng.flat.device
        self.tables = eng.table_params()
        self.state = {k: {"exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
                      for k, p in self.tables.items()}
        # bf16-table configuration (BASELINE.json configs[1] "bf16", SURVEY 8(d) C2: tables bf16,
        # Adam moments fp32): the four tables live as bf16 (half the row bytes of every gather,
        # segment reduce and table update); the model's fp32 table parameters hold the same
        # values widened, brought up to date by sync() (state_dict, eval forward, exports).
        if table_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("table_dtype must be torch.float32 or torch.bfloat16")
        self.bf16 = table_dtype == torch.bfloat16
        self.tables_lp = None
        if self.bf16:
            with torch.no_grad():
                self.tables_lp = {k: p.detach().to(torch.bfloat16) for k, p in self.tables.items()}
                for k, p in self.tables.items():
                    p.copy_(self.tables_lp[k])
        self.m_flat = torch.zeros_like(eng.flat)
        self.v_flat = torch.zeros_like(eng.flat)
        self.last_loss = None
        self.graph = bool(graph)
        # the device step clock is the default whenever the deferred schedule is on (both kinds
        # per launch, no host step arguments; bit-identical to the host-driven form)
        self.use_clock = (self.graph or deferred) if clock is None else bool(clock)
        if self.graph and not self.use_clock:
            raise ValueError("graph capture needs the step clock")
        self.clock = None
        if self.use_clock:
            if not deferred:
                raise ValueError("the step clock drives the deferred table Adam (deferred=True)")
            self.base_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            # ncf_step_clock {int32 t, int32 reserved, uint64 seed}: t = 0, seed of step 1
            self.clock = torch.tensor([0, self.base_seed], dtype=torch.int64, device=dev)
            eng.clock = self.clock
        self.deferred = None
        if overlap_sweep is None:    # the overlapped rolling sweep (deferred.py): on by default
            overlap_sweep = deferred_mod.OVERLAP_SWEEP
        if deferred:
            from .deferred import DeferredTableAdam
            self.deferred = DeferredTableAdam(eng, lr, betas, eps, weight_decay, sweep_every,
                                              moments=self.state, clock=self.clock,
                                              overlap_sweep=overlap_sweep and self.clock is not None,
                                              param_tables=self.tables_lp)
        self.warmup = warmup
        # independent kernels on side streams.  Off by default: measured slower on MI355X, eager
        # (0.63 vs 0.54 ms) and captured (0.71 vs 0.58 ms) — a cross-queue dependency costs more
        # than the overlap of these short kernels wins
        eng.concurrent = bool(concurrent)
        self._g = None
        self._static = None
        self._w = None
        self._eager_steps = 0
        # side streams whose work may outlive a step (SIDE_AHEAD; the dedup fork at "entry"):
        # when the step is dropped, the stream it was built on waits for them before the
        # caching allocator can hand their buffers (the model's, this step's) to new work there
        self._side_streams = []
        if self.deferred is not None and self.deferred._side is not None:
            self._side_streams.append(self.deferred._side)
        weakref.finalize(self, _join_side_streams, dev, self._side_streams)

    @property
    def lr(self):
        return self._lr

    @lr.setter
    def lr(self, value):
        """The learning rate of the steps not yet taken, for the dense parameters and the
        deferred table schedule alike (its per-step scalar table is refilled from step t + 1;
        a captured graph reads that table, so it needs no re-capture)."""
        self._lr = float(value)
        if self.deferred is not None:
            self.deferred.lr = self._lr

    def _body(self, user_ids, item_ids, targets, M):
        m = self.model
        eng = m.engine
        drop_p = float(m.dropout)
        seed = 0
        if drop_p > 0 and self.clock is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        prep = self.deferred.prepare if self.deferred is not None else None
        w = eng.forward(user_ids, item_ids, M, True, drop_p, seed, prepare=prep,
                        tables=self.tables_lp, bf16=self.bf16)
        # (REDUCE_ASYNC: the dense-gradient reductions beside the table Adam)
        d = self.deferred
        side = (d.side_stream() if EARLY_REDUCE and d is not None and d.overlap and not self.graph
                and not REDUCE_ASYNC else None)
        fa = d.fused_apply_args(w) if FUSE_APPLY and d is not None else None
        # (the late catch-up is read when the table apply has been queued, not here: the sweep
        # fork, and with it the next batch's prefetch, may sit in the backward — "mlp_bwd")
        done = self._tables_done if fa is not None else None
        eng.backward(w, user_ids, item_ids, None, targets, drop_p, seed, tables=self.tables_lp,
                     bf16=self.bf16, reduce_async=REDUCE_ASYNC and not self.graph,
                     reduce_side=side, fused_apply=fa, tables_done=done)
        st = _lib.stream_ptr(eng.flat.device)
        b1, b2 = self.betas
        split = (SPLIT_CLOSE and self.deferred is not None and self.clock is not None
                 and not self.graph and self.deferred.overlap)
        # (SIDE_AHEAD: no join of the side stream in the step unless a sweep part reading the
        # live clock was forked in it — the closed step's sweep could not run at the entry)
        free = self._ahead() and not d._live_pending
        if self.deferred is not None:
            self.deferred.apply(w, st, late_join=split or free)
        elif self.bf16:      # dense bf16 sweep (the reference schedule of the bf16 tables)
            D = self.model.mlp_embedding_dim
            for key, lp in self.tables_lp.items():
                slot = eng.slot_u if key.endswith("user") else eng.slot_i
                s_ = self.state[key]
                _lib.call("ncf_adam_table_bf16", ptr(lp), ptr(s_["exp_avg"]), ptr(s_["exp_avg_sq"]),
                          lp.shape[0], D, ptr(slot), ptr(w.G[key]), self.lr, b1, b2, self.eps,
                          self.wd, float(self.step_count + 1), st)
            eng.release_pending(st)
        else:
            hp = lambda p: (self.lr, b1, b2, self.eps, self.wd)  # noqa: E731
            key_of = {id(p): k for k, p in self.tables.items()}
            eng.adam_tables(hp, lambda p: self.state[key_of[id(p)]], float(self.step_count + 1), st)
        eng.join_reductions()
        if self.clock is not None and split:
            _lib.call("ncf_adam_flat_clock", ptr(eng.flat), ptr(eng.flat_grad), ptr(self.m_flat),
                      ptr(self.v_flat), eng.flat.numel(), ptr(self.deferred._table), 1,
                      ptr(self.clock), b1, b2, self.eps, self.wd, st)
            self.deferred.sweep_join()       # (the clock advance below changes its target)
            _lib.call("ncf_step_clock_advance", ptr(self.clock), self.base_seed, st)
        elif self.clock is not None:
            if self.deferred is not None and not free:
                self.deferred.sweep_join()   # (the clock advance below changes its target)
            _lib.call("ncf_adam_flat_clock_close", ptr(eng.flat), ptr(eng.flat_grad),
                      ptr(self.m_flat), ptr(self.v_flat), eng.flat.numel(),
                      ptr(self.deferred._table), 1, ptr(self.clock), b1, b2, self.eps, self.wd,
                      self.base_seed, st)
        else:
            _lib.call("ncf_adam_flat", ptr(eng.flat), ptr(eng.flat_grad), ptr(self.m_flat),
                      ptr(self.v_flat), eng.flat.numel(), self.lr, b1, b2, self.eps, self.wd,
                      float(self.step_count + 1), st)
        return w

    def _tables_done(self):
        """Engine hook, right after the embedding backward with the table apply fused in was
        queued: the late catch-up of the next batch's rows, if this step's prefetch sorted them
        (at the sweep fork, in the forward or the backward) and no early catch-up ran."""
        late, self._late_next = self._late_next, None
        if late is not None:
            self._late_catchup(*late)
        elif self._ahead():      # (the closed step's sweep may then run at the next entry)
            d = self.deferred
            ev = self._event()
            ev.record(_lib.stream_ptr(self.model.engine.flat.device))
            ev.wait(d.side_stream().cuda_stream)
            d.side_ordered()

    def _late_catchup(self, s, n):
        """deferred.LATE_CATCHUP: the next batch's rows (dedup set s, sorted on the side stream)
        caught up through this step there, after this step's table apply (queued just before, in
        the embedding backward) — beside the dense-gradient reductions; the step's sweep join
        (before the clock advance) waits for it."""
        d = self.deferred
        side = d.side_stream()
        clk = None
        ahead = self._ahead()
        if LATE_DETACHED and not ahead and d._late_clock is None:
            d._late_clock = torch.zeros_like(self.clock)
        ev = self._event()     # (also orders the copy below after the copy buffer's creation)
        ev.record(_lib.stream_ptr(self.model.engine.flat.device))
        ev.wait(side.cuda_stream)
        if ahead:
            d.side_ordered()
            clk = d.side_clock(side.cuda_stream)
        elif LATE_DETACHED:
            # the clock as this step's catch-up needs it, copied on the side stream ahead of the
            # step's join (the advance after that join cannot overtake the copy)
            clk = d._late_clock
            _lib.call("ncf_memcpy_async", ptr(clk), ptr(self.clock), 16, side.cuda_stream)
            d.sweep_done(side.cuda_stream)
            d._joined = False
        if _lib.PROFILE is not None:     # (the per-launch instrumentation times it on its stream)
            with torch.cuda.stream(side):
                d.late_catchup(s, n, side.cuda_stream, clk)
        else:
            d.late_catchup(s, n, side.cuda_stream, clk)
        if LATE_DETACHED or ahead:
            evs = getattr(self, "_late_evs", None)
            if evs is None:
                evs = self._late_evs = [_lib.RawEvent(stream_only=True) for _ in range(2)]
            evs.reverse()
            evs[0].record(side.cuda_stream)
            d._late_ev = evs[0]
        else:
            d.sweep_done(side.cuda_stream)
            d._joined = False

    # ---- pipelined dedup: the id sort of step t+1 runs on a side stream under step t
    def _event(self):
        """The next of a ring of stream-to-stream events (the pipelined dedup's fork / join:
        never waited on by the host; a wait is enqueued before its event is recorded again)."""
        ring = getattr(self, "_evring", None)
        if ring is None:
            ring = self._evring = [[_lib.RawEvent(stream_only=True) for _ in range(8)], 0]
        ring[1] = (ring[1] + 1) % len(ring[0])
        return ring[0][ring[1]]

    def _dedup_sets(self, w):
        """A ring of sets of the dedup outputs (sorted segments, unique ids, counts) for
        workspace w, used in turn by consecutive steps: the workspace's own buffers and a twin
        (a third with SIDE_AHEAD).  {"ring": [...], "i": the current step's set}."""
        k = 3 if self._ahead() else 2
        sets = w.cache.get(("dedup_sets", k))
        if sets is None:
            a = dict(emb_ws=w.emb_ws, uniq_u=w.uniq_u, uniq_i=w.uniq_i, num_unique=w.num_unique)
            ring = [a] + [{n: torch.empty_like(v) for n, v in a.items()} for _ in range(k - 1)]
            sets = w.cache[("dedup_sets", k)] = {"ring": ring, "i": 0}
        return sets

    @staticmethod
    def _next_set(sets):
        return sets["ring"][(sets["i"] + 1) % len(sets["ring"])]

    def _ahead(self):
        """SIDE_AHEAD applies: eager, the overlapped sweep, the late catch-up behind the fused
        table apply (deferred.EARLY_CATCHUP = False)."""
        d = self.deferred
        return (SIDE_AHEAD and not self.graph and d is not None and d.overlap and FUSE_APPLY
                and deferred_mod.LATE_CATCHUP and deferred_mod.EARLY_CATCHUP is False)

    def _prefetch_dedup(self, w, uid, iid, entry, side=None):
        """Dedup of the NEXT step's ids into the idle set, on the side stream, after `entry`
        (the start of this step: the run that last used that set is complete there).  With
        ``side`` (and no entry): on that stream, already ordered after such a point."""
        s = self._next_set(self._dedup_sets(w))
        eng = self.model.engine
        m = self.model
        if side is not None:
            self._enqueue_dedup(s, w, uid, iid, side)
            # its rows this step does not touch caught up through this step behind the sort
            # (early), or once this step's apply has run (late: _late_catchup)
            if not self.deferred.early_catchup(s, uid.numel(), side.cuda_stream) and \
                    deferred_mod.LATE_CATCHUP and FUSE_APPLY:
                self._late_next = (s, uid.numel())
            # the sweep's done-event re-recorded behind the sort: the step's sweep join (before
            # the clock advance) then orders the sort too, and the next step waits for nothing
            d = self.deferred
            d.sweep_done(side.cuda_stream)
            self._pending = (uid, iid, None)
            return
        if getattr(self, "_side", None) is None:
            self._side = _lib.side_stream(eng.flat.device)
            self._side_streams.append(self._side)
        side = self._side
        entry.wait(side.cuda_stream)
        self._enqueue_dedup(s, w, uid, iid, side)

    def _entry_side(self, w, uid, next):
        """SIDE_AHEAD, at the step's entry, on the deferred schedule's side stream (ordered
        after the previous step's table apply by its tables-done event, nothing recorded on the
        step's stream): the next batch's id sort into the next set of the ring, then the
        rolling sweep the previous step owes (deferred.sweep_owed, its target from the side
        clock)."""
        d = self.deferred
        side = d.side_stream()
        d.side_clock(side.cuda_stream)
        if next is not None and next[0].numel() == uid.numel():
            s = self._next_set(self._dedup_sets(w))
            self._enqueue_dedup(s, w, next[0], next[1], side)
            self._late_next = (s, next[0].numel())
        if d.sweep_owed(side.cuda_stream):
            self.model.engine.fork_hook = None

    def _enqueue_dedup(self, s, w, uid, iid, side):
        m = self.model
        u = uid.reshape(-1)
        i = iid.reshape(-1)
        s.pop("late_t", None)
        _lib.call("ncf_dedup_ids", ptr(u), ptr(i), u.numel(), w.g.D, m.num_users,
                  m.num_products, ptr(s["uniq_u"]), ptr(s["uniq_i"]), None, None,
                  ptr(s["num_unique"]), ptr(s["emb_ws"]), s["emb_ws"].numel(), side.cuda_stream)
        ev = self._event()
        ev.record(side.cuda_stream)
        self._pending = (uid, iid, ev)          # the caller's objects: matched by identity

    def _activate_dedup(self, w, uid, iid, ahead=False):
        """Point w at this step's dedup set: the prefetched one when it was made for these ids
        (the step then waits for its event instead of sorting), else the next set, sorted
        inline by the deferred Adam's prepare."""
        sets = self._dedup_sets(w)
        pend, self._pending = getattr(self, "_pending", None), None
        sets["i"] = (sets["i"] + 1) % len(sets["ring"])
        s = sets["ring"][sets["i"]]
        w.emb_ws, w.uniq_u, w.uniq_i, w.num_unique = s["emb_ws"], s["uniq_u"], s["uniq_i"], s["num_unique"]
        w.prededuped = None
        late_t, w.late_t = s.pop("late_t", None), None
        if pend is not None:
            cur = torch.cuda.current_stream(self.model.engine.flat.device)
            mine = pend[0] is uid and pend[1] is iid
            if pend[2] is None:               # sorted behind the sweep: joined with it
                self.deferred.sweep_join()
            elif not (ahead and mine and late_t is not None):
                pend[2].wait(cur.cuda_stream)  # (also orders a stale prefetch before reuse)
            # (else: the late catch-up queued behind that sort, which the step's prepare
            # waits for, orders it — deferred.late_join)
            if mine:
                w.prededuped = True
                w.late_t = late_t

    def __call__(self, user_ids: torch.Tensor, item_ids: torch.Tensor, targets: torch.Tensor,
                 M: Optional[int] = None, next=None):
        """One step.  ``next=(user_ids, item_ids)`` of the following step lets its id sort run
        on a side stream under this step (deferred clock path, eager; same results).  The next
        call must pass those very tensor objects, unmodified, to use the prefetched sort."""
        m = self.model
        M = M or (1 + m.negative_samples)
        self._late_next = None     # set by this step's prefetch (_prefetch_dedup / _entry_side)
        if not self.graph:
            pipe = self.deferred is not None and self.clock is not None and (
                next is not None or getattr(self, "_pending", None) is not None)
            ahead = self._ahead()
            if pipe:
                eng = m.engine
                eng.ensure_layout()
                w0 = eng.workspace(user_ids.numel(), M, True)
                self._activate_dedup(w0, user_ids, item_ids, ahead)
                if ahead:
                    self._entry_side(w0, user_ids, next)
                elif next is not None and next[0].numel() == user_ids.numel():
                    if DEDUP_FORK == "entry":
                        # (recorded only here: an event record costs the queue a few us)
                        entry = self._event()
                        entry.record(_lib.stream_ptr(eng.flat.device))
                        self._prefetch_dedup(w0, next[0], next[1], entry)
                    else:   # launched from the engine's fork point DEDUP_FORK of this step
                        pre = (w0, next[0], next[1])

                        def hook(at, pre=pre):
                            if eng.fork_hook is not hook:
                                return
                            d = self.deferred
                            if DEDUP_FORK == "sweep" and d.overlap and d.fork_part(at) is not None \
                                    and not d._joined:
                                # the overlapped sweep was just forked here: the sort queues
                                # behind it on its stream, ordered by the sweep's own fork
                                # (no event record of its own on the step's queue)
                                eng.fork_hook = None
                                self._prefetch_dedup(pre[0], pre[1], pre[2], None,
                                                     side=d.side_stream())
                            elif at == DEDUP_FORK or (DEDUP_FORK == "sweep" and at == "attn_bwd"):
                                eng.fork_hook = None
                                ev = self._event()
                                ev.record(_lib.stream_ptr(eng.flat.device))
                                self._prefetch_dedup(pre[0], pre[1], pre[2], ev)
                        eng.fork_hook = hook
            w = self._body(user_ids, item_ids, targets, M)
            m.engine.fork_hook = None     # (a fork point the step did not pass: no prefetch)
            if getattr(m, "validate_ids", True):
                m.engine.check_ids_async(w)     # out-of-range ids raise a few steps later
            self.step_count += 1
            m.engine.updates += 1
            self.last_loss = w.loss
            return w
        dev = m.engine.flat.device
        shape = (user_ids.numel(), item_ids.numel(), targets.numel(), M)
        d = self.deferred
        if d._hp_filled is not None and d._hp_filled != (d.lr,) + tuple(d.betas) + (d.eps,):
            # lr changed: refill steps > t in place.  The graph reads the table by address, so
            # it stays valid unless the buffer moved (then re-capture)
            table_at = d._table.data_ptr()
            d._ensure(d._filled)
            if d._table.data_ptr() != table_at:
                self._drop_graph()
        if self._g is not None and self._g_consts != d._consts():
            self._drop_graph()          # betas / eps / weight decay are launch arguments
        horizon_ok = d._filled >= d.t + 2
        if self._g is None or self._shape != shape or not horizon_ok:
            if self._eager_steps < self.warmup or not horizon_ok:
                # eager clock-driven steps: allocate every workspace, set kernel attributes
                w = self._body(user_ids, item_ids, targets, M)
                self._eager_steps += 1
                self.step_count += 1
                m.engine.updates += 1
                self.last_loss = w.loss
                self._drop_graph()
                return w
            self._capture(user_ids, item_ids, targets, M, shape, dev)
        su, si, stg = self._static
        su.copy_(user_ids.reshape(-1), non_blocking=True)
        si.copy_(item_ids.reshape(-1), non_blocking=True)
        stg.copy_(targets.reshape(stg.shape), non_blocking=True)
        self._g.replay()
        # host mirrors of what the replayed launches did on the device
        self.deferred.t += 1
        self.model.engine.pending = None
        self.model.engine.updates += 1
        self.step_count += 1
        self.last_loss = self._w.loss
        return self._w

    def eager(self, user_ids, item_ids, targets, M: Optional[int] = None):
        """One step through the launch sequence itself (never the captured graph) — the same
        kernels a replay runs; used for per-launch instrumentation."""
        w = self._body(user_ids, item_ids, targets, M or (1 + self.model.negative_samples))
        self.step_count += 1
        self.model.engine.updates += 1
        self.last_loss = w.loss
        return w

    def _drop_graph(self):
        """Release the captured step graph.  Replays are asynchronous: the last one may still be
        executing, and destroying its executable under it frees the kernel-argument buffers its
        queued dispatches read.  The stream is drained first (a re-capture is rare: a new batch
        geometry, the scalar horizon, a betas / eps / weight-decay change, a state load)."""
        if self._g is not None:
            torch.cuda.current_stream(self.model.engine.flat.device).synchronize()
            self._g = None

    def _capture(self, user_ids, item_ids, targets, M, shape, dev):
        d = self.deferred
        self._drop_graph()
        d._ensure(d.t + GRAPH_HORIZON)      # scalar table horizon: no host copies inside the graph
        self._static = (user_ids.reshape(-1).to(device=dev, dtype=torch.int64).clone(),
                        item_ids.reshape(-1).to(device=dev, dtype=torch.int64).clone(),
                        targets.reshape(-1, 1).to(device=dev, dtype=torch.float32).clone())
        t0, sc = d.t, self.step_count
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(g):
            self._w = self._body(*self._static, M)
        d.t, self.step_count = t0, sc        # capturing executes nothing
        self.model.engine.pending = None
        self._g, self._shape, self._g_consts = g, shape, d._consts()

    def sync(self):
        if self.deferred is not None:
            self.deferred.sync()
        elif self.bf16:
            with torch.no_grad():
                for k, p in self.tables.items():
                    p.copy_(self.tables_lp[k])

    def load_optimizer_state(self, state_dict):
        """Resume from a ``torch.optim.Adam(model.parameters())`` state_dict (what
        export_optimizer_state / checkpoint.save_checkpoint and the reference trainer write):
        moments and step of every trained parameter; the deferred schedule restarts with every
        row current at that step."""
        self.sync()
        eng = self.model.engine
        idx_of = {id(p): i for i, p in enumerate(self.model.parameters())}
        st = state_dict["state"]

        def entry(p, what):
            s = st.get(idx_of[id(p)])
            if s is None:
                raise KeyError(f"optimizer state has no entry for {what}")
            return s
        step = None
        for k, p in self.tables.items():
            s = entry(p, k)
            self.state[k]["exp_avg"].copy_(s["exp_avg"])
            self.state[k]["exp_avg_sq"].copy_(s["exp_avg_sq"])
            step = int(float(s["step"]))
        for name, p in eng.dense_params():
            s = entry(p, name)
            o, n, _ = eng.offsets[name]
            self.m_flat[o:o + n].copy_(s["exp_avg"].reshape(-1))
            self.v_flat[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
        self.step_count = step or 0
        d = self.deferred
        if d is not None:
            d.t = d.synced_t = self.step_count
            for stamp in d.stamp.values():
                stamp.fill_(self.step_count)
            d._ensure(d.t + 2)
        if self.clock is not None:
            self.clock[0] = self.step_count      # ncf_step_clock.t (reserved = 0)
        self._drop_graph()                       # re-capture from the restored state
        eng.updates += 1

    def export_optimizer_state(self, opt: torch.optim.Adam):
        self.sync()
        eng = self.model.engine
        step_t = torch.tensor(float(self.step_count))
        for k, p in self.tables.items():
            opt.state[p] = {"step": step_t, "exp_avg": self.state[k]["exp_avg"],
                            "exp_avg_sq": self.state[k]["exp_avg_sq"]}
        for name, p in eng.dense_params():
            o, n, shp = eng.offsets[name]
            opt.state[p] = {"step": step_t, "exp_avg": self.m_flat[o:o + n].view(shp),
                            "exp_avg_sq": self.v_flat[o:o + n].view(shp)}


class ModelTrainer:
    """Reference-compatible trainer (src/model/trainer.py:27-95, 216-337) minus BigQuery I/O."""

    def __init__(self, model: nn.Module, config: Dict[str, Any], num_gpus: int = 1):
        required = {"num_users", "num_products", "batch_size", "learning_rate"}
        missing = required - set(config.keys())
        if missing:
            raise ValueError(f"Missing required parameters in config: {missing}")
        self.model = model
        self.config = config
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.num_gpus = num_gpus
        self.negative_samples = config.get("negative_samples", 4)
        weight_decay = float(config.get("weight_decay", 1e-5))
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=config["learning_rate"],
                                          weight_decay=weight_decay)
        self.criterion = nn.BCELoss().to(self.device)
        self.model = self.model.to(self.device)

    def train_epoch(self, train_loader) -> float:
        """trainer.py:216-337.  The per-batch loss is summed on the device and read once at the
        end of the epoch (the reference reads it, and three accuracies, with .item() every
        batch for its progress bar: four host syncs per step)."""
        self.model.train()
        with torch.autograd.set_multithreading_enabled(not CALLING_THREAD_BACKWARD):
            return self._train_epoch(train_loader)

    def _train_epoch(self, train_loader) -> float:
        total_loss, num_batches = None, 0
        for batch_idx, (features, targets) in enumerate(train_loader):
            base_batch_size = len(features.lengths()) // len(features.keys())
            effective_batch_size = base_batch_size * (1 + self.negative_samples)
            if base_batch_size < 2:
                log.warning("Skipping small batch %d: size %d", batch_idx, base_batch_size)
                continue
            features = features.to(self.device)
            targets = targets.to(self.device)
            outputs = self.model(features)
            if outputs.shape != targets.shape:
                outputs = outputs.view(effective_batch_size, 1)
                targets = targets.view(effective_batch_size, 1)
            loss = self.criterion(outputs, targets)
            self.optimizer.zero_grad()
            loss.backward()
            self.optimizer.step()
            total_loss = loss.detach() if total_loss is None else total_loss + loss.detach()
            num_batches += 1
        avg = float(total_loss) / num_batches if num_batches > 0 else float("inf")
        log.info("Epoch complete - Average loss: %.4f", avg)
        return avg

    def validate(self, val_loader) -> Dict[str, float]:
        """trainer.py:350-410: eval forward (M = 1) over the loader, BCE loss, then
        calculate_metrics over every prediction with k = 1, 5, 10 and no negatives (each row is
        its own group, as in the reference); ``loss`` = mean per-batch loss."""
        from .metrics import calculate_metrics
        self.model.eval()
        total_loss = None
        outs, tgts = [], []
        with torch.no_grad():
            for features, targets in val_loader:
                features = features.to(self.device)
                targets = targets.to(self.device)
                outputs = self.model(features)
                loss = self.criterion(outputs, targets)
                total_loss = loss if total_loss is None else total_loss + loss
                outs.append(outputs)
                tgts.append(targets)
        all_out, all_t = torch.cat(outs, 0), torch.cat(tgts, 0)
        metrics = calculate_metrics(predictions=all_out, targets=all_t, k_values=[1, 5, 10],
                                    batch_size=len(all_t), negative_samples=0)
        metrics["loss"] = float(total_loss) / len(val_loader)
        metrics["val_loss"] = metrics["loss"]
        for name, value in metrics.items():
            log.info("- %s: %.4f", name, value)
        return metrics

    def train(self, train_loader, val_loader, num_epochs: int, early_stopping_patience: int = 5,
              checkpoint_dir: Optional[str] = None) -> Dict[str, list]:
        """trainer.py:412-546: epochs of train_epoch + validate with early stopping on the
        validation loss and (with ``checkpoint_dir``) per-epoch checkpoints in the trainer
        format (checkpoint.py; ``best_model.pt`` for the best, resume from the latest)."""
        import glob
        import os
        from .checkpoint import load_checkpoint, save_checkpoint
        best, patience, start = float("inf"), 0, 0
        history = {"train_loss": [], "val_loss": [], "val_hit_rate": [], "val_ndcg": [],
                   "learning_rate": []}
        if checkpoint_dir:
            os.makedirs(checkpoint_dir, exist_ok=True)
            found = sorted(glob.glob(os.path.join(checkpoint_dir, "checkpoint_epoch_*.pt")),
                           key=lambda p: int(p.rsplit("_", 1)[1].split(".")[0]))
            if found:
                start = load_checkpoint(found[-1], self.model, self.optimizer)
        epoch, val_metrics = start, None
        try:
            for epoch in range(start, num_epochs):
                history["train_loss"].append(self.train_epoch(train_loader))
                val_metrics = self.validate(val_loader)
                history["val_loss"].append(val_metrics["loss"])
                history["val_hit_rate"].append(val_metrics.get("hit_rate@10"))
                history["val_ndcg"].append(val_metrics.get("ndcg@10"))
                history["learning_rate"].append(self.optimizer.param_groups[0]["lr"])
                improved = val_metrics["loss"] < best
                if improved:
                    best, patience = val_metrics["loss"], 0
                else:
                    patience += 1
                if checkpoint_dir:
                    path = os.path.join(checkpoint_dir, f"checkpoint_epoch_{epoch + 1}.pt")
                    save_checkpoint(path, self.model, self.optimizer, epoch, val_metrics,
                                    self.config)
                    if improved:
                        save_checkpoint(os.path.join(checkpoint_dir, "best_model.pt"),
                                        self.model, self.optimizer, epoch, val_metrics,
                                        self.config)
                if patience >= early_stopping_patience:
                    log.info("Early stopping triggered after %d epochs", epoch + 1)
                    break
            return history
        except Exception:
            if checkpoint_dir:
                save_checkpoint(os.path.join(checkpoint_dir, "emergency_checkpoint.pt"),
                                self.model, self.optimizer, epoch, val_metrics, self.config)
            raise
