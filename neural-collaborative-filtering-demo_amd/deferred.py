"""Deferred dense-exact Adam for the embedding tables.

The reference's Adam (src/model/trainer.py:71-75, :285) updates EVERY row of every table every
step: the dense gradient is zero on rows the batch did not touch, but coupled weight decay
(g = 0 + wd * p) still moves them.  Streaming 140.8M parameters x 24 B per step
(3.4 GB at C2) is the whole cost of the dense schedule.

This schedule computes the same numbers lazily: each row carries ``stamp[row]`` (the last step
its p / exp_avg / exp_avg_sq reflect).  A step then
  1. deduplicates the batch ids (``ncf_dedup_ids``, before the forward),
  2. catches up exactly those rows by replaying their missed zero-gradient steps
     (``ncf_adam_rows_catchup``) so the forward gathers current values,
  3. after the backward applies this step's real gradient to those rows (``ncf_adam_rows_apply``),
  4. a rolling sweep brings one 1/``sweep_every`` slice of every table current each step (no row
     is ever more than ``sweep_every`` steps behind), and the whole table is swept before
     anything else reads it (state_dict, eval forward, embedding export) (``ncf_adam_sweep``).
Every replayed step uses the per-step fp32 scalars of the dense kernel and the same
contraction-free arithmetic, so the result is bit-identical to the dense sweep (tested); the
work moves from HBM traffic (24 B/element/step) to VALU (~15 flops/element/step, amortised).
"""
import ctypes
import itertools

import numpy as np
import torch

from . import _lib
from ._lib import ptr

_KINDS = (("user", "mf_user", "mlp_user"), ("item", "mf_item", "mlp_item"))
# Catch-up by claim (no id sort before the forward) when the batch was not sorted ahead;
# CLAIM_CATCHUP = False: sort inline, then catch up the unique rows (tested equal).  The
# claim path forks its id sort beside the forward (measured, drop-in step GPU-bound: 0.350-0.353
# ms against 0.381-0.399 forked at a backward fork point; round 3)
CLAIM_CATCHUP = True
_SERIAL = itertools.count(1)      # distinguishes schedules in workspace caches (ids recycle)
# Steps of per-step scalars filled past the furthest step asked for.  The replay kernels read the
# scalars of up to 8 steps past their target (replay_uniform's prefetch, csrc/adam.hip), so the
# pad must stay >= 16; tests shrink it to force table growth under a captured graph.
SCALAR_PAD = 4096
# Early catch-up: with the next batch sorted a step ahead (FusedTrainStep's
# next=), its rows that this step's batch does not touch are caught up through this step on the
# side stream, behind the rolling sweep and beside the backward; this step's own rows are locked
# by its catch-up (NCF_STAMP_LOCK) and skipped.  The next step's catch-up then finds its rows
# current.  Same replays, bit-identical (tested).  Off: measured slower at C2 (round 5,
# tools/step_ab.py, 3 interleaved runs each: 0.2942-0.2957 ms/step without, 0.3004 with, the
# replay beside the backward slows it more than it saves on the critical path; round 3 found
# the same for three placements of it).  Smaller batches leave CUs idle beside the backward
# (the reference's default batch of 256 groups fills 86 of 256 CUs) and the late catch-up's
# wait sits on their step's critical path; run r06zl / r06zm, tools/step_ab.py, 3 interleaved
# runs each, min ms/step late -> early: B = 256 groups 0.1622 -> 0.1516, 1,024 0.2131 -> 0.2027,
# 2,048 0.2180 -> 0.2143, 4,096 (C2) 0.2669 -> 0.2689.  None (the default): on for batches of at
# most EARLY_CATCHUP_ROWS rows (early_on); True / False: always / never.
EARLY_CATCHUP = None
EARLY_CATCHUP_ROWS = 10240


def early_on(n: int) -> bool:
    """Whether a batch of n rows takes the early catch-up (EARLY_CATCHUP)."""
    return bool(EARLY_CATCHUP) if EARLY_CATCHUP is not None else n <= EARLY_CATCHUP_ROWS
# Late catch-up: the same catch-up of the next batch's rows, queued once this step's table Adam
# has run inside the embedding backward (trainer.FUSE_APPLY) — on the side stream behind the
# sweep and the sort, beside the dense-gradient reductions (memory-bound, like it) instead of
# beside the compute-bound backward; nothing to lock (the step's rows already carry its stamp).
# The next step then skips its own catch-up launch for that batch.
LATE_CATCHUP = True
# HIP stream priority of the overlapped sweep's side stream (torch.cuda.Stream priority: 0 the
# default, -1 high)
SIDE_PRIORITY = 0
# The side stream's kernels on `SIDE_CU_KEEP` of every 8 CUs (a CU-masked stream, its own
# hardware queue); 0: a pool stream on every CU (the default, _lib.side_stream)
SIDE_CU_KEEP = 0
# The overlapped rolling sweep (below) for FusedTrainStep and the optimizer hook: on (False: the
# sweep on the step's own stream)
OVERLAP_SWEEP = True
# Fork point(s) of the overlapped sweep (None: the geometry's default, _default_fork; else a
# comma-separated list, see DeferredTableAdam.__init__)
SWEEP_FORK = None
# With the default fork point, batches of at most GATHER_FORK_ROWS rows fork the sweep before
# their gathers instead ("gather"): the small-batch step leaves most CUs idle beside its short
# kernels, and the sweep started earlier ends earlier (run r06zp, tools/step_ab.py, 3
# interleaved runs each, min ms/step tower -> gather: B = 256 groups 0.1506 -> 0.1420; run
# r06zr / r06zq: 512 groups 0.1732 -> 0.1693, 1,024 0.2018 -> 0.2042, 2,048 0.2172 -> 0.2165;
# C2, 4,096 groups, 0.2655 ->
# 0.2864: there the sweep beside the gather and the forward slows both)
GATHER_FORK_ROWS = 2560


class DeferredTableAdam:
    def __init__(self, engine, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 sweep_every: int = 64, moments=None, clock=None, overlap_sweep=None,
                 param_tables=None):
        self.engine = engine
        self._serial = next(_SERIAL)
        # clock (ncf_step_clock, device): every step-dependent value is read on the device, so
        # the launches of a step do not depend on the host counter (hipGraph capture)
        self.clock = clock
        self.lr, self.eps, self.wd = float(lr), float(eps), float(weight_decay)
        self.betas = (float(betas[0]), float(betas[1]))
        self.sweep_every = int(sweep_every)
        # the rows the schedule updates: the fp32 table parameters, or (bf16-table
        # configuration) bf16 tables that own the values, with the fp32 parameters a widened
        # copy brought up to date by sync()
        self.params = engine.table_params()
        self.tables = dict(param_tables) if param_tables is not None else self.params
        self.bf16 = self.tables["mf_user"].dtype == torch.bfloat16
        dev = self.tables["mf_user"].device
        self.state = moments or {k: {"exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
                                 for k, p in self.params.items()}     # (fp32 moments)
        m = engine.model
        self.stamp = {"user": torch.zeros(m.num_users, dtype=torch.int32, device=dev),
                      "item": torch.zeros(m.num_products, dtype=torch.int32, device=dev)}
        if engine.deferred is not None and engine.deferred is not self:
            engine.deferred.detach()    # the previous schedule settles its lagging rows first
        self.t = 0
        self.synced_t = 0
        self.late_skips = 0         # steps whose catch-up the previous step's late catch-up made
        self._table = torch.zeros(0, dtype=torch.float32, device=dev)
        self._filled = 0
        self._hp_filled = None      # (lr, beta1, beta2) the filled scalars were computed with
        # Overlapped rolling sweep (clock path; FusedTrainStep and the optimizer hook turn it
        # on): the sweep closing step T is launched during step T+1, after its catch-up, on a
        # side stream, and joined before the clock advance.  Rows of step T+1's batch are current
        # by then (stamp >= T) and skipped; every other row of the slice is touched by the sweep
        # alone.  Same arithmetic, bit-identical results (tested).
        # Invariant that lets the table apply run before the join (trainer.FUSE_APPLY: the apply
        # inside the embedding backward, the sweep possibly still running beside it): the sweep
        # targets clock->t (step_rel 0) and every row of the batch was caught up to t before the
        # fork (every engine fork point — tower, mlp_bwd, mlp_bwd_after, attn_bwd, emb_bwd,
        # reduce — lies after engine.forward's prepare; a part whose point the step never passes
        # is settled on the step's stream in apply(), behind the fused apply, where those rows
        # stand at t + 1 and are skipped all the same), so the sweep skips exactly the rows
        # the apply steps from t to t + 1: no row is stepped twice.  A fork point placed before
        # prepare, or a sweep target past t (step_rel > 0 in sweep_fork), would break this.
        self.overlap = bool(overlap_sweep)
        if self.overlap and clock is None:
            raise ValueError("the overlapped sweep needs the device step clock")
        # Where the engine forks it ("gather": after the catch-up, before the gathers;
        # "mlp_bwd": before the MLP tower backward; "mlp_bwd_after":
        # right after its launch (round 3: 0.337-0.344 vs 0.312 ms); "tower": before the tower
        # forward; "attn_bwd", "emb_bwd", "reduce": before those backward launches); the step
        # joins it before the table apply (a join before the clock-advancing close measured the
        # same, round 2).  Measured at C2 (one MI355X, ms/step): not overlapped 0.337; forked at
        # tower 0.325, mlp_bwd 0.313-0.317, attn_bwd 0.327, emb_bwd 0.342, reduce 0.322-0.325.  The
        # VALU-bound replay fills the issue slots the latency-bound tower and attention
        # backward leave idle (it stretches k_mlp_bwd from 80 to ~92 us and itself from 50
        # to ~96 us, both off the critical path's sum).
        # Several comma-separated fork points split the slice into that many consecutive row
        # ranges, one launched at each (ncf_adam_pairs_sweep_rolling_part).
        # Default: "tower" when the step runs the attention block and the tower fused
        # (tower_fused.hip: the sweep beside the fused forward and backward; round 5, 3
        # interleaved runs each: 0.2879-0.2908 ms/step, forked at mlp_bwd 0.3056-0.3074, the
        # unfused step 0.2972-0.3006), else "mlp_bwd" (unfused at "tower": 0.3107-0.3119).
        self.fork_points = SWEEP_FORK.split(",") if SWEEP_FORK else [self._default_fork(engine)]
        self._owed = []           # parts of a closed step's rolling sweep not launched yet
        self._rows_now = None     # the current step's batch rows (prepare; cleared by advance)
        self._side = None
        self._ev = None
        self._joined = True
        # a late catch-up left running past its step (trainer.LATE_DETACHED): the event the next
        # user of the tables waits for (late_join), and the clock copy it reads its target from
        self._late_ev = None
        self._late_clock = None
        self._side_t = None        # the t the side clock was last set to (side_clock)
        self._side_ordered_t = -1  # the side stream is ordered after the table apply closing t + 1
        self._live_pending = False  # a sweep part reading the live clock awaits the step's join
        engine.deferred = self
        if self.overlap and not torch.cuda.is_current_stream_capturing():
            self.side_stream()     # (picked and checked here, outside any stream capture)

    @staticmethod
    def _default_fork(engine):
        m = engine.model
        D, H, M = m.mlp_embedding_dim, m.num_heads, 1 + m.negative_samples
        fused = (m.mf_embedding_dim == D and
                 engine.attn_tower_step(D, H, M, list(m.mlp_hidden_dims)))
        return "tower" if fused else "mlp_bwd"

    # ---- per-step scalar table (index 4s .. 4s+3 = step s: gradient-step and zero-gradient-step
    #      scalars, ncf_adam_step_scalars)
    def _ensure(self, upto: int):
        b1, b2 = self.betas
        hp = (self.lr, b1, b2, self.eps)
        if upto <= self._filled and self._hp_filled == hp:
            return
        if self._hp_filled is None:
            first = 1
            last = max(upto, first) + SCALAR_PAD
        elif self._hp_filled != hp:
            # an lr (or beta) change affects only steps not yet taken: the scalars of steps
            # <= t stay as they were, so rows still behind replay those steps as taken.  The
            # filled horizon is refilled in place (no growth unless `upto` lies beyond it): a
            # captured step graph holds this buffer's address
            first = min(self._filled + 1, self.t + 1)
            last = self._filled if upto <= self._filled else upto + SCALAR_PAD
        else:
            first = self._filled + 1
            last = max(upto, first) + SCALAR_PAD
        first = max(1, first)
        last = max(last, first)
        host = np.empty(4 * (last - first + 1), dtype=np.float32)
        _lib.call("ncf_adam_step_scalars", self.lr, b1, b2, self.eps, first, last - first + 1,
                  host.ctypes.data)
        need = 4 * (last + 1)
        if self._table.numel() < need:
            dev = self._table.device
            if self._table.numel():
                # The table moves.  Kernels already queued read the old buffer by address: the
                # overlapped sweep on its side stream (apply ensures before it joins the sweep)
                # and a captured step graph still replaying.  Freeing it under them would let the
                # caching allocator hand it to other work (or, with the graph, leave it read after
                # the caller drops the graph), so the device is drained first — the table grows
                # once per doubling, rarely enough that the wait is noise.
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("deferred Adam: the per-step scalar table would move "
                                       "inside a graph capture (ensure the horizon before "
                                       "capturing)")
                torch.cuda.synchronize(dev)
            grown = torch.zeros(max(need, 2 * self._table.numel()), dtype=torch.float32,
                                device=dev)
            if self._table.numel():
                grown[:self._table.numel()].copy_(self._table)
            self._table = grown
        self._table[4 * first:4 * (last + 1)].copy_(torch.from_numpy(host))
        self._filled, self._hp_filled = last, hp

    def set_hparams(self, lr, betas, eps, weight_decay):
        """Change the hyper-parameters for the steps not yet taken.  lr lives only in the
        per-step scalar table (refilled from step t + 1); betas / eps / weight_decay also enter
        every replayed zero-gradient step, so rows still behind are first brought current with
        the old values (one full sweep, only when they change)."""
        betas = (float(betas[0]), float(betas[1]))
        if (betas, float(eps), float(weight_decay)) != (self.betas, self.eps, self.wd):
            self.sync()
            self.betas, self.eps, self.wd = betas, float(eps), float(weight_decay)
        self.lr = float(lr)

    def mark_current(self, t: int):
        """Every row of every table holds its value after step t (e.g. a dense step, or state
        just loaded): restart the schedule there."""
        self.t = self.synced_t = int(t)
        for stamp in self.stamp.values():
            stamp.fill_(int(t))
        self._owed, self._joined = [], True

    def rebind_moments(self, moments):
        """Use other exp_avg / exp_avg_sq tensors (e.g. after an optimizer state load)."""
        self.state = moments
        self.__dict__.pop("_sweep_pairs", None)
        self._gen = getattr(self, "_gen", 0) + 1

    def _pairs_for(self, w):
        """_pairs(w), cached on the workspace (its buffers, the tables and the moments are
        fixed while the key holds)."""
        key = ("pairs", self._serial, getattr(self, "_gen", 0), w.uniq_u.data_ptr(),
               w.uniq_i.data_ptr())
        p = w.cache.get(key)
        if p is None:
            p = w.cache[key] = self._pairs(w)
        return p

    def _consts(self):
        b1, b2 = self.betas
        return b1, b2, self.eps, self.wd

    def _ptrs(self, kind):
        _, a, b = next(k for k in _KINDS if k[0] == kind)
        s = self.state
        return (ptr(self.tables[a]), ptr(s[a]["exp_avg"]), ptr(s[a]["exp_avg_sq"]),
                ptr(self.tables[b]), ptr(s[b]["exp_avg"]), ptr(s[b]["exp_avg_sq"]))

    # ---- row-list primitives (also used by the row-sharded step)
    def catchup_rows(self, kind, row_ids, count_dev, kind_index, max_n, st):
        """Bring the listed unique rows of `kind` current through step self.t."""
        if self.clock is not None:
            if max_n > 0:
                self._ensure(self.t + 1)
                _lib.call("ncf_adam_rows_catchup_clock", *self._ptrs(kind),
                          self.engine.model.mlp_embedding_dim, ptr(row_ids), ptr(count_dev),
                          kind_index, max_n, ptr(self.stamp[kind]), 0, ptr(self.clock),
                          ptr(self._table), *self._consts(), st)
            return
        if self.t == 0 or max_n <= 0:
            return
        self._ensure(self.t)
        _lib.call("ncf_adam_rows_catchup", *self._ptrs(kind), self.engine.model.mlp_embedding_dim,
                  ptr(row_ids), ptr(count_dev), kind_index, max_n, ptr(self.stamp[kind]), self.t,
                  ptr(self._table), *self._consts(), st)

    def apply_rows(self, kind, row_ids, count_dev, kind_index, max_n, g_mf, g_mlp, st):
        """Step self.t + 1 on the listed rows (current through self.t) with their gradients."""
        step = self.t + 1
        self._ensure(step)
        if max_n <= 0:
            return
        p0, m0, v0, p1, m1, v1 = self._ptrs(kind)
        if self.clock is not None:
            _lib.call("ncf_adam_rows_apply_clock", p0, m0, v0, ptr(g_mf), p1, m1, v1, ptr(g_mlp),
                      self.engine.model.mlp_embedding_dim, ptr(row_ids), ptr(count_dev),
                      kind_index, max_n, ptr(self.stamp[kind]), 1, ptr(self.clock),
                      ptr(self._table), *self._consts(), st)
            return
        _lib.call("ncf_adam_rows_apply", p0, m0, v0, ptr(g_mf), p1, m1, v1, ptr(g_mlp),
                  self.engine.model.mlp_embedding_dim, ptr(row_ids), ptr(count_dev), kind_index,
                  max_n, ptr(self.stamp[kind]), step, ptr(self._table), *self._consts(), st)

    def advance(self, st):
        """Close step self.t + 1 (after apply_rows of every kind), then the rolling sweep: one
        1/sweep_every slice of every table is brought current each step, so no row is ever more
        than sweep_every steps behind and the catch-up work is spread evenly over the steps.
        With the overlapped sweep it is only owed here and launched by the next sweep_fork."""
        self.t += 1
        self._rows_now = None
        self.engine.pending = None
        if self.sweep_every and self.clock is not None and self.overlap:
            self._owed = list(range(len(self.fork_points)))
        elif self.sweep_every and self.clock is not None:
            self._rolling(st, 1)
        elif self.sweep_every:
            k = self.t % self.sweep_every
            for kind in ("user", "item"):
                rows = self.stamp[kind].numel()
                sl = (rows + self.sweep_every - 1) // self.sweep_every
                r0 = k * sl
                self._sweep_range(kind, r0, max(0, min(rows, r0 + sl) - r0), st)

    def _rolling(self, st, step_rel, part=0, nparts=1, clock=None):
        """Rolling sweep closing step clock->t + step_rel (slice of that step; part `part` of
        `nparts` consecutive row ranges of it); ``clock``: a side clock (side_clock) instead of
        the live one."""
        pairs = self.__dict__.get("_sweep_pairs") or self.__dict__.setdefault("_sweep_pairs",
                                                                               self._pairs())
        D = self.engine.model.mlp_embedding_dim
        clk = ptr(self.clock if clock is None else clock)
        if nparts == 1:
            _lib.call("ncf_adam_pairs_sweep_rolling", ctypes.addressof(pairs), 2, D,
                      self.sweep_every, step_rel, clk, ptr(self._table), *self._consts(), st)
        else:
            _lib.call("ncf_adam_pairs_sweep_rolling_part", ctypes.addressof(pairs), 2, D,
                      self.sweep_every, step_rel, part, nparts, clk, ptr(self._table),
                      *self._consts(), st)

    def sweep_fork(self, at="mlp_bwd"):
        """During step T+1 (clock->t = T, after its catch-up), at the engine's fork point `at`:
        launch the part of the owed sweep of step T registered there on the side stream; it
        overlaps everything the current stream does until sweep_join."""
        part = self.fork_part(at)
        if part is None or part not in self._owed:
            return
        side = self.side_stream().cuda_stream
        dev = self.clock.device
        # (C-ABI event calls: a launch tape of the step holds the fork and join in order)
        self._ev[0].record(_lib.stream_ptr(dev))
        self._ev[0].wait(side)
        if _lib.PROFILE is not None:     # per-launch instrumentation times it on its stream
            with torch.cuda.stream(self._side):
                self._rolling(side, 0, part, len(self.fork_points))
        else:     # (step_rel 0: the target is clock->t, which the batch's rows already reached)
            self._rolling(side, 0, part, len(self.fork_points))
        self._ev[1].record(side)
        self._owed.remove(part)
        self._joined = False
        self._live_pending = True      # (it reads the live clock: joined before the advance)

    def fork_part(self, at):
        """The part of the owed sweep forked at engine fork point `at`, or None: fork_points,
        except that with the default single fork point a batch of at most GATHER_FORK_ROWS rows
        forks it at "gather"."""
        if (SWEEP_FORK is None and len(self.fork_points) == 1 and self._rows_now is not None
                and self._rows_now <= GATHER_FORK_ROWS):
            return 0 if at == "gather" else None
        return self.fork_points.index(at) if at in self.fork_points else None

    def side_stream(self):
        """The overlapped sweep's stream (created on first use)."""
        if self._side is None:     # (one that runs beside the step's stream: _lib.side_stream)
            self._side = (_lib.masked_stream(self.clock.device, SIDE_CU_KEEP) if SIDE_CU_KEEP
                          else _lib.side_stream(self.clock.device, SIDE_PRIORITY))
            self._ev = (_lib.RawEvent(stream_only=True), _lib.RawEvent(stream_only=True))
        return self._side

    def sweep_done(self, stream: int):
        """The side stream's work queued so far (the sweep, then the next batch's sort behind
        it) is what the step's sweep join waits for."""
        self._ev[1].record(stream)

    def late_join(self, st=None):
        """Stream st (default: the current stream) waits for a late catch-up that was left
        running past the step that queued it (trainer.LATE_DETACHED): before anything on st
        reads or steps table rows again (the next prepare, a flush, a sync)."""
        ev, self._late_ev = self._late_ev, None
        if ev is not None:
            ev.wait(st if st is not None else _lib.stream_ptr(self.clock.device))

    def sweep_join(self):
        """The current stream waits for the side-stream sweep (before the step's apply and the
        clock advance that would change the sweep's target under it)."""
        if not self._joined:
            self._ev[1].wait(_lib.stream_ptr(self.clock.device))
            self._joined = True
            self._live_pending = False

    # ---- trainer.SIDE_AHEAD: the side stream's work off the step's queue
    def side_clock(self, st):
        """The side stream's own step clock, t = the host's step counter, set on stream st (the
        side stream) when that changed: the late catch-up and the sweep queued there read their
        targets from it, so the step's stream advances the live clock without joining them."""
        if self._late_clock is None:
            # (no fill: written by ncf_step_clock_set on the side stream before any reader)
            self._late_clock = torch.empty_like(self.clock)
        if self._side_t != self.t:
            _lib.call("ncf_step_clock_set", ptr(self._late_clock), self.t, 0, st)
            self._side_t = self.t
        return self._late_clock

    def side_ordered(self):
        """The side stream has waited for the table apply closing step t + 1 (the trainer's
        tables-done event): after this step's advance, its owed sweep may run there."""
        self._side_ordered_t = self.t

    def sweep_owed(self, side):
        """Every owed part of the closed step's rolling sweep on stream `side` now, its target
        (t) from the side clock, when that stream is ordered after the closed step's table
        apply (side_ordered; else the parts stay owed for the engine's fork points).  The
        batch rows of that step carry its stamp and are skipped, the next batch's rows were
        caught up ahead of it on the same stream (the late catch-up), every other row is the
        sweep's alone; a catch-up on the step's stream first joins it (prepare)."""
        if not self._owed or self._side_ordered_t != self.t - 1:
            return False
        clk = self.side_clock(side)
        n = len(self.fork_points)
        for part in sorted(self._owed):
            if _lib.PROFILE is not None:   # (per-launch instrumentation times it on its stream)
                with torch.cuda.stream(self._side):
                    self._rolling(side, 0, part, n, clock=clk)
            else:
                self._rolling(side, 0, part, n, clock=clk)
        self._owed = []
        self._ev[1].record(side)
        self._joined = False
        return True

    def _settle(self, st):
        """Parts of the owed sweep whose fork point this step did not pass: on stream st, now
        (before the step's apply closes the next step)."""
        for part in self._owed:
            self._rolling(st, 0, part, len(self.fork_points))
        self._owed = []

    def flush(self, st):
        """Settle any owed / in-flight sweep on the current stream (before full sweeps or
        anything that reads the tables from the host side)."""
        self.late_join(st)
        self.sweep_join()
        self._settle(st)

    def _pairs(self, w=None):
        """ncf_table_pair[2] (users, items) for the both-kinds launches of the clock path."""
        pairs = (_lib.TablePair * 2)()
        for k, (kind, a, b) in enumerate(_KINDS):
            p0, m0, v0, p1, m1, v1 = self._ptrs(kind)
            pr = pairs[k]
            pr.p0, pr.m0, pr.v0, pr.p1, pr.m1, pr.v1 = p0, m0, v0, p1, m1, v1
            pr.stamp, pr.rows = ptr(self.stamp[kind]), self.stamp[kind].numel()
            pr.param_dtype = _lib.DTYPE_BF16 if self.bf16 else _lib.DTYPE_F32
            if w is not None:
                pr.row_ids = ptr(w.uniq_u if k == 0 else w.uniq_i)
                pr.g0, pr.g1 = ptr(w.G[a]), ptr(w.G[b])
        return pairs

    # ---- engine hook: before the gathers of a training step
    def prepare(self, w, uid, iid, st):
        eng = self.engine
        m = eng.model
        n = w.g.n
        self._rows_now = n
        self.late_join(st)
        if (CLAIM_CATCHUP and self.clock is not None and n > 0 and not getattr(w, "prededuped", None)
                and not torch.cuda.is_current_stream_capturing()):
            self._prepare_claim(w, uid, iid, st)
            return
        if not getattr(w, "prededuped", None):   # else: sorted ahead on a side stream (trainer)
            _lib.call("ncf_dedup_ids", ptr(uid), ptr(iid), n, w.g.D, m.num_users, m.num_products,
                      ptr(w.uniq_u), ptr(w.uniq_i), None, None, ptr(w.num_unique), ptr(w.emb_ws),
                      w.emb_ws.numel(), st)
        w.prededuped = None
        w.deduped = True
        if self.clock is not None and n > 0:   # both kinds in one launch
            self._ensure(self.t + 1)
            if getattr(w, "late_t", None) == self.t:
                # (the late catch-up of the previous step brought this very set current through
                # step t: its catch-up would replay nothing)
                w.late_t = None
                self._locked = False
                self.late_skips += 1
                return
            # (a sweep still running on the side stream may hold rows of this batch: SIDE_AHEAD)
            self.sweep_join()
            pairs = self._pairs_for(w)
            # (locked: an early catch-up of the next batch may run during this step)
            lock = 1 if early_on(n) else 0
            _lib.call("ncf_adam_pairs_catchup_lock_clock", ctypes.addressof(pairs), 2,
                      m.mlp_embedding_dim, ptr(w.num_unique), n, 0, lock, ptr(self.clock),
                      ptr(self._table), *self._consts(), st)
            self._locked = bool(lock)
            return
        self.catchup_rows("user", w.uniq_u, w.num_unique, 0, n, st)
        self.catchup_rows("item", w.uniq_i, w.num_unique, 1, n, st)

    def _prepare_claim(self, w, uid, iid, st):
        """The step's rows caught up straight from the raw id lists (a claim per row,
        ncf_adam_pairs_catchup_claim_clock: no sort before the gathers), and the id sort the
        backward and the table apply need forked onto a side stream beside the forward; the
        engine joins it before the embedding backward (w.dedup_ev).  The reference call pattern
        (model(kjt) -> loss.backward() -> Adam.step(), trainer.py:258-285) has no next batch to
        sort ahead, so without this its sort sat on the critical path."""
        m = self.engine.model
        n = w.g.n
        self._ensure(self.t + 1)
        self.sweep_join()             # (a side sweep left running past its step: SIDE_AHEAD)
        pairs = self._pairs_for(w)
        self._locked = False          # (no early catch-up during a claim-path step)
        _lib.call("ncf_adam_pairs_catchup_claim_clock", ctypes.addressof(pairs), 2,
                  m.mlp_embedding_dim, ptr(uid), ptr(iid), n, 0, ptr(self.clock),
                  ptr(self._table), *self._consts(), st)
        if getattr(w, "dedup_ev", None) is not None:   # a previous sort never joined (no backward)
            w.dedup_ev.wait(st)
            w.dedup_ev = None
        w.prededuped = None
        w.deduped = True
        # uid / iid stay referenced until the engine joins the sort (w.dedup_refs): the caching
        # allocator cannot hand their memory to work the current stream queues before the join
        w.dedup_refs = (uid, iid)
        self.fork_claim_sort(w, st)

    def fork_claim_sort(self, w, st):
        """The id sort of a claim-path step (w.dedup_refs) on the side stream, after everything
        queued on stream st so far; joined through w.dedup_ev."""
        uid, iid = w.dedup_refs
        m = self.engine.model
        n = w.g.n
        dev = self.clock.device
        side = getattr(self, "_dedup_side", None)
        if side is None or side.device != dev:
            side = self._dedup_side = _lib.side_stream(dev, SIDE_PRIORITY)
            self._dedup_evs = [_lib.RawEvent(stream_only=True) for _ in range(2)]
        cur = st
        self._dedup_evs[0].record(cur)
        self._dedup_evs[0].wait(side.cuda_stream)
        _lib.call("ncf_dedup_ids", ptr(uid), ptr(iid), n, w.g.D, m.num_users, m.num_products,
                  ptr(w.uniq_u), ptr(w.uniq_i), None, None, ptr(w.num_unique), ptr(w.emb_ws),
                  w.emb_ws.numel(), side.cuda_stream)
        self._dedup_evs[1].record(side.cuda_stream)
        w.dedup_ev = self._dedup_evs[1]

    def early_catchup(self, rows, n, stream):
        """The next batch's unique rows (``rows``: a dedup set's uniq_u / uniq_i / num_unique)
        caught up through the step now running, on `stream` (ordered after their sort and
        joined before this step's apply).  Only when this step's catch-up locked its own rows;
        returns whether it was queued."""
        if not (early_on(n) and self.clock is not None and getattr(self, "_locked", False)
                and n > 0):
            return False
        self._catchup_next(rows, n, stream)
        return True

    def late_catchup(self, rows, n, stream, clock=None):
        """The next batch's unique rows (a dedup set, as early_catchup) caught up through the
        step now running, on `stream`, which must be ordered after this step's table apply (the
        apply fused into the embedding backward) and its sweep; the set is marked, so the next
        step's prepare skips its catch-up.  The caller joins `stream` before the clock advance."""
        if self.clock is None or n <= 0:
            return False
        self._catchup_next(rows, n, stream, clock)
        rows["late_t"] = self.t + 1
        return True

    def _catchup_next(self, rows, n, stream, clock=None):
        self._ensure(self.t + 2)
        cache = self.__dict__.setdefault("_early_pairs", {})
        key = (getattr(self, "_gen", 0), rows["uniq_u"].data_ptr(), rows["uniq_i"].data_ptr())
        pairs = cache.get(key)
        if pairs is None:
            if len(cache) > 8:
                cache.clear()
            pairs = cache[key] = self._pairs()
            for k, ids in enumerate((rows["uniq_u"], rows["uniq_i"])):
                pairs[k].row_ids = ptr(ids)
        _lib.call("ncf_adam_pairs_catchup_lock_clock", ctypes.addressof(pairs), 2,
                  self.engine.model.mlp_embedding_dim, ptr(rows["num_unique"]), n, 1, 0,
                  ptr(self.clock if clock is None else clock), ptr(self._table), *self._consts(),
                  stream)

    def fused_apply_args(self, w):
        """The arguments of the apply fused into the embedding backward (engine.backward
        fused_apply): this step's touched rows stepped where their gradient rows complete, as
        apply() would step them after it.  None without the device clock.  The overlapped sweep
        may still run beside that apply (joined later, in apply()/sweep_join): safe by the
        invariant stated in __init__ (sweep target t <= every batch row's stamp)."""
        if self.clock is None or w.g.n == 0:
            return None
        self._ensure(self.t + 1)
        pairs = self._pairs_for(w)
        return (ctypes.addressof(pairs), ptr(self.clock), ptr(self._table)) + self._consts()

    # ---- after the backward: this step's gradient on the touched rows
    def apply(self, w, st, late_join: bool = False):
        """``late_join`` (the step's table apply already ran inside the embedding backward): the
        side stream is not joined here; the caller joins it (sweep_join) before the clock
        advance.  Only when no sweep part is owed (those run on st and must follow the join)."""
        n = w.g.n
        if self.clock is not None:
            self._ensure(self.t + 1)
            if not (late_join and getattr(w, "applied", False) and not self._owed):
                self.sweep_join()
                self._settle(st)
            if n > 0 and not getattr(w, "applied", False):
                pairs = self._pairs_for(w)
                _lib.call("ncf_adam_pairs_apply_clock", ctypes.addressof(pairs), 2,
                          self.engine.model.mlp_embedding_dim, ptr(w.num_unique), n, 1,
                          ptr(self.clock), ptr(self._table), *self._consts(), st)
            w.applied = False
            self.advance(st)
            return
        self.apply_rows("user", w.uniq_u, w.num_unique, 0, n, w.G["mf_user"], w.G["mlp_user"], st)
        self.apply_rows("item", w.uniq_i, w.num_unique, 1, n, w.G["mf_item"], w.G["mlp_item"], st)
        self.advance(st)

    def _sweep_range(self, kind, row0, rows, st):
        if rows <= 0 or self.t == 0:
            return
        self._ensure(self.t)
        _lib.call("ncf_adam_sweep_bf16" if self.bf16 else "ncf_adam_sweep", *self._ptrs(kind), row0, rows,
                  self.engine.model.mlp_embedding_dim, ptr(self.stamp[kind]), self.t,
                  ptr(self._table), *self._consts(), st)

    def _sweep(self, st):
        if self.clock is not None:
            self.flush(st)
        for kind in ("user", "item"):
            self._sweep_range(kind, 0, self.stamp[kind].numel(), st)
        self.synced_t = self.t
        self.widen()

    def widen(self):
        """bf16 tables: the fp32 table parameters := the bf16 values (exactly representable)."""
        if self.bf16:
            with torch.no_grad():
                for k, p in self.params.items():
                    p.copy_(self.tables[k])

    def reload_params(self):
        """bf16 tables: take new fp32 parameter values (load_state_dict): round them into the
        bf16 tables and widen back, every row current."""
        if self.bf16:
            with torch.no_grad():
                for k, p in self.params.items():
                    self.tables[k].copy_(p)
            self.widen()

    def sync(self):
        """Catch every row up to the current step (tables + moments become the dense values)."""
        if self.clock is not None:
            self.late_join()
        if self.t == 0 or self.synced_t == self.t:
            return
        self._sweep(_lib.stream_ptr(self.tables["mf_user"].device))

    def detach(self):
        self.sync()
        if self.engine.deferred is self:
            self.engine.deferred = None
