"""Launch tapes for the reference call pattern (``model(kjt)`` -> ``loss.backward()`` ->
``optimizer.step()``, src/model/trainer.py:258-285).

That loop enters this package three times per step, and each entry runs the same Python host
code every step to issue the same C-ABI launches: measured on MI355X hosts (tools/dropin_host.py)
the host work of a step (0.45-0.87 ms) exceeds the GPU work (0.31 ms at C2), so the drop-in
step was host-bound.  A launch tape (``_lib.LaunchTape``) records the C-ABI calls of one such
entry while it runs for real; later steps replay them from C with the step's own id lists, loss
gradient and stream patched in.  The kernels, their order, their streams and their arguments are
those of the eager code, so results are bit-identical (``tests/test_gpu_dropin.py``).

One tape per phase and batch geometry (n, M, dropout):
  * forward  -- the deferred Adam's claim catch-up, the id sort forked beside the forward, the
    gathers, the attention block and the MLP tower (engine.forward with deferred.prepare);
  * backward -- the tower / attention / embedding backward and the gradient reductions, the
    overlapped sweep fork (engine.backward);
  * step     -- the table apply, the sweep join and the dense Adam with the clock advance
    (optim._Binding.run).
A tape is replayed only when the host state its Python code branches on equals the state it
was recorded in (``_pre`` keys) and the buffers it names are the same (``_signature``); the host
state the replayed code would have left is then set as that code sets it (``_post``).  Anything
else -- gradient accumulation, a frozen table, an lr change that moves the scalar table, an
instrumented run -- takes the eager path for that phase.  ENABLED = False turns tapes off.
"""

import torch

from . import _lib

ENABLED = True
RECORD_AFTER = 2          # consecutive eager steps of one geometry before its tapes are recorded


class _Entry:
    __slots__ = ("w", "fwd", "bwd", "step", "fwd_pre", "bwd_pre", "step_pre", "bwd_post",
                 "step_post", "dedup_ev")

    def __init__(self):
        for k in self.__slots__:
            setattr(self, k, None)


class StepTapes:
    """The tapes of one engine (NCFEngine.tapes)."""

    def __init__(self, eng):
        self.eng = eng
        self.entries = {}
        self.sig = None
        self.streak = (None, 0)
        self.replays = 0          # phases replayed (tests / bench read it)
        self.recorded = 0

    # ---- validity
    def _signature(self, light: int = 0):
        """Everything a tape holds by address or value beyond the step's ids / gradient /
        stream: a change drops every tape.  The forward checks all of it; within the step the
        backward checks the first 4 fields and the optimizer step the first 5 (`light`) — the
        rest cannot change between the three calls of one step without a forward."""
        eng = self.eng
        d = eng.deferred
        head = (id(d), d._table.data_ptr(), eng.flat.data_ptr(), eng.flat_grad.data_ptr(),
                d._consts())
        if light:
            return head[:light]
        tb = eng.table_params()
        return head + (d._serial, getattr(d, "_gen", 0), tuple(d.fork_points),
                       d.overlap, d.sweep_every, tuple(p.data_ptr() for p in tb.values()),
                       tuple(s["exp_avg"].data_ptr() for s in d.state.values()),
                       eng.clock.data_ptr(), eng.err_flag(eng.flat.device).data_ptr())

    def usable(self) -> bool:
        eng = self.eng
        d = eng.deferred
        return (ENABLED and d is not None and d.clock is not None and eng.clock is d.clock
                and not d.bf16 and eng.fork_hook is None and eng.timing is None
                and not eng.concurrent and _lib.PROFILE is None and _lib.tapes_available()
                and not torch.cuda.is_current_stream_capturing())

    def _horizon(self):
        """The per-step scalar table must cover the replayed step (the eager code's
        d._ensure(t + 1)); refilled in place from the host when needed, outside any tape.
        False when that moved the table (its address is in the tapes)."""
        d = self.eng.deferred
        b1, b2 = d.betas
        if d._filled >= d.t + 2 and d._hp_filled == (d.lr, b1, b2, d.eps):
            return True
        at = d._table.data_ptr()
        d._ensure(d.t + 2)
        return d._table.data_ptr() == at

    def _entry(self, key, create):
        sig = self._signature()
        if sig != self.sig:
            self.entries.clear()
            self.sig = sig
        e = self.entries.get(key)
        if e is None and create:
            e = self.entries[key] = _Entry()
        return e

    # ---- forward
    def _fwd_pre(self, w):
        eng = self.eng
        return (w is not None and eng.ws.get((w.g.n, w.g.M, True)) is w, eng.pending is None,
                w is not None and getattr(w, "dedup_ev", None) is None,
                w is not None and not getattr(w, "prededuped", None))

    def forward(self, uid, iid, M, drop_p, seed):
        """engine.forward(...) of a training step with the deferred prepare, replayed from the
        geometry's tape or recorded into it; None when the caller must run it eagerly."""
        if not self.usable():
            self.streak = (None, 0)
            return None
        eng = self.eng
        eng.ensure_layout()       # (a parameter re-assigned since: re-pack, the signature moves)
        n = uid.numel()
        key = (n, M, float(drop_p), int(seed))
        ks, cnt = self.streak
        cnt = cnt + 1 if ks == key else 1
        self.streak = (key, cnt)
        if not self._horizon():
            return None
        e = self._entry(key, create=cnt > RECORD_AFTER)
        if e is None:
            return None
        st = _lib.stream_ptr(uid.device)
        if e.fwd is not None and self._fwd_pre(e.w) == e.fwd_pre:
            w = e.w
            w.deduped = False
            e.fwd.replay((uid.data_ptr(), iid.data_ptr(), st))
            # host state as the recorded code leaves it (deferred._prepare_claim)
            w.deduped, w.prededuped = True, None
            w.dedup_ev, w.dedup_refs = e.dedup_ev, (uid, iid)
            self.replays += 1
            return w
        # record: the forward runs for real while the tape holds its calls
        w0 = eng.ws.get((n, M, True))
        pre = self._fwd_pre(w0)
        if not (pre[0] and pre[1] and pre[2] and pre[3]):
            return None           # (workspace not there yet, or a step left pending)
        tape = _lib.LaunchTape()
        with tape.record((uid.data_ptr(), 8 * n, iid.data_ptr(), 8 * n, st, 1)):
            w = eng.forward(uid, iid, M, True, drop_p, seed, prepare=eng.deferred.prepare)
        if tape.valid and w is w0 and getattr(w, "deduped", False) and w.dedup_ev is not None:
            e.w, e.fwd, e.fwd_pre, e.dedup_ev = w, tape, pre, w.dedup_ev
            e.bwd = e.step = None     # recorded against this forward's host state
            self.recorded += 1
        return w

    # ---- backward
    def _bwd_pre(self, e, w):
        eng = self.eng
        d = eng.deferred
        return (w is e.w, eng.pending is None, getattr(w, "dedup_ev", None) is e.dedup_ev,
                tuple(d._owed), d._joined, eng._zero_cols_of is eng.flat_grad,
                not getattr(eng, "_red_pending", False))

    def backward(self, w, uid, iid, gp, drop_p, seed):
        """engine.backward(w, uid, iid, gp, None, drop_p, seed) replayed or recorded; False
        when the caller must run it eagerly.  ``gp``: the loss gradient, contiguous fp32."""
        if not self.usable() or not self._horizon():
            return False
        n = w.g.n
        if self.sig is None or self._signature(4) != self.sig[:4]:
            self.entries.clear()
            self.sig = None
            return False
        e = self.entries.get((n, w.g.M, float(drop_p), int(seed)))
        if e is None or e.w is not w or e.fwd is None:
            return False
        eng = self.eng
        d = eng.deferred
        st = _lib.stream_ptr(gp.device)
        pre = self._bwd_pre(e, w)
        if e.bwd is not None and pre == e.bwd_pre:
            w.red_list.count = 0
            w.wgrads = []
            h = w.cache.get("head_args")
            if h is not None:         # (the loss gradient's and the ids' addresses: ncf_mlp_bwd)
                h.grad_prob, h.user_ids = gp.data_ptr(), uid.data_ptr()
            e.bwd.replay((uid.data_ptr(), iid.data_ptr(), gp.data_ptr(), st))
            owed, joined = e.bwd_post
            d._owed, d._joined = list(owed), joined
            w.slots_set = False
            w.dedup_ev = w.dedup_refs = None
            w.red_list.count = 0
            eng.pending = w
            self.replays += 1
            return True
        tape = _lib.LaunchTape()
        with tape.record((uid.data_ptr(), 8 * n, iid.data_ptr(), 8 * n, gp.data_ptr(), 4 * n,
                          st, 1)):
            eng.backward(w, uid, iid, gp, None, drop_p, seed)
        if tape.valid and not w.slots_set and not getattr(eng, "_red_pending", False):
            e.bwd, e.bwd_pre, e.bwd_post = tape, pre, (tuple(d._owed), d._joined)
            e.step = None
            self.recorded += 1
        return True

    # ---- optimizer step
    def _step_pre(self, e, w):
        d = self.eng.deferred
        return (w is e.w, self.eng.pending is w, tuple(d._owed), d._joined,
                not getattr(w, "slots_set", False))

    def step(self, w, run):
        """``run()`` = the step's launches (table apply + sweep join + dense Adam with the clock
        advance), replayed or recorded; False when the caller must call run() itself."""
        if not self.usable() or not self._horizon():
            return False
        # (betas / eps / weight decay are launch arguments here: checked with the addresses)
        if self.sig is None or self._signature(5) != self.sig[:5]:
            self.entries.clear()
            self.sig = None
            return False
        e = None
        for cand in self.entries.values():
            if cand.w is w and cand.bwd is not None:
                e = cand
                break
        if e is None:
            return False
        eng = self.eng
        d = eng.deferred
        st = _lib.stream_ptr(eng.flat.device)
        pre = self._step_pre(e, w)
        if e.step is not None and pre == e.step_pre:
            e.step.replay((st,))
            owed, joined = e.step_post
            d.t += 1                     # DeferredTableAdam.advance
            d._owed, d._joined = list(owed), joined
            eng.pending = None
            self.replays += 1
            return True
        tape = _lib.LaunchTape()
        t0 = d.t
        with tape.record((st, 1)):
            run()
        if tape.valid and d.t == t0 + 1 and eng.pending is None:
            e.step, e.step_pre, e.step_post = tape, pre, (tuple(d._owed), d._joined)
            self.recorded += 1
        return True


class SegmentTapes:
    """Launch tapes of the row-sharded step (distributed.ShardedTrainStep): its launches split
    at the host waits for split sizes into segments, each recorded once per key (geometry,
    plan-buffer set, pipelining state) and replayed with the step's pointers and scalars
    (ids of the next batch, targets, stream; claim token and row counts).  Same contract as
    StepTapes: replayed only from the host state it was recorded in, under an unchanged
    signature, with the host state it leaves set afterwards."""

    def __init__(self):
        self.entries = {}
        self.sig = None
        self.streak = {}
        self.replays = 0
        self.recorded = 0
        self._skip = False

    def usable(self, d, eng) -> bool:
        """The same guards as StepTapes.usable: a tape sees only C-ABI calls, so torch-side
        cross-stream ordering (engine.fork / join, a fork hook) and instrumentation rule it out."""
        self._skip = False
        return (ENABLED and d is not None and d.clock is not None and not d.bf16
                and not eng.concurrent and eng.fork_hook is None and eng.timing is None
                and _lib.PROFILE is None and _lib.tapes_available()
                and not torch.cuda.is_current_stream_capturing())

    def skip(self):
        """Run this step's segments eagerly (something in it is not replayable)."""
        self._skip = True

    @staticmethod
    def horizon(d):
        """The scalar table covers the step (outside any tape; an address change shows in the
        caller's signature)."""
        b1, b2 = d.betas
        if d._filled < d.t + 2 or d._hp_filled != (d.lr, b1, b2, d.eps):
            d._ensure(d.t + 2)

    def run(self, key, sig, pre, ranges, scalars, fn, post) -> bool:
        """Replay segment `key` (True) or run fn() eagerly, recording it once the key has come
        round RECORD_AFTER times (False).  ``ranges``: flat (base, size) pairs of the pointer
        slots; ``scalars``: the values of the scalar slots after them; ``post(None)`` returns
        the host state fn() leaves, ``post(state)`` sets it after a replay."""
        if sig != self.sig:
            self.entries.clear()
            self.sig = sig
        if self._skip:
            fn()
            return False
        e = self.entries.get(key)
        if e is not None and e[1] == pre:
            tape, _, state = e
            tape.replay(tuple(ranges[0::2]) + tuple(scalars))
            post(state)
            self.replays += 1
            return True
        cnt = self.streak.get(key, 0) + 1
        self.streak[key] = cnt
        if cnt <= RECORD_AFTER:
            fn()
            return False
        tape = _lib.LaunchTape()
        with tape.record(ranges):
            fn()
        if tape.valid:
            self.entries[key] = (tape, pre, post(None))
            self.recorded += 1
        return False
