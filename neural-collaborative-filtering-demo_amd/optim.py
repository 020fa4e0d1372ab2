"""Fused Adam for AdvancedNCF behind the reference's own optimizer construction.

The reference builds ``torch.optim.Adam(self.model.parameters(), lr=..., weight_decay=...)``
(src/model/trainer.py:71-75) and calls ``optimizer.zero_grad(); loss.backward();
optimizer.step()`` (:275-285).  That call site stays unchanged: a global optimizer step
pre-hook recognises the parameters of every live AdvancedNCF and updates them with the HIP
kernels instead of torch's per-tensor loop.  The first ``step()`` of a plain Adam binds the
(model, optimizer) pair (``_Binding``); from then on

  * embedding tables: the deferred dense-exact schedule (deferred.py) — the next training
    forward catches up exactly its rows, ``step()`` applies the step's gradient to them and
    sweeps one 1/64 slice of every table (bit-identical to torch's dense Adam, where coupled
    weight decay moves every row every step);
  * dense parameters: one flat Adam launch over the packed buffer;

all on the device step clock, with no host synchronisation.  The optimizer's own lr / betas /
eps / weight_decay are read every step (lr changes apply to steps not yet taken).  State is kept
in ``optimizer.state[p]`` under torch's keys (``step``, ``exp_avg``, ``exp_avg_sq``): every
parameter of the model shares one CPU ``step`` tensor, the moments are the kernels' own buffers
(dense ones views of a flat buffer), and the optimizer's ``state_dict`` / ``load_state_dict``
hooks bring lagging table rows current first, so the torch format stays exact.  The
parameters the fused step updated are taken out of the param groups for the duration of
torch's own step (so torch's loop never sees them) and put back afterwards.

``SCHEDULE = "dense"`` keeps the dense per-step table sweep instead (A/B and tests).  Optimizers
other than plain Adam (amsgrad, maximize, capturable, differentiable, tensor lr, other classes)
receive materialised dense table gradients and run unchanged.
"""
import weakref

import torch
import torch.optim.optimizer as _topt

from . import _lib
from ._lib import ptr

_models = weakref.WeakSet()
_hooks = {}
SCHEDULE = "deferred"      # or "dense": the per-step full-table sweep (ncf_adam_table)
# rolling-sweep period of the deferred table schedule behind torch.optim.Adam (the reference call
# pattern): 128 measured faster than 64 (drop-in leg 0.3289 / 0.328 against 0.3366 / 0.332
# ms/step, r5zq), as for FusedTrainStep and the row-sharded step
SWEEP_EVERY = 128


def register(model):
    _models.add(model)
    if "pre" not in _hooks:
        _hooks["pre"] = _topt.register_optimizer_step_pre_hook(_pre_hook)
        _hooks["post"] = _topt.register_optimizer_step_post_hook(_post_hook)


def _is_plain_adam(opt):
    if type(opt) is not torch.optim.Adam:
        return False
    for g in opt.param_groups:
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or \
                g.get("capturable") or g.get("decoupled_weight_decay", False):
            return False
        if isinstance(g["lr"], torch.Tensor):
            return False
    return True


def _models_in(opt):
    """The AdvancedNCF models whose four tables this optimizer holds (cached on the optimizer,
    re-derived when its parameter groups change)."""
    key = tuple(len(g["params"]) for g in opt.param_groups)
    c = opt.__dict__.get("_ncf_models")
    if c is not None and c[0] == key:
        out = [r() for r in c[1]]
        if all(m is not None for m in out):
            return [m for m in out if m.engine.flat is not None and m.engine.flat.is_cuda]
    ids = {id(p) for g in opt.param_groups for p in g["params"]}
    found = [m for m in list(_models)
             if all(id(p) in ids for p in m.engine.table_params().values())]
    opt.__dict__["_ncf_models"] = (key, [weakref.ref(m) for m in found])
    return [m for m in found if m.engine.flat is not None and m.engine.flat.is_cuda]


def _group_of(opt):
    """{id(param): its param_group} (cached on the optimizer while its groups keep their
    parameter lists)."""
    key = tuple((id(g), len(g["params"])) for g in opt.param_groups)
    c = opt.__dict__.get("_ncf_gmap")
    if c is not None and c[0] == key:
        return c[1]
    gmap = {}
    for g in opt.param_groups:
        for p in g["params"]:
            gmap[id(p)] = g
    opt.__dict__["_ncf_gmap"] = (key, gmap)
    return gmap


def _hp(g):
    b1, b2 = g["betas"]
    return float(g["lr"]), (float(b1), float(b2)), float(g["eps"]), float(g["weight_decay"])


def _fresh_moments(p):
    return torch.zeros_like(p, memory_format=torch.contiguous_format)


class _Binding:
    """One (AdvancedNCF, torch.optim.Adam) pair on the fused path: the deferred table schedule,
    the flat dense moments and the device step clock, adopted from / exposed as the optimizer's
    torch-format state."""

    def __init__(self, model, opt, group):
        from . import deferred as deferred_mod
        from .deferred import DeferredTableAdam
        eng = model.engine
        eng.ensure_layout()
        self.model = weakref.ref(model)
        self.opt = weakref.ref(opt)
        self.eng = eng
        dev = eng.flat.device
        self.tables = eng.table_params()
        self.dense = eng.dense_params()
        self.flat_ptr = eng.flat.data_ptr()
        self.hp = _hp(group)
        self.uniform = True          # every parameter so far stepped on the shared counter
        self.step_t = torch.tensor(0.0)
        self._step_np = self.step_t.numpy()   # (the same scalar: bumped without a torch op)
        self.m_flat = torch.zeros_like(eng.flat)
        self.v_flat = torch.zeros_like(eng.flat)
        self.moments = {k: {"exp_avg": _fresh_moments(p), "exp_avg_sq": _fresh_moments(p)}
                        for k, p in self.tables.items()}
        if eng.deferred is not None:          # another schedule (a FusedTrainStep) let go
            eng.deferred.detach()
        self.base_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.clock = torch.tensor([0, self.base_seed], dtype=torch.int64, device=dev)
        lr, betas, eps, wd = self.hp
        self.D = None
        # (the deferred schedule steps an MF and an MLP table as one pair of one width: with
        # mf_embedding_dim != mlp_embedding_dim the dense per-step sweep, equally exact, runs)
        if SCHEDULE == "deferred" and model.mf_embedding_dim == model.mlp_embedding_dim:
            self.D = DeferredTableAdam(eng, lr, betas, eps, wd, SWEEP_EVERY,
                                       moments=self.moments, clock=self.clock,
                                       overlap_sweep=deferred_mod.OVERLAP_SWEEP)
            eng.clock = self.clock
        self.adopt(opt)

    # ---- torch-format state <-> kernel buffers
    def adopt(self, opt):
        """Take over whatever the optimizer's state holds for this model (fresh, or loaded by
        load_state_dict: copied into the kernel buffers) and expose the kernel buffers there.
        Every row is current at that step afterwards."""
        eng = self.eng
        st = opt.state
        s0 = st.get(self.tables["mf_user"], {})
        step = int(float(s0["step"])) if "step" in s0 else 0
        self.step = step
        self.step_t.fill_(float(step))
        for k, p in self.tables.items():
            s = st[p]
            mine = self.moments[k]
            for key in ("exp_avg", "exp_avg_sq"):
                t = s.get(key)
                if t is not None and t is not mine[key]:
                    mine[key].copy_(t)
                s[key] = mine[key]
            s["step"] = self.step_t
        for name, p in self.dense:
            o, n, shp = eng.offsets[name]
            s = st[p]
            for key, buf in (("exp_avg", self.m_flat), ("exp_avg_sq", self.v_flat)):
                view = buf[o:o + n].view(shp)
                t = s.get(key)
                if t is not None and t.data_ptr() != view.data_ptr():
                    view.copy_(t.reshape(shp))
                s[key] = view
            s["step"] = self.step_t
        self.uniform = True
        if self.D is not None:
            self.D.rebind_moments(self.moments)
            self.D.mark_current(step)
            self.D._ensure(step + 1)
            self.clock[0] = step            # ncf_step_clock.t (reserved = 0)

    def sync(self):
        """Bring every lagging table row (and its moments) current: the tables and the
        optimizer state then hold exactly torch's dense values."""
        if self.D is not None:
            self.D.sync()

    def detach(self):
        self.sync()
        eng = self.eng
        if self.D is not None and eng.deferred is self.D:
            eng.deferred = None
        if eng.clock is self.clock:
            eng.clock = None
        self.D = None

    def valid(self, model):
        return self.eng is model.engine and self.eng.flat is not None and \
            self.eng.flat.data_ptr() == self.flat_ptr and \
            (self.D is None or self.eng.deferred is self.D)

    # ---- one optimizer step
    def step_tables_dense_grads(self, hp, st):
        """Tables holding dense .grad (gradient accumulation, frozen tables, user gradients):
        bring every row current, then torch's elementwise Adam on each graded table."""
        lr, (b1, b2), eps, wd = hp
        self.sync()
        stepped = False
        for k, p in self.tables.items():
            if p.grad is None:
                continue
            m = self.moments[k]
            _lib.call("ncf_adam_table_dense_grad", ptr(p), ptr(p.grad.contiguous()), ptr(m["exp_avg"]),
                      ptr(m["exp_avg_sq"]), p.numel(), lr, b1, b2, eps, wd,
                      float(self.step + 1), st)
            stepped = True
        return stepped

    def run(self, opt, gmap):
        """The fused step of this model; returns the parameters whose .grad torch must not
        see during its own step."""
        eng = self.eng
        dev = eng.flat.device
        st = _lib.stream_ptr(dev)
        group = gmap[id(self.tables["mf_user"])]
        if self.__dict__.get("_group") is not group:
            groups = {id(gmap[id(p)]) for p in self.tables.values()} | \
                {id(gmap[id(p)]) for _, p in self.dense}
            if len(groups) != 1:
                raise NotImplementedError("ncf_amd: the fused Adam needs every AdvancedNCF "
                                          "parameter in one param_group (lr/betas/eps/"
                                          "weight_decay shared)")
            self._group = group
        hp = _hp(group)
        if hp != self.hp:
            if self.D is not None:
                self.D.set_hparams(*hp)
            self.hp = hp
        lr, (b1, b2), eps, wd = hp
        w = eng.pending
        frozen = any(not p.requires_grad for p in self.tables.values())
        if w is not None and (frozen or any(p.grad is not None for p in self.tables.values())):
            eng.materialize_table_grads(accumulate=True)
            w = None
        table_grads = [p for p in self.tables.values() if p.grad is not None]
        views = eng.grad_views()
        if all(p.grad is gv for p, gv in views):
            # the common case: every dense .grad is the view the backward assigned
            dense_with, all_dense = self.dense, True
        else:
            dense_with = [(n, p) for n, p in self.dense if p.grad is not None]
            if w is None and not table_grads and not dense_with:
                return []
            # dense gradients handed in as other tensors than the flat buffer's views: copied
            # in first
            for p, gv in views:
                g = p.grad
                if g is not None and g is not gv and g.data_ptr() != gv.data_ptr():
                    gv.copy_(g)
            all_dense = len(dense_with) == len(self.dense)
        eng.updates += 1
        d = self.D
        clocked = d is not None and w is not None
        if clocked and all_dense and self.uniform and not getattr(w, "slots_set", False):
            # the common step: table apply + sweep + dense Adam with the clock advance, from
            # the launch tape of this geometry when there is one (tapes.py)
            def run():
                s_ = _lib.stream_ptr(dev)     # (the current stream: a capture's, under one)
                d.apply(w, s_)
                eng.pending = None
                d.sweep_join()        # (the clock advance below changes the sweep's target)
                _lib.call("ncf_adam_flat_clock_close", ptr(eng.flat), ptr(eng.flat_grad),
                          ptr(self.m_flat), ptr(self.v_flat), eng.flat.numel(), ptr(d._table), 1,
                          ptr(self.clock), b1, b2, eps, wd, self.base_seed, s_)
            tp = eng.tapes
            if tp is None or not tp.step(w, run):
                run()
            self.step += 1
            self._step_np += 1
            return self._all_params
        # --- tables
        if clocked:
            d.apply(w, st)             # this step's rows + the rolling 1/64 sweep (clock)
            if getattr(w, "slots_set", False):
                eng.reset_slots(w, st)
            eng.pending = None
        elif w is not None:            # SCHEDULE == "dense": sweep every row of every table
            hpf = lambda p: (lr, b1, b2, eps, wd)  # noqa: E731
            key_of = {id(p): k for k, p in self.tables.items()}
            eng.adam_tables(hpf, lambda p: self.moments[key_of[id(p)]], float(self.step + 1), st)
        elif table_grads:
            self.step_tables_dense_grads(hp, st)
            if d is not None:
                d.mark_current(self.step + 1)
        # --- dense parameters
        # the clock counts table steps (the deferred schedule's t): it advances iff they stepped
        tables_stepped = d is not None and (clocked or bool(table_grads))
        if all_dense and self.uniform and clocked:
            # the step's dense Adam + the clock advance in one launch (as FusedTrainStep)
            d.sweep_join()
            _lib.call("ncf_adam_flat_clock_close", ptr(eng.flat), ptr(eng.flat_grad),
                      ptr(self.m_flat), ptr(self.v_flat), eng.flat.numel(), ptr(d._table), 1,
                      ptr(self.clock), b1, b2, eps, wd, self.base_seed, st)
        else:
            step = float(self.step + 1)
            if all_dense and self.uniform:
                _lib.call("ncf_adam_flat", ptr(eng.flat), ptr(eng.flat_grad), ptr(self.m_flat),
                          ptr(self.v_flat), eng.flat.numel(), lr, b1, b2, eps, wd, step, st)
            else:
                # some dense parameters without a gradient (frozen / unused): each graded one
                # on its own (they share the model's step counter)
                self.uniform = self.uniform and all_dense
                for name, p in dense_with:
                    o, n, _ = eng.offsets[name]
                    _lib.call("ncf_adam_flat", ptr(eng.flat) + 4 * o, ptr(eng.flat_grad) + 4 * o,
                              ptr(self.m_flat) + 4 * o, ptr(self.v_flat) + 4 * o, n, lr, b1, b2,
                              eps, wd, step, st)
            if tables_stepped:
                _lib.call("ncf_step_clock_advance", ptr(self.clock), self.base_seed, st)
        self.step += 1
        self._step_np += 1
        return self._all_params

    @property
    def _all_params(self):
        c = self.__dict__.get("_allp")
        if c is None:
            c = self._allp = [p for _, p in self.dense] + list(self.tables.values())
        return c

    @property
    def _all_ids(self):
        """frozenset of id() of _all_params (what the pre-hook hides from torch's step)."""
        c = self.__dict__.get("_allids")
        if c is None:
            c = self._allids = frozenset(id(p) for p in self._all_params)
        return c


def _bindings(opt):
    b = opt.__dict__.get("_ncf_bind")
    if b is None:
        b = opt.__dict__["_ncf_bind"] = {}
        opt.register_state_dict_pre_hook(_opt_state_dict_pre)
        opt.register_load_state_dict_pre_hook(_opt_load_pre)
        opt.register_load_state_dict_post_hook(_opt_load_post)
    return b


def _opt_state_dict_pre(opt):
    for b in list(opt.__dict__.get("_ncf_bind", {}).values()):
        b.sync()


def _opt_load_pre(opt, state_dict):
    for b in list(opt.__dict__.get("_ncf_bind", {}).values()):
        b.sync()       # nothing owed from the old run may be replayed onto the loaded rows
    return None


def _opt_load_post(opt):
    for b in list(opt.__dict__.get("_ncf_bind", {}).values()):
        b.adopt(opt)


def binding_of(opt, model):
    """The fused-path binding of (optimizer, model), if that pair has stepped."""
    return opt.__dict__.get("_ncf_bind", {}).get(id(model))


def _restore_groups(opt):
    swap = opt.__dict__.pop("_ncf_swap", None)
    if swap:
        for g, ps in swap:
            g["params"] = ps


def _hide(opt, hk):
    """Take the parameters the fused step just updated (``hk``: frozenset of their id()) out of
    the param groups for the duration of torch's own step (restored by the post hook): torch's
    loop then never sees them — one list swap per group instead of hiding and restoring every
    .grad."""
    cache = opt.__dict__.setdefault("_ncf_keep", {})
    swap = []
    for g in opt.param_groups:
        ps = g["params"]
        c = cache.get(id(g))
        if c is None or c[0] is not ps or c[1] != len(ps) or (c[2] is not hk and c[2] != hk):
            c = cache[id(g)] = (ps, len(ps), hk, [p for p in ps if id(p) not in hk])
        if len(c[3]) != len(ps):
            swap.append((g, ps))
            g["params"] = c[3]
    opt._ncf_swap = swap


def _pre_hook(opt, args, kwargs):
    _restore_groups(opt)        # (a previous step that raised inside torch's body)
    models = _models_in(opt)
    if not models:
        return None
    if not _is_plain_adam(opt):
        for m in models:
            b = opt.__dict__.get("_ncf_bind", {}).pop(id(m), None)
            if b is not None:
                b.detach()
            elif m.engine.deferred is not None:
                m.engine.deferred.detach()
            m.engine.materialize_table_grads()
        return None
    gmap = _group_of(opt)
    binds = _bindings(opt)
    hidden = None
    for m in models:
        b = binds.get(id(m))
        if b is None or not b.valid(m):
            if b is not None:
                b.detach()
            b = binds[id(m)] = _Binding(m, opt, gmap[id(m.engine.table_params()["mf_user"])])
        if b.run(opt, gmap):
            hidden = b._all_ids if hidden is None else hidden | b._all_ids
    if hidden:
        _hide(opt, hidden)
    return None


def _post_hook(opt, args, kwargs):
    _restore_groups(opt)
