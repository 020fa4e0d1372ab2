"""Fused Adam for AdvancedNCF behind the reference's own optimizer construction.

The reference builds ``torch.optim.Adam(self.model.parameters(), lr=..., weight_decay=...)``
(src/model/trainer.py:71-75) and calls ``optimizer.zero_grad(); loss.backward();
optimizer.step()`` (:275-285).  That call site stays unchanged: a global optimizer step
pre-hook recognises the parameters of every live AdvancedNCF and updates them with the HIP
kernels instead of torch's per-tensor loop —

  * embedding tables: dense-exact Adam (every row decays) streaming the table once,
    touched rows' gradients read from the compact segment-reduce output via the slot map;
  * dense parameters: one flat Adam launch over the packed buffer;

with the optimizer's own lr / betas / eps / weight_decay, and state kept in
``optimizer.state[p]`` under torch's keys (``step``, ``exp_avg``, ``exp_avg_sq``) so
``optimizer.state_dict()`` / ``load_state_dict`` keep torch's format.  Their ``.grad`` is hidden
for the duration of torch's own step (so torch skips them) and restored afterwards.

Optimizers other than plain Adam (amsgrad, maximize, foreach/fused overrides are fine; other
classes) receive materialised dense table gradients and run unchanged.
"""
import weakref

import torch
import torch.optim.optimizer as _topt

from . import _lib
from ._lib import ptr

_models = weakref.WeakSet()
_hooks = {}


def register(model):
    _models.add(model)
    if "pre" not in _hooks:
        _hooks["pre"] = _topt.register_optimizer_step_pre_hook(_pre_hook)
        _hooks["post"] = _topt.register_optimizer_step_post_hook(_post_hook)


def note_pending(engine):
    pass


def _is_plain_adam(opt):
    if type(opt) is not torch.optim.Adam:
        return False
    for g in opt.param_groups:
        if g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or \
                g.get("decoupled_weight_decay", False):
            return False
        if isinstance(g["lr"], torch.Tensor):
            return False
    return True


def _models_in(opt):
    ids = {id(p) for g in opt.param_groups for p in g["params"]}
    out = []
    for m in list(_models):
        tb = m.engine.table_params()
        if all(id(p) in ids for p in tb.values()) and tb["mf_user"].is_cuda:
            out.append(m)
    return out


def _group_of(opt):
    gmap = {}
    for g in opt.param_groups:
        for p in g["params"]:
            gmap[id(p)] = g
    return gmap


def _state(opt, p, step_t):
    st = opt.state[p]
    if "exp_avg" not in st:
        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    st["step"] = step_t
    return st


class _DenseMoments:
    """Flat exp_avg / exp_avg_sq buffers parallel to the engine's flat parameter buffer."""

    def __init__(self, engine):
        self.m = torch.zeros_like(engine.flat)
        self.v = torch.zeros_like(engine.flat)
        self.flat_ptr = engine.flat.data_ptr()


def _pre_hook(opt, args, kwargs):
    models = _models_in(opt)
    if not models:
        return None
    stash = []
    if not _is_plain_adam(opt):
        for m in models:
            m.engine.materialize_table_grads()
        return None
    gmap = _group_of(opt)
    for m in models:
        eng = m.engine
        eng.ensure_layout() if eng.flat is None else None
        dev = eng.flat.device
        st = _lib.stream_ptr(dev)
        dense = eng.dense_params()
        tables = eng.table_params()
        have_dense = all(p.grad is not None for _, p in dense)
        have_tables = eng.pending is not None or any(p.grad is not None for p in tables.values())
        if not have_dense and not have_tables:
            continue
        # one step counter shared by every parameter of this model (they always step together)
        anyp = tables["mf_user"]
        st0 = opt.state[anyp].get("step")
        if isinstance(st0, torch.Tensor):
            step_t = st0
        else:
            step_t = torch.tensor(0.0, dtype=torch.float32)
        step_t += 1
        step = float(step_t.item())
        eng.updates += 1

        def hp(p):
            g = gmap[id(p)]
            b1, b2 = g["betas"]
            return float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"])

        # --- tables (dense-exact)
        eng.adam_tables(hp, lambda p: _state(opt, p, step_t), step, st)
        # --- dense params: flat buffers; moments exposed as views in optimizer.state
        mom = getattr(eng, "_moments", None)
        if mom is None or mom.flat_ptr != eng.flat.data_ptr():
            mom = _DenseMoments(eng)
            eng._moments = mom
            for name, p in dense:      # adopt existing state (e.g. after load_state_dict)
                s = opt.state.get(p)
                o, n, shp = eng.offsets[name]
                if s and "exp_avg" in s:
                    mom.m[o:o + n].copy_(s["exp_avg"].reshape(-1))
                    mom.v[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
        for name, p in dense:
            o, n, shp = eng.offsets[name]
            s = opt.state[p]
            mv, vv = mom.m[o:o + n].view(shp), mom.v[o:o + n].view(shp)
            if s.get("exp_avg") is not None and s["exp_avg"].data_ptr() != mv.data_ptr():
                mv.copy_(s["exp_avg"])
                vv.copy_(s["exp_avg_sq"])
            s["step"] = step_t
            s["exp_avg"], s["exp_avg_sq"] = mv, vv
            if p.grad is not None and p.grad.data_ptr() != eng.grad_view(name).data_ptr():
                eng.grad_view(name).copy_(p.grad)
        groups = {id(gmap[id(p)]) for _, p in dense}
        if have_dense and len(groups) == 1:
            lr, b1, b2, eps, wd = hp(dense[0][1])
            _lib.call("ncf_adam_flat", ptr(eng.flat), ptr(eng.flat_grad), ptr(mom.m), ptr(mom.v),
                      eng.flat.numel(), lr, b1, b2, eps, wd, step, st)
        elif have_dense:
            for name, p in dense:
                o, n, _ = eng.offsets[name]
                lr, b1, b2, eps, wd = hp(p)
                _lib.call("ncf_adam_flat", ptr(eng.flat[o:]), ptr(eng.flat_grad[o:]),
                          ptr(mom.m[o:]), ptr(mom.v[o:]), n, lr, b1, b2, eps, wd, step, st)
        for _, p in list(dense) + list(tables.items()):
            stash.append((p, p.grad))
            p.grad = None
    opt._ncf_stash = stash
    return None


def _post_hook(opt, args, kwargs):
    stash = getattr(opt, "_ncf_stash", None)
    if stash:
        for p, g in stash:
            p.grad = g
        opt._ncf_stash = None
