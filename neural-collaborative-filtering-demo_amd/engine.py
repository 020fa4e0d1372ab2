"""Kernel orchestration for the AdvancedNCF hot path (forward, backward, optimizer step).

One ``NCFEngine`` per model.  It owns the device workspaces, the flat layout of the dense
parameters (+ their gradient buffer) and the per-table slot maps, and it sequences the C-ABI
kernels of libncf_hip.so on torch's current HIP stream.  Reference stages (file:line in the
reference repo) are cited at each call.

Data layout in HBM (fp32 throughout — the reference computes in fp32):
  * embedding tables: row-major [rows, D] nn.Parameters (never copied, never densely graded);
  * dense parameters: ONE flat buffer, each used nn.Parameter a 16-B aligned view into it, and a
    parallel flat gradient buffer the backward kernels write into (p.grad are views of it);
  * per-batch activations: a workspace keyed by (N, M), reused across steps (no per-step allocs).
"""
import ctypes
import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _lib
from ._lib import ptr

LN_EPS = 1e-5
# bf16 configuration: the fused MLP tower's Linears on bf16 MFMA (False: fp32 MFMA)
BF16_MM = True
# fp32 configuration: the fused MLP tower's dX Linears on bf16 matrix cores through split
# operands (ncf_mlp_fwd_split / _bwd_split: six bf16 products per fp32 product, fp32-accurate)
# instead of the fp32 MFMA.  Measured (round 5, one MI355X, sweep not overlapped): k_mlp_bwd
# 78.0 vs 83.2 us, k_mlp_fwd 40.3 vs 42.2 us, step 0.309 vs 0.319 ms; but its last-bit
# differences move Adam's sign-flip decisions on near-zero gradients, so at full C2 size the
# step-1 probabilities sit 3.1e-5 from the fp32 oracle (as far as the fp64 trajectory does)
# instead of 2.4e-6: outside the full-size bound against the fp32 oracle (tests/
# test_gpu_fullsize.py).  Off: the headline keeps the fp32 oracle's trajectory.
TOWER_SPLIT = False
# C2 training geometry (D = 64, M = 5: the attention workgroup's 16 groups = the tower's 80-row
# tile): the attention block and the MLP tower as ONE launch per direction (tower_fused.hip,
# ncf_attn_mlp_fwd / ncf_attn_mlp_bwd; the same device code and bits as the two launches each
# way).  Measured at C2 (tools/step_ab.py, 3 interleaved runs each, ms/step): fused with the
# rolling sweep forked before it 0.2879-0.2908, two launches each way 0.2972-0.3006 (isolated:
# forward 57 against 22 + 42 us, backward 105-109 against 37 + 85 us).  False: two launches.
FUSE_ATTN_TOWER = True
# Batches of fewer interaction groups than this run the fused attention + tower in small-batch
# tiles (ncf_attn_mlp_*_small: 3 groups = 15 rows per workgroup instead of 16 groups = 80 rows),
# so a small batch spreads over more CUs (256 groups, the reference's default batch: 86
# workgroups instead of 16).  0: always the 80-row tiles.  Up to 768 groups (256 small
# workgroups, one per CU) the small tiles win; measured C2 steps (ms, small / 80-row tiles, run
# r06j/r06c): 256 groups 0.1657 / 0.2084, 768 groups 0.1827 / 0.2078, 1536 groups 0.2848 / 0.2209.
SMALL_TILE_GROUPS = 3 * 256 + 1
# SURVEY fact 6 (a training group's M rows hold one user): the gather writes the LN'd user rows
# once per group (group_rows = M) when every reader takes the group's row — the fused attention
# block and the fused tower's head backward (False: every row; the same bits, tested; measured
# at C2, 3 interleaved runs each: 0.3001-0.3012 against 0.3017-0.3031 ms/step, gather 11.5-11.8
# against 12.2-12.3 us)
GROUP_ROWS = True
# Fact 6 in the fused attention block: with the rows' user ids it projects Q once per group in
# every workgroup whose groups each hold one user (attn_block.hip ids_uniform; the stash backward
# reads the forward's recorded decision).  False (tests' per-row A/B): no ids are handed to the
# block and every row is gathered (no group rows), so every row's Q is projected.
ATTN_SHARE_Q = True
_WGRAD_ROWS = 160
# Geometry switches, read when an engine is built (tests and A/B runs set them before building a
# model): the one-launch MLP tower (False: per-layer GEMM + row launches), its fused weight
# gradients (False: the grouped weight-gradient launch), the one-launch attention block (False:
# projection GEMMs + attention.hip core), and the attention backward recomputing q/k/v/P/o
# instead of reading the forward's stash (off: measured slower, below)
MLP_FUSED = True
MLP_WGRAD = True
ATTN_BLOCK = True
ATTN_RC = False
# the fused attention forward's O stash (off: the backward recomputes O from the stashed P and V,
# attn_pv, the same bits, tested).  Measured at C2, 3 interleaved runs each: forward 22.3-23.1
# against 23.0-23.2 us, backward 38.3-38.9 against 37.9-38.0 us, forward HBM 25.7 against
# 31.0 MB per launch (gpurun_out/r4r_*)
_STASH_O = False


def _tptr(t) -> int:
    """A table given as a tensor or as a raw device pointer (int)."""
    return t if isinstance(t, int) else ptr(t)


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


@dataclass
class Geometry:
    n: int          # rows (samples) in the batch
    M: int          # rows per attention group (1 + negatives in training, 1 in eval)
    B: int          # groups
    D: int
    T: int
    H: int
    hidden: List[int]
    Dm: int = 0     # the MF tables' width (mf_embedding_dim); 0: the same as D


class Workspace:
    """Activation + scratch buffers for one (n, M) batch geometry."""

    def __init__(self, g: Geometry, device, train: bool):
        f = dict(device=device, dtype=torch.float32)
        n, D = g.n, g.D
        Dm = g.Dm or D
        self.g = g
        e = lambda *s: torch.empty(*s, **f)  # noqa: E731
        self.mf_pred, self.mlp_pred, self.prob = e(n), e(n), e(n)
        self.xu, self.xi, self.q, self.k, self.v, self.o, self.y = (e(n, D) for _ in range(7))
        self.umf = e(n, Dm) if train else None
        self.imf = e(n, Dm) if train else None
        if Dm != D:
            # split widths (mf_embedding_dim != mlp_embedding_dim): the gather and the embedding
            # backward run once per collection; each run's second pair of outputs is scratch
            self.split = {"rows_m": e(2, n, Dm), "rows_l": e(2, n, D), "pred": e(n),
                          "zero_w": torch.zeros(D, **f)}
        else:
            self.split = None
        self.P = e(max(1, g.B * g.H * g.M * g.M))
        self.r = [e(n, h) for h in g.hidden]
        self.a = [e(n, h) for h in g.hidden]
        self.mean = [e(n) for _ in g.hidden]
        self.rstd = [e(n) for _ in g.hidden]
        self.err = None             # the engine-wide sticky id-error flag (NCFEngine.workspace)
        self.train = train
        self.cache = {}             # ctypes argument blocks built once per workspace
        if not train:
            return
        self.dumf, self.dimf = e(n, Dm), e(n, Dm)
        self.dxu, self.dxi = e(n, D), e(n, D)
        self.dq, self.dk, self.dv, self.do, self.dy = (e(n, D) for _ in range(5))
        self.dS = e(max(1, g.B * g.H * g.M * g.M))
        self.dlin = [e(n, h) for h in g.hidden]
        self.da = [e(n, h) for h in g.hidden]
        self.loss = e(1)
        # Backward workspaces.  Every gradient reduction of the backward is deferred into
        # red_list and run by one ncf_reduce_batch at its end, so each producing call site keeps
        # its partials in its own slice of `red_ws` until then; the weight gradients are queued
        # in `wgrads` and run as one grouped launch (wg_ws holds their slab partials).
        sites = [("head", _lib.query("ncf_head_bwd_workspace", n, g.hidden[-1], max(D, Dm)))]
        for l, h in enumerate(g.hidden):
            sites.append((f"relu{l}", _lib.query("ncf_relu_ln_dropout_bwd_workspace", n, h)))
        mlp_ws = _lib.query("ncf_mlp_bwd_workspace", n)
        attn_ws = _lib.query("ncf_attn_block_bwd_workspace", g.B)
        if g.B < SMALL_TILE_GROUPS:     # (the small-batch tiles leave more partial sets)
            mlp_ws = max(mlp_ws, _lib.query("ncf_attn_mlp_bwd_workspace_small", g.B, 0))
            attn_ws = max(attn_ws, _lib.query("ncf_attn_mlp_bwd_workspace_small", g.B, 1))
        sites.append(("mlp", mlp_ws))
        sites.append(("attn", attn_ws))
        self.site_off, off = {}, 0
        for name, size in sites:
            self.site_off[name] = (off, size)
            off += _align4(size)
        self.red_ws = e(max(off, 1))
        self.red_list = _lib.ReduceList()
        self.red_scratch = e(1)
        self.wgrads = []            # weight gradients collected during a backward (grouped launch)
        self.wg_ws = []             # partials of the grouped launches in flight (one per slot)
        self.emb_ws = torch.empty(_lib.query("ncf_embedding_bwd_workspace", n, D),
                                  dtype=torch.uint8, device=device)
        self.G = {k: e(n, Dm if k.startswith("mf") else D)
                  for k in ("mf_user", "mlp_user", "mf_item", "mlp_item")}
        if Dm != D:      # the MF collection's own dedup workspace (its segment layout is per width)
            self.emb_ws_m = torch.empty(_lib.query("ncf_embedding_bwd_workspace", n, Dm),
                                        dtype=torch.uint8, device=device)
            self.split["uniq"] = torch.empty(2, max(1, n), dtype=torch.int64, device=device)
            self.split["num_unique"] = torch.zeros(2, dtype=torch.int32, device=device)
            self.split["ln"] = torch.empty(4, max(D, Dm), **f)
        self.uniq_u = torch.empty(max(1, n), dtype=torch.int64, device=device)
        self.uniq_i = torch.empty(max(1, n), dtype=torch.int64, device=device)
        self.num_unique = torch.zeros(2, dtype=torch.int32, device=device)

    @staticmethod
    def splits_for(m_out: int, k_out: int, rows: int) -> int:
        """Row slabs of a weight-gradient product: ~160 batch rows per wave (a few waves per SIMD
        over the grouped launch of a step), at most 256 slabs."""
        return max(1, min(256, math.ceil(max(rows, 1) / _WGRAD_ROWS)))

    def run_wgrads(self, st, slot: int = 0):
        """The weight gradients queued since the last call, as one grouped launch on stream
        ``st``; their slab reductions join the deferred list.  ``slot`` selects the partials
        buffer (groups in flight at the same time need distinct ones)."""
        if not self.wgrads:
            return
        descs = (_lib.WgradDesc * len(self.wgrads))()
        for d, (dY, ldy, X, ldx, dW, ldw, m_out, k_in, n, dbias) in zip(descs, self.wgrads):
            d.dy, d.x, d.dw, d.dbias = ptr(dY), ptr(X), ptr(dW), ptr(dbias)
            d.ldy, d.ldx, d.ldw = ldy, ldx, ldw
            d.m_out, d.k_in, d.n, d.slabs, d.accumulate = m_out, k_in, n, self.splits_for(m_out, k_in, n), 0
        addr = ctypes.addressof(descs)
        need = _lib.query("ncf_wgrad_grouped_workspace", addr, len(self.wgrads))
        while len(self.wg_ws) <= slot:
            self.wg_ws.append(torch.empty(1, dtype=torch.float32, device=self.red_ws.device))
        if self.wg_ws[slot].numel() < need:
            self.wg_ws[slot] = torch.empty(need, dtype=torch.float32, device=self.red_ws.device)
        ws = self.wg_ws[slot]
        _lib.call("ncf_wgrad_grouped", addr, len(self.wgrads), ptr(ws), ws.numel(),
                  self.red_list.address, st)
        self.wgrads = []

    def site(self, name: str) -> torch.Tensor:
        off, size = self.site_off[name]
        return self.red_ws[off:off + size]

    def run_reductions(self, st, scratch: str = "red_scratch"):
        """All gradient reductions deferred by this backward so far, in two launches (``scratch``:
        the workspace attribute of the scratch buffer — the early reductions on a side stream
        take a second one, so both batches can be in flight)."""
        lst = self.red_list
        if lst.count == 0:
            return
        need = _lib.query("ncf_reduce_batch_scratch", lst.address)
        buf = getattr(self, scratch, None)
        if buf is None or buf.numel() < need:
            buf = torch.empty(max(need, 1), dtype=torch.float32, device=self.red_ws.device)
            setattr(self, scratch, buf)
        _lib.call("ncf_reduce_batch", lst.address, ptr(buf), buf.numel(), st)
        lst.count = 0


class NCFEngine:
    """Binds an AdvancedNCF module to the HIP kernels."""

    def __init__(self, model):
        self.model = model
        self.fork_hook = None     # callable(at): side-stream work the caller forks at that point
        self.ws: Dict[tuple, Workspace] = {}
        self.flat = None
        self.flat_grad = None
        self.slot_u = None
        self.slot_i = None
        self.pending = None       # compact table grads of the last backward, not yet applied
        self.dense_names: List[str] = []
        self.offsets: Dict[str, tuple] = {}
        self.timing = None        # optional {table: (start_event, end_event)} for the bench
        self.deferred = None      # DeferredTableAdam holding rows behind, if any
        self.clock = None         # ncf_step_clock (device) of a clock-driven / captured step
        self._zero_cols_of = None  # flat_grad whose never-written mlp.0 temporal columns are 0
        self.concurrent = False   # fork independent work onto side streams (graph mode)
        self._side = None         # side streams (fork / join)
        self._events = None
        self._ev_i = 0
        self._mlp_ok = {}
        # the module's geometry switches as they were when this engine was built
        self._env_mlp_fused = bool(MLP_FUSED)
        self._env_mlp_wgrad = bool(MLP_WGRAD)
        self._env_attn_block = bool(ATTN_BLOCK)
        self._env_attn_rc = bool(ATTN_RC)
        from .tapes import StepTapes
        self.tapes = StepTapes(self)   # launch tapes of the reference call pattern (tapes.py)
        self.updates = 0          # parameter writes by the HIP kernels (torch's _version misses them)

    # ------------------------------------------------------------------ side streams
    # The step is a chain of latency-bound kernels that each fill a fraction of the GPU; work
    # that is independent of the chain (weight gradients, the q/k projections, the second id
    # kind) is forked onto side streams that start after everything queued so far on the
    # current stream and are joined back before their results are read.  Same kernels, same
    # inputs: results are bit-identical to the serial order.
    def fork(self, dev, k: int = 1):
        if not self.concurrent:   # serial: "side streams" are the current stream itself
            return [torch.cuda.current_stream(dev)] * k
        if self._side is None or self._side[0].device != dev:
            self._side = [_lib.side_stream(dev) for _ in range(2)]
            self._events = [torch.cuda.Event() for _ in range(16)]
        cur = torch.cuda.current_stream(dev)
        ev = self._next_event()
        ev.record(cur)
        for sd in self._side[:k]:
            sd.wait_event(ev)
        return self._side[:k]

    def join(self, dev, streams):
        if not self.concurrent:
            return
        cur = torch.cuda.current_stream(dev)
        for sd in streams:
            ev = self._next_event()
            ev.record(sd)
            cur.wait_event(ev)

    def _next_event(self):
        self._ev_i = (self._ev_i + 1) % len(self._events)
        return self._events[self._ev_i]

    # ------------------------------------------------------------------ parameter layout
    def dense_params(self):
        m = self.model
        ps = [("mf_norm.weight", m.mf_norm.weight), ("mf_norm.bias", m.mf_norm.bias),
              ("mlp_norm.weight", m.mlp_norm.weight), ("mlp_norm.bias", m.mlp_norm.bias)]
        att = m.user_product_attention
        for nm in ("q_proj", "k_proj", "v_proj", "out_proj"):
            lin = getattr(att, nm)
            ps += [(f"user_product_attention.{nm}.weight", lin.weight),
                   (f"user_product_attention.{nm}.bias", lin.bias)]
        for l in range(len(m.mlp_hidden_dims)):
            lin, ln = m.mlp[4 * l], m.mlp[4 * l + 2]
            ps += [(f"mlp.{4 * l}.weight", lin.weight), (f"mlp.{4 * l}.bias", lin.bias),
                   (f"mlp.{4 * l + 2}.weight", ln.weight), (f"mlp.{4 * l + 2}.bias", ln.bias)]
        ps += [("mf_output.weight", m.mf_output.weight), ("mf_output.bias", m.mf_output.bias),
               ("mlp_output.weight", m.mlp_output.weight), ("mlp_output.bias", m.mlp_output.bias),
               ("final.0.weight", m.final[0].weight), ("final.0.bias", m.final[0].bias)]
        return ps

    def table_params(self):
        # raw parameters: kernel plumbing must not trigger the bags' bring-current-on-read
        m = self.model
        mf, mlp = m.mf_embedding_collection.embedding_bags, m.mlp_embedding_collection.embedding_bags
        return {"mf_user": mf["user_id"].raw_weight(), "mf_item": mf["product_id"].raw_weight(),
                "mlp_user": mlp["user_id"].raw_weight(),
                "mlp_item": mlp["product_id"].raw_weight()}

    def flatten(self):
        """(Re)pack the used dense parameters into one 16-B aligned flat buffer (views)."""
        ps = self.dense_params()
        dev = ps[0][1].device
        total, offs = 0, {}
        for name, p in ps:
            offs[name] = (total, p.numel(), tuple(p.shape))
            total += _align4(p.numel())
        flat = torch.zeros(total, dtype=torch.float32, device=dev)
        for name, p in ps:
            o, n, shp = offs[name]
            flat[o:o + n].copy_(p.data.reshape(-1))
            p.data = flat[o:o + n].view(shp)
        self.flat = flat
        self._layout_key = self._pp_cache = None    # re-validated by ensure_layout
        self.flat_grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets = offs
        self.dense_names = [n for n, _ in ps]
        self.ws.clear()
        self.pending = None
        if dev.type == "cuda":
            m = self.model
            self.slot_u = torch.full((m.num_users,), -1, dtype=torch.int32, device=dev)
            self.slot_i = torch.full((m.num_products,), -1, dtype=torch.int32, device=dev)
        else:
            self.slot_u = self.slot_i = None

    def grad_view(self, name):
        o, n, shp = self.offsets[name]
        return self.flat_grad[o:o + n].view(shp)

    def gptr(self, name) -> int:
        """Device pointer of a parameter's slice of the flat gradient buffer."""
        return self.flat_grad.data_ptr() + 4 * self.offsets[name][0]

    def is_flat_view(self, p) -> bool:
        if self.flat is None:
            return False
        base = self.flat.data_ptr()
        return base <= p.data_ptr() < base + self.flat.numel() * 4

    def ensure_layout(self):
        """Re-pack when a dense parameter no longer views the flat buffer (.to(), assignment).
        Fast path: the parameter objects and their data pointers as recorded at the last pack
        (one data_ptr per parameter, no module traversal)."""
        key = getattr(self, "_layout_key", None)
        if key is not None and self.flat is not None:
            plist, ptrs = key
            if [p.data_ptr() for p in plist] == ptrs and self.model.mf_norm.weight is plist[0]:
                return
        ps = self.dense_params()
        if self.flat is None or any(not self.is_flat_view(p) for _, p in ps) or \
                self.flat.device != ps[0][1].device:
            self.flatten()
            ps = self.dense_params()
        plist = [p for _, p in ps]
        self._layout_key = (plist, [p.data_ptr() for p in plist])
        self._pp_cache = None

    def pp(self) -> dict:
        """Device pointers of the parameters and tables the launches pass (cached; valid while
        the layout checked by ensure_layout holds)."""
        c = getattr(self, "_pp_cache", None)
        if c is None:
            m = self.model
            att = m.user_product_attention
            c = {name: ptr(p) for name, p in self.dense_params()}
            c.update({"t_" + k: ptr(v) for k, v in self.table_params().items()})
            c["att_w"] = tuple(ptr(getattr(att, nm).weight) for nm in ("q_proj", "k_proj", "v_proj", "out_proj"))
            c["att_b"] = tuple(ptr(getattr(att, nm).bias) for nm in ("q_proj", "k_proj", "v_proj"))
            self._pp_cache = c
        return c

    # ------------------------------------------------------------------ helpers
    def _check_device(self):
        dev = self.model.mf_norm.weight.device
        if dev.type != "cuda":
            raise RuntimeError("ncf_amd: AdvancedNCF runs on the MI355X only (HIP kernels, no CPU "
                               "fallback); call model.to('cuda') first")
        _lib.load()
        return dev

    def workspace(self, n, M, train) -> Workspace:
        key = (n, M, train)
        w = self.ws.get(key)
        if w is None:
            m = self.model
            g = Geometry(n=n, M=M, B=n // M, D=m.mlp_embedding_dim, T=m.temporal_dim,
                         H=m.num_heads, hidden=list(m.mlp_hidden_dims),
                         Dm=m.mf_embedding_dim)
            dev = self.model.mf_norm.weight.device
            w = Workspace(g, dev, train)
            w.err = self.err_flag(dev)
            self.ws[key] = w
        return w

    def err_flag(self, dev) -> torch.Tensor:
        """One sticky out-of-range-id flag per engine, shared by every workspace's kernels: a
        bad id in any batch geometry (a short last batch included) raises it until a check
        reads and clears it."""
        f = getattr(self, "_err", None)
        if f is None or f.device != dev:
            f = self._err = torch.zeros(1, dtype=torch.int32, device=dev)
            self._err_async = None
        return f

    @staticmethod
    def _gemm(A, lda, a_t, Bm, ldb, b_t, C, ldc, M, N, K, bias=None, relu=False, accum=False, st=None):
        flags = (1 if relu else 0) | (2 if accum else 0)
        # weights-resident streaming kernel for the small-weight layers, LDS-tiled 128x64 kernel
        # for the 128x256 / 256x128 ones (measured per shape, tools/gemm_bench.py)
        if not a_t and K in (64, 128, 256) and N in (64, 128, 256) and K * N <= 16384 and K <= 128:
            _lib.call("ncf_gemm_rows", M, N, K, ptr(A), lda, ptr(Bm), ldb, int(b_t), ptr(C), ldc,
                      ptr(bias), flags, st)
            return
        _lib.call("ncf_gemm_f32", M, N, K, ptr(A), lda, int(a_t), ptr(Bm), ldb, int(b_t), ptr(C),
                  ldc, ptr(bias), flags, st)

    @staticmethod
    def _wgrad(w: Workspace, dY, ldy, X, ldx, dW, ldw, m_out, k_in, n, dbias=None):
        """Queue dW[m_out, k_in] = dYᵀ[m_out, n] · X[n, k_in] (+ dbias = column sums of dY) for the
        grouped launch at the end of the backward (Workspace.run_wgrads)."""
        w.wgrads.append((dY, ldy, X, ldx, dW, ldw, m_out, k_in, n, dbias))

    # ------------------------------------------------------------------ forward
    def sync_tables(self):
        """Bring every table row current if a deferred optimizer holds rows behind (no-op
        otherwise).  Called before anything other than the fused train step reads a table."""
        if self.deferred is not None:
            self.deferred.sync()
        if getattr(self, "_err_async", None) is not None:
            # a training run checked ids asynchronously: settle what its last steps saw
            self._err_async = None
            self.check_ids(None)

    def lagging(self) -> bool:
        """Whether a deferred optimizer holds table rows behind (a sync_tables would sweep)."""
        d = self.deferred
        return d is not None and d.t != 0 and d.synced_t != d.t

    def forward(self, uid: torch.Tensor, iid: torch.Tensor, M: int, train: bool,
                drop_p: float, seed: int, prepare=None, tables=None, rows=None,
                temporal=None, bf16: bool = False, table_ld: Optional[int] = None) -> Workspace:
        """AdvancedNCF.forward (architecture.py:258-381) on single-id bags; returns the workspace
        holding prob (and, when ``train``, everything the backward needs).  ``prepare(w, uid,
        iid, stream)`` runs before the gathers (the deferred Adam dedups the ids there and
        brings exactly those rows current).  ``temporal = (item_scale [n,D], factor, te [n,T])``
        is forward_simple's hour path (eval, M = 1): item rows scaled in the gather and the MLP
        fed [attention ‖ te] instead of [attention ‖ 0].  ``table_ld``: the ``tables`` rows are
        that many floats apart (the row-sharded step's received rows read in place)."""
        dev = self._check_device()
        self.ensure_layout()
        m = self.model
        n = uid.numel()
        if n % M != 0:
            # the reference's .view(batch_size, M, -1) (architecture.py:315) fails the same way
            raise RuntimeError(f"batch of {n} rows is not a multiple of samples_per_interaction={M}")
        uid = uid.to(device=dev, dtype=torch.int64).contiguous()
        iid = iid.to(device=dev, dtype=torch.int64).contiguous()
        w = self.workspace(n, M, train)
        if n == 0:
            return w
        st = _lib.stream_ptr(dev)
        D, H, T, hid = m.mlp_embedding_dim, m.num_heads, m.temporal_dim, list(m.mlp_hidden_dims)
        split = m.mf_embedding_dim != D
        if split and temporal is not None:
            # the reference scales the MLP item rows by (1 + 0.3 te) with te of the MF width
            # (architecture.py:436-456): a broadcast error there unless the widths agree
            raise RuntimeError(f"forward_simple(hour): the temporal scale has {m.mf_embedding_dim} "
                               f"columns, the MLP item rows {D}")
        if split and (bf16 or (table_ld is not None and table_ld != D)):
            raise ValueError("mf_embedding_dim != mlp_embedding_dim: fp32 tables, no table_ld")
        pp = self.pp()
        if tables is None:
            tbp = (pp["t_mf_user"], pp["t_mf_item"], pp["t_mlp_user"], pp["t_mlp_item"])
        else:
            tbp = tuple(_tptr(tables[k]) for k in ("mf_user", "mf_item", "mlp_user", "mlp_item"))
        n_users, n_items = rows or (m.num_users, m.num_products)
        # w.err is sticky (zeroed at creation and by check_ids): no per-step fill launch
        w.deduped = False
        if prepare is not None:
            prepare(w, uid, iid, st)
            self._sweep_fork("gather")     # (a fork point after prepare, before the gather)
        else:
            self.sync_tables()
        if temporal is not None and (train or M != 1):
            raise ValueError("the temporal (hour) path is forward_simple's: eval, one item per group")
        # a2-a4: 4 gathers + mf_norm/mlp_norm + GMF  (architecture.py:286-287, 305-312)
        t_scale, t_factor = (temporal[0], temporal[1]) if temporal is not None else (None, 0.0)
        G = M if (GROUP_ROWS and ATTN_SHARE_Q and train and M > 1 and temporal is None
                  and self.attn_block(D, H, M) and self.mlp_fused(D, hid)) else 0
        w.group_rows = G
        if split:
            # the two collections at their own widths (architecture.py:153-190, 305-312): the MF
            # run writes mf_pred (and the LN'd GMF rows for the backward), its MLP-side outputs
            # are scratch; the MLP run writes X_u / X_i, its GMF (a zero weight) is scratch
            Dm, sp = m.mf_embedding_dim, w.split
            mfu, mfi, mlu, mli = tbp
            _lib.call("ncf_gather_ln_gmf_scaled_fwd", ptr(uid), ptr(iid), n, mfu, mfi, mfu, mfi,
                      n_users, n_items, Dm, pp["mf_norm.weight"], pp["mf_norm.bias"],
                      pp["mf_norm.weight"], pp["mf_norm.bias"], pp["mf_output.weight"],
                      pp["mf_output.bias"], LN_EPS, None, 0.0, 0, ptr(w.mf_pred),
                      ptr(sp["rows_m"][0]), ptr(sp["rows_m"][1]), ptr(w.umf), ptr(w.imf),
                      ptr(w.err), st)
            _lib.call("ncf_gather_ln_gmf_scaled_fwd", ptr(uid), ptr(iid), n, mlu, mli, mlu, mli,
                      n_users, n_items, D, pp["mlp_norm.weight"], pp["mlp_norm.bias"],
                      pp["mlp_norm.weight"], pp["mlp_norm.bias"], ptr(sp["zero_w"]),
                      pp["mf_output.bias"], LN_EPS, None, 0.0, 0, ptr(sp["pred"]), ptr(w.xu),
                      ptr(w.xi), None, None, ptr(w.err), st)
        elif table_ld is not None and table_ld != D:
            if bf16 or temporal is not None:
                raise ValueError("table_ld: fp32 tables, no temporal scaling")
            _lib.call("ncf_gather_ln_gmf_ld_fwd", ptr(uid), ptr(iid), n, *tbp, n_users, n_items, D,
                      int(table_ld), pp["mf_norm.weight"], pp["mf_norm.bias"],
                      pp["mlp_norm.weight"], pp["mlp_norm.bias"], pp["mf_output.weight"],
                      pp["mf_output.bias"], LN_EPS, G, ptr(w.mf_pred), ptr(w.xu), ptr(w.xi),
                      ptr(w.umf), ptr(w.imf), ptr(w.err), st)
        elif bf16:    # bf16 tables (``tables`` holds them): rows widened to fp32 in the gather
            if temporal is not None:
                raise ValueError("the bf16-table configuration is a training configuration")
            _lib.call("ncf_gather_ln_gmf_bf16_fwd", ptr(uid), ptr(iid), n, *tbp, n_users,
                      n_items, D, pp["mf_norm.weight"], pp["mf_norm.bias"],
                      pp["mlp_norm.weight"], pp["mlp_norm.bias"], pp["mf_output.weight"],
                      pp["mf_output.bias"], LN_EPS, G, ptr(w.mf_pred), ptr(w.xu), ptr(w.xi),
                      ptr(w.umf), ptr(w.imf), ptr(w.err), st)
        else:
            _lib.call("ncf_gather_ln_gmf_scaled_fwd", ptr(uid), ptr(iid), n, *tbp, n_users,
                      n_items, D, pp["mf_norm.weight"], pp["mf_norm.bias"],
                      pp["mlp_norm.weight"], pp["mlp_norm.bias"], pp["mf_output.weight"],
                      pp["mf_output.bias"], LN_EPS, ptr(t_scale), float(t_factor), G,
                      ptr(w.mf_pred), ptr(w.xu), ptr(w.xi), ptr(w.umf), ptr(w.imf), ptr(w.err), st)
        # a5: MultiHeadAttention over each group of M rows (architecture.py:315-326)
        att = m.user_product_attention
        if train and temporal is None and self.attn_tower_step(D, H, M, hid):
            # a5 + a7 + a8 in one launch (tower_fused.hip): the attention block, then the tower
            # and head on its output tile in LDS
            self._sweep_fork("tower")
            _, addr, _, haddr = self._mlp_layers(w, train, bwd=False)
            mode = {"ncf_mlp_fwd": 0, "ncf_mlp_fwd_bf16": 1,
                    "ncf_mlp_fwd_split": 3}[self._tower_entry("ncf_mlp_fwd", bf16)]
            a_ = "user_product_attention."
            _lib.call("ncf_attn_mlp_fwd" + self._tiles(n // M), ptr(w.xu), ptr(w.xi), n // M, H,
                      pp[a_ + "q_proj.weight"], pp[a_ + "q_proj.bias"], pp[a_ + "k_proj.weight"],
                      pp[a_ + "k_proj.bias"], pp[a_ + "v_proj.weight"], pp[a_ + "v_proj.bias"],
                      pp[a_ + "out_proj.weight"], pp[a_ + "out_proj.bias"], drop_p, seed,
                      ptr(self.clock), ptr(w.q), ptr(w.k), ptr(w.v), ptr(w.P), ptr(w.y),
                      ptr(uid) if ATTN_SHARE_Q else None, addr, len(hid), haddr, LN_EPS,
                      pp["mlp_output.weight"], pp["mlp_output.bias"], ptr(w.mf_pred),
                      pp["final.0.weight"], pp["final.0.bias"], ptr(w.mlp_pred), ptr(w.prob),
                      mode, st)
            return w
        if temporal is None and self.attn_block(D, H, M):
            # projections + core + out_proj in one launch (attn_block.hip)
            # training: nothing stashed when the backward recomputes q/k/v/P/o (attn_rc)
            core = (train or M != 1) and not (train and self.attn_rc(D, H, M))
            a_ = "user_product_attention."
            _lib.call("ncf_attn_block_fwd", ptr(w.xu), ptr(w.xi), n // M, M, H, D,
                      pp[a_ + "q_proj.weight"], pp[a_ + "q_proj.bias"], pp[a_ + "k_proj.weight"],
                      pp[a_ + "k_proj.bias"], pp[a_ + "v_proj.weight"], pp[a_ + "v_proj.bias"],
                      pp[a_ + "out_proj.weight"], pp[a_ + "out_proj.bias"],
                      drop_p if train else 0.0, seed, ptr(self.clock),
                      ptr(w.q) if core else None, ptr(w.k) if core else None,
                      ptr(w.v) if core else None, ptr(w.P) if core else None,
                      ptr(w.o) if core and _STASH_O else None, ptr(w.y),
                      ptr(uid) if ATTN_SHARE_Q else None, st)
            # a7: MLP tower on [attn ‖ zeros_T] (architecture.py:329-344): the zero temporal
            # columns contribute nothing, so layer 0 reads only the first D columns of mlp.0.weight
            x, ldx, kin = w.y, D, D
        else:
            x, ldx, kin = self._attention_unfused(w, M, train, drop_p, seed, temporal, st)
        if train:
            self._sweep_fork("tower")
        if temporal is None and self.mlp_fused(D, hid):
            # a7 + a8: the whole tower and the head in one launch (mlp_tower.hip)
            _, addr, _, haddr = self._mlp_layers(w, train, bwd=False)
            _lib.call(self._tower_entry("ncf_mlp_fwd", bf16), ptr(x), n, D, addr,
                      len(hid),
                      haddr, LN_EPS, drop_p if train else 0.0, seed, ptr(self.clock),
                      pp["mlp_output.weight"],
                      pp["mlp_output.bias"], ptr(w.mf_pred), pp["final.0.weight"],
                      pp["final.0.bias"], ptr(w.mlp_pred), ptr(w.prob), st)
            return w
        for l, h in enumerate(hid):
            lin, ln = m.mlp[4 * l], m.mlp[4 * l + 2]
            ldw = lin.weight.shape[1]
            self._gemm(x, ldx, 0, lin.weight, ldw, 1, w.r[l], h, n, h, kin, bias=lin.bias,
                       relu=True, st=st)
            # (forward_simple(hour) in training mode passes its dropout here with train=False)
            _lib.call("ncf_relu_ln_dropout_fwd", ptr(w.r[l]), n, h, ptr(ln.weight), ptr(ln.bias),
                      LN_EPS, drop_p if train or temporal is not None else 0.0,
                      (seed + 0x9E37 * (l + 1)) & (2 ** 63 - 1),
                      ptr(self.clock), ptr(w.a[l]), ptr(w.mean[l]), ptr(w.rstd[l]), st)
            x, ldx, kin = w.a[l], h, h
        # a8: mlp_output + final Linear(2,1) + Sigmoid (architecture.py:345, 353-354)
        _lib.call("ncf_head_fwd", ptr(x), n, hid[-1], ptr(m.mlp_output.weight),
                  ptr(m.mlp_output.bias), ptr(w.mf_pred), ptr(m.final[0].weight),
                  ptr(m.final[0].bias), ptr(w.mlp_pred), ptr(w.prob), st)
        return w

    def mlp_fused(self, D: int, hid) -> bool:
        """Whether the one-launch MLP tower (mlp_tower.hip) covers this geometry;
        MLP_FUSED = False forces the per-layer launches (A/B measurement, parity tests)."""
        if not self._env_mlp_fused:
            return False
        if self.model.mf_embedding_dim != self.model.mlp_embedding_dim:
            return False        # (its head backward reads the GMF rows at the tower's width)
        key = (D, tuple(hid))
        ok = self._mlp_ok.get(key)
        if ok is None:
            h = (ctypes.c_int64 * len(hid))(*hid)
            ok = self._mlp_ok[key] = bool(_lib.query("ncf_mlp_fused_supported", D, len(hid),
                                                     ctypes.addressof(h)))
        return ok

    def mlp_fused_wgrad(self) -> bool:
        """The tower backward also computes the three MLP weight gradients (per-workgroup
        partials); MLP_WGRAD = False leaves them to the grouped weight-gradient launch."""
        return self._env_mlp_wgrad

    def _mlp_layers(self, w, train: bool, bwd: bool):
        """ncf_mlp_layer[] for the fused tower (cached per workspace: the parameter and buffer
        addresses are fixed for its lifetime)."""
        fw = self.mlp_fused_wgrad()
        key = ("mlp", train, bwd, fw)
        c = w.cache.get(key)
        if c is None:
            m = self.model
            hid = list(m.mlp_hidden_dims)
            arr = (_lib.MlpLayer * len(hid))()
            for l, L in enumerate(arr):
                lin, ln = m.mlp[4 * l], m.mlp[4 * l + 2]
                L.w, L.ldw, L.b = ptr(lin.weight), lin.weight.shape[1], ptr(lin.bias)
                L.gamma, L.beta = ptr(ln.weight), ptr(ln.bias)
                if train:
                    # with the weight gradients fused into the tower backward, that kernel
                    # recomputes the activations a from r: the forward does not store them
                    L.r, L.mean, L.rstd = ptr(w.r[l]), ptr(w.mean[l]), ptr(w.rstd[l])
                    L.a = None if fw else ptr(w.a[l])
                if bwd:
                    gv = self.grad_view
                    L.dbias = ptr(gv(f"mlp.{4 * l}.bias"))
                    L.dgamma, L.dbeta = ptr(gv(f"mlp.{4 * l + 2}.weight")), ptr(gv(f"mlp.{4 * l + 2}.bias"))
                    if fw:   # dlin stays in LDS (consumed by the fused weight gradients)
                        L.dw = ptr(gv(f"mlp.{4 * l}.weight"))
                    else:
                        L.dlin = ptr(w.dlin[l])
            harr = (ctypes.c_int64 * len(hid))(*hid)
            c = w.cache[key] = (arr, ctypes.addressof(arr), harr, ctypes.addressof(harr))
        return c

    def attn_block(self, D: int, H: int, M: int) -> bool:
        """Whether the one-launch attention block (attn_block.hip) covers this geometry;
        ATTN_BLOCK = False forces the unfused launches (A/B measurement, parity tests)."""
        if not self._env_attn_block:
            return False
        key = ("attn", D, H, M)
        ok = self._mlp_ok.get(key)
        if ok is None:
            ok = self._mlp_ok[key] = bool(_lib.query("ncf_attn_block_supported", D, H, M))
        return ok

    def attn_mlp_fused(self, D: int, H: int, M: int, hid) -> bool:
        """Whether the one-launch attention block + tower forward (tower_fused.hip) covers this
        geometry (D = 64, M = 5, [256, 128, 64]) and is switched on (FUSE_ATTN_TOWER)."""
        if not FUSE_ATTN_TOWER:
            return False
        key = ("attn_mlp", D, H, M, tuple(hid))
        ok = self._mlp_ok.get(key)
        if ok is None:
            harr = (ctypes.c_int64 * len(hid))(*hid)
            ok = self._mlp_ok[key] = bool(_lib.query("ncf_attn_mlp_fused_supported", D, H, M,
                                                      len(hid), ctypes.addressof(harr)))
        return ok

    @staticmethod
    def _tiles(groups: int) -> str:
        """The fused attention + tower entry points' suffix for a batch of `groups` groups:
        the small-batch tiles below SMALL_TILE_GROUPS."""
        return "_small" if groups < SMALL_TILE_GROUPS else ""

    def attn_tower_step(self, D: int, H: int, M: int, hid) -> bool:
        """Whether a training step of this geometry runs the attention block and the tower as
        one launch per direction (tower_fused.hip): the fused attention block with its stash,
        the fused tower with its weight gradients, and the fused kernels' geometry."""
        return (self.attn_block(D, H, M) and self.mlp_fused(D, hid) and self.mlp_fused_wgrad()
                and not self.attn_rc(D, H, M) and not _STASH_O
                and self.attn_mlp_fused(D, H, M, hid))

    @staticmethod
    def _tower_entry(base: str, bf16: bool) -> str:
        """The fused tower's entry point: bf16 tables -> single-term bf16 MFMA (BF16_MM); fp32
        -> split-operand bf16 MFMA (TOWER_SPLIT) or the fp32 MFMA."""
        if bf16 and BF16_MM:
            return base + "_bf16"
        return base + "_split" if (TOWER_SPLIT and not bf16) else base

    def attn_rc(self, D: int, H: int, M: int) -> bool:
        """Whether the training forward of the attention block stashes nothing and its backward
        recomputes q/k/v, the probabilities and o from the LN'd rows (ncf_attn_block_bwd_rc:
        27.9 MB less HBM traffic per C2 step).  Off by default (ATTN_RC):
        measured at C2 the forward gains 3 us and the backward loses 6-7 us (its serial
        re-projection + core prologue costs more than reading the stash back)."""
        if not self._env_attn_rc:
            return False
        key = ("attn_rc", D, H, M)
        ok = self._mlp_ok.get(key)
        if ok is None:
            ok = self._mlp_ok[key] = bool(_lib.query("ncf_attn_block_rc_supported", D, H, M))
        return ok

    def _attention_unfused(self, w, M, train, drop_p, seed, temporal, st):
        """a5 as separate launches (q/k/v projections, core, out_proj): any D, M <= 64, and the
        forward_simple(hour) MLP input [attn ‖ hour_E]."""
        m = self.model
        dev = w.xu.device
        n = w.g.n
        D, H = w.g.D, w.g.H
        att = m.user_product_attention
        if M == 1 and not train:
            # softmax over a single key is exactly 1 -> the core returns V unchanged
            self._gemm(w.xi, D, 0, att.v_proj.weight, D, 1, w.v, D, n, D, D, bias=att.v_proj.bias, st=st)
            src = w.v
            if temporal is not None and drop_p > 0:
                # forward_simple(hour) in training mode: the attention's nn.Dropout on that
                # weight of 1 (architecture.py:51): kept (x 1/(1-p)) or dropped per (row, head)
                _lib.call("ncf_dropout_rows", ptr(w.v), n, D, D // H, drop_p, seed, ptr(w.v),
                          None, st)
        else:
            side = self.fork(dev, 2)
            for sd, (X, lin, Y) in zip(side, ((w.xu, att.q_proj, w.q), (w.xi, att.k_proj, w.k))):
                with torch.cuda.stream(sd):
                    self._gemm(X, D, 0, lin.weight, D, 1, Y, D, n, D, D, bias=lin.bias,
                               st=_lib.stream_ptr(dev))
            self._gemm(w.xi, D, 0, att.v_proj.weight, D, 1, w.v, D, n, D, D, bias=att.v_proj.bias,
                       st=st)
            self.join(dev, side)
            _lib.call("ncf_attention_fwd", ptr(w.q), ptr(w.k), ptr(w.v), n // M, M, H, D,
                      drop_p if train else 0.0, seed, ptr(self.clock), ptr(w.P), ptr(w.o), st)
            src = w.o
        if temporal is None:
            self._gemm(src, D, 0, att.out_proj.weight, D, 1, w.y, D, n, D, D,
                       bias=att.out_proj.bias, st=st)
            # a7: MLP tower on [attn ‖ zeros_T] (architecture.py:329-344): the zero temporal
            # columns contribute nothing, so layer 0 reads only the first D columns of mlp.0.weight
            x, ldx, kin = w.y, D, D
        else:
            # forward_simple(hour): MLP input [attn ‖ hour_E[h]] (architecture.py:467-468)
            te = temporal[2]
            Tt = te.shape[1]
            yt = torch.empty(n, D + Tt, device=dev)
            self._gemm(src, D, 0, att.out_proj.weight, D, 1, yt, D + Tt, n, D, D,
                       bias=att.out_proj.bias, st=st)
            yt[:, D:].copy_(te)
            x, ldx, kin = yt, D + Tt, D + Tt
        return x, ldx, kin

    def check_ids(self, w: Optional[Workspace] = None):
        """Raise IndexError if any forward of this engine since the last check saw an
        out-of-range id (the engine-wide flag is sticky between checks; one host sync)."""
        f = getattr(self, "_err", None)
        if f is None:
            return
        if int(f.item()):
            f.zero_()
            raise IndexError("AdvancedNCF: user/product id out of range of the embedding tables")

    ID_CHECK_EVERY = 16

    def check_ids_async(self, w: Workspace):
        """Training-mode id validation without a host sync.  Every ID_CHECK_EVERY-th call
        copies the sticky error flag of w to pinned host memory behind an event; a later call
        whose event has completed reads it and raises IndexError.  An out-of-range id never
        touches memory out of bounds (the kernels read / update row 0 instead and raise the
        flag), so the error surfaces at most a few steps after the faulty batch ran on the
        GPU; ``check_ids`` (eval, and ``model.validate_ids = "sync"``) is immediate."""
        f = w.err
        a = getattr(self, "_err_async", None)
        if a is None:
            a = self._err_async = {"host": torch.zeros(1, dtype=torch.int32, pin_memory=True),
                                   "ev": torch.cuda.Event(), "pending": False, "k": 0}
        if a["pending"]:
            if not a["ev"].query():
                return
            a["pending"] = False
            if int(a["host"][0]):
                f.zero_()
                raise IndexError("AdvancedNCF: user/product id out of range of the embedding "
                                 "tables (seen by a training step in flight)")
        a["k"] += 1
        if a["k"] % self.ID_CHECK_EVERY:
            return
        a["host"].copy_(f, non_blocking=True)
        a["ev"].record()
        a["pending"] = True

    # ------------------------------------------------------------------ backward
    def _sweep_fork(self, at: str, w=None):
        """Launch the previous step's owed rolling sweep on its side stream when the overlapped
        sweep is on and `at` is one of its fork points (DeferredTableAdam.fork_points)."""
        d = self.deferred
        if d is not None and d.overlap:
            d.sweep_fork(at)
        hook = self.fork_hook
        if hook is not None:
            hook(at)

    def _zero_temporal_cols(self, m, hid, D, st):
        """Gradient columns of mlp.0 that see the all-zero temporal input: exactly 0, and no
        kernel ever writes them — zeroed once per gradient buffer."""
        if self._zero_cols_of is self.flat_grad:
            return
        ldw = m.mlp[0].weight.shape[1]
        if ldw > D:
            _lib.call("ncf_fill_2d", ptr(self.grad_view("mlp.0.weight")[:, D:]), hid[0], ldw - D,
                      ldw, 0.0, st)
        self._zero_cols_of = self.flat_grad

    def _attn_grad_ptrs(self, w):
        """Address of the 8 attention parameter-gradient pointers (q/k/v/out weight, bias)."""
        gp = w.cache.get("attn_grads")
        if gp is None:
            names = [f"user_product_attention.{nm}.{t}" for nm in ("q_proj", "k_proj", "v_proj",
                                                                    "out_proj")
                     for t in ("weight", "bias")]
            arr = (ctypes.c_void_p * 8)(*[ptr(self.grad_view(x)) for x in names])
            gp = w.cache["attn_grads"] = (arr, ctypes.addressof(arr))
        return gp[1]

    def backward(self, w: Workspace, uid, iid, grad_prob: Optional[torch.Tensor],
                 targets: Optional[torch.Tensor], drop_p: float, seed: int,
                 loss_denominator: float = 0.0, tables=None, rows=None, uniq=None,
                 reduce_async: bool = False, bf16: bool = False, grad_rows=None,
                 table_ld: Optional[int] = None, reduce_side=None, fused_apply=None,
                 tables_done=None):
        """Gradients of every used parameter.  Dense grads land in the flat grad buffer; table
        grads stay compact (self.pending) for the fused Adam step.  ``reduce_async``: the
        deferred reductions (every dense gradient) run on a side stream, beside whatever the
        caller queues next that does not read them (the table Adam); the caller must call
        ``join_reductions()`` before reading the dense gradients.  ``reduce_side`` (a stream
        whose queued work the step joins before its dense Adam): the tower and attention
        reductions run there right after the fused tower/attention backward, beside the
        embedding backward and the table Adam (join_reductions orders them).  ``fused_apply``
        (DeferredTableAdam.fused_apply_args): the table Adam's apply of this step runs inside the
        embedding backward (ncf_embedding_bwd_reduce_apply_clock; w.applied tells the deferred
        schedule).  ``tables_done()`` is called right after the embedding backward is queued
        (before the dense-gradient reductions).  ``grad_rows = (buf, rows_u,
        rows_i)``: the table gradients of unique row c go to row rows_*[c] of buf ([mf | mlp]
        halves, 2 D floats per row: the row-sharded step's send buffer) instead of w.G."""
        m = self.model
        g = w.g
        n, D, H, M, hid = g.n, g.D, g.H, g.M, g.hidden
        dev = w.prob.device
        st = _lib.stream_ptr(dev)
        uid = uid.to(device=dev, dtype=torch.int64).contiguous()
        iid = iid.to(device=dev, dtype=torch.int64).contiguous()
        gv = self.grad_view
        w.red_list.count = 0
        w.wgrads = []
        joins = []   # side streams to join before the deferred reductions
        # a12 + a8 backward (trainer.py:271; architecture.py:245-252)
        gp = None if grad_prob is None else grad_prob.reshape(-1).to(torch.float32).contiguous()
        tg = None if targets is None else targets.reshape(-1).to(device=dev, dtype=torch.float32).contiguous()
        fused = self.mlp_fused(D, hid)
        if not fused:
            _lib.call("ncf_head_bwd", ptr(w.prob), ptr(gp), ptr(tg), ptr(w.mf_pred), ptr(w.mlp_pred),
                      ptr(w.a[-1]), n, hid[-1], ptr(m.mlp_output.weight), ptr(m.final[0].weight),
                      ptr(w.umf), ptr(w.imf), g.Dm or D, ptr(m.mf_output.weight), ptr(w.da[-1]), ptr(w.dumf),
                      ptr(w.dimf), ptr(gv("mlp_output.weight")), ptr(gv("mlp_output.bias")),
                      ptr(gv("mf_output.weight")), ptr(gv("mf_output.bias")),
                      ptr(gv("final.0.weight")), ptr(gv("final.0.bias")), ptr(w.loss),
                      float(loss_denominator), ptr(w.site("head")), w.site("head").numel(),
                      w.red_list.address, st)
        # a7 backward, last layer first
        self._sweep_fork("mlp_bwd", w)
        if fused:   # head + relu/LN/dropout backward + dX of all layers in one launch
            _, addr, _, haddr = self._mlp_layers(w, True, bwd=True)
            h = w.cache.get("head_args")
            if h is None:
                h = w.cache["head_args"] = _lib.HeadArgs()
                h.mf_pred, h.mlp_pred, h.mf_user_ln, h.mf_item_ln = (
                    ptr(w.mf_pred), ptr(w.mlp_pred), ptr(w.umf), ptr(w.imf))
                h.mlp_out_w, h.final_w, h.mf_out_w = (
                    ptr(m.mlp_output.weight), ptr(m.final[0].weight), ptr(m.mf_output.weight))
                h.grad_mf_user_ln, h.grad_mf_item_ln = ptr(w.dumf), ptr(w.dimf)
                h.grad_mlp_out_w, h.grad_mlp_out_b = ptr(gv("mlp_output.weight")), ptr(gv("mlp_output.bias"))
                h.grad_mf_out_w, h.grad_mf_out_b = ptr(gv("mf_output.weight")), ptr(gv("mf_output.bias"))
                h.grad_final_w, h.grad_final_b = ptr(gv("final.0.weight")), ptr(gv("final.0.bias"))
            h.prob, h.grad_prob, h.targets, h.loss = ptr(w.prob), ptr(gp), ptr(tg), ptr(w.loss)
            h.loss_denominator = float(loss_denominator)
            # (the gather's source rows of the LN'd user rows: ncf_head_args.user_ids)
            h.user_ids, h.group_rows = ptr(uid), getattr(w, "group_rows", 0)
        fused_all = fused and self.mlp_fused_wgrad()
        pp = self.pp()
        fused_ta = fused_all and self.attn_tower_step(D, H, M, hid)
        if fused_ta:
            # tower + head backward, then the attention backward on the tower's input gradient
            # in LDS, in one launch (tower_fused.hip); the forward's stash q/k/v/P either way
            self._zero_temporal_cols(m, hid, D, st)
            mode = {"ncf_mlp_bwd": 0, "ncf_mlp_bwd_bf16": 1,
                    "ncf_mlp_bwd_split": 3}[self._tower_entry("ncf_mlp_bwd", bf16)]
            gpa = self._attn_grad_ptrs(w)
            ws = w.site("attn")
            _lib.call("ncf_attn_mlp_bwd" + self._tiles(n // M), n // M, H, ptr(w.y), addr, len(hid),
                      haddr, drop_p,
                      seed, ptr(self.clock), ctypes.addressof(h), ptr(w.site("mlp")),
                      w.site("mlp").numel(), ptr(w.q), ptr(w.k), ptr(w.v), ptr(w.P),
                      *pp["att_w"], ptr(w.xu), ptr(w.xi), gpa, ptr(ws), ws.numel(),
                      ptr(w.dxu), ptr(w.dxi), ptr(uid) if ATTN_SHARE_Q else None,
                      w.red_list.address, mode, st)
            self._sweep_fork("mlp_bwd_after")
            self._sweep_fork("attn_bwd", w)
        elif fused:
            _lib.call(self._tower_entry("ncf_mlp_bwd", bf16), None, n, D,
                      ptr(w.y), addr,
                      len(hid), haddr, drop_p, seed,
                      ptr(self.clock), ctypes.addressof(h), ptr(w.dy), ptr(w.site("mlp")),
                      w.site("mlp").numel(), w.red_list.address, st)
            self._sweep_fork("mlp_bwd_after")     # (a fork point right behind the tower backward)
        elif fused_all:
            self._zero_temporal_cols(m, hid, D, st)
        for l in (() if fused_all else reversed(range(len(hid)))):
            h = hid[l]
            lin, ln = m.mlp[4 * l], m.mlp[4 * l + 2]
            if not fused:
                _lib.call("ncf_relu_ln_dropout_bwd", ptr(w.da[l]), ptr(w.r[l]), ptr(w.mean[l]),
                          ptr(w.rstd[l]), ptr(ln.weight), n, h, drop_p,
                          (seed + 0x9E37 * (l + 1)) & (2 ** 63 - 1), ptr(self.clock),
                          ptr(w.dlin[l]), ptr(gv(f"mlp.{4 * l + 2}.weight")),
                          ptr(gv(f"mlp.{4 * l + 2}.bias")), ptr(gv(f"mlp.{4 * l}.bias")),
                          ptr(w.site(f"relu{l}")), w.site(f"relu{l}").numel(),
                          w.red_list.address, st)
            xin, kin = (w.y, D) if l == 0 else (w.a[l - 1], hid[l - 1])
            ldw = lin.weight.shape[1]
            dW = gv(f"mlp.{4 * l}.weight")
            if not (fused and self.mlp_fused_wgrad()):
                self._wgrad(w, w.dlin[l], h, xin, kin, dW, ldw, h, kin, n)
            if ldw > kin and self._zero_cols_of is not self.flat_grad:
                # gradient columns of mlp.0 that see the all-zero temporal input: exactly 0, and
                # no kernel ever writes them — zero once per gradient buffer
                _lib.call("ncf_fill_2d", ptr(dW[:, kin:]), h, ldw - kin, ldw, 0.0, st)
                self._zero_cols_of = self.flat_grad
            if l == 0:   # every MLP weight gradient is ready: one grouped launch on a side stream
                joins.extend(self.fork(dev, 1))
                with torch.cuda.stream(joins[-1]):
                    w.run_wgrads(_lib.stream_ptr(dev), slot=0)
            if not fused:
                dx = w.dy if l == 0 else w.da[l - 1]
                self._gemm(w.dlin[l], h, 0, lin.weight, ldw, 0, dx, kin, n, kin, h, st=st)
        # a5 backward: out_proj, core, q/k/v projections
        if fused_ta:
            pass     # (in the fused launch above)
        elif self.attn_block(D, H, M):
            self._sweep_fork("attn_bwd", w)
            # core + projections backward and the four Linear gradients in one launch
            gpa = self._attn_grad_ptrs(w)
            ws = w.site("attn")
            if self.attn_rc(D, H, M):
                wq, wk, wv, wo = pp["att_w"]
                bq, bk, bv = pp["att_b"]
                _lib.call("ncf_attn_block_bwd_rc", ptr(w.dy), ptr(w.xu), ptr(w.xi), n // M, M, H, D,
                          wq, bq, wk, bk, wv, bv, wo, drop_p, seed, ptr(self.clock), gpa,
                          ptr(ws), ws.numel(), w.red_list.address, ptr(w.dxu), ptr(w.dxi),
                          ptr(uid) if ATTN_SHARE_Q else None, st)
            else:
                _lib.call("ncf_attn_block_bwd", ptr(w.dy), ptr(w.q), ptr(w.k), ptr(w.v), ptr(w.P),
                          n // M, M, H, D, *pp["att_w"], drop_p, seed,
                          ptr(self.clock), ptr(w.o) if _STASH_O else None, ptr(w.xu), ptr(w.xi),
                          gpa, ptr(ws),
                          ws.numel(), w.red_list.address, None, None, None, ptr(w.dxu),
                          ptr(w.dxi), ptr(uid) if ATTN_SHARE_Q else None, st)
        else:
            self._sweep_fork("attn_bwd", w)
            self._attention_bwd_unfused(w, drop_p, seed, joins, st)
        if reduce_side is not None and fused_ta and not reduce_async:
            # the dense-gradient reductions of the fused backward on the side stream now, beside
            # the embedding backward and the table Adam (its own scratch; joined before the
            # flat Adam by join_reductions)
            ev = getattr(self, "_early_red_ev", None)
            if ev is None:
                ev = self._early_red_ev = (_lib.RawEvent(stream_only=True),
                                           _lib.RawEvent(stream_only=True))
            side = reduce_side.cuda_stream
            ev[0].record(st)
            ev[0].wait(side)
            w.run_reductions(side, scratch="red_scratch_side")
            ev[1].record(side)
            self._early_red_pending = True
        # a2/a3 backward: segment-reduce + mf_norm/mlp_norm backward (compact table grads)
        self._sweep_fork("emb_bwd", w)
        if tables is None:
            tbp = (pp["t_mf_user"], pp["t_mlp_user"], pp["t_mf_item"], pp["t_mlp_item"])
        else:
            tbp = tuple(_tptr(tables[k]) for k in ("mf_user", "mlp_user", "mf_item", "mlp_item"))
        G = w.G
        uq_u, uq_i = uniq if uniq is not None else (w.uniq_u, w.uniq_i)
        d_rows = rows or (m.num_users, m.num_products)
        w.slots_set = False
        ev = getattr(w, "dedup_ev", None)
        if ev is not None:   # the id sort forked beside the forward (deferred._prepare_claim)
            ev.wait(st)
            w.dedup_ev = w.dedup_refs = None
        if not getattr(w, "deduped", False):   # sort/deduplicate now (slot maps for the Adam)
            _lib.call("ncf_dedup_ids", ptr(uid), ptr(iid), n, D, m.num_users, m.num_products,
                      ptr(w.uniq_u), ptr(w.uniq_i), ptr(self.slot_u), ptr(self.slot_i),
                      ptr(w.num_unique), ptr(w.emb_ws), w.emb_ws.numel(), st)
            w.slots_set = True
        if table_ld is not None and table_ld != D and grad_rows is None:
            raise ValueError("table_ld: the backward takes it with grad_rows only")
        applied = False
        if w.split is not None:
            if grad_rows is not None or fused_apply is not None or bf16:
                raise ValueError("mf_embedding_dim != mlp_embedding_dim: the dense table schedule")
            self._embedding_bwd_split(w, uid, iid, tbp, d_rows, st)
        elif grad_rows is not None:
            if bf16:
                raise ValueError("grad_rows: fp32 tables only")
            gb, ru_, ri_ = grad_rows
            gmf, gml = ptr(gb), ptr(gb) + 4 * D
            _lib.call("ncf_embedding_bwd_reduce_rows", n, D, d_rows[0], d_rows[1],
                      ptr(w.dumf), ptr(w.dxu), ptr(w.dimf), ptr(w.dxi), *tbp,
                      pp["mf_norm.weight"], pp["mlp_norm.weight"], LN_EPS, gmf, gml, gmf, gml,
                      ptr(uq_u), ptr(uq_i), ptr(ru_), ptr(ri_), 2 * D, int(table_ld or D),
                      self.gptr("mf_norm.weight"), self.gptr("mf_norm.bias"),
                      self.gptr("mlp_norm.weight"), self.gptr("mlp_norm.bias"), ptr(w.emb_ws),
                      w.emb_ws.numel(), w.red_list.address, st)
        elif fused_apply is not None:
            pa, clk, tab, b1, b2, eps_a, wd = fused_apply
            _lib.call("ncf_embedding_bwd_reduce_apply_clock", n, D, d_rows[0], d_rows[1],
                      ptr(w.dumf), ptr(w.dxu), ptr(w.dimf), ptr(w.dxi),
                      pp["mf_norm.weight"], pp["mlp_norm.weight"], LN_EPS, ptr(G["mf_user"]),
                      ptr(G["mlp_user"]), ptr(G["mf_item"]), ptr(G["mlp_item"]), ptr(uq_u),
                      ptr(uq_i), self.gptr("mf_norm.weight"), self.gptr("mf_norm.bias"),
                      self.gptr("mlp_norm.weight"), self.gptr("mlp_norm.bias"), ptr(w.emb_ws),
                      w.emb_ws.numel(), w.red_list.address, pa, 1, clk, tab, b1, b2, eps_a, wd,
                      st)
            w.applied = applied = True
        else:
            _lib.call("ncf_embedding_bwd_reduce_bf16" if bf16 else "ncf_embedding_bwd_reduce", n,
                      D, d_rows[0], d_rows[1],
                      ptr(w.dumf), ptr(w.dxu), ptr(w.dimf), ptr(w.dxi), *tbp,
                      pp["mf_norm.weight"], pp["mlp_norm.weight"], LN_EPS, ptr(G["mf_user"]),
                      ptr(G["mlp_user"]), ptr(G["mf_item"]), ptr(G["mlp_item"]), ptr(uq_u),
                      ptr(uq_i), self.gptr("mf_norm.weight"), self.gptr("mf_norm.bias"),
                      self.gptr("mlp_norm.weight"), self.gptr("mlp_norm.bias"), ptr(w.emb_ws),
                      w.emb_ws.numel(), w.red_list.address, st)
        if tables_done is not None and applied:    # (only behind a queued table apply)
            tables_done()
        self.join(dev, joins)
        self._sweep_fork("reduce")
        if reduce_async:
            if getattr(self, "_red_side", None) is None:
                self._red_side = _lib.side_stream(dev)
                self._red_ev = (torch.cuda.Event(), torch.cuda.Event())
            side = self._red_side
            self._red_ev[0].record()
            side.wait_event(self._red_ev[0])
            with torch.cuda.stream(side):
                w.run_reductions(side.cuda_stream)
            self._red_ev[1].record(side)
            self._red_pending = True
        else:
            w.run_reductions(st)
        self.pending = w

    def _embedding_bwd_split(self, w, uid, iid, tbp, d_rows, st):
        """a2/a3 backward when the collections differ in width: the segment reduce + LayerNorm
        backward once per collection, each with its own dedup workspace (the segment layout is
        carved per width); each run's second table pair is scratch.  The inline dedup of the
        MLP run (above, with the slot maps) and the MF run's give the same unique-id order."""
        m = self.model
        n, D, Dm = w.g.n, w.g.D, w.g.Dm
        sp = w.split
        mfu, mlu, mfi, mli = tbp
        _lib.call("ncf_dedup_ids", ptr(uid), ptr(iid), n, Dm, m.num_users, m.num_products,
                  ptr(sp["uniq"][0]), ptr(sp["uniq"][1]), None, None, ptr(sp["num_unique"]),
                  ptr(w.emb_ws_m), w.emb_ws_m.numel(), st)
        G, sm, sl, ln = w.G, sp["rows_m"], sp["rows_l"], sp["ln"]
        _lib.call("ncf_embedding_bwd_reduce", n, Dm, d_rows[0], d_rows[1], ptr(w.dumf),
                  ptr(w.dumf), ptr(w.dimf), ptr(w.dimf), mfu, mfu, mfi, mfi,
                  self.pp()["mf_norm.weight"], self.pp()["mf_norm.weight"], LN_EPS,
                  ptr(G["mf_user"]), ptr(sm[0]), ptr(G["mf_item"]), ptr(sm[1]),
                  ptr(sp["uniq"][0]), ptr(sp["uniq"][1]), self.gptr("mf_norm.weight"),
                  self.gptr("mf_norm.bias"), ptr(ln[0]), ptr(ln[1]), ptr(w.emb_ws_m),
                  w.emb_ws_m.numel(), w.red_list.address, st)
        _lib.call("ncf_embedding_bwd_reduce", n, D, d_rows[0], d_rows[1], ptr(w.dxu), ptr(w.dxu),
                  ptr(w.dxi), ptr(w.dxi), mlu, mlu, mli, mli, self.pp()["mlp_norm.weight"],
                  self.pp()["mlp_norm.weight"], LN_EPS, ptr(sl[0]), ptr(G["mlp_user"]),
                  ptr(sl[1]), ptr(G["mlp_item"]), ptr(w.uniq_u), ptr(w.uniq_i), ptr(ln[2]),
                  ptr(ln[3]), self.gptr("mlp_norm.weight"), self.gptr("mlp_norm.bias"),
                  ptr(w.emb_ws), w.emb_ws.numel(), w.red_list.address, st)

    def join_reductions(self):
        """The current stream waits for the side-stream reductions of the last backward."""
        if getattr(self, "_red_pending", False):
            torch.cuda.current_stream(self.flat.device).wait_event(self._red_ev[1])
            self._red_pending = False
        if getattr(self, "_early_red_pending", False):
            self._early_red_ev[1].wait(_lib.stream_ptr(self.flat.device))
            self._early_red_pending = False

    def _attention_bwd_unfused(self, w, drop_p, seed, joins, st):
        """a5 backward as separate launches (any geometry the unfused forward takes)."""
        m = self.model
        g = w.g
        n, D, H, M = g.n, g.D, g.H, g.M
        dev = w.prob.device
        gv = self.grad_view
        att = m.user_product_attention
        src = w.o
        self._wgrad(w, w.dy, D, src, D, gv("user_product_attention.out_proj.weight"), D, D, D, n,
                    dbias=gv("user_product_attention.out_proj.bias"))
        self._gemm(w.dy, D, 0, att.out_proj.weight, D, 0, w.do, D, n, D, D, st=st)
        _lib.call("ncf_attention_bwd", ptr(w.q), ptr(w.k), ptr(w.v), ptr(w.P), ptr(w.do), n // M, M,
                  H, D, drop_p, seed, ptr(self.clock), ptr(w.dS), ptr(w.dq), ptr(w.dk), ptr(w.dv), st)
        for nm, dX, X in (("q_proj", w.dq, w.xu), ("k_proj", w.dk, w.xi), ("v_proj", w.dv, w.xi)):
            self._wgrad(w, dX, D, X, D, gv(f"user_product_attention.{nm}.weight"), D, D, D, n,
                        dbias=gv(f"user_product_attention.{nm}.bias"))
        # attention weight gradients and dxu on side streams, dxi on this one
        side = self.fork(dev, 2)
        with torch.cuda.stream(side[0]):
            w.run_wgrads(_lib.stream_ptr(dev), slot=1)
        with torch.cuda.stream(side[1]):
            self._gemm(w.dq, D, 0, att.q_proj.weight, D, 0, w.dxu, D, n, D, D,
                       st=_lib.stream_ptr(dev))
        self._gemm(w.dk, D, 0, att.k_proj.weight, D, 0, w.dxi, D, n, D, D, st=st)
        self._gemm(w.dv, D, 0, att.v_proj.weight, D, 0, w.dxi, D, n, D, D, accum=True, st=st)
        self.join(dev, side[1:])
        joins.append(side[0])

    # ------------------------------------------------------------------ optimizer
    def table_state_tensors(self):
        return self.table_params()

    def adam_tables(self, hp_for, state_for, step: float, st):
        """Dense-exact Adam over the four tables using the pending compact grads."""
        w = self.pending
        tb = self.table_params()
        for key, p in tb.items():
            D = p.shape[1]       # (the MF and MLP collections may differ in width)
            if w is None and p.grad is None:
                continue  # torch.optim.Adam skips parameters whose grad is None
            lr, b1, b2, eps, wd = hp_for(p)
            s = state_for(p)
            if w is None:
                # dense gradient present (materialised / user-provided): elementwise Adam
                g = p.grad.contiguous()
                _lib.call("ncf_adam_flat", ptr(p), ptr(g), ptr(s["exp_avg"]),
                          ptr(s["exp_avg_sq"]), p.numel(), lr, b1, b2, eps, wd, step, st)
                continue
            kind = 0 if key.endswith("user") else 1
            slot = self.slot_u if kind == 0 else self.slot_i
            ev = self.timing.get(key) if self.timing else None
            if ev:
                ev[0].record()
            _lib.call("ncf_adam_table", ptr(p), ptr(s["exp_avg"]), ptr(s["exp_avg_sq"]),
                      p.shape[0], D, ptr(slot), ptr(w.G[key]), lr, b1, b2, eps, wd, step, st)
            if ev:
                ev[1].record()
        self.release_pending(st)

    def reset_slots(self, w, st):
        """Clear the slot-map entries a backward's inline dedup set (rows of w)."""
        n = w.g.n
        _lib.call("ncf_slot_reset", ptr(w.uniq_u), ptr(w.num_unique), 0, ptr(self.slot_u), n, st)
        _lib.call("ncf_slot_reset", ptr(w.uniq_i), ptr(w.num_unique), 1, ptr(self.slot_i), n, st)
        w.slots_set = False

    def release_pending(self, st):
        w = self.pending
        if w is None:
            return
        self.reset_slots(w, st)
        self.pending = None

    def materialize_table_grads(self, accumulate: bool = False):
        """Write dense [rows, D] gradients into the tables' .grad (for optimizers other than
        the fused Adam, gradient accumulation, or inspection), then release the compact
        buffers.  ``accumulate``: add to an existing .grad instead of replacing it.  Tables
        with requires_grad=False get no gradient (as autograd gives them none)."""
        w = self.pending
        if w is None:
            return
        st = _lib.stream_ptr(w.prob.device)
        for key, p in self.table_params().items():
            if not p.requires_grad:
                continue
            D = p.shape[1]
            kind = 0 if key.endswith("user") else 1
            add = accumulate and p.grad is not None
            dst = torch.zeros_like(p) if (add or p.grad is None) else p.grad.zero_()
            _lib.call("ncf_scatter_compact_rows", ptr(dst), D,
                      ptr(w.uniq_u if kind == 0 else w.uniq_i), ptr(w.num_unique), kind,
                      ptr(w.G[key]), w.g.n, st)
            if add:
                p.grad.add_(dst)
            elif p.grad is None:
                p.grad = dst
        self.release_pending(st)

    def grad_views(self):
        """{name: view of the flat gradient buffer} of the dense parameters (cached per
        buffer: assigning them as .grad after each backward allocates nothing)."""
        c = getattr(self, "_grad_views", None)
        if c is None or c[0] is not self.flat_grad:
            c = self._grad_views = (self.flat_grad,
                                    [(p, self.grad_view(n)) for n, p in self.dense_params()])
        return c[1]
