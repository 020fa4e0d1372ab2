"""Row-sharded multi-GPU training step — one process per GPU, RCCL over xGMI.

Partitioning: every embedding table is row-sharded by ``owner(id) = id mod W``, local row
``id div W`` (each rank holds ``ceil(rows / W)`` rows of each of the four tables, their Adam
moments and deferred-Adam stamps).  Dense parameters are replicated.  Each rank trains on its own
batch of B groups (weak scaling); the W local batches form one global batch whose loss is the mean
over all W*N samples — a W-rank step equals the 1-rank step on the concatenated batch.

Per step and per id kind (users, items):
  1. dedup the local ids (radix sort), bucket the unique ids by owner          [kernels]
  2. all_to_all of per-owner counts (host splits), then of the ids             [RCCL]
  3. owners dedup what they received, bring those rows current (deferred
     dense-exact Adam catch-up) and gather the GMF+MLP rows                    [kernels]
  4. all_to_all of the rows back; requesters scatter them into mini tables     [RCCL, kernels]
  5. forward + backward on the mini tables with remapped ids (the 1-GPU kernels)
  6. all_to_all of the compact row gradients to the owners, who sum them in a
     fixed order (source rank, then sender order) and apply the step          [RCCL, kernels]
  7. one all_reduce of the flat dense-gradient buffer, replicated dense Adam   [RCCL, kernel]
The exchange protocol (``ShardExchange`` + ``ShardedTrainStep``) is device-agnostic; the ops
backend does the per-rank work: ``HipShardOps`` (this file, the product path) or, in the CPU
``gloo`` tests, a torch reference backend.
"""
import ctypes
import math
import random
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import ptr


class ShardExchange:
    """The collectives of the sharded step (torch.distributed: RCCL on GPU, gloo on CPU)."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device

    def exchange_counts_dev(self, counts: torch.Tensor):
        """Device counts [2 * W] (kind-major) -> (send, recv) host lists per kind, with ONE
        device-to-host copy for both (the only host sync of a step)."""
        W = self.world
        send = counts.view(2, W).t().contiguous()          # [W, 2]: per destination
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        both = torch.cat([send, recv]).cpu().tolist()
        s, r = both[:W], both[W:]
        return ([[s[d][0] for d in range(W)], [s[d][1] for d in range(W)]],
                [[r[x][0] for x in range(W)], [r[x][1] for x in range(W)]])

    def exchange_counts(self, counts: List[List[int]]) -> List[List[int]]:
        """counts[kind][dst] -> recv[kind][src] (one all_to_all of a [W, 2] int64 tensor)."""
        W = self.world
        send = torch.tensor([[counts[0][d], counts[1][d]] for d in range(W)], dtype=torch.int64,
                            device=self.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        r = recv.cpu().tolist()
        return [[r[s][0] for s in range(W)], [r[s][1] for s in range(W)]]

    def exchange(self, t: torch.Tensor, send_splits: List[int], recv_splits: List[int]):
        out = torch.empty((sum(recv_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t[:sum(send_splits)].contiguous(), recv_splits, send_splits,
                               group=self.group)
        return out

    def all_reduce_(self, t: torch.Tensor):
        dist.all_reduce(t, group=self.group)
        return t


@dataclass
class Plan:
    send: list          # per kind: unique ids in owner order
    perm: list          # per kind: send slot -> local compact index
    counts: Optional[list] = None   # per kind: per-owner counts (host ints)
    recv_counts: Optional[list] = None
    counts_dev: Optional[torch.Tensor] = None   # device counts (HIP backend: one sync later)


class ShardedTrainStep:
    """One data-parallel + row-sharded training step: the protocol above over an ops backend."""

    def __init__(self, ops, exchange: ShardExchange):
        self.ops, self.x = ops, exchange

    def __call__(self, user_ids, item_ids, targets):
        ops, X = self.ops, self.x
        n = user_ids.numel()
        ded = ops.dedup(user_ids, item_ids)
        plan = ops.bucket(ded, X.world)
        if plan.counts_dev is not None:
            plan.counts, plan.recv_counts = X.exchange_counts_dev(plan.counts_dev)
        else:
            plan.recv_counts = X.exchange_counts(plan.counts)
        recv = [X.exchange(plan.send[k], plan.counts[k], plan.recv_counts[k]) for k in (0, 1)]
        own = ops.owner_prepare(recv)
        rows = [ops.owner_gather(own, k, recv[k]) for k in (0, 1)]
        back = [X.exchange(rows[k], plan.recv_counts[k], plan.counts[k]) for k in (0, 1)]
        grads, loss = ops.compute(ded, plan, back, user_ids, item_ids, targets,
                                  loss_denominator=n * X.world)
        got = [X.exchange(grads[k], plan.counts[k], plan.recv_counts[k]) for k in (0, 1)]
        ops.owner_apply(own, got)
        X.all_reduce_(ops.dense_grad())
        ops.dense_step()
        return loss


class HipShardOps:
    """Per-rank work of the sharded step on the MI355X (HIP kernels through the C-ABI)."""

    def __init__(self, model, num_users: int, num_items: int, world: int, lr=1e-3,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, sweep_every=64):
        from .deferred import DeferredTableAdam
        self.model, self.U, self.I, self.W = model, num_users, num_items, world
        self.Ru, self.Ri = model.num_users, model.num_products      # shard rows
        if self.Ru < math.ceil(num_users / world) or self.Ri < math.ceil(num_items / world):
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
                                          clock=self.clock)
        self.m_flat = torch.zeros_like(self.eng.flat)
        self.v_flat = torch.zeros_like(self.eng.flat)
        self.step_count = 0
        self.rng = random.Random(self.base_seed)     # dropout seeds without a device sync
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.last_loss = None

    def _st(self):
        return _lib.stream_ptr(self.dev)

    def _ws(self, n):
        return torch.empty(_lib.query("ncf_embedding_bwd_workspace", max(n, 1), self.D),
                           dtype=torch.uint8, device=self.dev)

    # 1. local dedup + inverse map
    def dedup(self, uid, iid):
        n = uid.numel()
        w = self.eng.workspace(n, self.M, True)
        st = self._st()
        _lib.call("ncf_dedup_ids", ptr(uid), ptr(iid), n, self.D, self.U, self.I, ptr(w.uniq_u),
                  ptr(w.uniq_i), None, None, ptr(w.num_unique), ptr(w.emb_ws), w.emb_ws.numel(), st)
        inv_u = torch.empty(n, dtype=torch.int64, device=self.dev)
        inv_i = torch.empty(n, dtype=torch.int64, device=self.dev)
        _lib.call("ncf_dedup_inverse", n, n, self.U, self.I, self.D, ptr(inv_u), ptr(inv_i),
                  ptr(w.emb_ws), w.emb_ws.numel(), st)
        return {"w": w, "n": n, "inv": (inv_u, inv_i)}

    def bucket(self, ded, world):
        w, n = ded["w"], ded["n"]
        send = [torch.empty(max(n, 1), dtype=torch.int64, device=self.dev) for _ in range(2)]
        perm = [torch.empty(max(n, 1), dtype=torch.int32, device=self.dev) for _ in range(2)]
        counts = torch.zeros(2 * world, dtype=torch.int64, device=self.dev)
        ws = self._ws(n)
        _lib.call("ncf_owner_bucket", ptr(w.uniq_u), ptr(w.uniq_i), ptr(w.num_unique), n, world,
                  ptr(send[0]), ptr(send[1]), ptr(perm[0]), ptr(perm[1]), ptr(counts), ptr(ws),
                  ws.numel(), self._st())
        return Plan(send=send, perm=perm, counts_dev=counts)      # split sizes fetched later

    # 3. owner side: dedup received ids (already local rows), catch their rows up
    def owner_prepare(self, recv):
        st = self._st()
        rn = [r.numel() for r in recv]
        nmax = max(rn)
        uq = [torch.empty(max(nmax, 1), dtype=torch.int64, device=self.dev) for _ in range(2)]
        cnt = torch.zeros(2, dtype=torch.int32, device=self.dev)
        ws = self._ws(nmax)
        _lib.call("ncf_dedup_ids2", ptr(recv[0]), rn[0], self.Ru, ptr(recv[1]), rn[1], self.Ri,
                  self.D, ptr(uq[0]), ptr(uq[1]), None, None, ptr(cnt), ptr(ws), ws.numel(), st)
        d = self.deferred
        if nmax > 0:
            d._ensure(d.t + 1)
            pairs = self._pairs(uq)
            _lib.call("ncf_adam_pairs_catchup_clock", ctypes.addressof(pairs), 2, self.D,
                      ptr(cnt), nmax, 0, ptr(self.clock), ptr(d._table), *d._consts(), st)
        return {"rn": rn, "uniq": uq, "cnt": cnt, "ws": ws}

    def _pairs(self, uq, G=None):
        pairs = self.deferred._pairs()
        for k in (0, 1):
            pairs[k].row_ids = ptr(uq[k])
            if G is not None:
                pairs[k].g0, pairs[k].g1 = ptr(G[2 * k]), ptr(G[2 * k + 1])
        return pairs

    def owner_gather(self, own, k, recv_ids):
        n = recv_ids.numel()
        out = torch.empty(max(n, 1), 2 * self.D, device=self.dev)
        tb = self.eng.table_params()
        t0, t1 = (tb["mf_user"], tb["mlp_user"]) if k == 0 else (tb["mf_item"], tb["mlp_item"])
        _lib.call("ncf_gather_shard_rows", ptr(recv_ids), n, 1, ptr(t0), ptr(t1),
                  self.Ru if k == 0 else self.Ri, self.D, ptr(out), ptr(self.err), self._st())
        return out[:n]

    # 5. forward + backward on the mini tables
    def compute(self, ded, plan, back, uid, iid, targets, loss_denominator):
        st = self._st()
        eng, w = self.eng, ded["w"]
        nu, ni = sum(plan.counts[0]), sum(plan.counts[1])
        mini = {k: torch.empty(max(c, 1), self.D, device=self.dev)
                for k, c in (("mf_user", nu), ("mlp_user", nu), ("mf_item", ni), ("mlp_item", ni))}
        _lib.call("ncf_perm_rows", ptr(back[0]), ptr(plan.perm[0]), nu, self.D,
                  ptr(mini["mf_user"]), ptr(mini["mlp_user"]), 0, st)
        _lib.call("ncf_perm_rows", ptr(back[1]), ptr(plan.perm[1]), ni, self.D,
                  ptr(mini["mf_item"]), ptr(mini["mlp_item"]), 0, st)
        m = self.model
        drop_p = float(m.dropout)
        seed = self.rng.getrandbits(62) if drop_p > 0 else 0
        inv_u, inv_i = ded["inv"]

        def mark(wk, u, i, s):
            wk.deduped = True
        eng.forward(inv_u, inv_i, self.M, True, drop_p, seed, prepare=mark, tables=mini,
                    rows=(max(nu, 1), max(ni, 1)))
        ar_u = torch.arange(max(nu, 1), dtype=torch.int64, device=self.dev)
        ar_i = torch.arange(max(ni, 1), dtype=torch.int64, device=self.dev)
        eng.backward(w, inv_u, inv_i, None, targets, drop_p, seed,
                     loss_denominator=loss_denominator, tables=mini, rows=(self.U, self.I),
                     uniq=(ar_u, ar_i))
        eng.pending = None
        out = []
        for k, (a, b), c in ((0, ("mf_user", "mlp_user"), nu), (1, ("mf_item", "mlp_item"), ni)):
            g = torch.empty(max(c, 1), 2 * self.D, device=self.dev)
            _lib.call("ncf_perm_rows", ptr(g), ptr(plan.perm[k]), c, self.D, ptr(w.G[a]),
                      ptr(w.G[b]), 1, st)
            out.append(g[:c])
        self.last_loss = w.loss
        return out, w.loss

    # 6. owner side: sum received gradients per unique row, apply the step
    def owner_apply(self, own, got):
        st = self._st()
        rn, uq, cnt, ws = own["rn"], own["uniq"], own["cnt"], own["ws"]
        G = [torch.empty(max(rn[k], 1), self.D, device=self.dev) for k in (0, 0, 1, 1)]
        _lib.call("ncf_segment_sum_rows", rn[0], rn[1], self.Ru, self.Ri, self.D, ptr(got[0]),
                  ptr(got[1]), ptr(G[0]), ptr(G[1]), ptr(G[2]), ptr(G[3]), ptr(ws), ws.numel(), st)
        d = self.deferred
        nmax = max(rn)
        d._ensure(d.t + 1)
        if nmax > 0:
            pairs = self._pairs(uq, G)
            _lib.call("ncf_adam_pairs_apply_clock", ctypes.addressof(pairs), 2, self.D, ptr(cnt),
                      nmax, 1, ptr(self.clock), ptr(d._table), *d._consts(), st)
        d.advance(st)                               # rolling sweep of step t + 1 (clock)

    def dense_grad(self):
        return self.eng.flat_grad

    def dense_step(self):
        self.step_count += 1
        self.eng.updates += 1
        b1, b2 = self.betas
        st = self._st()
        _lib.call("ncf_adam_flat_clock", ptr(self.eng.flat), ptr(self.eng.flat_grad),
                  ptr(self.m_flat), ptr(self.v_flat), self.eng.flat.numel(),
                  ptr(self.deferred._table), 1, ptr(self.clock), b1, b2, self.eps, self.wd, st)
        _lib.call("ncf_step_clock_advance", ptr(self.clock), self.base_seed, st)


def shard_rows(rows: int, world: int) -> int:
    return (rows + world - 1) // world


def make_sharded_step(model_factory, num_users, num_items, group=None, **adam):
    """Build the local shard model (tables of ceil(rows / W) rows) and its sharded step.
    Dense parameters are broadcast from rank 0 so every replica starts identical."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    model = model_factory(shard_rows(num_users, world), shard_rows(num_items, world))
    dev = model.mf_norm.weight.device
    eng = model.engine
    eng.ensure_layout()
    dist.broadcast(eng.flat, src=0, group=group)
    ops = HipShardOps(model, num_users, num_items, world, **adam)
    return model, ShardedTrainStep(ops, ShardExchange(group, dev))
