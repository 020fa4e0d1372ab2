"""World-size-2 gloo test of the row-sharded data-parallel step on CPU.

It runs the product's exchange protocol (ncf_amd.distributed.ShardExchange + ShardedTrainStep:
count/id/row/gradient all-to-alls, global-mean loss scaling, dense all-reduce, owner-side
gradient sums) with a torch reference backend for the per-rank kernels (test infrastructure: the
HIP kernels need a GPU), and checks the SURVEY §8(e) parity criterion: a 2-rank step on a global
batch equals the 1-rank step on the concatenated batch (oracle, same init)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.parity import assert_params_close, zone_from_grads

U, I, D, T, H, HID, B, M = 97, 41, 16, 8, 2, [32, 16], 6, 5
TABLES = {"mf_user": "mf_embedding_collection.embedding_bags.user_id.weight",
          "mlp_user": "mlp_embedding_collection.embedding_bags.user_id.weight",
          "mf_item": "mf_embedding_collection.embedding_bags.product_id.weight",
          "mlp_item": "mlp_embedding_collection.embedding_bags.product_id.weight"}


def global_setup():
    import _ncf_pkg
    ncf = _ncf_pkg.load()
    torch.manual_seed(0)
    m = ncf.AdvancedNCF(U, I, 5, 24, D, D, T, HID, H, 0.0, M - 1)
    params = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    batches = []
    for _ in range(2):           # 2 steps x 2 ranks
        per_rank = []
        for _r in range(2):
            u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
            i = torch.randint(0, I, (B * M,), generator=g)
            t = torch.zeros(B, M)
            t[:, 0] = 1
            per_rank.append((u, i, t.reshape(-1, 1)))
        batches.append(per_rank)
    return params, batches


class TorchShardOps:
    """Reference backend (CPU, oracle math) implementing HipShardOps' interface."""

    def __init__(self, params, rank, world):
        from oracle import ncf_oracle as O
        self.O = O
        self.rank, self.W = rank, world
        self.names = O.used_param_names(list(params), len(HID))
        self.p = {k: v.clone() for k, v in params.items()}
        for key, name in TABLES.items():
            self.p[name] = params[name][rank::world].clone()      # rows with id % W == rank
        self.dense_names = [k for k in self.names if k not in TABLES.values()]
        self.opt = O.AdamState(lr=1e-3, weight_decay=1e-5)

    def mark_entry(self):
        pass

    def begin(self, plan):
        pass

    def plan(self, uid, iid, world):
        """Keys (id mod W) * R + id div W, deduplicated: compact order = owner order; the send
        buffer is destination-major (per destination: its user rows, then its item rows)."""
        from ncf_amd.distributed import Plan
        W = world
        uniq, inv, local, owner = [], [], [], []
        for ids, rows in ((uid, U), (iid, I)):
            R = -(-rows // W)
            keys = (ids % W) * R + ids // W
            uq, iv = torch.unique(keys, return_inverse=True)
            uniq.append(uq)
            inv.append(iv)
            owner.append(uq // R)
            local.append(uq % R)
        counts = [[int((owner[k] == d).sum()) for k in (0, 1)] for d in range(W)]
        send, spos = [], [torch.empty(len(uniq[0]), dtype=torch.long),
                          torch.empty(len(uniq[1]), dtype=torch.long)]
        off = 0
        for d in range(W):
            for k in (0, 1):
                sel = (owner[k] == d).nonzero().reshape(-1)
                spos[k][sel] = torch.arange(off, off + len(sel))
                send.append(local[k][sel])
                off += len(sel)
        return Plan(send=torch.cat(send), counts=counts,
                    extra={"inv": inv, "spos": spos, "n": uid.numel()})

    def owner_prepare(self, recv, plan):
        kind = torch.empty(len(recv), dtype=torch.long)
        src = torch.empty(len(recv), dtype=torch.long)
        off = 0
        for s_, (a, b) in enumerate(plan.recv_counts):
            kind[off:off + a], kind[off + a:off + a + b] = 0, 1
            src[off:off + a + b] = s_
            off += a + b
        return {"kind": kind, "src": src, "rows": recv.long()}

    def owner_gather(self, own, recv):
        out = torch.empty(len(recv), 2 * D)
        for k, (a, b) in enumerate(((TABLES["mf_user"], TABLES["mlp_user"]),
                                    (TABLES["mf_item"], TABLES["mlp_item"]))):
            sel = own["kind"] == k
            loc = own["rows"][sel]
            out[sel] = torch.cat([self.p[a][loc], self.p[b][loc]], 1)
        return out

    def compute(self, plan, back, uid, iid, targets, loss_denominator):
        O = self.O
        leaves = {}
        spos = plan.extra["spos"]
        for k, (a, b) in enumerate(((TABLES["mf_user"], TABLES["mlp_user"]),
                                    (TABLES["mf_item"], TABLES["mlp_item"]))):
            rows = back[spos[k]]
            leaves[a] = rows[:, :D].clone().requires_grad_(True)
            leaves[b] = rows[:, D:].clone().requires_grad_(True)
        for k in self.dense_names:
            leaves[k] = self.p[k].clone().requires_grad_(True)
        full = dict(self.p)
        full.update(leaves)
        inv_u, inv_i = plan.extra["inv"]
        prob = O.forward(full, inv_u, inv_i, training=True, negative_samples=M - 1, num_heads=H,
                         temporal_dim=T, n_layers=len(HID))
        loss = O.bce_loss(prob, targets) * (plan.extra["n"] / loss_denominator)
        keys = list(leaves)
        gr = dict(zip(keys, torch.autograd.grad(loss, [leaves[k] for k in keys])))
        self.dgrad = torch.cat([gr[k].reshape(-1) for k in self.dense_names])
        out = torch.empty(len(spos[0]) + len(spos[1]), 2 * D)
        for k, (a, b) in enumerate(((TABLES["mf_user"], TABLES["mlp_user"]),
                                    (TABLES["mf_item"], TABLES["mlp_item"]))):
            out[spos[k]] = torch.cat([gr[a], gr[b]], 1)
        return out, loss.detach()

    def owner_apply(self, own, got):
        """Per-row sums in source-rank order (the received order is rank-major)."""
        self.tgrad = {}
        for k, (a, b) in enumerate(((TABLES["mf_user"], TABLES["mlp_user"]),
                                    (TABLES["mf_item"], TABLES["mlp_item"]))):
            sel = own["kind"] == k
            ga, gb = torch.zeros_like(self.p[a]), torch.zeros_like(self.p[b])
            ga.index_add_(0, own["rows"][sel], got[sel][:, :D])
            gb.index_add_(0, own["rows"][sel], got[sel][:, D:])
            self.tgrad[a], self.tgrad[b] = ga, gb

    def dense_grad(self):
        return self.dgrad

    def dense_step(self):
        grads, o = dict(self.tgrad), 0
        for k in self.dense_names:
            n = self.p[k].numel()
            grads[k] = self.dgrad[o:o + n].view_as(self.p[k])
            o += n
        self.opt.step(self.p, grads)


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _ncf_pkg
    _ncf_pkg.load()
    from ncf_amd.distributed import ShardExchange, ShardedTrainStep
    params, batches = global_setup()
    ops = TorchShardOps(params, rank, world)
    plan_group = dist.new_group(list(range(world)))      # the plan's own communicator
    step = ShardedTrainStep(ops, ShardExchange(None, torch.device("cpu"), plan_group))
    losses = []
    for s in range(len(batches)):
        u, i, t = batches[s][rank]
        nxt = batches[s + 1][rank][:2] if s + 1 < len(batches) else None   # pipelined plan
        losses.append(float(step(u, i, t, next=nxt)))
    torch.save({"p": ops.p, "losses": losses}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_step_equals_single_rank_global_batch():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    from oracle import ncf_oracle as O
    params, batches = global_setup()
    ref = {k: v.clone() for k, v in params.items()}
    opt = O.AdamState(lr=1e-3, weight_decay=1e-5)
    zones = {}
    for s in range(len(batches)):
        u = torch.cat([b[0] for b in batches[s]])
        i = torch.cat([b[1] for b in batches[s]])
        t = torch.cat([b[2] for b in batches[s]])
        before = {k: v.clone() for k, v in ref.items()}
        _, loss, grads = O.train_step(ref, opt, u, i, t, negative_samples=M - 1, num_heads=H,
                                      temporal_dim=T, n_layers=len(HID))
        for k, v in grads.items():
            zones.setdefault(k, []).append(zone_from_grads(v.numpy(), before[k].numpy(), 1e-5))
        # the global loss is the sum of the ranks' contributions
        assert abs(sum(r["losses"][s] for r in res) - float(loss)) < 1e-5
    for name, zs in zones.items():
        if name in TABLES.values():
            got = torch.empty_like(ref[name])
            for r in range(world):
                got[r::world] = res[r]["p"][name]
        else:
            got = res[0]["p"][name]
            assert torch.equal(got, res[1]["p"][name]), name     # replicas stay identical
        assert_params_close(name, got.numpy(), ref[name].numpy(), zs, 1e-3, atol=2e-6)


# ----------------------------------------------------------------------------- C5 item shards
SU, SI, SK = 23, 301, 7


def _score_setup():
    import _ncf_pkg
    ncf = _ncf_pkg.load()
    torch.manual_seed(2)
    m = ncf.AdvancedNCF(SU, SI, 5, 24, D, D, T, HID, H, 0.0, M - 1)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def _ref_merge(s, i, k):
    """(score desc, item id asc) top-k with empty slots (id < 0) last — the merge's contract."""
    key_s = torch.where(i >= 0, s.double(), torch.full_like(s.double(), -1.0))
    out_s, out_i = [], []
    for r in range(s.shape[0]):
        order = sorted(range(s.shape[1]), key=lambda j: (-key_s[r, j].item(), i[r, j].item()))[:k]
        out_s.append(torch.stack([s[r, j] if i[r, j] >= 0 else s.new_zeros(()) for j in order]))
        out_i.append(torch.stack([i[r, j] for j in order]))
    return torch.stack(out_s), torch.stack(out_i)


def _score_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ncf_oracle as O
    p = _score_setup()
    from ncf_amd.scoring import shard_items, sharded_score_topk
    users = torch.arange(SU)

    def local_topk(u, k):    # oracle scores of this rank's shard (the HIP scorer needs a GPU)
        ids = shard_items(SI, world, rank)
        sc = O.score_factorised(p, u, ids, temporal_dim=T, n_layers=len(HID)).float()
        return _ref_merge(sc, ids.expand(len(u), -1), k)

    s, i = sharded_score_topk(None, users, SK, local_topk=local_topk, merge=_ref_merge)
    torch.save({"s": s, "i": i}, os.path.join(out_dir, f"score{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_item_sharded_scoring_collective_layout():
    """the per-shard top-k lists all-gathered over 2 gloo ranks and merged equal the
    single-rank top-k over the whole catalogue, on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_score_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"score{r}.pt"), weights_only=True) for r in range(world)]
    from oracle import ncf_oracle as O
    p = _score_setup()
    sc = O.score_factorised(p, torch.arange(SU), torch.arange(SI), temporal_dim=T,
                            n_layers=len(HID)).float()
    rs, ri = _ref_merge(sc, torch.arange(SI).expand(SU, -1), SK)
    for r in res:
        assert torch.equal(r["i"], ri)
        assert torch.equal(r["s"], rs)
