"""The row-sharded step's HIP path at world size 2, two processes on ONE MI355X.

RCCL cannot put two ranks on one device, so the collectives here go over gloo with host round
trips (``HostCopyExchange``, test infrastructure); everything else is the product path:
HipShardOps (plan kernels on the side stream, owner-side sort-free dedup, deferred Adam on the
shards, mini-table forward/backward, rank-ordered gradient sums) and the pipelined protocol of
ShardedTrainStep.  Parity criterion: two ranks stepping on their halves equal
one rank stepping on the concatenated batch (the CPU oracle), within the F2 tolerances."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.parity import assert_params_close, zone_from_grads

pytestmark = pytest.mark.gpu

U, I, D, T, H, HID, B, M = 301, 97, 64, 32, 4, [256, 128, 64], 8, 5
TABLES = {"mf_user": "mf_embedding_collection.embedding_bags.user_id.weight",
          "mlp_user": "mlp_embedding_collection.embedding_bags.user_id.weight",
          "mf_item": "mf_embedding_collection.embedding_bags.product_id.weight",
          "mlp_item": "mlp_embedding_collection.embedding_bags.product_id.weight"}
STEPS = 6   # (>= 6: the overlapped rolling sweep runs on the plan stream across several steps)


def setup():
    import _ncf_pkg
    ncf = _ncf_pkg.load()
    torch.manual_seed(0)
    m = ncf.AdvancedNCF(U, I, 5, 24, D, D, T, HID, H, 0.0, M - 1)
    params = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    batches = []
    for _ in range(STEPS):
        per_rank = []
        for _r in range(2):
            u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
            i = (torch.rand(B * M, generator=g) ** 2 * I).long()
            t = torch.zeros(B, M)
            t[:, 0] = 1
            per_rank.append((u, i, t.reshape(-1, 1)))
        batches.append(per_rank)
    return ncf, params, batches


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    ncf, params, batches = setup()
    from ncf_amd.distributed import HipShardOps, ShardExchange, ShardedTrainStep

    class HostCopyExchange(ShardExchange):
        """gloo collectives on host copies (two ranks share one GPU: no RCCL)."""

        def counts_issue(self, plan):
            W = self.world
            with torch.cuda.stream(plan.stream):     # the plan kernels run on the side stream
                send = plan.counts.view(W, 2).cpu()
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.plan_group)
            plan.send_counts, plan.recv_counts = send.tolist(), recv.tolist()

        def exchange(self, t, send_splits, recv_splits, side=False, slot=None):
            src = t[:sum(send_splits)].cpu()
            out = torch.empty((sum(recv_splits),) + tuple(t.shape[1:]), dtype=t.dtype)
            dist.all_to_all_single(out, src, recv_splits, send_splits,
                                   group=self.plan_group if side else self.group)
            return out.to(t.device)

        def all_reduce_(self, t):
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
            return t

        def all_reduce_start(self, t):
            self.all_reduce_(t)
            return None

    R = {"user": -(-U // world), "item": -(-I // world)}
    model = ncf.AdvancedNCF(R["user"], R["item"], 5, 24, D, D, T, HID, H, 0.0, M - 1)
    sd = dict(params)
    for key, name in TABLES.items():           # local row l <-> global id l * W + rank
        full = params[name][rank::world]
        shard = torch.zeros(R[key.split("_")[1]], D)
        shard[:full.shape[0]] = full
        sd[name] = shard
    model.load_state_dict(sd, strict=True)
    model = model.to(dev).train()
    ops = HipShardOps(model, U, I, world, lr=1e-3, weight_decay=1e-5)
    step = ShardedTrainStep(ops, HostCopyExchange(None, dev, dist.new_group([0, 1])))
    dev_batches = [[(u.to(dev), i.to(dev), t.to(dev)) for (u, i, t) in b] for b in batches]
    losses = []
    for s in range(STEPS):
        u, i, t = dev_batches[s][rank]
        nxt = dev_batches[s + 1][rank][:2] if s + 1 < STEPS else None     # pipelined plan
        losses.append(float(step(u, i, t, next=nxt)))
    ops.check()
    out = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save({"p": out, "losses": losses}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_hip_sharded_step_world2_equals_single_rank_global_batch():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    from oracle import ncf_oracle as O
    _, params, batches = setup()
    ref = {k: v.clone() for k, v in params.items()}
    opt = O.AdamState(lr=1e-3, weight_decay=1e-5)
    zones = {}
    for s in range(STEPS):
        u = torch.cat([b[0] for b in batches[s]])
        i = torch.cat([b[1] for b in batches[s]])
        t = torch.cat([b[2] for b in batches[s]])
        before = {k: v.clone() for k, v in ref.items()}
        _, loss, grads = O.train_step(ref, opt, u, i, t, negative_samples=M - 1, num_heads=H,
                                      temporal_dim=T, n_layers=len(HID))
        for k, v in grads.items():
            zones.setdefault(k, []).append(zone_from_grads(v.numpy(), before[k].numpy(), 1e-5))
        assert abs(sum(r["losses"][s] for r in res) - float(loss)) < 2e-6
    for name, zs in zones.items():
        if name in TABLES.values():
            got = torch.empty_like(ref[name])
            for r in range(world):
                got[r::world] = res[r]["p"][name][:ref[name][r::world].shape[0]]
        else:
            got = res[0]["p"][name]
            assert torch.equal(got, res[1]["p"][name]), name     # replicas stay identical
        assert_params_close(name, got.numpy(), ref[name].numpy(), zs, 1e-3, atol=2e-6)
