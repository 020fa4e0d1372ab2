"""C4 at full size on ONE MI355X (BASELINE.json configs[3]): 50M users x 5M items,
D = 128, H = 4, MLP [256,128,64].  The fp32 tables (56.3 GB) + Adam moments (112.6 GB) fit one
GPU's 288 GB of HBM.  Size-independent properties (the CPU oracle cannot hold this model):

* ids at the very top of both ranges train (int64 row offsets: user row 49,999,999 starts at
  element 6.4e9 > 2^31), and the loss stays finite;
* the 3-radix-pass dedup (26-bit user ids) equals np.unique on the step's ids;
* after sync(), rows no batch touched hold exactly what the dense kernel (ncf_adam_table with
  every slot empty, the reference's dense Adam on a zero gradient + coupled decay) gives when
  replayed on their initial values for the same steps — bitwise, parameters and moments.
"""
import numpy as np
import pytest
import torch

import _ncf_pkg

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")
U, I, D, B, M, STEPS = 50_000_000, 5_000_000, 128, 4096, 5, 4
TABLES = {"mf_user": "mf_embedding_collection.embedding_bags.user_id.weight",
          "mlp_user": "mlp_embedding_collection.embedding_bags.user_id.weight",
          "mf_item": "mf_embedding_collection.embedding_bags.product_id.weight",
          "mlp_item": "mlp_embedding_collection.embedding_bags.product_id.weight"}


def test_c4_full_size_one_gpu():
    from ncf_amd import _lib
    from ncf_amd.trainer import FusedTrainStep
    if torch.cuda.get_device_properties(0).total_memory < 250e9:
        pytest.skip("needs a 288 GB MI355X")
    torch.cuda.empty_cache()
    torch.manual_seed(5)
    with torch.device(DEV):
        m = ncf.AdvancedNCF(U, I, 5, 24, D, D, 32, [256, 128, 64], 4, 0.0, M - 1).train()
    g = torch.Generator(device=DEV).manual_seed(6)
    batches = []
    for s in range(STEPS):
        u = torch.randint(0, U, (B,), generator=g, device=DEV).repeat_interleave(M)
        i = torch.randint(0, I, (B * M,), generator=g, device=DEV)
        if s == 0:
            u[:M] = U - 1
            i[:3] = torch.tensor([I - 1, I - 2, 0], device=DEV)
        t = torch.zeros(B, M, device=DEV)
        t[:, 0] = 1
        batches.append((u, i, t.reshape(-1, 1)))
    # rows no batch touches (sampled across each table, the last rows included)
    seen_u = torch.cat([b[0] for b in batches]).unique().cpu().numpy()
    seen_i = torch.cat([b[1] for b in batches]).unique().cpu().numpy()
    cand_u = np.array([1, 12_345, U // 2 + 7, 2 ** 31 // D + 3, U - 3, U - 2])
    cand_i = np.array([3, I // 2 + 1, I - 7, I - 4])
    rows = {"user": torch.from_numpy(np.setdiff1d(cand_u, seen_u)).to(DEV),
            "item": torch.from_numpy(np.setdiff1d(cand_i, seen_i)).to(DEV)}
    tb = m.engine.table_params()
    init = {k: tb[k][rows["user" if k.endswith("user") else "item"]].clone() for k in TABLES}
    top0 = tb["mlp_user"][U - 1].clone()

    # the 3-pass radix dedup (ids up to 2^26) vs np.unique
    u0, i0 = batches[0][0], batches[0][1]
    n = u0.numel()
    ws = torch.empty(_lib.query("ncf_embedding_bwd_workspace", n, D), dtype=torch.uint8, device=DEV)
    uq = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(2)]
    cnt = torch.zeros(2, dtype=torch.int32, device=DEV)
    _lib.call("ncf_dedup_ids", u0.data_ptr(), i0.data_ptr(), n, D, U, I, uq[0].data_ptr(),
              uq[1].data_ptr(), None, None, cnt.data_ptr(), ws.data_ptr(), ws.numel(),
              _lib.stream_ptr(DEV))
    nu, ni = cnt.tolist()
    assert np.array_equal(uq[0][:nu].cpu().numpy(), np.unique(u0.cpu().numpy()))
    assert np.array_equal(uq[1][:ni].cpu().numpy(), np.unique(i0.cpu().numpy()))
    assert uq[0][nu - 1].item() == U - 1

    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    for s, (u, i, t) in enumerate(batches):
        step(u, i, t, next=batches[s + 1][:2] if s + 1 < STEPS else None)
        assert np.isfinite(float(step.last_loss.item()))
    step.sync()
    assert not m.engine.lagging()
    # the top rows are finite, and user U-1 (in batch 0) was trained: its first moment is not
    # what zero-gradient steps (coupled decay only, ~(1-b1) wd p) would leave
    assert torch.isfinite(tb["mlp_user"][U - 1]).all() and torch.isfinite(tb["mlp_item"][I - 1]).all()
    decay_only = 1e-5 * top0.abs().max().item()
    assert step.state["mlp_user"]["exp_avg"][U - 1].abs().max().item() > 10 * decay_only

    # untouched rows == the dense kernel replayed on their initial values (bitwise)
    st = _lib.stream_ptr(DEV)
    for k in TABLES:
        r = rows["user" if k.endswith("user") else "item"]
        p = init[k].clone()
        ea, eas = torch.zeros_like(p), torch.zeros_like(p)
        slot = torch.full((p.shape[0],), -1, dtype=torch.int32, device=DEV)
        for s in range(1, STEPS + 1):
            _lib.call("ncf_adam_table", p.data_ptr(), ea.data_ptr(), eas.data_ptr(), p.shape[0], D,
                      slot.data_ptr(), None, 1e-3, 0.9, 0.999, 1e-8, 1e-5, float(s), st)
        assert torch.equal(tb[k][r], p), k
        assert torch.equal(step.state[k]["exp_avg"][r], ea), k
        assert torch.equal(step.state[k]["exp_avg_sq"][r], eas), k
    del step, m
    torch.cuda.empty_cache()
