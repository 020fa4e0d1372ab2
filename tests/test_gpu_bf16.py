"""The bf16-table configuration (BASELINE.json configs[1] "bf16"; SURVEY 8(d) C2: tables bf16,
Adam moments fp32) on the MI355X.

* Its deferred schedule reproduces its own dense schedule (every table swept every step,
  ncf_adam_table_bf16) bit for bit: parameters (bf16) and moments (fp32).
* Against the fp32 CPU oracle (oracle/ncf_oracle.py, pinned to the reference's goldens) over
  100 training steps: every step's loss within 1% and the final eval probabilities within 2e-2
  (SURVEY 8(c) bf16 tolerances); the fp32 parity path stays the reference (test_gpu_parity).
"""
import numpy as np
import pytest
import torch

import _ncf_pkg
from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
ncf = _ncf_pkg.load()
DEV = torch.device("cuda:0")


def _batches(U, I, B, M, n, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        u = torch.randint(0, U, (B,), generator=g).repeat_interleave(M)
        i = (torch.rand(B * M, generator=g) ** 2 * I).long().clamp_max(I - 1)
        t = torch.zeros(B, M)
        t[:, 0] = 1
        out.append((u, i, t.reshape(-1, 1)))
    return out


def _run_bf16(deferred, steps, U=3000, I=500, B=64, seed=31):
    from ncf_amd.trainer import FusedTrainStep
    torch.manual_seed(seed)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.0, 4).to(DEV)
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, deferred=deferred,
                          table_dtype=torch.bfloat16)
    for u, i, t in _batches(U, I, B, 5, steps, seed + 1):
        step(u.to(DEV), i.to(DEV), t.to(DEV))
    step.sync()
    return ({k: v.detach().cpu().clone() for k, v in step.tables_lp.items()},
            {k: (v["exp_avg"].cpu().clone(), v["exp_avg_sq"].cpu().clone())
             for k, v in step.state.items()}, m)


def test_bf16_deferred_bitwise_equals_dense_bf16():
    a_t, a_m, _ = _run_bf16(False, 70)
    b_t, b_m, mb = _run_bf16(True, 70)
    for k in a_t:
        assert a_t[k].dtype == torch.bfloat16
        assert torch.equal(a_t[k], b_t[k]), k
        assert torch.equal(a_m[k][0], b_m[k][0]) and torch.equal(a_m[k][1], b_m[k][1]), k
    # the model's fp32 table parameters hold the bf16 values after sync (state_dict readers)
    sd = mb.state_dict()
    assert torch.equal(sd["mlp_embedding_collection.embedding_bags.user_id.weight"].cpu(),
                       b_t["mlp_user"].float())


def test_bf16_tables_track_fp32_oracle_over_100_steps():
    from ncf_amd.trainer import FusedTrainStep
    U, I, B, M, steps = 1000, 300, 32, 5, 100
    torch.manual_seed(7)
    m = ncf.AdvancedNCF(U, I, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.0, M - 1)
    ref = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, table_dtype=torch.bfloat16)
    oopt = O.AdamState(lr=1e-3, weight_decay=1e-5)
    worst = 0.0
    for u, i, t in _batches(U, I, B, M, steps, 8):
        w = step(u.to(DEV), i.to(DEV), t.to(DEV))
        _, oloss, _ = O.train_step(ref, oopt, u, i, t, negative_samples=M - 1, num_heads=4,
                                   temporal_dim=32, n_layers=3)
        rel = abs(float(w.loss.item()) - float(oloss)) / float(oloss)
        worst = max(worst, rel)
    assert worst < 0.01, f"loss drifted {worst:.4%} from the fp32 oracle"
    eu = torch.randint(0, U, (200,), generator=torch.Generator().manual_seed(9))
    ei = torch.randint(0, I, (200,), generator=torch.Generator().manual_seed(10))
    m.eval()
    with torch.no_grad():
        got = m.forward_simple(eu.to(DEV), ei.to(DEV)).cpu()
    want = O.forward(ref, eu, ei, training=False, negative_samples=M - 1, num_heads=4,
                     temporal_dim=32, n_layers=3).reshape(-1)
    assert (got - want).abs().max().item() < 2e-2
    assert np.isfinite(got.numpy()).all()
