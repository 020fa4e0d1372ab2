"""bench.py's own launcher (`--gpus N` outside torchrun) and its priming rule, on the CPU:
`--dry-launch` ranks join a gloo group from the environment the launcher sets and report."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=120)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_starts_n_ranks_that_agree(n):
    r, lines = _run(["--gpus", str(n), "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["dry_launch"] and rec["n_gpus"] == n
    assert rec["ranks"] == list(range(n)) and rec["worlds_agree"]


def test_gpus_1_runs_in_process():
    r, lines = _run(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["ranks"] == [0] and rec["local_ranks_env"] is None


def test_gpus_n_refuses_without_enough_devices():
    # no GPU in this container: asking for 2 must fail loudly, not run one rank
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    r, lines = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and not lines
    assert "only" in r.stderr and "visible" in r.stderr


def test_priming_rule():
    import bench
    assert bench.steady_state(128, 5, 64) and bench.steady_state(0, 128, 64)
    assert not bench.steady_state(0, 5, 64) and not bench.steady_state(100, 5, None)

    class A:
        prime = -1
    assert bench.prime_steps(A) == 2 * bench.SWEEP_EVERY
    A.prime = 3
    assert bench.prime_steps(A) == 3


def test_embedding_rooflines_byte_models():
    """bench.embedding_rooflines prices the scatter by the entry point that ran: the plain
    reduce N (16 D + 16) + U 16 D, the reduce with the table Adam fused in
    N (16 D + 16) + U (56 D + 4) (its parameter rows out, moment rows in and out, the stamp);
    and the PMC summary quoted first is the round's final one."""
    import bench
    N, D, U = 20480, 64, (4000, 20000)
    per = {"ncf_gather_ln_gmf_scaled_fwd": [None] * 10}
    for kern, per_row in (("ncf_embedding_bwd_reduce", 16 * D),
                          ("ncf_embedding_bwd_reduce_apply_clock", 56 * D + 4)):
        totals = {"ncf_gather_ln_gmf_scaled_fwd": 0.01, kern: 0.03}
        p = dict(per, **{kern: [None] * 10})
        hbm = bench.embedding_rooflines(totals, p, 10, N, D, 5, U, pmc=False)
        assert hbm["scatter"]["entry_point"] == kern
        assert hbm["scatter"]["bytes_per_launch"] == N * (16 * D + 16) + sum(U) * per_row
    src = bench.pmc_traffic("k_attn_mlp_bwd")
    assert src is None or src["source"].startswith(bench.PMC_SUMMARIES[-1])
