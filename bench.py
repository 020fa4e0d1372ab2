#!/usr/bin/env python3
"""Benchmark: AdvancedNCF training samples/s (+ inference pairs/s) on MI355X.

Workload (BASELINE.json configs[1]): 1,000,000 users x 100,000 items, D=64,
4 attention heads, MLP [256,128,64], T=32; B=4096 interaction groups x M=5 rows (1 positive +
4 negatives) = 20,480 samples per step per GPU.  A step is one full ModelTrainer.train_epoch
batch: forward, BCE, backward, dense-exact Adam over all 140.8M embedding parameters + the dense
parameters (src/model/trainer.py:253-285).  Synthetic data: users uniform, positive items
Zipf(1.05), negatives uniform; random-init weights.  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

``--gpus N`` without a torchrun environment (no WORLD_SIZE) starts the N rank processes itself
(torchrun's env: RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) before this
process touches the GPU, and exits with their status; fewer than N visible GPUs is an error.

Every timed leg first runs ``prime`` steps (2 x the deferred Adam's sweep_every = 256 by
default) before its W counted warm-up steps: the deferred table schedule replays, per swept
row, the zero-gradient steps since that row's stamp, and every stamp starts at 0, so before
step 2 x sweep_every a sweep replays less than its steady-state share.  Priming puts every leg
in steady state whatever W is (``adam_steady_state`` per leg).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import platform
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import _ncf_pkg  # noqa: E402

METRIC = "train samples/sec + infer pairs/sec, 1M×100K d=64 AdvancedNCF @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA = the f32 vector rate
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)


# C-ABI entry point -> the kernel symbol rocprofv3 reports for it
KERNEL_SYMBOL = {"ncf_attn_block_fwd": "k_attn_block_fwd", "ncf_attn_block_bwd": "k_attn_block_bwd",
                 "ncf_mlp_fwd": "k_mlp_fwd", "ncf_mlp_bwd": "k_mlp_bwd",
                 "ncf_mlp_fwd_split": "k_mlp_fwd", "ncf_mlp_bwd_split": "k_mlp_bwd",
                 "ncf_wgrad_grouped": "k_wgrad_grouped",
                 "ncf_attn_mlp_fwd": "k_attn_mlp_fwd", "ncf_attn_mlp_bwd": "k_attn_mlp_bwd",
                 "ncf_attn_mlp_fwd_small": "k_attn_mlp_fwd", "ncf_attn_mlp_bwd_small": "k_attn_mlp_bwd"}
# the tower's Linears on bf16 matrix cores through split operands: 6 bf16 products per fp32
# product (engine.TOWER_SPLIT); their roofline is quoted as fp32-equivalent work against the fp32
# MFMA peak, with the executed bf16 products against the bf16 peak beside it
SPLIT_PRODUCTS = 6
SPLIT_NAMES = ("ncf_mlp_fwd_split", "ncf_mlp_bwd_split")


PMC_SUMMARIES = ("r06_c5_pmc_traffic.json", "r06_pmc_traffic.json")   # (run r06k)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/*_pmc_traffic.json, made by tools/pmc_traffic.py from separate FETCH_SIZE and
    WRITE_SIZE passes, gfx950 FETCH_SIZE x2 correction applied); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    # the summaries taken at the round's final HEAD first (then the newest name)
    for name in PMC_SUMMARIES:
        pref = os.path.join(ROOT, "profiles", name)
        if pref in files:
            files.remove(pref)
            files.append(pref)
    if not kernel:
        return None
    for fn in reversed(files):   # the newest summary that has the kernel
        with open(fn) as f:
            k = json.load(f).get("kernels", {}).get(kernel)
        if k:
            return {"bytes_per_launch": k["hbm_bytes_per_launch"],
                    "source": f"{os.path.basename(fn)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                              f"separate passes)"}
    return None


ISO_STEPS = 40   # steps of the roofline kernel's isolated (sweep not overlapped) measurement
N_BATCHES = 256  # distinct resident batches the timed legs cycle through (not 8)
# VALU issue of the deferred-Adam replay (tools/isa_replay_count.py on csrc/adam.hip, gfx950):
# per zero-gradient element-step of the fp32 table-pair replay loop (D = 64): 4.94 plain VALU
# (v_mul / v_fma(c) / v_mov), 1.63 packed (v_pk_fma / v_pk_mul: 2 lane-slots each), 2
# transcendental (v_sqrt, v_rcp: quarter rate, 4 slots each) -> 16.19 lane issue slots.  D = 128
# (C4): 1.25 plain + 3 packed + 2 transcendental -> 15.25.  Recount with the script after any
# change to adam0 / the replay loop.
ADAM_REPLAY_SLOTS = {64: 16.19, 128: 15.25}
# chip VALU issue rate: 256 CUs x 4 SIMDs x 32 lanes per cycle x 2.4 GHz = 78.64 T lane-slots/s
# (= the 157.3 TF fp32 vector peak with an FMA counted as 2 flops; MI355X_MICROARCH.md)
VALU_SLOTS_PEAK_T = 78.64
SWEEP_EVERY = 128  # the longest rolling-sweep period of the legs (FusedTrainStep's; optim.py: 64)


def prime_steps(args) -> int:
    """Untimed steps run before the counted warm-up of every training leg: 2 x sweep_every
    (the deferred schedule's steady state, see the module docstring) unless --prime says."""
    return 2 * SWEEP_EVERY if args.prime < 0 else args.prime


def steady_state(prime: int, warmup: int, sweep_every) -> bool:
    """Whether a leg's timed steps run with the deferred sweep in steady state: every row has
    been swept at least once after its first sweep cycle before timing starts."""
    return bool(sweep_every) and prime + warmup >= 2 * int(sweep_every)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, dry: bool) -> int:
    """`bench.py --gpus n` outside torchrun: start n rank processes of this script with
    torchrun's environment, one per GPU, and return their exit status (the first failure; the
    other ranks are then stopped, by PID).  Runs before anything here touches the GPU
    (torch.cuda.device_count() does not initialise it on this image)."""
    if not dry:
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} asked for {n} GPUs but only {have} are visible; "
                  "refusing to run a smaller job", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:          # a rank failed: the others would wait in collectives
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def dry_launch() -> None:
    """--dry-launch: each rank joins a gloo group from the env and checks that all ranks agree
    on the world size (no GPU); rank 0 prints one JSON line.  Tests the --gpus N launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([world, rank, 1], dtype=torch.int64)
    if world > 1:
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        dist.destroy_process_group()
    else:
        lst = [t]
    if rank == 0:
        print(json.dumps({"dry_launch": True, "n_gpus": world,
                          "ranks": sorted(int(x[1]) for x in lst),
                          "worlds_agree": all(int(x[0]) == world for x in lst),
                          "local_ranks_env": os.environ.get("LOCAL_RANK")}), flush=True)


def zipf_sampler(n_items, s, device):
    w = 1.0 / torch.arange(1, n_items + 1, dtype=torch.float64) ** s
    cdf = torch.cumsum(w / w.sum(), 0).to(device=device, dtype=torch.float64)
    perm = torch.randperm(n_items, generator=torch.Generator().manual_seed(7)).to(device)

    def sample(k, gen):
        u = torch.rand(k, generator=gen, device=device, dtype=torch.float64)
        idx = torch.searchsorted(cdf, u).clamp_max(n_items - 1)
        return perm[idx]
    return sample


def make_batches(U, I, B, M, count, device, seed):
    gen = torch.Generator(device=device).manual_seed(seed)
    zipf = zipf_sampler(I, 1.05, device)
    out = []
    for _ in range(count):
        users = torch.randint(0, U, (B,), generator=gen, device=device).repeat_interleave(M)
        pos = zipf(B, gen)
        neg = torch.randint(0, I, (B, M - 1), generator=gen, device=device)
        items = torch.cat([pos[:, None], neg], 1).reshape(-1).contiguous()
        t = torch.zeros(B, M, device=device)
        t[:, 0] = 1
        out.append((users.contiguous(), items, t.reshape(-1, 1)))
    return out


def host_cpu():
    """(cores this process may run on, CPU model): the affinity mask capped by the cgroup CPU
    quota (a GPU box's share of a larger host), and the /proc/cpuinfo (lscpu) model name."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            cores = max(1, min(cores, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, model


def cpu_baseline(model_sd, cfg, batches_cpu, budget_s):
    """The CPU oracle (fp32 PyTorch restatement of the reference math, oracle/ncf_oracle.py)
    timed on this host's cores on a bounded sample of the same workload, with every core this
    process may use."""
    from oracle import ncf_oracle as O
    threads, cpu_model = host_cpu()
    torch.set_num_threads(threads)
    p = {k: v.detach().cpu().clone() for k, v in model_sd.items()}
    opt = O.AdamState(lr=1e-3, weight_decay=1e-5)
    U, I, D, T, H, hid, B, M = cfg
    kw = dict(negative_samples=M - 1, num_heads=H, temporal_dim=T, n_layers=len(hid))
    u, i, t = batches_cpu[0]
    O.train_step(p, opt, u, i, t, **kw)            # warm-up (allocations, first-touch)
    times = []
    k = 0
    t_all = time.perf_counter()
    while True:
        u, i, t = batches_cpu[(k + 1) % len(batches_cpu)]
        t0 = time.perf_counter()
        O.train_step(p, opt, u, i, t, **kw)
        times.append(time.perf_counter() - t0)
        k += 1
        if time.perf_counter() - t_all > budget_s or k >= 20:
            break
    med = sorted(times)[len(times) // 2]
    return {"value": (B * M) / med, "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model,
            "sample": f"{k} timed train steps (B={B} groups x M={M}, full {U} x {I} tables, "
                      f"D={D}, fp32, dense Adam) after 1 warm-up; median step {med * 1e3:.1f} ms; "
                      f"{threads} threads on {cpu_model}"}


def cpu_infer_baseline(model_sd, iu, ii, H, T, n_layers, budget_s):
    """the C2 eval forward (M = 1) on the CPU oracle over the same N resident
    pairs, full tables, every core this process may use; median of <= 5 calls within budget."""
    from oracle import ncf_oracle as O
    threads, cpu_model = host_cpu()
    torch.set_num_threads(threads)
    p = {k: v.detach().cpu() for k, v in model_sd.items()}
    kw = dict(training=False, negative_samples=4, num_heads=H, temporal_dim=T, n_layers=n_layers)
    with torch.no_grad():
        O.forward(p, iu, ii, **kw)          # warm-up
        times = []
        t_all = time.perf_counter()
        while len(times) < 5 and time.perf_counter() - t_all < budget_s:
            t0 = time.perf_counter()
            O.forward(p, iu, ii, **kw)
            times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": round(iu.numel() / med, 1), "unit": "pairs/s", "cores": threads,
            "kind": "port", "cpu_model": cpu_model,
            "sample": f"oracle eval forward over the same {iu.numel()} pairs (full 1M x 100K "
                      f"tables, fp32), median of {len(times)} calls: {med * 1e3:.1f} ms"}


def embedding_rooflines(totals, per, steps, N, D, grows, nu_ni, pmc=True):
    """HBM rooflines of the embedding gather and scatter from per-launch event times (SURVEY
    8(d) algorithmic bytes per launch):
      gather  (ncf_gather_ln_gmf_scaled_fwd), group_rows = M (fact 6: a group's user rows read
              and its LN'd user rows written once): per row the item GMF + MLP rows in and out,
              two int64 ids and mf_pred = N (16 D + 20), per group the user's two rows in and out
              = (N / M) 16 D; every row written (group_rows 0): N (16 D + 16 + 16 D + 4);
      scatter (ncf_embedding_bwd_reduce): 4 gradient rows in per sample + 2 ids, per unique row
              the 2 table rows (LN recompute) in and 2 compact gradient rows out
              = N (16 D + 16) + (n_u + n_i) 16 D;
      scatter + apply (ncf_embedding_bwd_reduce_apply_clock, the table Adam fused in): the same,
              and per unique row its 2 parameter rows out and 4 moment rows in and out, and the
              stamp = N (16 D + 16) + (n_u + n_i) (56 D + 4)."""
    g_bytes = (N * (16 * D + 20) + (N // grows) * 16 * D if grows > 1
               else N * (16 * D + 16 + 16 * D + 4))
    hbm = {}
    fused = "ncf_embedding_bwd_reduce_apply_clock" in totals
    for name, kern, nbytes in (
            ("gather", "ncf_gather_ln_gmf_scaled_fwd", g_bytes),
            ("scatter", "ncf_embedding_bwd_reduce_apply_clock" if fused else "ncf_embedding_bwd_reduce",
             N * (16 * D + 16) + (sum(nu_ni) * ((56 * D + 4) if fused else 16 * D)
                                  if nu_ni else 0))):
        if kern in totals:
            launches = len(per.get(kern, [])) / steps
            ms = totals[kern] / max(launches, 1)
            gbs = nbytes / (ms * 1e-3) / 1e9
            # (the committed PMC summaries are of the C2 launch: not quoted for other sizes)
            pm = pmc_traffic({"ncf_gather_ln_gmf_scaled_fwd": "k_gather_ln_gmf",
                              "ncf_embedding_bwd_reduce": "k_piece_reduce_ln",
                              "ncf_embedding_bwd_reduce_apply_clock": "k_piece_reduce_ln"}[kern]) \
                if pmc else None
            hbm[name] = {"entry_point": kern, "bytes_per_launch": nbytes, "ms_per_launch": round(ms, 4),
                         "achieved_GBps": round(gbs, 1), "peak_GBps": HBM_PEAK_GBS,
                         "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": pm["bytes_per_launch"] if pm else None}
    if "gather" in hbm:
        hbm["gather"]["group_rows"] = grows
        hbm["gather"]["round3_count_bytes"] = N * (16 * D + 16 + 16 * D + 4)
    if "scatter" in hbm:
        hbm["scatter"]["unique_rows"] = nu_ni
        hbm["scatter"]["note"] = ("segment reduce + LN backward (+ the multi-piece fix-up)"
                                  + (" with the table Adam apply fused in" if fused else "")
                                  + "; the id sort before it (ncf_dedup_ids) is listed in "
                                  "kernel_ms_per_step")
    return hbm


def profiled_steps(step, batches, first, count, pipelined=True):
    """count FusedTrainStep steps with HIP events around every C-ABI call: (per entry point
    [(args, ms)], ms per step per entry point)."""
    from ncf_amd import _lib as L
    L.PROFILE = []
    torch.cuda.synchronize()
    for s in range(first, first + count):
        u, i, t = batches[s % len(batches)]
        if pipelined:
            step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
        else:
            step(u, i, t)
    torch.cuda.synchronize()
    prof, L.PROFILE = L.PROFILE, None
    per = {}
    for name, a, e0, e1 in prof:
        per.setdefault(name, []).append((a, e0.elapsed_time(e1)))
    return per, {k: sum(d for _, d in v) / count for k, v in per.items()}


def embedding_large(ncf, dev, cfg, groups, warmup, steps):
    """the embedding gather / scatter rooflines where their launch latency is
    amortised — SURVEY 8(d)'s strong-scaling global batch (32,768 groups x M = 163,840 rows) on
    ONE GPU, the same C2 tables and step (FusedTrainStep), per-launch HIP events."""
    from ncf_amd.trainer import FusedTrainStep
    U, I, D, T, H, hid, _, M = cfg
    N = groups * M
    torch.manual_seed(555)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    batches = make_batches(U, I, groups, M, 8, dev, seed=321)
    for s in range(warmup):
        u, i, t = batches[s % len(batches)]
        step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(warmup, warmup + steps):
        u, i, t = batches[s % len(batches)]
        step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    per, totals = profiled_steps(step, batches, warmup + steps, steps)
    w = next(iter(m.engine.ws.values()))
    nu_ni = [int(x) for x in w.num_unique.cpu().tolist()]
    hbm = embedding_rooflines(totals, per, steps, N, D, int(getattr(w, "group_rows", 0)), nu_ni,
                              pmc=False)
    out = {"config": f"C2 tables (1M x 100K, D=64), {groups} groups x M={M} = {N} rows per step "
                     "on one GPU (SURVEY 8(d) strong-scaling global batch)",
           "rows_per_step": N, "ms_per_step": round(dt / steps * 1e3, 4),
           "value": round(N * steps / dt, 1), "unit": "samples/s", **hbm,
           "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(totals.items(), key=lambda x: -x[1])}}
    del step, m, batches
    torch.cuda.empty_cache()
    return out


def small_batch_train(ncf, dev, cfg, warmup, steps, prime, init_sd=None, cpu_budget=0.0):
    """C2 at the reference's default batch (batch_size 256,
    /root/reference/config/config.yaml:65; N = 1,280 rows): the same FusedTrainStep.  Here the
    dense-exact Adam's full-table replay (140.8M element-steps per step whatever the batch) sets
    the pace, not the batch.  With ``init_sd``: the CPU oracle on the same configuration (BASELINE.md
    section 2 quotes 4,037 samples/s on 8 cores for the reference itself)."""
    from ncf_amd.trainer import FusedTrainStep
    U, I, D, T, H, hid, B, M = cfg
    torch.manual_seed(1234)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)
    batches = make_batches(U, I, B, M, N_BATCHES, dev, seed=256)

    def run(first, count):
        for s in range(first, first + count):
            u, i, t = batches[s % len(batches)]
            step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
    run(0, prime + warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(prime + warmup, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    per, totals = profiled_steps(step, batches, prime + warmup + steps, min(steps, 50))
    out = {"config": f"C2 at the reference's default batch: B={B} groups x M={M} = {B * M} rows "
                     "(config.yaml:65), 1M x 100K, D=64, FusedTrainStep",
           "value": round(B * M * steps / dt, 1), "unit": "samples/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "prime_steps": prime,
           "adam_steady_state": steady_state(prime, warmup, step.deferred.sweep_every),
           "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(totals.items(), key=lambda x: -x[1])},
           "reference_cpu_published": {"value": 4037, "unit": "samples/s",
                                       "source": "BASELINE.md section 2 (8-core Xeon, measured by "
                                                 "the survey on the reference itself)"}}
    del step, m
    torch.cuda.empty_cache()
    if init_sd is not None:
        cpu_b = [(u.cpu(), i.cpu(), t.cpu()) for (u, i, t) in batches[:4]]
        out["cpu_baseline"] = cpu_baseline(init_sd, cfg, cpu_b, cpu_budget)
        out["vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    del batches
    return out


C1 = dict(U=943, I=1682, D=16, T=32, H=1, hid=[64, 32], B=256, M=5)


def c1_line(ncf, dev, warmup, steps, prime, cpu_budget, with_cpu):
    """BASELINE.json configs[0] / SURVEY 8(d) C1 (MovieLens-100K-shaped: 943 users x 1682 items,
    D=16, H=1, MLP [64, 32], B=256 x M=5): the reference's CPU configuration.  The CPU oracle
    timed on the host's cores (the baseline SURVEY 8(d) asks for), and the same step on the GPU
    (FusedTrainStep; D = 16 runs the unfused attention / tower kernels)."""
    from ncf_amd.trainer import FusedTrainStep
    c = C1
    U, I, D, T, H, hid, B, M = c["U"], c["I"], c["D"], c["T"], c["H"], c["hid"], c["B"], c["M"]
    cfg = (U, I, D, T, H, hid, B, M)
    torch.manual_seed(11)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1)
    init = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    batches = make_batches(U, I, B, M, 64, dev, seed=943)
    out = {"config": "C1: 943 users x 1682 items, D=16, H=1, MLP [64,32], T=32, B=256 x M=5, "
                     "dropout 0.2, Adam lr 1e-3 wd 1e-5 (dense-exact)"}
    try:
        step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5)

        def run(first, count):
            for s in range(first, first + count):
                u, i, t = batches[s % len(batches)]
                step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
        run(0, prime + warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(prime + warmup, steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out.update({"value": round(B * M * steps / dt, 1), "unit": "samples/s",
                    "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps})
        del step
    except Exception as e:     # recorded, not fatal to the headline
        out["gpu_error"] = f"{type(e).__name__}: {e}"[:300]
    if with_cpu:
        cpu_b = [(u.cpu(), i.cpu(), t.cpu()) for (u, i, t) in batches[:4]]
        out["cpu_baseline"] = cpu_baseline(init, cfg, cpu_b, cpu_budget)
        if "value" in out:
            out["vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    del m, batches
    torch.cuda.empty_cache()
    return out


def dropin_train(ncf, dev, cfg, batches, warmup, steps, prime=0):
    """The reference's own call pattern on the fused path (src/model/trainer.py:258-285):
    ``out = model(kjt); loss = nn.BCELoss()(out, t); optimizer.zero_grad(); loss.backward();
    optimizer.step()`` with ``torch.optim.Adam(model.parameters(), lr, weight_decay)`` — the
    nn.Module / optimizer surface the north star keeps identical (autograd + the step hook
    driving the deferred dense-exact table schedule).  Same C2 workload and batches as the
    headline; timed after the same steady-state warm-up.  Second figure: the same loop plus the
    reference's per-batch ``loss.item()`` (trainer.py:289), a host sync every step."""
    U, I, D, T, H, hid, B, M = cfg
    torch.manual_seed(1234)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    feats = []
    for u, i, t in batches:
        kj = ncf.KeyedJaggedTensor.from_lengths_sync(
            keys=["user_id", "product_id"], values=torch.cat([u, i]),
            lengths=torch.ones(2 * u.numel(), dtype=torch.long, device=dev))
        feats.append((kj, t))

    def run(first, count, item=False):
        for s in range(first, first + count):
            f, t = feats[s % len(feats)]
            out = m(f)
            loss = crit(out, t)
            opt.zero_grad()
            loss.backward()
            opt.step()
            if item:
                loss.item()
        return loss

    run(0, prime + warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = run(prime + warmup, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_item = min(steps, 100)
    t1 = time.perf_counter()
    run(prime + warmup + steps, n_item, item=True)
    torch.cuda.synchronize()
    dt_item = time.perf_counter() - t1
    # the same loop with the backward on the calling thread (what ncf_amd.trainer.Trainer's
    # train_epoch does: torch.autograd.set_multithreading_enabled(False) around the epoch)
    with torch.autograd.set_multithreading_enabled(False):
        run(prime + warmup + steps + n_item, 20)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        run(prime + warmup + steps + n_item + 20, steps)
        torch.cuda.synchronize()
        dt_ct = time.perf_counter() - t2
    # per-phase breakdown (a separate region: host perf_counter around each call of the loop,
    # and a torch event on the current stream at each phase boundary).  host_us: the Python
    # call's duration; gpu_us: stream time from the phase's first enqueued work to its last
    # (includes any wait of the stream for the host inside the phase)
    phases = ("forward", "bce", "zero_grad", "backward", "step")
    nb = min(steps, 50)
    host = {k: 0.0 for k in phases}
    evs = []
    first = prime + warmup + steps + n_item + 20 + steps
    torch.cuda.synchronize()
    for s_ in range(first, first + nb):
        f, t = feats[s_ % len(feats)]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(len(phases) + 1)]
        e[0].record()
        h0 = time.perf_counter()
        out = m(f)
        h1 = time.perf_counter()
        e[1].record()
        l_ = crit(out, t)
        h2 = time.perf_counter()
        e[2].record()
        opt.zero_grad()
        h3 = time.perf_counter()
        e[3].record()
        l_.backward()
        h4 = time.perf_counter()
        e[4].record()
        opt.step()
        h5 = time.perf_counter()
        e[5].record()
        for k, a, b in zip(phases, (h0, h1, h2, h3, h4), (h1, h2, h3, h4, h5)):
            host[k] += b - a
        evs.append(e)
    torch.cuda.synchronize()
    gpu = {k: sum(e[j].elapsed_time(e[j + 1]) for e in evs) / nb * 1e3
           for j, k in enumerate(phases)}
    breakdown = {k: {"host_us": round(host[k] / nb * 1e6, 1), "gpu_us": round(gpu[k], 1)}
                 for k in phases}
    from ncf_amd import optim as _o
    b = _o.binding_of(opt, m)
    out = {"pattern": "model(kjt) -> nn.BCELoss -> zero_grad -> backward -> torch.optim.Adam.step "
                      "(trainer.py:258-285), deferred dense-exact table schedule via the step hook",
           "value": round(B * M * steps / dt, 1), "unit": "samples/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "prime_steps": prime,
           "adam_steady_state": steady_state(prime, warmup, b.D.sweep_every if b is not None
                                             and b.D is not None else None),
           "schedule": "deferred" if b is not None and b.D is not None else "dense",
           "final_loss": round(float(loss.detach()), 6),
           "calling_thread_backward": {"ms_per_step": round(dt_ct / steps * 1e3, 4),
                                       "value": round(B * M * steps / dt_ct, 1), "steps": steps,
                                       "note": "the same loop under torch.autograd."
                                               "set_multithreading_enabled(False), as "
                                               "ncf_amd.trainer.Trainer.train_epoch runs it"},
           "with_loss_item": {"ms_per_step": round(dt_item / n_item * 1e3, 4),
                              "value": round(B * M * n_item / dt_item, 1), "steps": n_item,
                              "note": "plus loss.item() every batch (trainer.py:289)"},
           "phases": breakdown,
           "phases_note": f"{nb} steps after the timed ones; host_us = the Python call, gpu_us = "
                          "stream time between torch events at the phase boundaries"}
    del m, opt, feats
    torch.cuda.empty_cache()
    return out


def bf16_train(ncf, dev, cfg, batches, warmup, steps, prime=0):
    """The C2 configuration as BASELINE.json configs[1] states it ("bf16"; SURVEY 8(d): tables
    bf16, Adam moments fp32): the same step as the headline with the four tables held as bf16
    (FusedTrainStep(table_dtype=torch.bfloat16)); every other tensor and all arithmetic fp32.
    A separate, labelled line: the fp32 step is the parity path and the headline."""
    from ncf_amd.trainer import FusedTrainStep
    U, I, D, T, H, hid, B, M = cfg
    torch.manual_seed(1234)
    m = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, table_dtype=torch.bfloat16)

    def run(first, count):
        for s in range(first, first + count):
            u, i, t = batches[s % len(batches)]
            step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
    run(0, prime + warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(prime + warmup, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"config": "C2 with bf16 tables (fp32 Adam moments, fp32 compute), FusedTrainStep",
           "value": round(B * M * steps / dt, 1), "unit": "samples/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "prime_steps": prime,
           "adam_steady_state": steady_state(prime, warmup, step.deferred.sweep_every),
           "table_bytes": 2 * (U + I) * D * 2, "final_loss": round(float(step.last_loss.item()), 6),
           "tolerance": "vs fp32 oracle: loss within 1% per step over 100 steps, eval prob "
                        "abs <= 2e-2 (tests/test_gpu_bf16.py)"}
    del step, m
    torch.cuda.empty_cache()
    return out


C4 = dict(U=50_000_000, I=5_000_000, D=128, T=32, H=4, hid=[256, 128, 64], B=4096, M=5)


def c4_train(ncf, dev, warmup, steps, prime=0):
    """BASELINE.json configs[3] / SURVEY 8(d) C4 on ONE MI355X: 50M users x 5M items, D=128,
    H=4 (hd 32), MLP [256,128,64], B=4096 groups x M=5.  The four fp32 tables (56.3 GB) and
    their Adam moments (112.6 GB) are resident in one GPU's 288 GB HBM, built there directly
    (torch.device context: no 56 GB host staging).  Same step as the headline (FusedTrainStep:
    forward, fused BCE, backward, deferred dense-exact Adam over all 14.08B table parameters),
    timed after the deferred schedule's steady-state warm-up.  D = 128 runs the fused attention
    block (8 groups per workgroup) and the fused MLP tower (128-wide input)."""
    from ncf_amd import _lib as L
    from ncf_amd.trainer import FusedTrainStep
    c = C4
    U, I, D, T, H, hid, B, M = c["U"], c["I"], c["D"], c["T"], c["H"], c["hid"], c["B"], c["M"]
    torch.manual_seed(4444)
    t0 = time.perf_counter()
    with torch.device(dev):
        model = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    batches = make_batches(U, I, B, M, 8, dev, seed=777)
    # ids at the top of both id ranges (int64 row offsets past 2^31 elements)
    batches[0][0][:M] = U - 1
    batches[0][1][:3] = torch.tensor([I - 1, I - 2, 0], device=dev)

    def run(first, count):
        for s in range(first, first + count):
            u, i, t = batches[s % len(batches)]
            step(u, i, t, next=batches[(s + 1) % len(batches)][:2])
    run(0, prime + warmup)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    run(prime + warmup, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - ta
    loss = float(step.last_loss.item())
    L.PROFILE = []
    for s in range(prime + warmup + steps, prime + warmup + steps + 20):
        u, i, t = batches[s % len(batches)]
        step(u, i, t)
    torch.cuda.synchronize()
    prof, L.PROFILE = L.PROFILE, None
    per = {}
    for name, _, e0, e1 in prof:
        per[name] = per.get(name, 0.0) + e0.elapsed_time(e1) / 20
    # The same kernels with the rolling sweep on the step's own stream: overlapped, the sweep
    # (the C4 step's bound on one GPU: 14.08B table parameters) holds the CUs the Linear kernels
    # wait for, so their in-step spans above measure the sweep, not them
    dfr = step.deferred
    iso = {}
    if dfr is not None and getattr(dfr, "overlap", False):
        dfr.overlap = False
        L.PROFILE = []
        for s in range(prime + warmup + steps + 20, prime + warmup + steps + 30):
            u, i, t = batches[s % len(batches)]
            step(u, i, t)
        torch.cuda.synchronize()
        prof, L.PROFILE = L.PROFILE, None
        for name, _, e0, e1 in prof:
            iso[name] = iso.get(name, 0.0) + e0.elapsed_time(e1) / 10
        # the table Adam's exact work from the stamps (sweep on the step's stream)
        acct = table_adam_accounting(step, batches, prime + warmup + steps + 30, 4, dfr, D)
        dfr.overlap = True
    else:
        acct = None
    lin = ("ncf_attn_block_fwd", "ncf_attn_block_bwd", "ncf_mlp_fwd", "ncf_mlp_bwd",
           "ncf_mlp_fwd_split", "ncf_mlp_bwd_split",
           "ncf_gemm_rows", "ncf_gemm_f32", "ncf_wgrad_grouped", "ncf_relu_ln_dropout_fwd",
           "ncf_relu_ln_dropout_bwd", "ncf_attention_fwd", "ncf_attention_bwd")
    mem = torch.cuda.max_memory_allocated(dev)
    out = {"config": "C4: 50M users x 5M items, D=128, H=4, MLP [256,128,64], T=32, B=4096 x M=5, "
                     "dropout 0.2, Adam lr 1e-3 wd 1e-5 (dense-exact, deferred), 1 GPU",
           "value": round(B * M * steps / dt, 1), "unit": "samples/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "prime_steps": prime,
           "adam_steady_state": steady_state(prime, warmup, step.deferred.sweep_every),
           "table_params": 2 * (U + I) * D, "hbm_peak_GB": round(mem / 1e9, 1),
           "build_s": round(build_s, 1), "final_loss": round(loss, 6),
           "finite": bool(math.isfinite(loss)),
           # per-launch kernel times: measured with the rolling sweep on the step's own stream,
           # where a launch's event span is its own kernel's
           "kernel_ms_per_step": {
               k: round(v, 4) for k, v in sorted(iso.items(), key=lambda x: -x[1])},
           # the default (overlapped) step: event spans on the launching stream while the sweep
           # runs beside it on another — the time a launch's stream waited, not its kernel time
           "launch_span_ms_per_step_overlapped": {
               k: round(v, 4) for k, v in sorted(per.items(), key=lambda x: -x[1])},
           "linear_ms_per_step": round(sum(v for k, v in iso.items() if k in lin), 4),
           "linear_kernels": "fused attention block + fused MLP tower (D = 128)"
           if "ncf_attn_block_fwd" in iso and ("ncf_mlp_fwd" in iso or "ncf_mlp_fwd_split" in iso)
           else "unfused",
           "table_adam_roofline": table_adam_roofline(acct, D) if acct else None}
    del step, model, batches
    torch.cuda.empty_cache()
    return out


def c5_scoring(dev, n_users, n_items, n_query, ks, cpu_budget, world=1, rank=0):
    """C5 (BASELINE.json configs[4]): n_query users x n_items top-K with the factorised MFMA
    scorer (ncf_amd.scoring), timed with inputs resident; plus the reference serving path
    (forward_simple over items) on the CPU oracle for a bounded slice.  With world > 1 the
    catalogue is item-sharded: each rank scans its 1/W of the items, the per-rank
    top-K lists are all-gathered and merged (fixed total work: strong scaling); the time is the
    max over ranks."""
    import ncf_amd
    from ncf_amd import _lib as L
    from ncf_amd.scoring import SPLIT_SCAN, SPLIT_TERMS, ItemIndex, shard_items, sharded_score_topk
    torch.manual_seed(4321)
    m = ncf_amd.AdvancedNCF(n_users, n_items, 10, 50).to(dev).eval()
    users = torch.randperm(n_users, device=dev)[:n_query]
    shard = shard_items(n_items, world, rank) if world > 1 else None
    n_local = n_items if shard is None else shard.numel()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx = ItemIndex(m, items=shard)
    torch.cuda.synchronize()
    index_cold_ms = (time.perf_counter() - t0) * 1e3
    # the rebuild a parameter change costs (GraphedScorer rebuilds on every model update): the
    # first build above also pays first-use allocations and code-object loads
    t0 = time.perf_counter()
    idx = ItemIndex(m, items=shard)
    torch.cuda.synchronize()
    index_ms = (time.perf_counter() - t0) * 1e3
    # the rebuild's launches with HIP events: its roofline.  Per item it runs
    # the eval forward with M = 1 (attention: v and out projections, 2 x 2 D^2 flop; tower + head
    # 2 (D h1 + h1 h2 + h2 h3)), the GMF row's LayerNorm, the bias and the bf16 split planes
    L.PROFILE = []
    idx = ItemIndex(m, items=shard)
    torch.cuda.synchronize()
    iprof, L.PROFILE = L.PROFILE, None
    ims = {}
    for name, _, e0, e1 in iprof:
        ims[name] = ims.get(name, 0.0) + e0.elapsed_time(e1)
    D_ = 64
    mlp_f_ = 2.0 * (D_ * 256 + 256 * 128 + 128 * 64)
    idx_flops = n_local * (4.0 * D_ * D_ + mlp_f_)
    idx_tf = idx_flops / (index_ms * 1e-3) / 1e12
    mf_ms = ims.get("ncf_mlp_fwd", 0.0) + ims.get("ncf_mlp_fwd_split", 0.0)
    mf_tf = n_local * mlp_f_ / (mf_ms * 1e-3) / 1e12 if mf_ms else 0.0
    item_index = {"ms": round(index_ms, 3), "first_build_ms": round(index_cold_ms, 3),
                  "kernel_ms": {k: round(v, 4) for k, v in sorted(ims.items(), key=lambda x: -x[1])},
                  "flops": idx_flops,
                  "roofline": {"bound": "mfma", "kernel": "k_mlp_fwd (item tower, M = 1)",
                               "achieved": round(mf_tf, 2), "peak": FP32_MFMA_PEAK_TFS,
                               "unit": "TFLOP/s", "frac": round(mf_tf / FP32_MFMA_PEAK_TFS, 4),
                               "ms": round(mf_ms, 4)},
                  "whole_build": {"achieved": round(idx_tf, 2), "peak": FP32_MFMA_PEAK_TFS,
                                  "unit": "TFLOP/s", "frac": round(idx_tf / FP32_MFMA_PEAK_TFS, 4),
                                  "note": "all item-side flops / the rebuild's wall time"}}

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt)
        return dt

    out = {"config": f"{n_query} users x {n_items} items (model {n_users} x {n_items}, D=64), "
                     "top-K over the whole catalogue, factorised fp32-accurate MFMA scan "
                     + (f"(bf16 matrix cores, {SPLIT_TERMS}-term operand split"
                        + (", candidates re-scored in fp32)" if SPLIT_TERMS < 3 else ")")
                        if SPLIT_SCAN else "(fp32 MFMA)")
                     + ", hipGraph-captured"
                     + (f", item-sharded over {world} GPUs (all-gather + merge)" if world > 1 else ""),
           "scaling": "strong", "n_gpus": world, "item_index_ms": round(index_ms, 3),
           "item_index_first_build_ms": round(index_cold_ms, 3), "item_index": item_index}
    for k in ks:
        # the served form: the per-shard pipeline captured once as a hipGraph and replayed
        # (GraphedScorer); the eager launches are timed beside it with per-launch HIP events
        # for the scan kernel's roofline
        sharded_score_topk(m, users, k, idx, graph=True)
        torch.cuda.synchronize()
        best = min(timed(lambda: sharded_score_topk(m, users, k, idx, graph=True))
                   for _ in range(3))
        sharded_score_topk(m, users, k, idx)
        torch.cuda.synchronize()
        eager, prof = 1e9, None
        for _ in range(3):
            L.PROFILE = []
            dt = timed(lambda: sharded_score_topk(m, users, k, idx))
            if dt < eager:
                eager, prof = dt, L.PROFILE
            L.PROFILE = None
        kname = "ncf_score_collect_split" if SPLIT_SCAN else "ncf_score_collect"
        # (mean over the k = 10 and k = 100 launches of the profiled micro-benchmark)
        ctraffic = pmc_traffic("k_collect3" if SPLIT_SCAN else "k_collect")
        coll = sum(e0.elapsed_time(e1) for name, _, e0, e1 in prof if name == kname)
        algo_tf = 2.0 * 64 * n_query * n_local / (coll * 1e-3) / 1e12   # 128 flop per pair
        if SPLIT_SCAN:
            # executed matrix work: the bf16 products of the operand splits per pair (1 term:
            # a0b0; 2 terms: a0b0 + a0b1 + a1b0; 3 terms: six)
            nprod = {1: 1, 2: 3, 3: 6}[SPLIT_TERMS]
            tf, peak = nprod * algo_tf, BF16_MFMA_PEAK_TFS
            kdesc = f"k_collect3 (v_mfma_f32_32x32x16_bf16, {nprod} split products per pair)"
        else:
            tf, peak = algo_tf, FP32_MFMA_PEAK_TFS
            kdesc = "k_collect (v_mfma_f32_32x32x2_f32)"
        out[f"k{k}"] = {"ms": round(best * 1e3, 3), "pairs_per_s": round(n_query * n_items / best, 1),
                        "launch": "hipGraph replay (GraphedScorer)",
                        "eager_ms": round(eager * 1e3, 3), "collect_ms": round(coll, 3),
                        "roofline": {"bound": "mfma", "kernel": kdesc,
                                     "achieved": round(tf, 2), "peak": peak,
                                     "unit": "TFLOP/s", "frac": round(tf / peak, 4),
                                     "flops_per_pair": 128 * (nprod if SPLIT_SCAN else 1),
                                     "traffic": ctraffic["bytes_per_launch"] if ctraffic else None,
                                     "traffic_source": ctraffic["source"] if ctraffic else None,
                                     "algorithmic_tflops": round(algo_tf, 2),
                                     "algorithmic_frac_of_fp32_peak":
                                         round(algo_tf / FP32_MFMA_PEAK_TFS, 4)}}
    if cpu_budget > 0 and rank == 0 and world == 1:
        # the reference serving path (app.py:43-77: forward_simple over the items,
        # then nlargest) on the CPU oracle for a 100-user slice, extrapolated linearly to the
        # whole 10K x 1M job and labelled so.  Each user scores a 100K-item slice of the
        # catalogue (the literal per-pair forward is ~1 us per pair on the host); stops early
        # when the time budget runs out and extrapolates from the users done.
        from oracle import ncf_oracle as O
        threads, cpu_model = host_cpu()
        torch.set_num_threads(threads)
        p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        n_cpu = min(n_items, 100_000)
        items = torch.arange(n_cpu)
        ucpu = users[:100].cpu()
        with torch.no_grad():     # warm-up
            O.forward_simple(p, torch.full((n_cpu,), int(ucpu[0]), dtype=torch.int64), items,
                             num_heads=4, temporal_dim=32, n_layers=3)
        done = 0
        t0 = time.perf_counter()
        with torch.no_grad():
            for uu in ucpu.tolist():
                sc = O.forward_simple(p, torch.full((n_cpu,), uu, dtype=torch.int64), items,
                                      num_heads=4, temporal_dim=32, n_layers=3)
                torch.topk(sc.reshape(-1), max(ks))
                done += 1
                if time.perf_counter() - t0 > cpu_budget:
                    break
        dt = time.perf_counter() - t0
        rate = done * n_cpu / dt
        out["cpu_baseline"] = {"value": round(rate, 1), "unit": "pairs/s", "cores": threads,
                               "kind": "port", "cpu_model": cpu_model,
                               "sample": f"oracle forward_simple + topk({max(ks)}) (the reference "
                                         f"serving path, literal per-pair forward) for {done} "
                                         f"users x {n_cpu} items, {threads} threads",
                               "extrapolated_full_job_s": round(n_query * n_items / rate, 1),
                               "extrapolated_note": f"linear extrapolation to {n_query} users x "
                                                    f"{n_items} items (labelled: not run)"}
    del m, idx
    torch.cuda.empty_cache()
    return out


CATCHUP_NAMES = ("ncf_adam_pairs_catchup_claim_clock", "ncf_adam_pairs_catchup_clock")


def table_adam_accounting(step_fn, batches, first, n, dfr, D):
    """The deferred table Adam's exact work over n steps, from the per-row stamps: before and
    after each step (host syncs; a separate region, the sweep on the step's own stream) the
    stamp arrays are read, so every row's replayed / applied steps are counted.  A touched row
    (in the batch) takes (delta - 1) zero-gradient steps in the catch-up and one gradient step in
    the apply; any other row whose stamp moved was replayed by the rolling sweep.  Each row step
    is 2 D element-steps (the GMF and MLP tables of the kind).  Kernel times: HIP events around
    each launch.  Returns {part: (element_steps per step, ms per step)}."""
    from ncf_amd import _lib as L
    es = {"catchup": 0, "apply": 0, "sweep": 0}
    ms = {}
    for s_ in range(first, first + n):
        u, i, t = batches[s_ % len(batches)]
        torch.cuda.synchronize()
        s0 = {k: v.clone() for k, v in dfr.stamp.items()}
        L.PROFILE = []
        step_fn(u, i, t)
        torch.cuda.synchronize()
        prof, L.PROFILE = L.PROFILE, None
        for name, _, e0, e1 in prof:
            ms[name] = ms.get(name, 0.0) + e0.elapsed_time(e1)
        for kind, ids in (("user", u), ("item", i)):
            d = (dfr.stamp[kind] - s0[kind]).long()
            touched = torch.zeros(d.numel(), dtype=torch.bool, device=d.device)
            touched[ids.reshape(-1)] = True
            es["apply"] += int(touched.sum())
            es["catchup"] += int((d[touched] - 1).clamp_min(0).sum())
            es["sweep"] += int(d[~touched].sum())
        del s0
    kms = {"catchup": sum(ms.get(k, 0.0) for k in CATCHUP_NAMES),
           "apply": ms.get("ncf_adam_pairs_apply_clock", 0.0),
           "sweep": ms.get("ncf_adam_pairs_sweep_rolling", 0.0)}
    return {k: (es[k] * 2 * D / n, kms[k] / n) for k in es}


def table_adam_roofline(acct, D):
    """VALU-issue roofline of the replay kernels (catch-up, rolling sweep: zero-gradient
    element-steps x ADAM_REPLAY_SLOTS lane issue slots each, against VALU_SLOTS_PEAK_T) and the
    HBM roofline of the apply (per touched element: p, m, v read and written + the gradient
    read = 28 B)."""
    slots = ADAM_REPLAY_SLOTS[D]
    out = {}
    for k in ("catchup", "sweep"):
        n_es, t_ms = acct[k]
        a = n_es * slots / (t_ms * 1e-3) / 1e12 if t_ms > 0 else 0.0
        out[k] = {"bound": "valu", "element_steps": int(n_es), "ms": round(t_ms, 4),
                  "achieved": round(a, 2), "peak": VALU_SLOTS_PEAK_T, "unit": "T lane-slots/s",
                  "frac": round(a / VALU_SLOTS_PEAK_T, 4)}
    n_es, t_ms = acct["apply"]
    gbs = n_es * 28.0 / (t_ms * 1e-3) / 1e9 if t_ms > 0 else 0.0
    out["apply"] = {"bound": "hbm", "element_steps": int(n_es), "ms": round(t_ms, 4),
                    "bytes": int(n_es * 28), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    z_es = acct["catchup"][0] + acct["sweep"][0]
    z_ms = acct["catchup"][1] + acct["sweep"][1]
    a = z_es * slots / (z_ms * 1e-3) / 1e12 if z_ms > 0 else 0.0
    out["replay"] = {"bound": "valu", "achieved": round(a, 2), "peak": VALU_SLOTS_PEAK_T,
                     "unit": "T lane-slots/s", "frac": round(a / VALU_SLOTS_PEAK_T, 4),
                     "element_steps": int(z_es), "ms": round(z_ms, 4),
                     "slots_per_element_step": slots,
                     "slots_source": "tools/isa_replay_count.py (gfx950 ISA of the replay loop: "
                                     "plain VALU 1, packed 2, transcendental 4 slots)"}
    out["element_steps_per_step"] = int(z_es + n_es)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the deferred table Adam reaches steady state after 2 x sweep_every (= 256) steps: before
    # that its rolling sweep replays fewer zero-gradient steps per row than it will later, so
    # the default warm-up covers that transient and the timed region spans >= 3 sweep cycles
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prime", type=int, default=-1,
                    help="untimed priming steps before the warm-up of every training leg "
                         "(default 2 x sweep_every = 256: deferred-Adam steady state)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="test the --gpus N launcher: ranks join a gloo group and report (no GPU)")
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--groups", type=int, default=4096, help="interaction groups per GPU per step")
    ap.add_argument("--batches", type=int, default=N_BATCHES,
                    help="distinct resident batches the timed legs cycle through")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--infer-pairs", type=int, default=65536)
    ap.add_argument("--no-score", action="store_true", help="skip the C5 scoring measurement")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the reference-call-pattern (model + torch.optim.Adam) line")
    ap.add_argument("--no-clock", action="store_true",
                    help="host-driven Adam step arguments instead of the device step clock")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a captured hipGraph (measured ~3%% slower than host "
                         "launches on MI355X: the host enqueue is already below the GPU time)")
    ap.add_argument("--score-users", type=int, default=10_000)
    ap.add_argument("--score-items", type=int, default=1_000_000)
    ap.add_argument("--sharded", action="store_true",
                    help="use the row-sharded DP step even at world size 1 (exercises the N>1 path)")
    ap.add_argument("--config", default="c2", choices=("c2", "c4"),
                    help="c4: only the C4 (50M x 5M, D=128) training line on one GPU")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 line of the default run")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the B=256, C1 and large-batch embedding lines")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here before anything touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dry_launch))
    if args.dry_launch:
        dry_launch()
        return
    prime = prime_steps(args)
    if args.config == "c4":
        torch.cuda.set_device(0)
        ncf = _ncf_pkg.load()
        rec = c4_train(ncf, torch.device("cuda", 0), args.warmup, args.steps, prime)
        print(json.dumps({"metric": METRIC, **rec, "n_gpus": 1, "higher_is_better": True,
                          "dtype": "fp32", "data": "synthetic (users uniform, items Zipf(1.05))"}),
              flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr,
              flush=True)
    sharded = world > 1 or args.sharded
    if sharded:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ncf = _ncf_pkg.load()
    from ncf_amd.trainer import FusedTrainStep

    U, I, D, T, H, hid = args.users, args.items, 64, 32, 4, [256, 128, 64]
    B, M = args.groups, 5
    N = B * M
    torch.manual_seed(1234)
    init_sd = None
    if sharded:
        # row-sharded tables (owner = id mod W) + replicated dense params; RCCL all-to-alls
        from ncf_amd.distributed import make_sharded_step

        def factory(ru, ri):
            torch.manual_seed(1234 + rank)
            return ncf.AdvancedNCF(ru, ri, 10, 50, D, D, T, hid, H, 0.2, M - 1).to(dev).train()
        model, step = make_sharded_step(factory, U, I, lr=1e-3, weight_decay=1e-5)
    else:
        model = ncf.AdvancedNCF(U, I, 10, 50, D, D, T, hid, H, 0.2, M - 1)
        if rank == 0 and not args.no_cpu_baseline:
            init_sd = {k: v.clone() for k, v in model.state_dict().items()}
        model = model.to(dev).train()
        step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, graph=args.graph,
                              clock=False if args.no_clock else None)
    batches = make_batches(U, I, B, M, args.batches, dev, seed=100 + rank)
    torch.cuda.synchronize()

    # the single-GPU step sorts the next batch's ids on a side stream under the current step
    # (FusedTrainStep(next=...)); the instrumented eager pass below does not
    pipelined = not sharded and not args.graph and not args.no_clock

    def run_steps(fn, first, count):
        """count steps over the resident batches from index `first`; the row-sharded step plans
        the following batch under each step (pipelined input distribution)."""
        for s in range(first, first + count):
            u, i, t = batches[s % len(batches)]
            if sharded or (pipelined and fn is step):
                fn(u, i, t, next=batches[(s + 1) % len(batches)][:2])
            else:
                fn(u, i, t)

    # --- priming (deferred-Adam steady state) + warm-up
    run_steps(step, 0, prime + args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(step, prime + args.warmup, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_step = elapsed / args.steps * 1e3
    # the same timed region cycling over 8 of the resident batches (the round-3 headline's
    # reuse cycle, whose rows and Adam state fit the 256 MB Infinity Cache), reported beside
    # the headline once
    cyc8 = None
    if not sharded:
        b8 = batches[:8]
        torch.cuda.synchronize()
        t8 = time.perf_counter()
        for s_ in range(args.steps):
            u, i, t = b8[s_ % 8]
            if pipelined:
                step(u, i, t, next=b8[(s_ + 1) % 8][:2])
            else:
                step(u, i, t)
        torch.cuda.synchronize()
        dt8 = time.perf_counter() - t8
        cyc8 = {"ms_per_step": round(dt8 / args.steps * 1e3, 4),
                "value": round(N * args.steps / dt8, 1),
                "note": "same step cycling over 8 resident batches (round 3's bench); the "
                        f"headline cycles over {args.batches} distinct batches"}
    samples_s = N * world * args.steps / elapsed
    last = step.ops.last_loss if sharded else step.last_loss
    loss = float(last.item()) if last is not None else float("nan")
    # second timed region, same K steps, with live per-launch HIP events (torch events on the
    # stream the kernels run on) around every C-ABI call: per-kernel durations for the roofline.
    # Kept separate because recording 2 events per launch costs host time that would otherwise
    # leak into the headline number.
    from ncf_amd import _lib as L
    L.PROFILE = []
    torch.cuda.synchronize()
    # the headline's own launch sequence (the pipelined step: the next batch sorted ahead, the
    # sorted catch-up); with --graph the eager launches a replay runs (a graph cannot be
    # instrumented per launch)
    run = step.eager if (args.graph and hasattr(step, "eager")) else step
    run_steps(run, prime + args.warmup + args.steps, args.steps)
    torch.cuda.synchronize()
    prof, L.PROFILE = L.PROFILE, None

    # per-entry-point GPU time; roofline of the dominant kernel class
    per = {}
    for name, a, e0, e1 in prof:
        per.setdefault(name, []).append((a, e0.elapsed_time(e1)))
    totals = {k: sum(d for _, d in v) / args.steps for k, v in per.items()}   # ms per step
    # fp32 MFMA kernels carrying the Linear layers.  Algorithmic FLOPs (temporal
    # columns dropped): per sample 3 x 2 x (4 D^2 + D h1 + h1 h2 + h2 h3) = 442,368 at C2 =
    #   ncf_attn_block_fwd  2 x 4 D^2          (q/k/v/out projections)
    #   ncf_attn_block_bwd  2 x 8 D^2          (dO, dXu, 2 x dXi, 4 weight gradients)
    #   ncf_mlp_fwd         2 x (D h1 + h1 h2 + h2 h3)
    #   ncf_mlp_bwd         2 x (D h1 + h1 h2 + h2 h3)   (dX of the three Linears), plus the
    #                       same again for their weight gradients when computed inside it
    #   ncf_wgrad_grouped   2 x (D h1 + h1 h2 + h2 h3)   (the MLP weight gradients, unfused path)
    #   ncf_attn_mlp_fwd / _bwd: the attention block and the tower fused into one launch per
    #                       direction (tower_fused.hip, D = 64 / M = 5): the sums of the above
    # plus any unfused ncf_gemm_* launch (2 M N K, first three arguments).
    mlp_f = 2.0 * (D * hid[0] + hid[0] * hid[1] + hid[1] * hid[2])
    # (with the weight gradients fused into the tower backward, ncf_mlp_bwd carries dX + dW)
    per_sample = {"ncf_attn_block_fwd": 8.0 * D * D, "ncf_attn_block_bwd": 16.0 * D * D,
                  "ncf_mlp_fwd": mlp_f, "ncf_mlp_fwd_split": mlp_f,
                  "ncf_mlp_bwd": mlp_f if "ncf_wgrad_grouped" in totals else 2.0 * mlp_f,
                  "ncf_mlp_bwd_split": 2.0 * mlp_f,
                  "ncf_wgrad_grouped": mlp_f,
                  "ncf_attn_mlp_fwd": 8.0 * D * D + mlp_f,
                  "ncf_attn_mlp_bwd": 16.0 * D * D + 2.0 * mlp_f,
                  "ncf_attn_mlp_fwd_small": 8.0 * D * D + mlp_f,
                  "ncf_attn_mlp_bwd_small": 16.0 * D * D + 2.0 * mlp_f}
    gemm_names = ("ncf_gemm_direct", "ncf_gemm_f32", "ncf_gemm_rows", "ncf_gemm_f32_splitk")
    mfma = {}
    for k, f in per_sample.items():
        if k in totals:
            fl = f * N
            mfma[k] = {"ms": round(totals[k], 4), "gflop": round(fl / 1e9, 4),
                       "tflops": round(fl / (totals[k] * 1e-3) / 1e12, 2)}
    gemm_ms = sum(totals.get(k, 0.0) for k in per_sample) + sum(totals.get(k, 0.0) for k in gemm_names)
    gemm_flops = sum(f * N for k, f in per_sample.items() if k in totals) + sum(
        2.0 * a[0] * a[1] * a[2] for k in gemm_names for a, _ in per.get(k, [])) / args.steps
    gemm_launches = sum(len(per.get(k, [])) for k in list(per_sample) + list(gemm_names)) / args.steps
    achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12
    # the dominant MFMA kernel by time: its own roofline (per launch)
    dom = max(mfma, key=lambda k: mfma[k]["ms"]) if mfma else None
    dom_launches = len(per.get(dom, [])) / args.steps if dom else 0
    dom_ms = totals[dom] / max(dom_launches, 1) if dom else 0.0
    dom_flops = per_sample[dom] * N / max(dom_launches, 1) if dom else 0.0
    dom_tf = dom_flops / (dom_ms * 1e-3) / 1e12 if dom else 0.0
    traffic = pmc_traffic(KERNEL_SYMBOL.get(dom)) if dom else None
    # The rolling table sweep runs on a side stream beside the backward (deferred.py, overlapped
    # sweep): the times above are the kernels as they run in the step, sharing the CUs with it.
    # The dominant kernel alone: a short third region with the sweep back on the step's stream.
    iso = None
    dfr0 = getattr(step, "deferred", None)
    if dom and dfr0 is not None and getattr(dfr0, "overlap", False):
        dfr0.flush(L.stream_ptr(dev))
        dfr0.overlap = False
        L.PROFILE = []
        run_steps(run, prime + args.warmup + 2 * args.steps, ISO_STEPS)
        torch.cuda.synchronize()
        prof2, L.PROFILE = L.PROFILE, None
        dfr0.overlap = True
        ds = [e0.elapsed_time(e1) for name, _, e0, e1 in prof2 if name == dom]
        if ds:
            iso_ms = sum(ds) / len(ds)
            iso_tf = dom_flops / (iso_ms * 1e-3) / 1e12
            iso = {"ms_per_launch": round(iso_ms, 4), "achieved": round(iso_tf, 2),
                   "frac": round(iso_tf / FP32_MFMA_PEAK_TFS, 4), "steps": ISO_STEPS,
                   "note": "the same kernel with the rolling sweep on the step's own stream "
                           "(not overlapped)"}
    adam_rf = None
    if dfr0 is not None and getattr(dfr0, "clock", None) is not None and not sharded:
        dfr0.flush(L.stream_ptr(dev))
        ov = dfr0.overlap
        dfr0.overlap = False
        acct = table_adam_accounting(run, batches, prime + args.warmup + 2 * args.steps + ISO_STEPS,
                                     8, dfr0, D)
        dfr0.overlap = ov
        adam_rf = table_adam_roofline(acct, D)
        adam_rf["note"] = ("8 steps with the rolling sweep on the step's own stream, per-row "
                           "stamps read before and after each (exact element-steps)")
    # table-update work of the deferred dense-exact Adam: algorithmic = the dense schedule's
    # 24 B per table element per step (what the reference's Adam must move), priced per step
    tab_ms = sum(totals.get(k, 0.0) for k in ("ncf_adam_rows_catchup", "ncf_adam_rows_apply",
                                                "ncf_adam_sweep", "ncf_adam_table",
                                                "ncf_adam_rows_catchup_clock",
                                                "ncf_adam_rows_apply_clock",
                                                "ncf_adam_sweep_rolling",
                                                "ncf_adam_pairs_catchup_clock",
                                                "ncf_adam_pairs_catchup_claim_clock",
                                                "ncf_adam_pairs_catchup_lock_clock",
                                                "ncf_adam_pairs_apply_clock",
                                                "ncf_adam_pairs_sweep_rolling"))
    sweep_ms = sum(totals.get(k, 0.0) for k in ("ncf_adam_pairs_sweep_rolling",
                                                "ncf_adam_sweep_rolling", "ncf_adam_sweep"))
    dfr = step.deferred if hasattr(step, "deferred") else getattr(
        getattr(step, "ops", None), "deferred", None)
    sweep_every = int(dfr.sweep_every) if dfr is not None else None
    # steady state: every stamp has been refreshed by a full sweep cycle after the first one
    # (rows start at stamp 0, so during steps < 2 x sweep_every a swept slice replays fewer
    # zero-gradient steps than later)
    steady = steady_state(prime, args.warmup, sweep_every)
    # embedding gather / scatter: algorithmic HBM bytes per launch
    #   gather  (ncf_gather_ln_gmf_scaled_fwd): 4 rows of D fp32 + 2 int64 ids in, 4 LN'd rows
    #           (MLP + GMF, training) + mf_pred out = N (16 D + 16 + 16 D + 4)
    #   scatter (ncf_embedding_bwd_reduce): 4 gradient rows in per sample, per unique row the 2
    #           table rows (LN recompute) in and 2 compact gradient rows out = N (16 D + 16) +
    #           (n_u + n_i) 16 D
    nu_ni = None
    grows = 0
    try:
        ws_any = next(iter(model.engine.ws.values()))
        nu_ni = [int(x) for x in ws_any.num_unique.cpu().tolist()]
        grows = int(getattr(ws_any, "group_rows", 0))
    except Exception:
        pass
    hbm = embedding_rooflines(totals, per, args.steps, N, D, grows, nu_ni)
    # --- inference pairs/s: eval forward (M = 1) on resident pairs
    model.eval()
    npairs = args.infer_pairs
    g = torch.Generator(device=dev).manual_seed(9)
    iu = torch.randint(0, model.num_users, (npairs,), generator=g, device=dev)
    ii = torch.randint(0, model.num_products, (npairs,), generator=g, device=dev)
    eng = model.engine
    with torch.no_grad():
        for _ in range(3):
            eng.forward(iu, ii, 1, False, 0.0, 0)
        torch.cuda.synchronize()
        ti = time.perf_counter()
        reps = 20
        for _ in range(reps):
            eng.forward(iu, ii, 1, False, 0.0, 0)
        torch.cuda.synchronize()
        infer_s = (time.perf_counter() - ti) / reps
    infer_pairs = npairs * world / infer_s
    # per-launch profile of the eval forward (HIP events around each C-ABI call)
    L.PROFILE = []
    with torch.no_grad():
        for _ in range(reps):
            eng.forward(iu, ii, 1, False, 0.0, 0)
    torch.cuda.synchronize()
    prof_i, L.PROFILE = L.PROFILE, None
    inf_ms = {}
    for name, _, e0, e1 in prof_i:
        inf_ms[name] = inf_ms.get(name, 0.0) + e0.elapsed_time(e1) / reps
    # algorithmic work per pair of the executed eval path (M = 1: softmax of one key is 1, so
    # the attention output is out_proj(v_proj(x_item)); q / k projections are dead math and not
    # executed): gather 4 D-float rows + 2 int64 ids in, 2 LN'd MLP rows + mf_pred out; the
    # attention block 2 x 2 D^2 flop; the tower + head 2 (D h1 + h1 h2 + h2 h3) flop
    inf_work = {"ncf_gather_ln_gmf_scaled_fwd": ("hbm", npairs * (16 * D + 16 + 8 * D + 4)),
                "ncf_attn_block_fwd": ("mfma", npairs * 4.0 * D * D),
                "ncf_mlp_fwd": ("mfma", npairs * mlp_f),
                "ncf_mlp_fwd_split": ("mfma", npairs * mlp_f)}
    inf_k = {}
    for name, (bound, work) in inf_work.items():
        if name in inf_ms:
            t_ = inf_ms[name] * 1e-3
            if bound == "hbm":
                a = work / t_ / 1e9
                inf_k[name] = {"bound": "hbm", "ms": round(inf_ms[name], 4), "bytes": int(work),
                               "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(a / HBM_PEAK_GBS, 4)}
            else:
                a = work / t_ / 1e12
                inf_k[name] = {"bound": "mfma", "ms": round(inf_ms[name], 4), "flops": work,
                               "achieved": round(a, 2), "peak": FP32_MFMA_PEAK_TFS,
                               "unit": "TFLOP/s", "frac": round(a / FP32_MFMA_PEAK_TFS, 4)}
    inf_dom = max(inf_k, key=lambda k: inf_k[k]["ms"]) if inf_k else None
    infer = {"pairs_per_s": round(infer_pairs, 1), "ms_per_call": round(infer_s * 1e3, 4),
             "pairs_per_call": npairs,
             "roofline": dict(inf_k[inf_dom], kernel=KERNEL_SYMBOL.get(inf_dom, inf_dom),
                              entry_point=inf_dom) if inf_dom else None,
             "kernels": inf_k,
             "flops_per_pair": 4.0 * D * D + mlp_f,
             "kernel_ms_per_call": {k: round(v, 4) for k, v in inf_ms.items()}}
    if init_sd is not None:
        infer["cpu_baseline"] = cpu_infer_baseline(init_sd, iu.cpu(), ii.cpu(), H, T,
                                                   len(hid), args.cpu_budget)

    dropin = None
    if not sharded and not args.no_dropin:
        dropin = dropin_train(ncf, dev, (U, I, D, T, H, hid, B, M), batches, args.warmup,
                              args.steps, prime)
        dropin["vs_fused_step"] = round(dropin["value"] / samples_s, 4)
        ct = dropin["calling_thread_backward"]
        ct["vs_fused_step"] = round(ct["value"] / samples_s, 4)

    bf16 = None
    if not sharded:
        bf16 = bf16_train(ncf, dev, (U, I, D, T, H, hid, B, M), batches, args.warmup, args.steps,
                          prime)
        bf16["vs_fp32_step"] = round(bf16["value"] / samples_s, 4)

    b256 = c1 = emb_large = None
    if not sharded and not args.no_extra:
        # the reference's default batch (config.yaml:65), C1 (configs[0]) and the embedding
        # kernels at the strong-scaling global batch on one GPU
        b256 = small_batch_train(ncf, dev, (U, I, D, T, H, hid, 256, M), args.warmup, args.steps,
                                 prime, init_sd, args.cpu_budget)
        emb_large = embedding_large(ncf, dev, (U, I, D, T, H, hid, B, M), 32768, 10, 20)
        c1 = c1_line(ncf, dev, args.warmup, args.steps, prime, args.cpu_budget,
                     init_sd is not None)

    c4 = None
    if not sharded and not args.no_c4:
        # C4 (170 GB resident) in a child process: its own allocator, nothing of it survives
        # into this one; a failure is recorded instead of costing the headline line
        import subprocess
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--config", "c4",
                                "--warmup", str(args.warmup), "--steps", str(args.steps),
                                "--prime", str(prime)],
                               capture_output=True, text=True, timeout=600)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            c4 = json.loads(line[-1]) if r.returncode == 0 and line else {
                "error": f"rc={r.returncode}", "stderr_tail": r.stderr[-800:]}
            c4.pop("metric", None)
        except subprocess.TimeoutExpired:
            c4 = {"error": "timeout"}

    cpu = None
    if init_sd is not None:
        cpu_batches = [(u.cpu(), i.cpu(), t.cpu()) for (u, i, t) in batches[:4]]
        cpu = cpu_baseline(init_sd, (U, I, D, T, H, hid, B, M), cpu_batches, args.cpu_budget)
    score = None
    if not args.no_score:
        # (C5's CPU leg: the 100-user slice SURVEY 8(d) names, ~30 s of oracle work)
        score = c5_scoring(dev, 1_000_000, args.score_items, args.score_users, (10, 100),
                           0 if args.no_cpu_baseline else 45, world=world, rank=rank)

    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(samples_s, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: users uniform, positive items Zipf(1.05), 4 uniform negatives; random-init weights",
            "config": {"workload": "C2 train step: 1M users x 100K items, D=64, H=4, MLP [256,128,64], "
                                   "T=32, dropout 0.2, Adam lr 1e-3 wd 1e-5 (dense-exact)",
                       "global_batch": N * world, "groups_per_gpu": B, "samples_per_group": M,
                       "launch": ("host launches (row-sharded step)" if sharded else
                                  "hipGraph replay of the captured step" if args.graph else
                                  "host launches"),
                       "parallelism": (f"dp{world} + row-sharded tables (RCCL all-to-all), "
                                       "dense all-reduce") if sharded else "single-gpu",
                       **({"exchange": type(step.x).__name__} if sharded else {})},
            "roofline": {"bound": "mfma", "kernel": KERNEL_SYMBOL.get(dom, dom),
                         "entry_point": dom,
                         "achieved": round(dom_tf, 2), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": round(dom_tf / FP32_MFMA_PEAK_TFS, 4),
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "flops_per_launch": dom_flops, "ms_per_launch": round(dom_ms, 4),
                         **({"matrix_cores": "bf16 (v_mfma_f32_16x16x32_bf16) on split operands: "
                                             f"{SPLIT_PRODUCTS} bf16 products per fp32 product, "
                                             "fp32-accurate; achieved/frac are fp32-equivalent "
                                             "work against the fp32 MFMA peak",
                             "executed_bf16_tflops": round(SPLIT_PRODUCTS * dom_tf, 2),
                             "executed_frac_of_bf16_peak":
                                 round(SPLIT_PRODUCTS * dom_tf / BF16_MFMA_PEAK_TFS, 4)}
                            if dom in SPLIT_NAMES else {}),
                         **({"overlap": "measured in the step, beside the rolling table sweep "
                                        "on a side stream", "isolated": iso} if iso else {})},
            "mfma_class": {"kernels": "k_attn_mlp_fwd/bwd (the attention block and the tower "
                                      "fused, D = 64) or k_attn_block_fwd/bwd + k_mlp_fwd/bwd, + "
                                      "k_wgrad_grouped when unfused "
                                      "(every Linear of the step: fp32 MFMA "
                                      "v_mfma_f32_16x16x4_f32, the tower on split-operand bf16 "
                                      "MFMA when the *_split entry points run; fp32-equivalent "
                                      "work against the fp32 MFMA peak)",
                           "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFS,
                           "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFS, 4),
                           "flops_per_step": gemm_flops, "launches_per_step": gemm_launches,
                           "per_kernel": mfma,
                         "ms_per_step": round(gemm_ms, 4)},
            "embedding_hbm": hbm,
            "adam_steady_state": steady,
            "prime_steps": prime,
            "table_adam": {"kernels": "deferred dense-exact Adam (catch-up + apply + 1/%s sweep%s)"
                                      % (sweep_every, "; the apply runs inside the embedding "
                                         "backward (ncf_embedding_bwd_reduce_apply_clock) and is "
                                         "not counted here" if "ncf_embedding_bwd_reduce_apply_clock"
                                         in totals else ""),
                           "ms_per_step": round(tab_ms, 4),
                           "sweep_us_per_step": round(1e3 * sweep_ms, 2),
                           "sweep_overlapped": bool(dfr is not None and getattr(dfr, "overlap", False)),
                           "sweep_note": "with sweep_overlapped the sweep's time is its span on the "
                                         "side stream, beside the backward kernels",
                           "sweep_every": sweep_every,
                           "steps_before_timing": prime + args.warmup,
                           "element_steps_per_step": 2 * (U + I) * D,
                           "note": "every table element takes one Adam step per step (dense-exact); "
                                   "the roofline is the replay's VALU issue rate",
                           "roofline": adam_rf},
            "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(totals.items(), key=lambda x: -x[1])},
            "cpu_baseline": cpu,
            "dropin_train": dropin,
            "infer_pairs_per_s": round(infer_pairs, 1),
            "infer_config": f"eval forward (M=1), {npairs} resident (user,item) pairs per GPU",
            "infer": infer,
            "headline_8_batch_cycle": cyc8,
            "resident_batches": args.batches,
            "c5_scoring": score,
            "c2_bf16_tables": bf16,
            "c2_b256": b256,
            "c1_train": c1,
            "embedding_hbm_large": emb_large,
            "c4_train": c4,
            "final_loss": round(loss, 6),
        }
        print(json.dumps(rec), flush=True)
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
