#!/bin/bash
# Round-3: world-1 sharded step, sweep serial vs overlapped: which kernels stretch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
B="python3 -u bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline --no-score --no-c4"
K="ncf_mlp_bwd ncf_mlp_fwd ncf_attn_block_fwd ncf_attn_block_bwd ncf_adam_pairs_sweep_rolling ncf_shard_plan ncf_embedding_bwd_reduce ncf_reduce_batch ncf_adam_pairs_apply_clock ncf_adam_pairs_catchup_clock ncf_shard_owner_prepare ncf_comm_alltoallv ncf_comm_allreduce_sum_f32"
MASTER_PORT=29581 step r3aa_ser 300 $B && python3 tools/bench_summ.py gpurun_out/r3aa_ser.log $K
MASTER_PORT=29582 NCF_SHARD_OVERLAP_SWEEP=1 step r3aa_ov 300 $B && python3 tools/bench_summ.py gpurun_out/r3aa_ov.log $K
