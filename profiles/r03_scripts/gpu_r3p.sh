#!/bin/bash
# Round-3: kernel timelines of the world-1 sharded step (sweep serial / overlapped) and the fused step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || { tail -40 "gpurun_out/$name.log"; exit $rc; }; }
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
B="python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-score --no-c4 --no-dropin"
step r3p_prof_sh 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3p_prof_sh -o run -- $B --sharded
f=$(find gpurun_out/r3p_prof_sh -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r3p_tl_sh.txt; tail -36 gpurun_out/r3p_tl_sh.txt
export MASTER_PORT=29556 NCF_SHARD_OVERLAP_SWEEP=1
step r3p_prof_shov 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3p_prof_shov -o run -- $B --sharded
f=$(find gpurun_out/r3p_prof_shov -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r3p_tl_shov.txt; tail -36 gpurun_out/r3p_tl_shov.txt
unset NCF_SHARD_OVERLAP_SWEEP RANK LOCAL_RANK WORLD_SIZE
step r3p_prof_fused 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3p_prof_fused -o run -- $B
f=$(find gpurun_out/r3p_prof_fused -name '*kernel_trace.csv' | head -1); python3 tools/prof_summary.py "$f" k_gather_ln_gmf -v > gpurun_out/r3p_tl_fused.txt; tail -30 gpurun_out/r3p_tl_fused.txt
rm -rf gpurun_out/r3p_prof_sh gpurun_out/r3p_prof_shov gpurun_out/r3p_prof_fused
